cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d in 0 1 4 5; do
 for k in nt_plain nn; do
  FD_GEMM_CFG_NT=8 FD_GEMM_CFG_NN=8 FD_GEMM_DIAG=$d timeout -k 10 60 python scripts/gemm_one.py $k 4096 768 3072 30 2>&1 | grep -v amdgpu.ids | sed "s/^/diag=$d /"
 done
done
