#!/bin/bash
# GEMM bottleneck diagnosis: timing with loads / MFMA / stores removed, plus L2 hit rate.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gdiag; mkdir -p $O
run() { timeout -k 10 120 python scripts/gemm_one.py "$@" 2>/dev/null | grep -v amdgpu.ids; }
for cfg in "nt_plain 4096 3072 768 4" "nt_plain 4096 3072 768 2" "nt_plain 4096 2304 768 2" "nt_plain 4096 768 3072 1" "nt_plain 4096 4096 4096 0" "nt_plain 4096 4096 4096 4" "nt_plain 8192 8192 8192 0"; do
  set -- $cfg
  for d in 0 1 2 4 3; do
    echo -n "diag=$d "; FD_GEMM_TILE=$5 FD_GEMM_DIAG=$d run $1 $2 $3 $4 50
  done
done | tee $O/timing.txt
for cfg in "nt_plain 4096 3072 768 4" "nt_plain 4096 3072 768 2" "nt_plain 4096 4096 4096 0"; do
  set -- $cfg
  FD_GEMM_TILE=$5 timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_$1_$3_$5 -- python3 scripts/gemm_one.py $1 $2 $3 $4 10 > $O/pmc_$1_$3_$5.log 2>&1
done
echo done
