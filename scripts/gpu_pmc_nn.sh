#!/bin/bash
# PMC comparison of the NN (MN-major B) and NT (K-major B) kernels on one shape.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pmcnn}; mkdir -p $O
for k in nt_plain nn; do
  FD_GEMM_CFG_NT=8 FD_GEMM_CFG_NN=8 timeout -k 10 120 python scripts/gemm_one.py $k 4096 768 3072 20 2>&1 | grep -v amdgpu.ids
  FD_GEMM_CFG_NT=8 FD_GEMM_CFG_NN=8 timeout -k 10 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/$k -- python3 scripts/gemm_one.py $k 4096 768 3072 10 > $O/$k.log 2>&1 || exit 1
  FD_GEMM_CFG_NT=8 FD_GEMM_CFG_NN=8 timeout -k 10 180 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM_RD --output-format csv -d $O/${k}_b -- python3 scripts/gemm_one.py $k 4096 768 3072 10 > $O/${k}_b.log 2>&1 || exit 1
done
echo done
