#!/bin/bash
# In-step sweep of the wide NT GEMM tile (FD_GEMM_WIDE_CFG: QKV / FFN1 forward), interleaved
set -o pipefail
OUT=gpurun_out/${1:-r6cfg}
mkdir -p $OUT
for i in 1 2; do
  for c in -1 10 21 1 6; do
    FD_GEMM_WIDE_CFG=$c timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality \
      > $OUT/cfg${c}_$i.json.log 2>&1 || exit 1
  done
done
