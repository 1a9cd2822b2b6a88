#!/bin/bash
# In-step sweep of the narrow (N = 768) GEMM tile (FD_GEMM_NARROW_CFG), interleaved
set -o pipefail
OUT=gpurun_out/${1:-r6cfg2}
mkdir -p $OUT
for i in 1 2; do
  for c in 24 0 8 18; do
    FD_GEMM_NARROW_CFG=$c timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality \
      > $OUT/cfg${c}_$i.json.log 2>&1 || exit 1
  done
done
