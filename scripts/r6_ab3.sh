#!/bin/bash
# next-launch weight prefetch in LN waits + plain GEMM epilogues (FD_LN_PREFETCH), loss granules: tests + A/B
set -o pipefail
OUT=gpurun_out/r6ab3
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for pf in 0 1; do
    FD_LN_PREFETCH=$pf timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality \
      > $OUT/ab_pf${pf}_$i.json.log 2>&1 || exit 1
  done
done
