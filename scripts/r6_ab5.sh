#!/bin/bash
# dW mixed schedule: short-K tiles first (FD_DWB_SHORT_FIRST) vs last; isolated probe + step A/B
set -o pipefail
OUT=gpurun_out/r6ab5
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dw_batch_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
FD_DWB_SHORT_FIRST=1 timeout -k 10 300 python -u -m pytest tests/test_dw_batch_gpu.py -x -q -k mixed --timeout 120 --timeout-method thread >> $OUT/tests.log 2>&1 || exit 1
FD_DWB_SHORT_FIRST=0 timeout -k 10 120 python3 scripts/dwb_tail_probe.py > $OUT/probe_sf0.txt 2>&1 || exit 1
FD_DWB_SHORT_FIRST=1 timeout -k 10 120 python3 scripts/dwb_tail_probe.py > $OUT/probe_sf1.txt 2>&1 || exit 1
for i in 1 2 3; do
  for sf in 0 1; do
    FD_DWB_SHORT_FIRST=$sf timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality \
      > $OUT/ab_sf${sf}_$i.json.log 2>&1 || exit 1
  done
done
