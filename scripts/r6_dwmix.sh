#!/bin/bash
# Mixed-tile all-layer dW schedule: bitwise tests, isolated subsets probe, interleaved step A/B.
set -o pipefail
OUT=gpurun_out/r6mix
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_dw_batch_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
FD_DWB_MIX=0 timeout -k 10 120 python3 scripts/dwb_tail_probe.py > $OUT/probe_plain.txt 2>&1 || exit 1
FD_DWB_MIX=1 timeout -k 10 120 python3 scripts/dwb_tail_probe.py > $OUT/probe_mixed.txt 2>&1 || exit 1
for i in 1 2; do
  for m in 0 1; do
    FD_DWB_MIX=$m timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality >> $OUT/ab_mix$m.json.log 2>&1 || exit 1
  done
done
