#!/bin/bash
# Final-code check on one lease: the GPU suite, the driver's exact bench command, and the
# distillation config (BASELINE config 5) with its quality half (3 epochs + FedAvg + eval).
set -o pipefail
OUT=gpurun_out/${1:-r6final}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 \
  || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_cmd.json.log 2> $OUT/driver_cmd.err || exit 1
grep -o '"ms_per_step": [0-9.]*' $OUT/driver_cmd.json.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 50 --warmup 10 --teacher --seq-len 256 --batch-size 64 \
  > $OUT/kd.json.log 2> $OUT/kd.err || { tail -5 $OUT/kd.err; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"aggregated_f1": [0-9.]*\|"aggregated_accuracy": [0-9.]*' $OUT/kd.json.log
