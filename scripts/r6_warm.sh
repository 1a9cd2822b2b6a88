#!/bin/bash
# FedAvg lift from a shared warm start (the reference fine-tunes a pretrained DistilBERT): calibrated profile
set -o pipefail
OUT=gpurun_out/r6warm
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --data-profile calibrated --virtual-clients 2 \
  --warm-start-epochs 1 > $OUT/calib_2x1_warm1.json.log 2> $OUT/calib_2x1_warm1.err || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --data-profile calibrated --virtual-clients 2 \
  > $OUT/calib_2x1_cold.json.log 2> $OUT/calib_2x1_cold.err || exit 1
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --data-profile calibrated --virtual-clients 8 \
  --rounds 3 --warm-start-epochs 1 > $OUT/calib_8x3_warm1.json.log 2> $OUT/calib_8x3_warm1.err || exit 1
