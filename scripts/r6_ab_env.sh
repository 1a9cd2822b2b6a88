#!/bin/bash
# Generic interleaved in-step A/B of one environment knob: scripts/r6_ab_env.sh <outdir> <VAR> <val...>
set -o pipefail
OUT=gpurun_out/$1; VAR=$2; shift 2
mkdir -p $OUT
for i in 1 2 3; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 120 python3 bench.py --gpus 1 --steps ${STEPS:-50} --warmup 10 --no-quality \
      > $OUT/ab_${v}_$i.json.log 2>&1 || exit 1
  done
done
