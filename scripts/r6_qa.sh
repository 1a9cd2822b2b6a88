#!/bin/bash
# Fused QKV + attention forward (FD_FUSE_QKV_ATTN modes): bitwise tests, then the step A/B
# usage: scripts/r6_qa.sh <outdir> <modes...>
set -o pipefail
OUT=gpurun_out/${1:-r6qa}; shift
MODES=${@:-0 1}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_qkv_attn_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  for f in $MODES; do
    FD_FUSE_QKV_ATTN=$f timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality \
      > $OUT/ab_qa${f}_$i.json.log 2>&1 || exit 1
  done
done
