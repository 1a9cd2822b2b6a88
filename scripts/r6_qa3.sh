#!/bin/bash
# per-(sequence, head) projection + attention: tests, kernel stats, step A/B against mode 0
set -o pipefail
OUT=gpurun_out/${1:-r6qa3}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_qkv_attn_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
FD_FUSE_QKV_ATTN=2 bash scripts/gpu.sh prof ${1:-r6qa3}_prof2 > /dev/null || exit 1
for i in 1 2 3; do
  for f in 0 2; do
    FD_FUSE_QKV_ATTN=$f timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality \
      > $OUT/ab_qa${f}_$i.json.log 2>&1 || exit 1
  done
done
