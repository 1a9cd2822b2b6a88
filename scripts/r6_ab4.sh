#!/bin/bash
# alternative next-launch prefetch targets: the forward qkv for the attention backward (FD_PF_ATTN_BWD),
# the forward u for the FFN2 dX epilogue (FD_PF_FFN2_U)
set -o pipefail
OUT=gpurun_out/r6ab4
mkdir -p $OUT
FD_PF_ATTN_BWD=1 FD_PF_FFN2_U=1 timeout -k 10 300 python -u -m pytest tests/test_numerics_gpu.py tests/test_prune_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for i in 1 2; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    FD_PF_ATTN_BWD=$1 FD_PF_FFN2_U=$2 timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality \
      > $OUT/ab_attn$1_u$2_$i.json.log 2>&1 || exit 1
  done
done
