#!/bin/bash
# Short-batch attention (every sequence <= 128 tokens at S = 256: the S <= 128 kernels alone, no
# 64-row launches; FD_ATTN_SHORT): GPU tests, then the distillation config with it on / off.
set -o pipefail
OUT=gpurun_out/${1:-r6short}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_packed_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_prune_gpu.py tests/test_qkv_attn_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for cfg in "FD_ATTN_SHORT=1" "FD_ATTN_SHORT=0"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality --teacher --seq-len 256 \
      --batch-size 64 > $OUT/kd_${tag}_$i.json.log 2>&1 || { tail -5 $OUT/kd_${tag}_$i.json.log; exit 1; }
    echo "$cfg pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/kd_${tag}_$i.json.log) $(grep -o '"hip_graphs": [0-9]*' $OUT/kd_${tag}_$i.json.log)"
  done
done
