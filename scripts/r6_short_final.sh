#!/bin/bash
# Short mode's final form (keep bits + compact [CLS] rows, no producer-GEMM fusions) vs the length split alone.
set -o pipefail
OUT=gpurun_out/${1:-r6shortfinal}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_packed_gpu.py tests/test_prune_gpu.py tests/test_qkv_attn_gpu.py -x -q \
  --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for cfg in "FD_ATTN_SHORT=1" "FD_ATTN_SHORT=0" "FD_ATTN_SHORT_FUSED=1"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality --teacher --seq-len 256 \
      --batch-size 64 > $OUT/kd_${tag}_$i.json.log 2>&1 || { tail -5 $OUT/kd_${tag}_$i.json.log; exit 1; }
    echo "$cfg pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/kd_${tag}_$i.json.log)"
  done
done
