#!/bin/bash
# Which fused S <= 128 path pays in short mode at seq256 bs64 (distillation config): each knob off in turn.
set -o pipefail
OUT=gpurun_out/${1:-r6shortparts}
mkdir -p $OUT
for i in 1 2; do
  for cfg in "FD_ATTN_SHORT=1" "FD_FUSE_QKV_ATTN=0" "FD_FUSE_ATTN_BWD=0" "FD_ATTN_CLS_COMPACT=0" "FD_ATTN_SHORT=0"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality --teacher --seq-len 256 \
      --batch-size 64 > $OUT/kd_${tag}_$i.json.log 2>&1 || { tail -5 $OUT/kd_${tag}_$i.json.log; exit 1; }
    echo "$cfg pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/kd_${tag}_$i.json.log)"
  done
done
