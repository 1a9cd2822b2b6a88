#!/bin/bash
# Distillation config (BASELINE config 5: seq256 bs64, BERT-base teacher) under this round's late defaults
set -o pipefail
OUT=gpurun_out/${1:-r6kd}
mkdir -p $OUT
for i in 1 2; do
  for cfg in "FD_PACK_QUANTUM=64 FD_REMAT_GELU=0" "FD_PACK_QUANTUM=128 FD_REMAT_GELU=1"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality --teacher --seq-len 256 \
      --batch-size 64 > $OUT/kd_${tag}_$i.json.log 2>&1 || exit 1
    echo "$cfg pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/kd_${tag}_$i.json.log) $(grep -o '"hip_graphs": [0-9]*' $OUT/kd_${tag}_$i.json.log)"
  done
done
