#!/bin/bash
# Varlen attention split dispatch at S > 128 (FD_ATTN_SPLIT): its GPU tests, then the distillation
# config (BASELINE config 5: seq256 bs64, BERT-base teacher) with the split on / off, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r6split}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_packed_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for i in 1 2; do
  for cfg in "FD_ATTN_SPLIT=1" "FD_ATTN_SPLIT=0"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality --teacher --seq-len 256 \
      --batch-size 64 > $OUT/kd_${tag}_$i.json.log 2>&1 || { tail -5 $OUT/kd_${tag}_$i.json.log; exit 1; }
    echo "$cfg pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/kd_${tag}_$i.json.log) $(grep -o '"hip_graphs": [0-9]*' $OUT/kd_${tag}_$i.json.log)"
  done
done
