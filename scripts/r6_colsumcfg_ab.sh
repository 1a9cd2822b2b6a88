#!/bin/bash
# GELU' dX GEMM with column sums at M >= 3584: 128 x 128 tiles (new) vs 128 x 64 (FD_GEMM_CFG_NN override
# cannot isolate it: the A/B runs this tree's .so against a copy built from the previous gemm.hip).
set -o pipefail
OUT=gpurun_out/${1:-r6colsum}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_packed_gpu.py -x -q --timeout 120 \
  --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for so in "_so/_hip_kernels.so" "_so_prev/_hip_kernels.so"; do
    tag=$(echo $so | tr '/.' '__')
    FD_SO_OUT=$so timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality --teacher --seq-len 256 \
      --batch-size 64 > $OUT/kd_${tag}_$i.json.log 2>&1 || { tail -5 $OUT/kd_${tag}_$i.json.log; exit 1; }
    echo "kd $so pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/kd_${tag}_$i.json.log)"
  done
done
