#!/bin/bash
# Large-M wide NT GEMM tile pick (FD_GEMM_BIG_CFG 6 vs the old 3): GEMM tests, then the distillation
# config and bs256 inference, interleaved.
set -o pipefail
OUT=gpurun_out/${1:-r6bigcfg}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
  for cfg in "FD_GEMM_BIG_CFG=6" "FD_GEMM_BIG_CFG=3"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality --teacher --seq-len 256 \
      --batch-size 64 > $OUT/kd_${tag}_$i.json.log 2>&1 || { tail -5 $OUT/kd_${tag}_$i.json.log; exit 1; }
    echo "kd $cfg pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/kd_${tag}_$i.json.log)"
    env $cfg timeout -k 10 300 python3 bench.py --mode infer --batch-size 256 > $OUT/inf_${tag}_$i.json.log 2>&1 \
      || { tail -5 $OUT/inf_${tag}_$i.json.log; exit 1; }
    echo "infer bs256 $cfg pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/inf_${tag}_$i.json.log)"
  done
done
