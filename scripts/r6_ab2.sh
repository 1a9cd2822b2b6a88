#!/bin/bash
# LN-epilogue weight prefetch (FD_LN_PREFETCH) and dW problem order (FD_DWB_ORDER): tests + probe + step A/B
set -o pipefail
OUT=gpurun_out/r6ab2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_fused_ln_gpu.py tests/test_prune_gpu.py tests/test_numerics_gpu.py tests/test_dw_batch_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 120 python3 scripts/dwb_tail_probe.py > $OUT/probe_mixed.txt 2>&1 || exit 1
for i in 1 2; do
  for cfg in "0 0" "1 0" "0 1" "1 1"; do
    set -- $cfg
    FD_LN_PREFETCH=$1 FD_DWB_ORDER=$2 timeout -k 10 120 python3 bench.py --gpus 1 --steps 50 --warmup 10 --no-quality \
      > $OUT/ab_pf$1_ord$2_$i.json.log 2>&1 || exit 1
  done
done
