#!/bin/bash
set -o pipefail
OUT=gpurun_out/r6qa4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_qkv_attn_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
bash scripts/r6_knobs.sh r6qa4 FD_FUSE_QKV_ATTN=0,2 > gpurun_out/r6qa4.txt 2>&1
