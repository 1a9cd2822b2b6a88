#!/bin/bash
# fused attention backward incl. the pruned block's compact form: tests, A/B, kernel stats
set -o pipefail
OUT=gpurun_out/r6abw3
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_qkv_attn_gpu.py tests/test_prune_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
bash scripts/r6_knobs.sh r6abw3 FD_FUSE_ATTN_BWD=0,1 FD_FUSE_ATTN_BWD=1,0 > gpurun_out/r6abw3.txt 2>&1 || exit 1
FD_FUSE_ATTN_BWD=1 bash scripts/gpu.sh prof r6abw3_prof1 > /dev/null
