#!/bin/bash
# 3-slot projection ring: tests, then same-lease A/Bs of the fused backward and of its compact form
set -o pipefail
OUT=gpurun_out/r6abw4
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_qkv_attn_gpu.py tests/test_prune_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
bash scripts/r6_knobs.sh r6abw4 FD_FUSE_ATTN_BWD=1,0 FD_FUSE_ATTN_BWD_CLS=1,0 FD_FUSE_ATTN_BWD=1,0 > gpurun_out/r6abw4.txt 2>&1 || exit 1
FD_FUSE_ATTN_BWD=1 bash scripts/gpu.sh prof r6abw4_prof1 > /dev/null && FD_FUSE_ATTN_BWD=0 bash scripts/gpu.sh prof r6abw4_prof0 > /dev/null
