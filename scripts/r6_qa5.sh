#!/bin/bash
set -o pipefail
bash scripts/r6_knobs.sh r6qa5 FD_FUSE_QKV_ATTN=0,2 FD_FUSE_QKV_ATTN=2,0 > gpurun_out/r6qa5.txt 2>&1 || exit 1
FD_FUSE_QKV_ATTN=2 bash scripts/gpu.sh prof r6qa5_prof2 > /dev/null
