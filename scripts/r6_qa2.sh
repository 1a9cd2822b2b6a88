#!/bin/bash
# Kernel stats of the timed step with the fused QKV + attention launch on / off
set -o pipefail
FD_FUSE_QKV_ATTN=1 bash scripts/gpu.sh prof r6qa_prof1 > /dev/null || exit 1
FD_FUSE_QKV_ATTN=0 bash scripts/gpu.sh prof r6qa_prof0 > /dev/null || exit 1
