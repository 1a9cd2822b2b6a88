#!/bin/bash
# Kernel stats of the timed step per FD_FUSE_QKV_ATTN mode (usage: scripts/r6_qa2.sh <modes...>)
set -o pipefail
for m in ${@:-1 0}; do
  FD_FUSE_QKV_ATTN=$m bash scripts/gpu.sh prof r6qa_prof$m > /dev/null || exit 1
done
