#!/bin/bash
# Interleaved A/B of two kernel-library builds on one box: ab/old.so vs ab/new.so copied over
# _so/_hip_kernels.so before each headline bench run (200 steps, no quality protocol).
#   bash scripts/gpu_ab_so.sh <name> <reps>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab_so}; mkdir -p $O
SO=_so/_hip_kernels.so
for i in $(seq ${2:-3}); do
  for v in old new; do
    cp ab/$v.so $SO
    timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-quality > $O/${v}_$i.log 2>&1 || { tail -5 $O/${v}_$i.log; cp ab/new.so $SO; exit 1; }
    echo "$v rep$i $(python -c "import json; d=json.loads(open('$O/${v}_$i.log').read().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
cp ab/new.so $SO
