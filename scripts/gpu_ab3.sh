#!/bin/bash
# Interleaved A/B/C of environment settings on one box:
#   bash scripts/gpu_ab3.sh <name> <reps> "<env A>" "<env B>" ["<env C>" ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab3}; mkdir -p $O
reps=${2:-2}; shift 2
for i in $(seq $reps); do
  j=0
  for E in "$@"; do
    j=$((j + 1))
    env $E timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-quality > $O/v${j}_$i.log 2>&1 || { tail -5 $O/v${j}_$i.log; exit 1; }
    echo "v$j.$i [$E] $(python -c "import json,sys; d=json.loads(open('$O/v${j}_$i.log').read().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
