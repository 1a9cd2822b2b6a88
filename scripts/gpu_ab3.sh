#!/bin/bash
# Interleaved A/B/C of bench configurations on one box:
#   bash scripts/gpu_ab3.sh <name> <reps> "<env+flags A>" "<env+flags B>" ["<env+flags C>" ...]
# Each arm is "VAR=x VAR2=y -- --bench-flag ..." (env before --, bench flags after).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab}; mkdir -p $O
reps=${2:-2}; shift 2
for i in $(seq $reps); do
  a=0
  for arm in "$@"; do
    a=$((a+1))
    envs="${arm%%--*}"; flags=""
    [[ "$arm" == *--* ]] && flags="${arm#*--}"
    env $envs timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-quality $flags > $O/arm${a}_$i.log 2>&1 || { tail -5 $O/arm${a}_$i.log; exit 1; }
    echo "arm$a rep$i [$arm] $(python -c "import json,sys; d=json.loads(open('$O/arm${a}_$i.log').read().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
