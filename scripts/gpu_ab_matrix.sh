#!/bin/bash
# Interleaved matrix of environment settings on one box (bench.py --steps 200 --no-quality):
#   bash scripts/gpu_ab_matrix.sh <name> <reps> "<env 1>" "<env 2>" ...   ("-" = no setting)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abm}; mkdir -p $O
R=${2:-2}; shift 2
for i in $(seq $R); do
  j=0
  for E in "$@"; do
    j=$((j+1))
    [ "$E" = "-" ] && E=""
    env $E timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-quality > $O/v${j}_$i.log 2>&1 || { tail -5 $O/v${j}_$i.log; exit 1; }
    echo "v$j rep$i [$E] $(python -c "import json,sys; d=json.loads(open('$O/v${j}_$i.log').read().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
