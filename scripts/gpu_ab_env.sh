#!/bin/bash
# A/B of an environment setting on one box: bash scripts/gpu_ab_env.sh <name> "<env A>" "<env B>" [reps] [bench flags]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abenv}; mkdir -p $O
for i in $(seq ${4:-2}); do
  for v in A B; do
    if [ $v = A ]; then E="$2"; else E="$3"; fi
    env $E timeout -k 10 300 python bench.py --steps 200 --warmup 10 $5 > $O/$v$i.log 2>&1 || { tail -5 $O/$v$i.log; exit 1; }
    echo "$v$i [$E] $(python -c "import json,sys; d=json.loads(open('$O/$v$i.log').read().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
