#!/bin/bash
# A/B of bench.py flags on one box: bash scripts/gpu_ab.sh <name> "<flags A>" "<flags B>" [reps]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab}; mkdir -p $O
for i in $(seq ${4:-2}); do
  for v in A B; do
    if [ $v = A ]; then F="$2"; else F="$3"; fi
    timeout -k 10 300 python bench.py --steps 200 --warmup 10 $F > $O/$v$i.log 2>&1 || { tail -5 $O/$v$i.log; exit 1; }
    echo "$v$i [$F] $(python -c "import json,sys; d=json.loads(open('$O/$v$i.log').read().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
