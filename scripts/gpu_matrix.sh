#!/bin/bash
# Interleaved bench matrix on one box: bash scripts/gpu_matrix.sh <name> <reps> "ENV|FLAGS" "ENV|FLAGS" ...
# (ENV may be empty or "X=1 Y=2"; FLAGS are bench.py flags)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-matrix}; mkdir -p $O
reps=${2:-2}; shift 2
for i in $(seq $reps); do
  k=0
  for v in "$@"; do
    k=$((k+1)); E="${v%%|*}"; F="${v#*|}"
    env $E timeout -k 10 300 python bench.py --steps 200 --warmup 10 $F > $O/v${k}_$i.log 2>&1 || { tail -5 $O/v${k}_$i.log; exit 1; }
    echo "v$k.$i [$E|$F] $(python -c "import json,sys; d=json.loads(open('$O/v${k}_$i.log').read().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
