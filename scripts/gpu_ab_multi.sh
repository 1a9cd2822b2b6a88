#!/bin/bash
# Targeted GPU tests, then an interleaved A/B/C.. of environment settings on one box:
#   bash scripts/gpu_ab_multi.sh <name> <reps> "<tests or ->" "<env A>" "<env B>" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-abmulti}; mkdir -p $O
REPS=${2:-2}; TESTS="$3"; shift 3
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; tail -4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
fi
for i in $(seq $REPS); do
  n=0
  for E in "$@"; do
    n=$((n+1))
    env $E timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-quality > $O/arm${n}_$i.log 2>&1 || { tail -5 $O/arm${n}_$i.log; exit 1; }
    echo "arm$n rep$i [$E] $(python -c "import json,sys; d=json.loads(open('$O/arm${n}_$i.log').read().splitlines()[-1]); print(d['ms_per_step'])")"
  done
done
