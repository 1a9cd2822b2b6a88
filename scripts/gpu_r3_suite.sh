#!/bin/bash
# Full GPU suite without -x (every failure listed), then bisect knobs on one named test.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3suite}; mkdir -p $O
[ -x ab/l2_fill ] && { timeout -k 10 90 ./ab/l2_fill > $O/l2_fill.txt 2>&1; r=$?; cat $O/l2_fill.txt; [ $r -ne 0 ] && exit $r; }
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -15 $O/tests.log
[ $rc -ge 124 ] && exit $rc
shift
for envs in "$@"; do
  echo "== $envs"
  env $envs timeout -k 10 200 python -u -m pytest tests/test_dp_gpu.py -x -q --timeout 150 --timeout-method thread > $O/bisect.log 2>&1
  r=$?; tail -2 $O/bisect.log; [ $r -ge 124 ] && exit $r
done
exit 0
