#!/bin/bash
# Round-2 GPU check: smoke (native-load proof), headline bench (N=1, with the quality
# protocol), then the GPU test suite.  Each step has its own time limit; any failure stops.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit $?
tail -1 gpurun_out/bench.log
if [ -z "${SKIP_TESTS}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${TEST_ARGS} \
    > gpurun_out/gputests.log 2>&1 || { tail -30 gpurun_out/gputests.log; exit 1; }
  tail -3 gpurun_out/gputests.log
fi
