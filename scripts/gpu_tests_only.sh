#!/bin/bash
# GPU tests only (optionally a subset: TESTS="tests/x.py tests/y.py"), output under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gputests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|SKIPPED|passed|failed" gpurun_out/gputests.log | tail -40
exit $rc
