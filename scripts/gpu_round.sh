#!/bin/bash
# tests (failures do not stop the run; a crash / timeout does), then bench + kernel-stats profile,
# then any extra command given as arguments.  Output under gpurun_out/<name>.
name=$1; shift
bash scripts/gpu.sh tests "$name"; rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stopping"; exit $rc; fi
bash scripts/gpu.sh bench "$name" && bash scripts/gpu.sh prof "$name" || exit $?
if [ $# -gt 0 ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
  timeout -k 10 "${EXTRA_TIMEOUT:-300}" "$@" > "gpurun_out/$name/extra.log" 2>&1; rc=$?; tail -30 "gpurun_out/$name/extra.log"; exit $rc
fi
