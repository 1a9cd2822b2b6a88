#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-dpdiag}; mkdir -p $O; shift
for envs in "$@"; do
  echo "== $envs"
  env $envs timeout -k 10 120 python -u scripts/dp_diag.py > $O/diag.log 2>&1; r=$?
  grep -v amdgpu.ids $O/diag.log | tail -12; [ $r -ne 0 ] && exit $r
done
exit 0
