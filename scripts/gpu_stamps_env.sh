#!/bin/bash
# In-kernel phase stamps (ab/stamps.so) of the one-round GEMMs under several env settings.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-stampsenv}; mkdir -p $O; shift
n=0
for E in "$@"; do
  n=$((n+1))
  echo "== [$E]"
  env FD_SO_OUT=ab/stamps.so $E timeout -k 10 200 python -u scripts/gemm_stamps.py > $O/s$n.txt 2>&1; r=$?
  grep -v amdgpu.ids $O/s$n.txt | tail -8; [ $r -ne 0 ] && exit $r
done
exit 0
