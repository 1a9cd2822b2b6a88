#!/bin/bash
# In-kernel phase stamps of the one-round GEMMs (ab/stamps.so diagnostic build) + the headline bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-stamps}; mkdir -p $O
FD_SO_OUT=ab/stamps.so timeout -k 10 300 python -u scripts/gemm_stamps.py > $O/stamps.txt 2>&1; rc=$?
cat $O/stamps.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-300
