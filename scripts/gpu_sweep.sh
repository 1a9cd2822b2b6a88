#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-sweep}; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or linear" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
# only numerical failures (rc 1) may continue; a crash / fault / timeout ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 900 python scripts/gemm_sweep.py ${2:-2688} > $O/sweep.txt 2>&1; rc=$?; tail -22 $O/sweep.txt; exit $rc
