#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-attn}; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "attention" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --teacher --seq-len 256 --batch-size 64 > $O/kd.log 2>&1 && tail -1 $O/kd.log &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --seq-len 256 --batch-size 64 > $O/s256.log 2>&1 && tail -1 $O/s256.log &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 && tail -1 $O/bench.log
