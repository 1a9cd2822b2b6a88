#!/bin/bash
# GEMM correctness (kernel tests) + timing on the DistilBERT shapes + full bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-gcheck}; mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "gemm or linear" > $O/tests.log 2>&1 && tail -2 $O/tests.log &&
timeout -k 10 300 python scripts/gemm_bench.py > $O/gemm_bench.log 2>&1 && grep -v amdgpu.ids $O/gemm_bench.log &&
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > $O/bench.log 2>&1 && tail -1 $O/bench.log
