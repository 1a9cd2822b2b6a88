#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/attn2; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_prune_gpu.py tests/test_packed_gpu.py tests/test_model_gpu.py tests/test_numerics_gpu.py tests/test_splitk_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -B5 -A30 "Error\|assert" $O/tests.log | head -60; exit $r; }
FD_SO_OUT=ab/astamps.so timeout -k 10 120 python -u scripts/attn_stamps.py 32 > $O/astamps.txt 2>&1; grep -v amdgpu $O/astamps.txt | head -2
bash scripts/gpu_ab_so.sh attn_ab 3 || exit 1
bash scripts/gpu_attn_pmc.sh attn_pmc2 > /dev/null 2>&1; echo pmc done
