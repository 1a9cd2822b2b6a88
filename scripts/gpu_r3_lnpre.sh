#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lnpre; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_ln_gpu.py tests/test_prune_gpu.py tests/test_packed_gpu.py tests/test_model_gpu.py tests/test_numerics_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1; r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && exit $r
FD_SO_OUT=ab/stamps.so timeout -k 10 200 python -u scripts/gemm_stamps.py > $O/stamps.txt 2>&1; grep -v amdgpu $O/stamps.txt | head -5
bash scripts/gpu_ab_so.sh lnpre_ab 3 || exit 1
bash scripts/gpu_attn_pmc.sh attn_pmc
