cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fused_ln_gpu.py tests/test_splitk_gpu.py tests/test_packed_gpu.py tests/test_prune_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dk_tests.log 2>&1; r=$?; tail -3 gpurun_out/dk_tests.log; [ $r -ne 0 ] && exit $r
FD_SO_OUT=ab/astamps.so timeout -k 10 120 python -u scripts/attn_stamps.py 32 > gpurun_out/astamps2.txt 2>&1; grep -v amdgpu gpurun_out/astamps2.txt
bash scripts/gpu_ab_so.sh dk_ab 3 || exit 1
timeout -k 10 600 python -u scripts/curve_bisect.py > gpurun_out/curve_bisect.txt 2>&1; cat gpurun_out/curve_bisect.txt
