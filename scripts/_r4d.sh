O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_fused_ln_gpu.py tests/test_model_gpu.py tests/test_fused_adam_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
DX_LAYOUTS=1 timeout -k 10 300 python scripts/da_bench.py > $O/dx_layouts.txt 2>&1; rc=$?; cat $O/dx_layouts.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1
bash scripts/gpu.sh pmc r4d_pmc
