O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "direct_a" tests/test_fused_ln_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/da_bench.py > $O/da_bench.txt 2>&1; rc=$?; cat $O/da_bench.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/ln_fused_bench.py 2688 24,50,51 > $O/ln_bench.txt 2>&1; rc=$?; cat $O/ln_bench.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python scripts/curve_bisect.py > $O/curve_bisect.txt 2>&1; rc=$?; tail -8 $O/curve_bisect.txt; exit $rc
