O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_packed_gpu.py tests/test_prune_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/attn_bench.py > $O/attn.txt 2>&1 && grep "B=  32" $O/attn.txt &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-200 &&
bash scripts/gpu.sh prof r4l
echo done
