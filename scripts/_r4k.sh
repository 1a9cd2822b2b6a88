O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_dw_batch_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/dwb_bench.py 2688 11,11 > $O/dwb.txt 2>&1 && grep -v amdgpu $O/dwb.txt &&
timeout -k 10 120 python scripts/overlap_probe.py > $O/overlap.txt 2>&1 && grep -v amdgpu $O/overlap.txt &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-200 &&
FD_DW_ADAM_ASYNC=1 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench_async.log 2>&1 && tail -n 1 $O/bench_async.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench2.log 2>&1 && tail -n 1 $O/bench2.log | cut -c1-200 &&
FD_DW_ADAM_ASYNC=1 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench_async2.log 2>&1 && tail -n 1 $O/bench_async2.log | cut -c1-200
echo done
