O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_dw_batch_gpu.py tests/test_kernels_gpu.py tests/test_packed_gpu.py tests/test_prune_gpu.py tests/test_fused_adam_gpu.py tests/test_model_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/dwb_bench.py 2688 11,25,26,11,25,26 > $O/dwb.txt 2>&1 && grep -v amdgpu $O/dwb.txt &&
FD_GEMM_DIAG=1 timeout -k 10 120 python scripts/dwb_bench.py 2688 11,25,26 > $O/dwb_diag1.txt 2>&1 && echo diag1 && grep -v amdgpu $O/dwb_diag1.txt &&
timeout -k 10 120 python scripts/attn_bench.py > $O/attn_split.txt 2>&1 && FD_ATTN_BWD_SPLIT=0 timeout -k 10 120 python scripts/attn_bench.py > $O/attn_nosplit.txt 2>&1 && grep "B=  32" $O/attn_split.txt $O/attn_nosplit.txt &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench.log 2>&1 && tail -n 1 $O/bench.log | cut -c1-220 &&
FD_ATTN_BWD_SPLIT=0 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench_nosplit.log 2>&1 && tail -n 1 $O/bench_nosplit.log | cut -c1-220 &&
FD_GEMM_DWB_CFG=25 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench_dwb25.log 2>&1 && tail -n 1 $O/bench_dwb25.log | cut -c1-220 &&
FD_GEMM_DWB_CFG=26 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench_dwb26.log 2>&1 && tail -n 1 $O/bench_dwb26.log | cut -c1-220
FD_ATTN_FWD_SPLIT=1 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench_fsplit.log 2>&1 && tail -n 1 $O/bench_fsplit.log | cut -c1-220
bash scripts/gpu.sh prof r4i
echo done
