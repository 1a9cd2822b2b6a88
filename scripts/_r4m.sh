O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_dw_batch_gpu.py tests/test_fused_adam_gpu.py tests/test_model_gpu.py tests/test_prune_gpu.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -n 4 $O/tests.log; [ $rc -ne 0 ] && exit $rc
for arm in 1 0 1 0; do FD_DW_TAIL=$arm timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-quality > $O/bench_tail$arm.log 2>&1 || exit 1; echo "tail=$arm $(tail -n 1 $O/bench_tail$arm.log | cut -c150-230)"; done
bash scripts/gpu.sh prof r4m
echo done
