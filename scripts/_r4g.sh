O=gpurun_out/r4g; mkdir -p $O
bash scripts/gpu.sh tests r4g; rc=$?; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu.sh bench r4g --steps 50 --warmup 10 --no-quality && bash scripts/gpu.sh prof r4g &&
FD_GEMM_LN_DIAG=128 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-quality > $O/bench_nodma.log 2>&1 && tail -n 1 $O/bench_nodma.log | cut -c1-200
timeout -k 10 120 python scripts/attn_bench.py > $O/attn.txt 2>&1; cat $O/attn.txt
echo done
