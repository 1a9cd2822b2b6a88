O=gpurun_out/r4j; mkdir -p $O
bash scripts/gpu.sh tests r4j; rc=$?; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --steps 50 --warmup 10 > $O/bench_q.log 2>&1 && tail -n 1 $O/bench_q.log | cut -c1-400 &&
bash scripts/gpu.sh prof r4j && timeout -k 10 120 python scripts/attn_bench.py > $O/attn.txt 2>&1 && grep "B=  32" $O/attn.txt
echo done
