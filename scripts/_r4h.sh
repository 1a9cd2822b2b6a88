O=gpurun_out/r4h; mkdir -p $O
for d in 0 1 4 5; do FD_GEMM_DIAG=$d timeout -k 10 120 python scripts/dwb_bench.py 2688 11,1 > $O/dwb_diag$d.txt 2>&1 || exit 1; echo "diag $d"; cat $O/dwb_diag$d.txt; done
echo done
