O=gpurun_out/r4h; mkdir -p $O
for d in 0 1 4 5; do FD_GEMM_DIAG=$d timeout -k 10 120 python scripts/dwb_bench.py 2688 11,1 > $O/dwb_diag$d.txt 2>&1 || exit 1; echo "diag $d"; grep -v amdgpu $O/dwb_diag$d.txt; done
timeout -k 10 900 python scripts/kd_vs_ce.py 225745 3 0.1,0.5,0.9 42,43 > $O/kd_vs_ce.txt 2>&1; tail -n 9 $O/kd_vs_ce.txt
echo done
