O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 200 python scripts/cfg_sweep_ffn.py 2688 > $O/ffn_sweep.txt 2>&1; grep -v amdgpu $O/ffn_sweep.txt
timeout -k 10 200 python scripts/gemm_bench.py 2688 > $O/gemm_vs_blas.txt 2>&1; grep -v amdgpu $O/gemm_vs_blas.txt
echo done
