O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 120 python scripts/overlap_probe.py > $O/overlap.txt 2>&1; grep -v amdgpu $O/overlap.txt
timeout -k 10 120 python scripts/overlap_probe.py > $O/overlap2.txt 2>&1; grep -v amdgpu $O/overlap2.txt
echo done
