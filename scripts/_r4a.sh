bash scripts/gpu.sh tests r4b; rc=$?; [ $rc -ge 124 ] && exit $rc
bash scripts/gpu.sh bench r4b && bash scripts/gpu.sh prof r4b &&
timeout -k 10 900 python scripts/curve_bisect.py > gpurun_out/r4b/curve_bisect.txt 2>&1; rc2=$?; tail -12 gpurun_out/r4b/curve_bisect.txt; exit $rc2
