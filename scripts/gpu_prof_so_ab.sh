#!/bin/bash
# rocprofv3 kernel stats of the headline step for two kernel-library builds (ab/old.so, ab/new.so)
#   bash scripts/gpu_prof_so_ab.sh <name>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-prof_so_ab}; mkdir -p $O
SO=_so/_hip_kernels.so
for v in old new; do
  cp ab/$v.so $SO
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw_$v -- python3 bench.py --steps 30 --warmup 3 --spinup-seconds 0 --no-quality > $O/bench_$v.log 2>&1 || { tail -5 $O/bench_$v.log; cp ab/new.so $SO; exit 1; }
  f=$(find $O/raw_$v -name "*kernel_stats.csv" | head -1) && python scripts/kstats.py "$f" auto 45 > $O/kstats_$v.txt
done
cp ab/new.so $SO
