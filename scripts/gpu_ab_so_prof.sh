#!/bin/bash
# Per-kernel A/B of two kernel-library builds (ab/old.so vs ab/new.so): rocprofv3 kernel stats
# of a short bench run for each, then the kstats table.  bash scripts/gpu_ab_so_prof.sh <name>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab_so_prof}; mkdir -p $O
SO=detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd/ops/_hip_kernels.cpython-310-x86_64-linux-gnu.so
for v in old new; do
  cp ab/$v.so $SO
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw_$v -- python3 bench.py --steps 40 --warmup 3 --spinup-seconds 0 --no-quality > $O/prof_$v.log 2>&1 || { tail -5 $O/prof_$v.log; cp ab/new.so $SO; exit 1; }
  f=$(find $O/raw_$v -name "*kernel_stats.csv" | head -1) && python scripts/kstats.py "$f" auto 30 > $O/kstats_$v.txt && echo "== $v" && head -16 $O/kstats_$v.txt
done
cp ab/new.so $SO
