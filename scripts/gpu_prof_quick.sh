#!/bin/bash
# Kernel stats of a short headline bench (no quality protocol): bash scripts/gpu_prof_quick.sh <name> [ENV=V ...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-profq}; shift; mkdir -p $O
for E in "$@"; do export "$E"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -- python3 bench.py --steps 20 --warmup 3 --spinup-seconds 0 --no-quality > $O/prof_bench.log 2>&1 &&
f=$(find $O/raw -name "*kernel_stats.csv" | head -1) && python scripts/kstats.py "$f" auto 30 > $O/kernel_stats.txt && head -14 $O/kernel_stats.txt
