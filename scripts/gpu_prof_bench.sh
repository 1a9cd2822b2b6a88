#!/bin/bash
# rocprofv3 kernel stats of the headline bench (bs32 seq128), summarised per step.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-prof}; mkdir -p $O
STEPS=${2:-20}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -- python3 bench.py --steps $STEPS --warmup 3 --spinup-seconds 0 --no-quality > $O/bench.log 2>&1 &&
f=$(find $O/raw -name "*kernel_stats.csv" | head -1) && python scripts/kstats.py "$f" auto 45 > $O/kernel_stats.txt && cat $O/kernel_stats.txt && tail -1 $O/bench.log
