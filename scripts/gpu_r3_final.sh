#!/bin/bash
# Round 3 record: full GPU suite, headline bench (quality protocol), kernel stats, KD config bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
tail -4 $O/tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-250 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -- python3 bench.py --steps 20 --warmup 3 --spinup-seconds 0 --no-quality > $O/prof_bench.log 2>&1 &&
f=$(find $O/raw -name "*kernel_stats.csv" | head -1) && python scripts/kstats.py "$f" auto 40 > $O/kernel_stats.txt && head -12 $O/kernel_stats.txt &&
timeout -k 10 600 python bench.py --steps 30 --warmup 5 --teacher --seq-len 256 --batch-size 64 > $O/kd.log 2>&1 && tail -1 $O/kd.log | cut -c1-200
