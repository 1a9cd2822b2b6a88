#!/bin/bash
# GPU round trip: all GPU tests, headline bench, rocprofv3 kernel stats of the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-full}; mkdir -p $O
timeout -k 10 900 python -m pytest tests/ -x -q -m gpu > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 && tail -1 $O/bench.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -- python3 bench.py --steps 20 --warmup 3 --spinup-seconds 0 --no-quality > $O/prof_bench.log 2>&1 &&
f=$(find $O/raw -name "*kernel_stats.csv" | head -1) && python scripts/kstats.py "$f" auto 40 > $O/kernel_stats.txt && head -30 $O/kernel_stats.txt
