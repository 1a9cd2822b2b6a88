#!/bin/bash
# Quick GPU check: model/kernel/DP GPU tests, then the headline bench, then kernel stats.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-quick}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/ > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > $O/bench.log 2>&1 && tail -1 $O/bench.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -- python3 bench.py --steps 20 --warmup 3 --spinup-seconds 0 --no-quality > $O/prof_bench.log 2>&1 &&
f=$(find $O/raw -name "*kernel_stats.csv" | head -1) && python scripts/kstats.py "$f" auto 45 > $O/kernel_stats.txt && head -25 $O/kernel_stats.txt
