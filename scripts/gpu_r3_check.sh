#!/bin/bash
# Targeted GPU tests + headline bench + kernel stats (round 3 iteration loop).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r3chk}; mkdir -p $O
shift
TESTS=${@:-tests/}
timeout -k 10 900 python -u -m pytest $TESTS -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log
if [ $rc -ne 0 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > $O/bench.log 2>&1 && tail -1 $O/bench.log | cut -c1-400 &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/raw -- python3 bench.py --steps 20 --warmup 3 --spinup-seconds 0 --no-quality > $O/prof_bench.log 2>&1 &&
f=$(find $O/raw -name "*kernel_stats.csv" | head -1) && python scripts/kstats.py "$f" auto 40 > $O/kernel_stats.txt && head -24 $O/kernel_stats.txt
