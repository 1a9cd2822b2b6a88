#!/bin/bash
# Round-6 record on one lease: GPU suite, kernel stats of the timed step, then the driver's exact
# command twice (the second with --step-events: per-step GPU times inside the 20-step window).
set -o pipefail
OUT=gpurun_out/${1:-r6rec}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
bash scripts/gpu.sh prof ${1:-r6rec}_prof > /dev/null || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver_cmd.json.log 2> $OUT/driver_cmd.err || exit 1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --step-events > $OUT/driver_cmd_events.json.log 2> $OUT/driver_cmd_events.err || exit 1
