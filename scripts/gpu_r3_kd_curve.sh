#!/bin/bash
# Round 3: loss-curve bias control (torch bf16 autocast) + the distillation config's quality protocol.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
BISECT_QUICK=1 timeout -k 10 600 python -u scripts/curve_bisect.py > gpurun_out/curve_bisect2.txt 2>&1; cat gpurun_out/curve_bisect2.txt
timeout -k 10 900 python bench.py --steps 30 --warmup 5 --teacher --seq-len 256 --batch-size 64 > gpurun_out/kd_quality.log 2>&1; r=$?
tail -1 gpurun_out/kd_quality.log | cut -c1-300; exit $r
