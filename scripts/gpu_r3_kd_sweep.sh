#!/bin/bash
# KD quality protocol variants (config 5: seq256 bs64): learning rate / CE weight / epochs.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kd_sweep
n=0
for V in "$@"; do
  n=$((n+1))
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --teacher --seq-len 256 --batch-size 64 $V > gpurun_out/kd_sweep/v$n.log 2>&1 || { tail -5 gpurun_out/kd_sweep/v$n.log; exit 1; }
  echo "[$V] $(tail -1 gpurun_out/kd_sweep/v$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ['aggregated_f1','aggregated_accuracy_pct','teacher_test_f1','quality_epoch_losses','quality_wall_s']})")"
done
