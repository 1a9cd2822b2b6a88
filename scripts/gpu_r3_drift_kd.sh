#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u scripts/drift_diag.py > gpurun_out/drift.txt 2>&1; grep -v amdgpu gpurun_out/drift.txt
timeout -k 10 900 python bench.py --steps 30 --warmup 5 --teacher --seq-len 256 --batch-size 64 > gpurun_out/kd_quality2.log 2>&1; r=$?
tail -1 gpurun_out/kd_quality2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ['aggregated_f1','aggregated_accuracy_pct','teacher_test_f1','teacher_test_accuracy_pct','quality_epoch_losses','ms_per_step']})"; exit $r
