#!/bin/bash
# Interleaved A/B of environment settings on the distillation config (seq256 bs64 + BERT-base
# teacher):  scripts/ab_kd.sh <name> <reps> "<env A>" "<env B>" ...   (timed steps only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
name=$1; reps=$2; shift 2
O=gpurun_out/$name; mkdir -p "$O"
for r in $(seq 1 "$reps"); do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    timeout -k 10 400 env $setting python bench.py --teacher --seq-len 256 --batch-size 64 --steps 30 --warmup 5 \
      --no-quality --spinup-seconds 0 > "$O/kd_${i}_${r}.log" 2>&1 || { echo "setting '$setting' failed"; tail -5 "$O/kd_${i}_${r}.log"; exit 1; }
    ms=$(tail -1 "$O/kd_${i}_${r}.log" | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "rep $r  [$setting]  $ms ms/step" | tee -a "$O/ab_kd.txt"
  done
done
