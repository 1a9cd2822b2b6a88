#!/bin/bash
# Interleaved A/B of environment settings on one box:  scripts/ab.sh <name> <reps> "<env A>" "<env B>" ...
# Each setting runs bench.py (--no-quality, 60 timed steps) <reps> times, round-robin; prints ms/step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
name=$1; reps=$2; shift 2
O=gpurun_out/$name; mkdir -p "$O"
for r in $(seq 1 "$reps"); do
  i=0
  for setting in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 env $setting python bench.py --steps 60 --warmup 10 --no-quality --spinup-seconds 0 \
      > "$O/ab_${i}_${r}.log" 2>&1 || { echo "setting '$setting' failed"; tail -5 "$O/ab_${i}_${r}.log"; exit 1; }
    ms=$(tail -1 "$O/ab_${i}_${r}.log" | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")
    echo "rep $r  [$setting]  $ms ms/step" | tee -a "$O/ab.txt"
  done
done
