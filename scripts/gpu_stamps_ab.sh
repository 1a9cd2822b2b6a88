#!/bin/bash
# Phase stamps (ab/stamps.so) + an environment A/B of the headline bench on the same box.
#   bash scripts/gpu_stamps_ab.sh <name> "<env A>" "<env B>" [reps]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-stamps_ab}; mkdir -p $O
FD_SO_OUT=ab/stamps.so timeout -k 10 300 python -u scripts/gemm_stamps.py > $O/stamps.txt 2>&1 || { tail -20 $O/stamps.txt; exit 1; }
head -12 $O/stamps.txt
bash scripts/gpu_ab_env.sh ${1:-stamps_ab} "$2" "$3" ${4:-3} --no-quality
