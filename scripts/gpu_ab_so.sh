#!/bin/bash
# A/B of two builds of the kernel library on one box: ab/old.so vs ab/new.so (bench.py, alternating).
# bash scripts/gpu_ab_so.sh <name> [reps] [extra bench flags]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab_so}; mkdir -p $O
SO=detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd/ops/_hip_kernels.cpython-310-x86_64-linux-gnu.so
for i in $(seq ${2:-3}); do
  for v in old new; do
    cp ab/$v.so $SO
    timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-quality $3 > $O/$v$i.log 2>&1 || { tail -5 $O/$v$i.log; exit 1; }
    echo "$v$i $(python -c "import json; d=json.loads(open('$O/$v$i.log').read().splitlines()[-1]); print(d['ms_per_step'], d['value'])")"
  done
done
cp ab/new.so $SO
