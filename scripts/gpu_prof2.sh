#!/bin/bash
# Kernel traces of two bench variants: bash scripts/gpu_prof2.sh <name> "ENV|FLAGS" "ENV|FLAGS"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-prof2}; mkdir -p $O
k=0
for v in "$2" "$3"; do
  k=$((k+1)); E="${v%%|*}"; F="${v#*|}"
  for kv in $E; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/raw$k -- python3 bench.py --steps 20 --warmup 3 --spinup-seconds 0 --no-quality $F > $O/prof$k.log 2>&1 || { tail -5 $O/prof$k.log; exit 1; }
  for kv in $E; do unset "${kv%%=*}"; done
  f=$(find $O/raw$k -name "*kernel_trace.csv" | head -1) && python scripts/step_timeline.py "$f" 15 > $O/timeline$k.txt && echo "== v$k [$v]" && head -16 $O/timeline$k.txt
done
