#!/bin/bash
# Re-check older defaults against the current step: interleaved 200-step pairs per knob.
# usage: scripts/r6_knobs.sh <outdir> "VAR=a,b,c" ["VAR2=x,y" ...]   (first value = the default; "unset" = not set)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
for spec in "$@"; do
  VAR=${spec%%=*}; VALS=${spec#*=}
  for i in 1 2; do
    for v in ${VALS//,/ }; do
      if [ "$v" = unset ]; then E="env -u $VAR"; else E="env $VAR=$v"; fi
      $E timeout -k 10 150 python3 bench.py --gpus 1 --steps 200 --warmup 10 --no-quality \
        > $OUT/${VAR}_${v}_$i.json.log 2>&1 || exit 1
      echo "$VAR=$v pair $i $(grep -o '"ms_per_step": [0-9.]*' $OUT/${VAR}_${v}_$i.json.log)"
    done
  done
done
