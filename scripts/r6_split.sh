#!/bin/bash
# Graph-chain capture (FD_GRAPH_SPLIT): tests, then the driver's command with per-step events
set -o pipefail
OUT=gpurun_out/${1:-r6split}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_graph_split_gpu.py tests/test_packed_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || exit 1
for i in 1 2; do
  for sp in none 0 0,2; do
    v=$sp; [ "$sp" = none ] && v=
    FD_GRAPH_SPLIT=$v timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --step-events \
      > $OUT/split_${sp}_$i.json.log 2> $OUT/split_${sp}_$i.err || exit 1
  done
done
