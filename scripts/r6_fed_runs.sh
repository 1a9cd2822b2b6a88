#!/bin/bash
# Round-6 federated records on one GPU (run under gpurun from the repo root):
#  1. BASELINE.json config 4's quality half: 8 virtual clients x 3 FedAvg rounds, default and
#     calibrated generator profiles (bench.py --virtual-clients 8 --rounds 3)
#  2. the 8-rank bench path rehearsed on one shared GPU (gloo; every rank a client)
#  3. cli scaling --gpus 1,2,4,8 in the same gloo mode (report columns)
set -o pipefail
OUT=gpurun_out/r6fed
mkdir -p $OUT
for prof in default calibrated; do
  timeout -k 10 420 python3 bench.py --gpus 1 --steps 20 --warmup 5 --virtual-clients 8 --rounds 3 \
    --data-profile $prof > $OUT/fedavg_8x3_$prof.json.log 2> $OUT/fedavg_8x3_$prof.err || exit 1
done
FEDDDOS_BACKEND=gloo timeout -k 10 420 python3 bench.py --gpus 8 --steps 10 --warmup 3 \
  > $OUT/bench_8rank_gloo_shared_gpu.json.log 2> $OUT/bench_8rank_gloo_shared_gpu.err || exit 1
FEDDDOS_BACKEND=gloo timeout -k 10 420 python3 -m detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd scaling \
  --gpus 1,2,4,8 --steps 10 --warmup 3 --out $OUT/scaling_gloo_shared_gpu.json --no-quality \
  > $OUT/scaling_gloo_shared_gpu.txt 2> $OUT/scaling_gloo_shared_gpu.err || exit 1
