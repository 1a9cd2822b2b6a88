#!/bin/bash
# BASELINE.json config 2: one client, bs32 seq128, 3 local epochs + FedAvg, synthetic 10 % CICIDS2017.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-acc1}; mkdir -p $O
W=/tmp/${1:-acc1}_work; rm -rf $W; mkdir -p $W
timeout -k 10 600 python -m detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd \
  client --batch-size 32 --resume false --out-dir $W > $O/log.txt 2>&1
rc=$?
cp $W/*.csv $W/*.json $O/ 2>/dev/null
grep -E "Epoch|Accuracy|updated|batches_per_sec|train" $O/log.txt | grep -v "^\s*$" | tail -14
exit $rc
