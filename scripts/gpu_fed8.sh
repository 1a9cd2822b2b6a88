#!/bin/bash
# BASELINE.json config 4 in miniature on a 1-GPU box: 8 federated clients (8 ranks sharing
# the one MI355X, gloo for the FedAvg collective since RCCL needs a GPU per rank),
# DistilBERT-base, seq128 bs32, 3 local epochs x 3 rounds on synthetic CICIDS2017.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-fed8}; mkdir -p $O
W=/tmp/${1:-fed8}_work; rm -rf $W; mkdir -p $W   # checkpoints (265 MB each) stay off gpurun_out
N=${2:-8}; R=${3:-3}
FEDDDOS_BACKEND=gloo timeout -k 10 1080 python -m detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd \
  launch --nproc $N --port 29555 --batch-size 32 --rounds $R --out-dir $W --resume false --plots true \
  --heartbeat-stale-s 120 > $O/log.txt 2>&1
rc=$?
cp $W/*.csv $W/*.json $O/ 2>/dev/null; cp -r $W/client1_plots $O/ 2>/dev/null
grep -E "Test Accuracy|Epoch \[|updated with aggregated" $O/log.txt | tail -40
python - "$O" <<'PY'
import json, sys
rep = json.load(open(sys.argv[1] + "/federated_report.json"))  # copied from the work dir
for c in rep["clients"]:
    print(c)
print(rep["phases_s"])
PY
exit $rc
