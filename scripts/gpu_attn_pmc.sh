#!/bin/bash
# PMC passes over the attention kernels alone (scripts/attn_pmc.py), one counter group per pass.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-attn_pmc}; mkdir -p $O
run() {
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O/$n -- python3 scripts/attn_pmc.py > $O/$n.log 2>&1 ||
    { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }
}
run p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA &&
run p2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE &&
python - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(f"{O}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "attn" not in k:
            continue
        k = k.split("(")[0].split("::")[-1]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    n = max(cnt[(k, "SQ_WAVE_CYCLES")], 1)
    print(k)
    for c in sorted(d):
        print(f"   {c:28s} {d[c] / max(cnt[(k, c)], 1):14.1f}  (per dispatch)")
PY
