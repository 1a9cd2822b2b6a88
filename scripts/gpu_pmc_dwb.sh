#!/bin/bash
# PMC passes over the isolated all-layer weight-gradient launch (scripts/dwb_bench.py), one config.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pmc_dwb}; CFG=${2:-8}; mkdir -p $O
run() {
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O/$n -- python3 scripts/dwb_bench.py 2688 $CFG > $O/$n.log 2>&1 ||
    { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE &&
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE &&
python - "$O" <<'PY'
import csv, glob, os, sys, collections
root = sys.argv[1]
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "dw_batch" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:28s} {tot[k] / max(n[k], 1):16.1f}  (mean per dispatch over {n[k]} records)")
w = tot.get("SQ_WAVE_CYCLES", 0)
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        print(f"{k} / SQ_WAVE_CYCLES = {tot.get(k, 0) / w:.3f}")
if tot.get("GRBM_GUI_ACTIVE"):
    print(f"MFMA busy = {tot['SQ_VALU_MFMA_BUSY_CYCLES'] / (tot['GRBM_GUI_ACTIVE'] / 8 * 1024):.3f}")
if tot.get("SQ_LDS_IDX_ACTIVE"):
    print(f"LDS bank conflict rate = {tot['SQ_LDS_BANK_CONFLICT'] / tot['SQ_LDS_IDX_ACTIVE']:.3f}")
PY
