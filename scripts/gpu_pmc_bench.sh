#!/bin/bash
# rocprofv3 PMC counters of the headline training step (bs32 seq128, eager so every
# dispatch is attributed), one pass per counter group (gfx950 slot limits: 8 SQ,
# 4 TCC with FETCH_SIZE = 3 / WRITE_SIZE = 2, 2 GRBM), then a per-kernel summary.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pmc}; mkdir -p $O
ARGS="bench.py --no-graph --steps ${2:-4} --warmup 2 --spinup-seconds 0 --no-quality"
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O/$n -- python3 $ARGS > $O/$n.log 2>&1 ||
    { echo "pass $n failed"; tail -5 $O/$n.log; exit 1; }
}
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || true
run sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT &&
run l2 TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
run rd FETCH_SIZE GRBM_GUI_ACTIVE &&
run wr WRITE_SIZE GRBM_GUI_ACTIVE &&
python scripts/pmc_summary.py $O > $O/pmc_summary.txt && cat $O/pmc_summary.txt
