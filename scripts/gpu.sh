#!/bin/bash
# One parameterised GPU runner (replaces the round 1-3 single-use gpu_*.sh wrappers).
#
#   scripts/gpu.sh <task> <outdir-name> [extra args...]
#
# tasks (every GPU step under its own timeout, chained with &&; output under gpurun_out/<name>):
#   tests   [pytest args]   the GPU suite (-m gpu), or the named test files / -k filters
#   bench   [bench args]    bench.py (default --steps 50 --warmup 10), last JSON line kept
#   prof    [bench args]    rocprofv3 --kernel-trace --stats of the timed step -> kernel_stats.txt
#   pmc                     PMC counter passes of the eager step (gfx950 slot limits) -> pmc_summary.txt
#   record                  tests + bench + prof + the distillation (config 5) bench: the round record
#   run     <cmd...>        any command (a script of scripts/), under a 600 s limit
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
task=$1; name=${2:-$1}; shift 2 2>/dev/null
O=gpurun_out/$name; mkdir -p "$O"

tests() {
  local args=("$@"); [ ${#args[@]} -eq 0 ] && args=(tests/ -m gpu)
  timeout -k 10 1000 python -u -m pytest "${args[@]}" -q --timeout 200 --timeout-method thread > "$O/tests.log" 2>&1
  local rc=$?; tail -6 "$O/tests.log"; return $rc
}
bench() {
  local args=("$@"); [ ${#args[@]} -eq 0 ] && args=(--steps 50 --warmup 10)
  timeout -k 10 600 python bench.py "${args[@]}" > "$O/bench.log" 2>&1 && tail -1 "$O/bench.log" | cut -c1-400
}
prof() {
  local args=("$@"); [ ${#args[@]} -eq 0 ] && args=(--steps 20 --warmup 3)
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/raw" -- \
      python3 bench.py "${args[@]}" --spinup-seconds 0 --no-quality > "$O/prof.log" 2>&1 &&
    f=$(find "$O/raw" -name "*kernel_stats.csv" | head -1) &&
    python scripts/kstats.py "$f" auto 45 > "$O/kernel_stats.txt" && head -16 "$O/kernel_stats.txt"
}
pmc() {
  local A="bench.py --no-graph --steps 4 --warmup 2 --spinup-seconds 0 --no-quality"
  pass() {  # name, counters...
    local n=$1; shift
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d "$O/$n" -- python3 $A \
      > "$O/$n.log" 2>&1 || { echo "pass $n failed"; tail -5 "$O/$n.log"; return 1; }
  }
  pass sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
       SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT &&
    pass l2 TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VALU GRBM_GUI_ACTIVE &&
    pass rd FETCH_SIZE GRBM_GUI_ACTIVE &&
    pass wr WRITE_SIZE GRBM_GUI_ACTIVE &&
    python scripts/pmc_summary.py "$O" > "$O/pmc_summary.txt" && head -40 "$O/pmc_summary.txt"
}

case "$task" in
  tests) tests "$@" ;;
  bench) bench "$@" ;;
  prof) prof "$@" ;;
  pmc) pmc ;;
  record)
    tests && bench && prof &&
      timeout -k 10 600 python bench.py --steps 30 --warmup 5 --teacher --seq-len 256 --batch-size 64 \
        > "$O/kd.log" 2>&1 && tail -1 "$O/kd.log" | cut -c1-300 ;;
  run) timeout -k 10 600 "$@" > "$O/run.log" 2>&1; rc=$?; tail -30 "$O/run.log"; exit $rc ;;
  *) echo "usage: scripts/gpu.sh tests|bench|prof|pmc|record|run <name> [args]"; exit 2 ;;
esac
