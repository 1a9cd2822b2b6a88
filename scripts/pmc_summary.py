"""Per-kernel PMC summary of scripts/gpu_pmc_bench.sh output.

Reads every counter_collection.csv (and kernel_trace.csv for durations) under the
pass directories and prints, per kernel family: calls per step, mean time, MFMA
busy share, LDS bank-conflict rate, L2 hit rate and HBM read/write bandwidth.

Conventions (MI355X_MICROARCH.md "rocprofv3 PMC slots"):
  MFMA busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)  (rocprofv3's MfmaUtil;
               the per-dispatch CSV value of GRBM_GUI_ACTIVE is summed over the 8 XCDs, the derived
               metric takes the max -- calibrated: FFN1 fwd at 594 TFLOP/s = 24 % of 2.5 PF reads 22.6 %)
  LDS conf   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  L2 hit     = TCC_HIT / (TCC_HIT + TCC_MISS)
  HBM rd/wr  = FETCH_SIZE / WRITE_SIZE (KiB) / kernel time; on gfx950 FETCH_SIZE reads
               ~1/2 of a wide coalesced stream's bytes, so rd is a lower bound.
"""
import collections
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
CUS = 256


def family(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = name.replace("void ", "")
    m = re.match(r"([A-Za-z0-9_:]+(<[^()]*>)?)", name)
    return (m.group(1) if m else name)[:72]


counters = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(lambda: collections.defaultdict(int))
dur = collections.defaultdict(float)
ncalls = collections.Counter()
for f in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
    pas = os.path.relpath(f, root).split(os.sep)[0]
    seen = set()
    for r in csv.DictReader(open(f)):
        k = family(r["Kernel_Name"])
        counters[k][(pas, r["Counter_Name"])] += float(r["Counter_Value"])
        key = (pas, r.get("Dispatch_Id") or r.get("Correlation_Id"))
        if key not in seen:
            seen.add(key)
            calls[k][pas] += 1
for f in glob.glob(os.path.join(root, "rd", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = family(r["Kernel_Name"])
        dur[k] += (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9
        ncalls[k] += 1

steps_kernel = next((k for k in ncalls if "step_kernel" in k), None)
steps = ncalls[steps_kernel] / 2 if steps_kernel else 1.0
print(f"{'kernel':72s} {'calls/st':>8s} {'avg_us':>7s} {'mfma%':>6s} {'ldsconf':>7s} {'L2hit':>6s} "
      f"{'rdGB/s':>7s} {'wrGB/s':>7s}")
tot = 0.0
for k in sorted(dur, key=lambda k: -dur[k]):
    c = counters[k]
    n = ncalls[k]
    t = dur[k] / max(n, 1)
    tot += dur[k]
    per = lambda name, pas: c[(pas, name)] / max(calls[k][pas], 1)  # noqa: E731  per-dispatch mean
    gui = per("GRBM_GUI_ACTIVE", "sq") / 8
    mf = per("SQ_VALU_MFMA_BUSY_CYCLES", "sq") / (gui * CUS * 4) if gui else 0.0
    la = c[("sq", "SQ_LDS_IDX_ACTIVE")]
    lds = c[("sq", "SQ_LDS_BANK_CONFLICT")] / la if la else 0.0
    hm = c[("l2", "TCC_HIT_sum")] + c[("l2", "TCC_MISS_sum")]
    hit = c[("l2", "TCC_HIT_sum")] / hm if hm else 0.0
    rd = per("FETCH_SIZE", "rd") * 1024 / t / 1e9 if t else 0.0
    wr = per("WRITE_SIZE", "wr") * 1024 / t / 1e9 if t else 0.0
    print(f"{k:72s} {n / steps:8.1f} {t * 1e6:7.1f} {100 * mf:6.1f} {100 * lds:6.1f}% {100 * hit:5.1f}% "
          f"{rd:7.0f} {wr:7.0f}")
print(f"eager GPU time per step: {tot / steps * 1e3:.3f} ms over {steps:g} steps (counters serialise dispatches)")
