"""Per-step GPU timeline from a rocprofv3 kernel_trace.csv: for each training step
(delimited by the Adam kernel) the wall span, the summed kernel time, the idle gap
total, and the top kernels by time -- where the step's milliseconds go."""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ends = [i for i, r in enumerate(rows) if "adam_kernel" in r["Kernel_Name"] or "gemm_dw_batch_kernel" in r["Kernel_Name"]]
spans = []
for a, b in zip(ends[:-1], ends[1:]):
    ks = rows[a + 1:b + 1]
    t0, t1 = int(rows[a]["End_Timestamp"]), int(ks[-1]["End_Timestamp"])
    busy, prev_end, gaps = 0, t0, []
    for r in ks:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s > prev_end:
            gaps.append(s - prev_end)
        busy += e - max(s, prev_end) if e > prev_end else 0
        prev_end = max(prev_end, e)
    spans.append((t1 - t0, busy, sum(gaps), len(ks), ks))
sel = spans[-last:]
n = len(sel)
print(f"steps {n}: wall {sum(s[0] for s in sel)/n/1e3:.1f} us, kernel-busy {sum(s[1] for s in sel)/n/1e3:.1f} us, "
      f"idle {sum(s[2] for s in sel)/n/1e3:.1f} us, kernels/step {sum(s[3] for s in sel)/n:.0f}")
agg = defaultdict(lambda: [0, 0])
for s in sel:
    for r in s[4]:
        k = r["Kernel_Name"][:90]
        agg[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[k][1] += 1
for k, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:30]:
    print(f"{t/n/1e3:8.1f} us {c/n:5.1f}x  {k}")
