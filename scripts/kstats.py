"""Summarise a rocprofv3 kernel_stats.csv: top kernels, per-step ms."""
import csv, sys
path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
arg = sys.argv[2] if len(sys.argv) > 2 else "1"
if arg == "auto":
    # the all-layer weight-gradient launch runs once per training step (so did the Adam launch,
    # which now runs inside it)
    steps = float(next(r['Calls'] for r in rows if 'gemm_dw_batch_kernel' in r['Name'] or 'adam_kernel' in r['Name']))
else:
    steps = float(arg)
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"{'ms/step':>8} {'%':>6} {'calls':>6} {'avg_us':>8}  kernel")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} {float(r['Percentage']):6.2f} {r['Calls']:>6} {float(r['AverageNs'])/1e3:8.1f}  {r['Name'][:100]}")
print(f"total GPU ms/step: {tot/1e6/steps:.3f}")
