"""Summarise a rocprofv3 kernel_stats CSV (per training step: total / steps)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 7.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {float(r['Percentage']):6.2f}% "
          f"calls/step={int(r['Calls'])/steps:6.1f} avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:95]}")
print(f"total {tot/1e6/steps:.2f} ms/step")
