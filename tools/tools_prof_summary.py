"""Summarise a rocprofv3 kernel_stats CSV per training step.

    python tools/tools_prof_summary.py STATS.csv [STEPS | auto] [TOP]

STEPS = auto counts the executed steps from a kernel that runs exactly once per step (the fused
AdamW, adamw_kernel), so eager warm-ups, graph-capture warm-ups and replays are all counted.
"""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv"
rows = [r for r in csv.DictReader(open(path)) if "busy_kernel" not in r["Name"]]   # bench's probe pre-roll
arg = sys.argv[2] if len(sys.argv) > 2 else "auto"
if arg == "auto":
    marks = [r for r in rows if r["Name"].startswith("mrg::adamw_kernel")]
    steps = float(sum(int(r["Calls"]) for r in marks)) if marks else 1.0
else:
    steps = float(arg)
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"# {path}: {steps:g} executed steps (per-step figures below)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 22]:
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step {float(r['Percentage']):6.2f}% "
          f"calls/step={int(r['Calls'])/steps:6.1f} avg={float(r['AverageNs'])/1e3:8.1f}us  {r['Name'][:95]}")
print(f"total kernel time {tot/1e6/steps:.2f} ms/step")
