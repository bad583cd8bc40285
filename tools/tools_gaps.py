"""Idle gaps of a graph-replayed step from a rocprofv3 kernel trace (tools_gpu_gaps.sh).

    python tools/tools_gaps.py gpurun_out/gaps/run_kernel_trace.csv
Steps are delimited by adamw_kernel; the last `--steps` replays before the eager probe steps.
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ends = [i for i, e in enumerate(ev) if "adamw_kernel" in e[2]]
# the graph replays: consecutive adamw's, pick the 3 steps before the last 3 (probe steps are eager)
segs = [(ends[i] + 1, ends[i + 1]) for i in range(len(ends) - 1)]
for a, b in segs[-6:-3]:
    seg = ev[a:b + 1]
    t0, t1 = seg[0][0], max(e[1] for e in seg)
    busy, cur_s, cur_e = 0, seg[0][0], seg[0][1]
    gaps = defaultdict(float)
    for s, e, n in seg[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps[n.split("(")[0].split("<")[0][-40:]] += (s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    print(f"step: wall {(t1 - t0) / 1e6:.3f} ms busy {busy / 1e6:.3f} ms idle {(t1 - t0 - busy) / 1e6:.3f} ms "
          f"kernels {len(seg)}")
    for k, v in sorted(gaps.items(), key=lambda kv: -kv[1])[:8]:
        print(f"   gap before {k:42s} {v / 1e3:8.1f} us")
