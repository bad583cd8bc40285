"""Concurrency of a graph-replayed step from a rocprofv3 kernel trace: per kernel family, the time
it ran and how much of that another kernel ran beside it (e.g. side-stream weight-gradient GEMMs
under the latency-bound LSTM recurrences).

    python tools/tools_overlap.py gpurun_out/ovl/run_kernel_trace.csv
Steps are delimited by adamw_kernel; the graph replays before the eager probe steps are used.
"""
import csv
import sys
from collections import defaultdict


def fam(n):
    n = n.split("(")[0]
    for k in ("lstm_fwd", "lstm_bwd", "gemm_x6", "splitk", "attn_bwd", "attn_fwd", "resln", "gemm_rows", "adamw",
              "loss"):
        if k in n:
            return k
    return "other"


rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ends = [i for i, e in enumerate(ev) if "adamw_kernel" in e[2] and "inc" not in e[2]]
segs = [(ends[i] + 1, ends[i + 1]) for i in range(len(ends) - 1)]
for a, b in segs[-6:-3]:
    seg = ev[a:b + 1]
    t0, t1 = seg[0][0], max(e[1] for e in seg)
    run = defaultdict(float)
    ovl = defaultdict(float)
    with_ = defaultdict(lambda: defaultdict(float))
    for i, (s, e, n) in enumerate(seg):
        f = fam(n)
        run[f] += e - s
        # union of other kernels' intervals intersected with [s, e]
        iv = sorted((max(s, s2), min(e, e2), fam(n2)) for j, (s2, e2, n2) in enumerate(seg)
                    if j != i and s2 < e and e2 > s)
        cur_s = cur_e = None
        tot = 0
        for x, y, f2 in iv:
            with_[f][f2] += y - x
            if cur_e is None or x > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = x, y
            else:
                cur_e = max(cur_e, y)
        if cur_e is not None:
            tot += cur_e - cur_s
        ovl[f] += tot
    print(f"step wall {(t1 - t0) / 1e6:.3f} ms, kernel time {sum(run.values()) / 1e6:.3f} ms")
    for f in sorted(run, key=lambda k: -run[k]):
        top = ", ".join(f"{k} {v / 1e6:.2f}" for k, v in sorted(with_[f].items(), key=lambda kv: -kv[1])[:3])
        print(f"  {f:10s} ran {run[f] / 1e6:7.3f} ms, with others beside it {ovl[f] / 1e6:7.3f} ms  [{top}]")
