"""Timeline of graph-replayed steps from a rocprofv3 kernel trace: per step the wall time, the time
any kernel runs (union of intervals), the idle gaps (no kernel on the GPU) and, per kernel family,
the union of its intervals and its launch count.

    python tools/tools_timeline.py gpurun_out/X/run_kernel_trace.csv [steps to show]
Steps are delimited by adamw_kernel; the replays before the eager probe steps are used.
"""
import csv
import sys
from collections import defaultdict


def fam(n):
    n = n.split("(")[0]
    for k in ("lstm_fwd_mx", "lstm_bwd_mx", "lstm_fwd", "lstm_bwd", "gemm_x6g_wgrad", "gemm_x6g", "gemm_x6",
              "gemm_rows", "splitk", "attn_bwd", "attn_fwd", "resln_param", "resln_fwd", "resln_bwd", "transpose",
              "adamw", "loss", "Fill", "copy", "elementwise", "Cat"):
        if k in n:
            return k
    return "other"


def union(iv):
    iv = sorted(iv)
    tot, cur0, cur1 = 0, None, None
    for a, b in iv:
        if cur1 is None or a > cur1:
            if cur1 is not None:
                tot += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    if cur1 is not None:
        tot += cur1 - cur0
    return tot


rows = list(csv.DictReader(open(sys.argv[1])))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ends = [i for i, e in enumerate(ev) if "adamw_kernel" in e[2] and "inc" not in e[2]]
segs = [(ends[i] + 1, ends[i + 1]) for i in range(len(ends) - 1)]
show = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for a, b in segs[-3 - show:-3]:
    seg = ev[a:b + 1]
    t0, t1 = seg[0][0], max(e[1] for e in seg)
    busy = union([(s, e) for s, e, _ in seg])
    print(f"step wall {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle {(t1 - t0 - busy) / 1e6:.3f} ms, "
          f"{len(seg)} kernels")
    by = defaultdict(list)
    for s, e, n in seg:
        by[fam(n)].append((s, e))
    for f, iv in sorted(by.items(), key=lambda kv: -union(kv[1])):
        print(f"  {f:16s} {union(iv) / 1e6:7.3f} ms  n={len(iv):4d}  sum={sum(e - s for s, e in iv) / 1e6:7.3f} ms")
