"""Per-family kernel time per step of the graph-replayed bench step from a rocprofv3 kernel trace,
the cross-check of bench.py's live probe (bench.trace_check).

    python tools/tools_trace_roofline.py <run_kernel_trace.csv> profiles/r03_trace_roofline.json

Steps are delimited by adamw_kernel.  "replay": the median over the graph-replayed steps (the first
segment, capture / warm-up tail, and the last two dropped); "probe": the mean over the last two
segments, the bench's eager one-stream probe steps, launch for launch what bench.py brackets live.
A family's time is the SUM of its kernels' durations (what the probe's brackets add up), split-K
reduce and row-sum helpers counted with the GEMMs.
"""
import csv
import json
import statistics
import sys

FAMS = {
    "gemm": ("gemm_", "splitk_reduce", "asum_reduce"),
    "lstm_fwd": ("lstm_fwd_kernel", "lstm_fwd_mx_kernel"),
    "lstm_bwd": ("lstm_bwd_kernel", "lstm_bwd_mx_kernel"),
    "attn_fwd": ("attn_fwd",),
    "attn_bwd": ("attn_bwd",),
}


def fam(name):
    n = name.split("(")[0]
    for f, keys in FAMS.items():
        if any(k in n for k in keys):
            return f
    return None


def main():
    src, dst = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else None)
    rows = list(csv.DictReader(open(src)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    ends = [i for i, e in enumerate(ev) if "adamw_kernel" in e[2] and "inc" not in e[2]]
    allsegs = [(ends[i] + 1, ends[i + 1]) for i in range(len(ends) - 1)]
    segs, probe = allsegs[1:-2], allsegs[-2:]
    per = {f: [] for f in FAMS}
    pper = {f: [] for f in FAMS}
    kinds = {f: set() for f in FAMS}
    walls = []
    for a, b in probe:
        acc = {f: 0.0 for f in FAMS}
        for s, e, n in ev[a:b + 1]:
            f = fam(n)
            if f:
                acc[f] += (e - s) / 1e6
        for f in FAMS:
            pper[f].append(acc[f])
    for a, b in segs:
        seg = ev[a:b + 1]
        walls.append((max(e[1] for e in seg) - seg[0][0]) / 1e6)
        acc = {f: [0.0, 0] for f in FAMS}
        for s, e, n in seg:
            f = fam(n)
            if f:
                acc[f][0] += (e - s) / 1e6
                acc[f][1] += 1
                kinds[f].add(n.split("(")[0].replace("void ", "").split("<")[0])
        for f in FAMS:
            per[f].append(acc[f])
    doc = {"source": src, "replayed_steps": len(segs), "step_wall_ms": round(statistics.median(walls), 3),
           "families": {}}
    for f, v in per.items():
        if not v:
            continue
        ms = statistics.median(x[0] for x in v)
        n = statistics.median(x[1] for x in v)
        doc["families"][f] = {"replay_ms_per_step": round(ms, 4), "kernels_per_step": n,
                              "probe_ms_per_step": round(sum(pper[f]) / max(1, len(pper[f])), 4),
                              "kernels": sorted(kinds[f])}
    txt = json.dumps(doc, indent=1)
    if dst:
        open(dst, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
