"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools_pmc.sh) into per-kernel HBM bytes per launch.

    python tools/tools_pmc_summary.py gpurun_out/r02/pmc profiles/r02_pmc_summary.json

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE (KiB) is doubled on gfx950
(it tallies 128-B requests at 64 B); WRITE_SIZE is taken as is.
"""
import collections
import csv
import json
import os
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
dst = sys.argv[2] if len(sys.argv) > 2 else None


def family(name):
    m = re.search(r"mrg::(\w+)(<[^>(]*>)?", name)
    if not m:
        return None
    return m.group(1) + (m.group(2) or "")


def load(counter):
    path = os.path.join(src, counter, "pmc_counter_collection.csv")
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        f = family(r["Kernel_Name"])
        if f:
            out[f].append(float(r["Counter_Value"]) * 1024.0)
    return out


fetch, write = load("FETCH_SIZE"), load("WRITE_SIZE")
summary = {}
for k in sorted(set(fetch) | set(write)):
    rd = [2.0 * v for v in fetch.get(k, [])]
    wr = write.get(k, [])
    if not rd or not wr:
        continue
    summary[k] = {"dispatches": len(rd), "read_bytes_per_launch": sum(rd) / len(rd),
                  "write_bytes_per_launch": sum(wr) / len(wr),
                  "hbm_bytes_per_launch": sum(rd) / len(rd) + sum(wr) / len(wr)}


def fam_total(prefix, extra=()):
    """Bytes per launch of the kernels matching `prefix`; kernels matching `extra` (helpers issued
    inside the same library call, e.g. the split-K slab reduce of a weight-gradient GEMM) add their
    bytes but not their dispatches, so the figure is per library launch, like the bench's probe."""
    prefixes = (prefix,) if isinstance(prefix, str) else prefix
    ks = [k for k in summary if k.startswith(prefixes)]
    xs = [k for k in summary if extra and k.startswith(tuple(extra))]
    n = sum(summary[k]["dispatches"] for k in ks)
    if not n:
        return None
    tot = sum(summary[k]["hbm_bytes_per_launch"] * summary[k]["dispatches"] for k in ks + xs)
    return {"dispatches": n, "hbm_bytes_per_launch": tot / n, "variants": ks, "helpers": xs}


doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over "
                 "`bench.py --graph 0 --cpu-baseline 0 --steps 1 --warmup 1`; FETCH_SIZE x2 (gfx950 correction)",
       "families": dict({p: fam_total(p) for p in ("lstm_fwd_kernel", "lstm_bwd_kernel", "gemm_x6_kernel", "gemm_f32_kernel",
                                                   "splitk_reduce", "attn_fwd_kernel", "attn_bwd", "resln",
                                                   "adamw_kernel")},
                        lstm_fwd=fam_total(("lstm_fwd_kernel", "lstm_fwd_mx_kernel")),
                        lstm_bwd=fam_total(("lstm_bwd_kernel", "lstm_bwd_mx_kernel")),
                        gemm_all=fam_total(("gemm_x6_kernel", "gemm_x6g_kernel", "gemm_x6g_wgrad_kernel", "gemm_x6w_kernel",
                                            "gemm_x6r_kernel",
                                            "gemm_rows_kernel", "gemm_f32_kernel", "gemm_bf16"),
                                           extra=("splitk_reduce",))),
       "kernels": summary}
txt = json.dumps(doc, indent=1)
if dst:
    open(dst, "w").write(txt + "\n")
for k, v in sorted(summary.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"] * kv[1]["dispatches"])[:25]:
    print(f"{k:55s} n={v['dispatches']:4d}  rd={v['read_bytes_per_launch']/1e6:9.2f} MB  "
          f"wr={v['write_bytes_per_launch']/1e6:9.2f} MB")
print(json.dumps(doc["families"]["lstm_fwd_kernel"]))
