"""Per-kernel SQ counter summary from tools_step_pmc.sh (averages per dispatch)."""
import collections
import csv
import re
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/spmc"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ("p1", "p2"):
    for r in csv.DictReader(open(f"{src}/{p}/p_counter_collection.csv")):
        m = re.search(r"mrg::(\w+)(<[^>(]*>)?", r["Kernel_Name"])
        if m:
            agg[m.group(1) + (m.group(2) or "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
keys = ["SQ_WAVES", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
        "SQ_INSTS_VMEM_WR", "SQ_LDS_BANK_CONFLICT"]
for k, c in sorted(agg.items()):
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    wc = avg.get("SQ_WAVE_CYCLES", 0) or 1
    busy = avg.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
    print(f"{k[:46]:46s} n={len(c.get('SQ_WAVES', [])):3d} " +
          " ".join(f"{n[3:]}={avg.get(n, 0):.3g}" for n in keys) +
          f" wait_any={avg.get('SQ_WAIT_ANY', 0) / wc:.2f} wait_inst={avg.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}"
          f" active={avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} lds_wait={avg.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}"
          f" mfma_busy={busy:.3g} busy_cyc={avg.get('SQ_BUSY_CYCLES', 0):.3g}")
