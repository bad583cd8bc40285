"""Per-stage phases of the persistent generation loop (gen.hip gen_loop_kernel, block 0's shader-clock
stamps of row group 0.s 16 members): median ns of each stage, the members. spread, and whether the hand-offs stayed in one
XCD's L2.  Usage: python tools/gen_stamps.py [T]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib  # noqa: E402
from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 60
dev = torch.device("cuda", 0)
mc, oc, me = C.lstmformer_config(ratio=1)
torch.manual_seed(0)
m = Metaformer(mc, oc, me).to(dev).eval()
batch = make_batch(B=64, T=T, lead=12, seed=1234, device=dev)
mask = torch.ones(T, dtype=torch.bool, device=dev)
lib = _lib.load()
buf = torch.zeros(T, 16, 32, dtype=torch.int64, device=dev)   # [frame][member of row group 0][slot]
with torch.no_grad():
    m._generate(batch, sampling_mask=mask)
    torch.cuda.synchronize()
    lib.mrg_gen_loop_debug_stamps(buf.data_ptr())
    m._generate(batch, sampling_mask=mask)
    torch.cuda.synchronize()
    lib.mrg_gen_loop_debug_stamps(None)
s = buf.cpu()
local = min(int(s[0, jm, 31]) for jm in range(16))
s[0, :, 31] = s[0, :, 30]
names = ["S1 lstm", "S2 mixer", "S3 integ", "S4 cat", "S5 ffn"]
fr = s[1:T - 1]
d = (s[2:, 0, 0] - s[1:-1, 0, 0]).double()
print(f"local hand-offs: {local}; frame median {int(d.median()) * 10} ns (member 0; 100 MHz real-time stamps)")
print(f"  {'stage (member 0 durations)':24s} {'ns':>6s}   spread over members at its end (median / p90), slowest member")


def row(nm, k, prev):
    cur = fr[:, 0, k]
    end = fr[:, :, k].double()
    rel = end - end.min(dim=1, keepdim=True).values
    spread = rel.max(dim=1).values
    slow = torch.bincount(rel.argmax(dim=1), minlength=16)
    print(f"  {nm:24s} {int((cur - prev).median()) * 10:6d}   {int(spread.median()) * 10:6d} / "
          f"{int(spread.quantile(0.9)) * 10:6d}   member {int(slow.argmax())} ({int(slow.max())} of {len(rel)})")
    return cur


prev = fr[:, 0, 0]
for k in range(5):
    for i, nm in enumerate(names):
        prev = row(f"block {k} {nm}", 1 + 5 * k + i, prev)
row("output", 30, prev)
