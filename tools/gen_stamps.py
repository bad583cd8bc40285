"""Per-stage phases of the persistent generation loop (gen.hip gen_loop_kernel, block 0's shader-clock
stamps): median cycles of each stage over the frames, and whether the group's hand-offs stayed in one
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
buf = torch.zeros(T, 32, dtype=torch.int64, device=dev)
with torch.no_grad():
    m._generate(batch, sampling_mask=mask)
    torch.cuda.synchronize()
    lib.mrg_gen_loop_debug_stamps(buf.data_ptr())
    m._generate(batch, sampling_mask=mask)
    torch.cuda.synchronize()
    lib.mrg_gen_loop_debug_stamps(None)
s = buf.cpu()
local = int(s[0, 31])
s[0, 31] = s[0, 30]
names = ["S1 lstm", "S2 mixer", "S3 integ", "S4 cat", "S5 ffn"]
fr = s[1:T - 1]
print(f"local hand-offs: {local}; frame cycles median {int((s[2:, 0] - s[1:-1, 0]).median())}")
prev = fr[:, 0]
for k in range(5):
    for i, nm in enumerate(names):
        cur = fr[:, 1 + 5 * k + i]
        print(f"block {k} {nm:10s} {int((cur - prev).median()):6d} cycles")
        prev = cur
print(f"output        {int((fr[:, 30] - prev).median()):6d} cycles")
