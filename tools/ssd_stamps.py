"""Per-stage phases of the persistent scheduled-sampling decode loop (ssd_loop.hip ssd_loop_kernel,
block 0's shader-clock stamps) at bench.py's C3 shape (LSTMwithSample, B=64, T frames, lead 12):
median cycles of each stage over the frames and whether the group's hand-offs stayed in one XCD's L2.
Usage: python tools/ssd_stamps.py [T]."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib  # noqa: E402
from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd.model import LSTMwithSample  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 300
dev = torch.device("cuda", 0)
mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=True)
torch.manual_seed(0)
m = LSTMwithSample(mc, oc, me)
m.current_epoch = 30
m = m.to(dev)
batch = make_batch(B=64, T=T, lead=12, seed=1234, device=dev)
mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5).to(dev)
lib = _lib.load()
buf = torch.zeros(T, 16, dtype=torch.int64, device=dev)
m.training_step(batch, sampling_mask=mask)["loss"].backward()
torch.cuda.synchronize()
lib.mrg_ssd_loop_debug_stamps(buf.data_ptr())
m.training_step(batch, sampling_mask=mask)["loss"].backward()
torch.cuda.synchronize()
lib.mrg_ssd_loop_debug_stamps(None)
s = buf.cpu()
local = int(s[0, 15])
s[0, 15] = 0
used = [k for k in range(15) if int(s[1, k]) != 0]   # slot 0, then per layer / FFN stage (decode.hip order)
nl = (max(used) - 2) // 2
names = {1: "layer 0 X0 build", 2: "layer 0 gates + publish"}
for i in range(1, nl):
    names[1 + 2 * i] = f"layer {i} gather"
    names[2 + 2 * i] = f"layer {i} LN + gates + publish"
names[1 + 2 * nl] = "ffn gather"
names[2 + 2 * nl] = "ffn LN / Z / y / select"
fr = s[1:T - 1]
d = (s[2:, 0] - s[1:-1, 0]).double()
print(f"local hand-offs: {local}; layers {nl}; frame median {int(d.median())} shader-clock cycles")
prev = fr[:, 0]
for k in used[1:]:
    cur = fr[:, k]
    print(f"{names.get(k, k)!s:32s} {int((cur - prev).median()):6d} cycles")
    prev = cur
