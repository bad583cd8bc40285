"""Per-stage phases of the persistent scheduled-sampling decode loops (ssd_loop.hip: ssd_loop_kernel
forward, ssd_loop_bwd_kernel backward; the 100 MHz real-time stamps of group 0's 16 members) at bench.py's C3 shape
(LSTMwithSample, B=64, T frames, lead 12): median ns of each stage, the members' spread at its end over the frames and whether the
group's hand-offs stayed in one XCD's L2.  Usage: python tools/ssd_stamps.py [T]."""
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
fwd = torch.zeros(T, 16, 16, dtype=torch.int64, device=dev)   # [frame][member of group 0][slot]
bwd = torch.zeros(T, 16, 16, dtype=torch.int64, device=dev)
m.training_step(batch, sampling_mask=mask)["loss"].backward()
torch.cuda.synchronize()
lib.mrg_ssd_loop_debug_stamps(fwd.data_ptr())
lib.mrg_ssd_loop_bwd_debug_stamps(bwd.data_ptr())
m.training_step(batch, sampling_mask=mask)["loss"].backward()
torch.cuda.synchronize()
lib.mrg_ssd_loop_debug_stamps(None)
lib.mrg_ssd_loop_bwd_debug_stamps(None)


def report(title, s, names):
    s = s.cpu()
    local = [int(s[0, j, 15]) for j in range(16)]
    hwid = [int(s[0, j, 14]) for j in range(16)]
    s[0, :, 14:] = 0
    used = [k for k in range(14) if int(s[1, 0, k]) != 0]
    fr = s[1:T - 1]                       # [frames][member][slot]
    d = (s[2:, 0, 0] - s[1:-1, 0, 0]).double()
    print(f"{title}: local hand-offs {min(local)}; per frame median {int(d.median()) * 10} ns (member 0)")
    cus = [((h >> 8) & 15, (h >> 12) & 1, (h >> 13) & 7) for h in hwid]
    print("  members' (CU, SH, SE):", cus, f"distinct CUs {len(set(cus))}")
    prev = fr[:, 0, 0]
    print(f"  {'stage (member 0 durations)':34s} {'ns':>6s}   spread over members at its end (median / p90), slowest member")
    for k in used[1:]:
        cur = fr[:, 0, k]
        end = fr[:, :, k].double()
        rel = end - end.min(dim=1, keepdim=True).values
        spread = rel.max(dim=1).values
        slow = torch.bincount(rel.argmax(dim=1), minlength=16)
        print(f"  {names(k)!s:34s} {int((cur - prev).median()) * 10:6d}   {int(spread.median()) * 10:6d} / "
              f"{int(spread.quantile(0.9)) * 10:6d}   member {int(slow.argmax())} ({int(slow.max())} of {len(rel)})")
        prev = cur


nl = 2
fn = {1: "layer 0 X0 build", 2: "layer 0 gates + publish"}
for i in range(1, nl):
    fn[1 + 2 * i] = f"layer {i} gather"
    fn[2 + 2 * i] = f"layer {i} LN + gates + publish"
fn[1 + 2 * nl] = "ffn gather"
fn[2 + 2 * nl] = "ffn LN / Z / y / select"
report("forward", fwd, lambda k: fn.get(k, k))
bn = {1: "F gather dyx", 2: "F dy / dz / du / LN / cell / P publish"}
for q in range(nl - 1):
    bn[3 + 2 * q] = f"B{nl - 2 - q} gather partials + sums"
    bn[4 + 2 * q] = f"B{nl - 2 - q} dX / LN / cell / " + ("P publish" if nl - 2 - q > 0 else "dyx publish")
report("backward", bwd, lambda k: bn.get(k, k))
