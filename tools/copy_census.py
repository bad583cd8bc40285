"""Diagnostics: which ATen ops of the headline training step launch torch's own kernels (copies,
fills, elementwise), and from where?  One eager step (B = 64, T = 300, as bench.py) under a
TorchDispatchMode that records every ATen op whose output lands on the GPU, keyed by the innermost
frame inside this repository; the library's own kernels never pass through ATen, so what is
listed is exactly the torch-launched work (the `__amd_rocclr_copyBuffer`, `elementwise_kernel`,
... rows of a kernel trace).  Metadata-only ops (views, empty) are skipped.

    python tools/copy_census.py            (GPU box)
"""
import os
import sys
import traceback
from collections import Counter

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402

# ops that allocate or alias without launching a kernel
SKIP = {"empty", "empty_strided", "empty_like", "view", "_unsafe_view", "reshape", "as_strided", "t", "transpose",
        "permute", "unsqueeze", "squeeze", "expand", "slice", "select", "detach", "alias", "split", "unbind",
        "chunk", "narrow", "split_with_sizes", "_reshape_alias", "lift_fresh", "set_", "resize_", "record_stream",
        "is_nonzero", "item", "_local_scalar_dense", "size", "stride", "numel", "dim", "is_same_size",
        "new_empty", "new_empty_strided", "unfold", "view_as", "_to_copy_meta"}


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.count = Counter()
        self.every = Counter()   # every op seen, by name (skipped ones included)

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.overloadpacket.__name__
        self.every[name] += 1
        if name in SKIP:
            return out
        outs = out if isinstance(out, (tuple, list)) else (out,)
        if not any(isinstance(o, torch.Tensor) and o.is_cuda and o.numel() > 0 for o in outs):
            return out
        where = "?"
        for fr in reversed(traceback.extract_stack()[:-1]):
            if fr.filename.startswith(ROOT) and not fr.filename.endswith("copy_census.py"):
                where = f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno} ({fr.name})"
                break
        self.count[(name, where)] += 1
        return out


def main():
    dev = torch.device("cuda", 0)
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to(dev)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=64, T=300, seed=1234, device=dev)
    one = torch.ones((), device=dev)

    def step():
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward(one)
        opt.step()
    for _ in range(2):   # warm: weight copies / planes made, allocator settled
        step()
    torch.cuda.synchronize()
    cen = Census()
    with cen:
        step()
    torch.cuda.synchronize()
    total = sum(cen.count.values())
    print(f"{total} torch-launched ATen ops in one step; every op seen: {dict(cen.every)}", flush=True)
    for (name, where), n in sorted(cen.count.items(), key=lambda kv: -kv[1]):
        print(f"{n:5d}  {name:28s} {where}", flush=True)


if __name__ == "__main__":
    main()
