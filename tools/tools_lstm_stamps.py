"""Diagnostics: where a persistent LSTM step spends its time (in-kernel s_memtime stamps, block 0).

    python tools/tools_lstm_stamps.py            (on a GPU box)
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib, functional as Fn  # noqa: E402

H, B, T = int(os.environ.get("H", "256")), 64, 300
dev = "cuda:0"
lib = _lib.load()
FWD = ["gemv", "reduce+pre", "sync1", "cell+publish", "gather", "sync2"]
BWD = ["gather", "cell-bwd", "sync1", "gemv", "reduce+publish", "sync2"]
if os.environ.get("MX") == "2":   # the MFMA form's phases (lstm_mx.hip)
    lib.mrg_lstm_set_mx(2, 0)
    FWD = ["mfma+pre", "sync1", "cell+publish", "gather+split", "sync2", "-"]
    BWD = ["gather", "cell-bwd+split", "sync1", "mfma", "publish+io", "sync2"]


def report(name, st, labels):
    st = st.cpu().numpy().astype("float64")
    d = st[5:T - 5]
    steps = d[1:, 0] - d[:-1, 0]
    phases = [d[:, i + 1] - d[:, i] for i in range(6)]
    print(f"{name}: cycles/step median {sorted(steps)[len(steps)//2]:.0f}  " +
          "  ".join(f"{l}={sorted(p)[len(p)//2]:.0f}" for l, p in zip(labels, phases)))


def run(nprob, force_bs=0):
    g = torch.Generator().manual_seed(0)
    probs = []
    for _ in range(nprob):
        w = [torch.nn.Parameter((torch.randn(4 * H, H, generator=g) * 0.05).to(dev)) for _ in range(2)]
        bb = [torch.nn.Parameter((torch.randn(4 * H, generator=g) * 0.05).to(dev)) for _ in range(2)]
        x = torch.randn(B, T, H, generator=g).to(dev).requires_grad_(True)
        probs.append((x, w[0], w[1], bb[0], bb[1]))
    st = torch.zeros(T * 8, dtype=torch.int64, device=dev)
    for it in range(3):
        rec = it == 2
        lib.mrg_lstm_debug_stamps(ctypes.c_void_p(st.data_ptr()) if rec else None)
        Fn.probe_start("lstm_fwd", "lstm_bwd")
        ys = Fn.lstm_layers_batched(probs, force_bs=force_bs)
        torch.cuda.synchronize()
        if rec:
            report(f"fwd nprob={nprob} bs={force_bs}", st.view(T, 8), FWD)
        sum(y.sum() for y in ys).backward()
        torch.cuda.synchronize()
        lib.mrg_lstm_debug_stamps(None)
        times = Fn.probe_stop()
        if rec:
            report(f"bwd nprob={nprob} bs={force_bs}", st.view(T, 8), BWD)
            print("   launch ms:", {k: [round(x, 3) for x in v] for k, v in times.items()})
    Fn.check_errors()


if __name__ == "__main__":
    for grp in [int(g) for g in os.environ.get("GROUPS", "8").split(",")]:
        _lib.check(lib.mrg_lstm_config(grp), "config")
        print(f"== group256 = {grp}")
        cfgs = os.environ.get("STAMP_CFGS", "1:0,2:0,3:0,1:2,1:4,2:4,4:4,1:8")
        for nprob, bs in [tuple(int(v) for v in c.split(":")) for c in cfgs.split(",")]:
            run(nprob, bs)
