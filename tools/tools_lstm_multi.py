"""Per-step cost of the H = 256, B = 64 recurrence with n independent problems per launch, by form and
batch tile: is a (block, time-chunk) wavefront over the metaformer blocks' single-problem recurrences
 worth it?  Kernel-bound probes (the recurrence kernels only), fwd and bwd.

    python tools/tools_lstm_multi.py          (GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402


def run(n, T, mx, bs, dev):
    lib = _lib.load()
    B, H = 64, 256
    g = torch.Generator(device="cpu").manual_seed(0)
    probs = []
    for _ in range(n):
        x = torch.randn(B, T, H, generator=g).to(dev).requires_grad_(True)
        ws = [(torch.randn(4 * H, H, generator=g) * 0.06).to(dev).requires_grad_(True),
              (torch.randn(4 * H, H, generator=g) * 0.06).to(dev).requires_grad_(True),
              (torch.randn(4 * H, generator=g) * 0.06).to(dev).requires_grad_(True),
              (torch.randn(4 * H, generator=g) * 0.06).to(dev).requires_grad_(True)]
        probs.append((x, *ws))
    prev = lib.mrg_lstm_set_mx(mx, 0)
    try:
        for it in range(3):
            if it == 2:
                Fn.probe_start("lstm_fwd", "lstm_bwd", kernel=True)
            ys = Fn.lstm_layers_batched(probs, force_bs=bs)
            sum((y * 1.0).sum() for y in ys).backward()
        per = Fn.probe_stop()
    finally:
        lib.mrg_lstm_set_mx(prev, 0)
    Fn.check_errors()
    f, b = sum(per.get("lstm_fwd", [0])), sum(per.get("lstm_bwd", [0]))
    print(f"n={n} T={T} mx={mx} bs={bs}: fwd {f * 1e3:7.1f} us ({f * 1e6 / T:6.0f} ns/step)  "
          f"bwd {b * 1e3:7.1f} us ({b * 1e6 / T:6.0f} ns/step)", flush=True)


def main():
    dev = torch.device("cuda:0")
    for n, mx, bs in ((1, 0, 0), (1, 0, 1), (1, 0, 2), (2, 0, 2), (2, 0, 4), (3, 0, 4), (4, 0, 4), (4, 0, 8),
                      (1, 2, 0), (2, 2, 0), (3, 2, 0), (4, 2, 0)):
        for T in (100, 300):
            try:
                run(n, T, mx, bs, dev)
            except Exception as e:   # a shape the launcher refuses
                print(f"n={n} T={T} mx={mx} bs={bs}: {str(e)[:120]}", flush=True)


if __name__ == "__main__":
    main()
