"""Solo (one-workgroup, LDS-exchange) recurrence groups at H <= 128 vs the multi-member hand-off
groups: per-step cost (kernel-bound probes) and agreement of outputs / weight gradients, B = 64,
T = 300, n independent problems per launch.

    python tools/tools_lstm_solo.py          (GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402


def run(H, n, T, solo, dev):
    lib = _lib.load()
    B = 64
    g = torch.Generator(device="cpu").manual_seed(H + n)
    probs = []
    for _ in range(n):
        x = torch.randn(B, T, H, generator=g).to(dev).requires_grad_(True)
        s = 1.0 / H ** 0.5
        ws = [(torch.randn(4 * H, H, generator=g) * s).to(dev).requires_grad_(True),
              (torch.randn(4 * H, H, generator=g) * s).to(dev).requires_grad_(True),
              (torch.randn(4 * H, generator=g) * s).to(dev).requires_grad_(True),
              (torch.randn(4 * H, generator=g) * s).to(dev).requires_grad_(True)]
        probs.append((x, *ws))
    prev = lib.mrg_lstm_set_solo(solo)
    try:
        for it in range(3):
            for p in probs:
                for t in p:
                    t.grad = None
            if it == 2:
                Fn.probe_start("lstm_fwd", "lstm_bwd", kernel=True)
            ys = Fn.lstm_layers_batched(probs)
            sum((y * y).sum() for y in ys).backward()
        per = Fn.probe_stop()
    finally:
        lib.mrg_lstm_set_solo(prev)
    Fn.check_errors()
    f, b = sum(per.get("lstm_fwd", [0])), sum(per.get("lstm_bwd", [0]))
    out = [y.detach().clone() for y in ys] + [p[0].grad.clone() for p in probs] + [p[2].grad.clone() for p in probs]
    return f, b, out


def main():
    dev = torch.device("cuda:0")
    T = 300
    for H in (128, 64, 32):
        for n in (1, 2, 4):
            res = {}
            for solo in (0, 1):
                res[solo] = run(H, n, T, solo, dev)
            d = max(((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item()
                    for a, b in zip(res[1][2], res[0][2]))
            print(f"H={H} n={n}: ring fwd {res[0][0] * 1e6 / T:6.0f} bwd {res[0][1] * 1e6 / T:6.0f} ns/step | "
                  f"solo fwd {res[1][0] * 1e6 / T:6.0f} bwd {res[1][1] * 1e6 / T:6.0f} ns/step | "
                  f"max rel diff (y, dx, dW_hh) {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
