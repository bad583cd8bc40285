"""LSTM recurrence launch time vs group size (members per batch-row group) and problems per launch.

    python tools/tools_lstm_groups.py        (on a GPU box)

H = 256, B = 64, T = 300 (the lstmformer encoder layers); fwd = one persistent forward launch of
nprob independent recurrences, bwd = the matching backward launch (timed from the probes).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib, functional as Fn  # noqa: E402

DEV = "cuda:0"


def main():
    lib = _lib.load()
    H, B, T = 256, 64, 300
    g = torch.Generator().manual_seed(0)
    nps = [int(v) for v in os.environ.get("NPROB", "1,2,3").split(",")]
    bss = [int(v) for v in os.environ.get("FORCE_BS", "0").split(",")]
    gs = [int(v) for v in os.environ.get("GROUPS", "8,16").split(",")]
    if "MX" in os.environ:   # 0: VALU form only, 2: MFMA form whenever it fits (lstm_mx.hip)
        lib.mrg_lstm_set_mx(int(os.environ["MX"]), 0)   # returns the previous mode
    for G, nprob, fbs in [(G, n, b) for G in gs for n in nps for b in bss]:
            _lib.check(lib.mrg_lstm_config(G), "cfg")
            probs = []
            for _ in range(nprob):
                w = [(torch.randn(4 * H, H, generator=g) * 0.06).to(DEV).requires_grad_(True) for _ in range(2)]
                bb = [(torch.randn(4 * H, generator=g) * 0.06).to(DEV).requires_grad_(True) for _ in range(2)]
                x = torch.randn(B, T, H, generator=g).to(DEV).requires_grad_(True)
                probs.append((x, w[0], w[1], bb[0], bb[1]))
            try:
                for _ in range(2):
                    ys = Fn.lstm_layers_batched(probs, force_bs=fbs)
                    sum(y.sum() for y in ys).backward()
            except RuntimeError as e:
                print(f"G={G:2d} nprob={nprob} bs={fbs}  {e}", flush=True)
                continue
            torch.cuda.synchronize()
            Fn.probe_start("lstm_fwd", "lstm_bwd")
            for _ in range(5):
                ys = Fn.lstm_layers_batched(probs, force_bs=fbs)
                sum(y.sum() for y in ys).backward()
            t = Fn.probe_stop()
            Fn.check_errors()
            f = sorted(t.get("lstm_fwd", [0]))[len(t.get("lstm_fwd", [0])) // 2]
            b = sorted(t.get("lstm_bwd", [0]))[len(t.get("lstm_bwd", [0])) // 2]
            print(f"G={G:2d} nprob={nprob:2d} bs={fbs:2d}  fwd {f * 1e3:7.1f} us ({f * 1e3 / T:5.2f} us/step)  "
                  f"bwd {b * 1e3:7.1f} us ({b * 1e3 / T:5.2f} us/step)", flush=True)


if __name__ == "__main__":
    main()
