"""Diagnostics: capture the headline step (bench.py's schedule) and replay it REPS times, printing a
marker line before the replays -- for runtime logs of the HIP graph executor (AMD_LOG_LEVEL) or a
kernel trace of the replays alone.

    AMD_LOG_LEVEL=4 python tools/replay_once.py [REPS]        (GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd.graphs import capture  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402


def main(reps):
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
    replay = capture(step, 2, preserve=opt.state_tensors())
    torch.cuda.synchronize()
    print("=== REPLAYS START ===", file=sys.stderr, flush=True)
    sync = os.environ.get("SYNC") == "1"   # 1: synchronize after every replay (no host run-ahead)
    import time
    for i in range(reps):
        t0 = time.perf_counter()
        replay()
        t1 = time.perf_counter()
        if sync:
            torch.cuda.synchronize()
        print(f"replay {i}: host {1e3 * (t1 - t0):.2f} ms", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    print("=== REPLAYS END ===", file=sys.stderr, flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 1)
