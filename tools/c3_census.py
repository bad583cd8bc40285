"""Kernel census of bench.py's launch-bound secondary lines: the C3 scheduled-sampling train step
(LSTMwithSample, B=64, T=300, lead 12, epoch 30, mask refreshed from the host RNG before each replay)
or lstmformer generation (Metaformer.prediction, B=64 x 300 frames), each captured as one HIP graph
exactly as bench.secondary does and replayed REPS times, for
`rocprofv3 --kernel-trace --stats -- python3 tools/c3_census.py [c3|gen] [REPS]`; per-step figures =
the stats divided by REPS + 2 (the capture's two eager warm-up runs also launch).  Prints ms/step.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd.graphs import capture  # noqa: E402
from multimodalreactiongeneration_amd.model import LSTMwithSample, Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402


def main(which, reps):
    dev = torch.device("cuda", 0)
    B, T = 64, 300
    pre = None
    if which == "c3":
        mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=True)
        torch.manual_seed(0)
        m = LSTMwithSample(mc, oc, me)
        m.current_epoch = 30
        m = m.to(dev)
        opt = m.configure_optimizers()["optimizer"]
        batch = make_batch(B=B, T=T, lead=12, seed=1234, device=dev)
        mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5).to(dev)
        rng = np.random.RandomState(7)

        def pre():
            mask.copy_(torch.from_numpy(rng.rand(T) < 0.5), non_blocking=True)

        def step():
            opt.zero_grad()
            m.training_step(batch, sampling_mask=mask)["loss"].backward()
            opt.step()
        replay = capture(step, 2, preserve=opt.state_tensors())
    else:
        mc, oc, me = C.lstmformer_config(ratio=1)
        torch.manual_seed(0)
        m = Metaformer(mc, oc, me).to(dev).eval()
        batch = make_batch(B=B, T=T, lead=12, seed=1234, device=dev)
        gmask = torch.ones(T, dtype=torch.bool, device=dev)

        def step():
            with torch.no_grad():
                m._generate(batch, sampling_mask=gmask)
        replay = capture(step, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        if pre is not None:
            pre()
        replay()
    torch.cuda.synchronize()
    print(f"{which}: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms/step over {reps} replays "
          f"(+2 eager capture warm-ups in the trace)", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "c3", int(sys.argv[2]) if len(sys.argv) > 2 else 10)
