"""simple_lstm (BASELINE configs[1]) graph-replayed steps in fp32 then bf16, for a kernel trace.

    rocprofv3 --kernel-trace --stats -d DIR -o run -- python3 tools/tools_c2_prof.py     (GPU box)
    python3 tools/tools_timeline.py DIR/run_kernel_trace.csv 6    (last 3 fp32-replay steps + bf16)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd.graphs import capture  # noqa: E402
from multimodalreactiongeneration_amd.model import SimpleLSTM  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_simple_batch  # noqa: E402


def main():
    dev = "cuda:0"
    for prec in ("32", "bf16"):
        cfg, oc, me = C.simple_lstm_config()
        torch.manual_seed(0)
        m = SimpleLSTM(cfg, oc, me).set_precision(prec).to(dev)
        opt = m.configure_optimizers()["optimizer"]
        batch = make_simple_batch(B=64, T=300, device=dev)

        def step():
            opt.zero_grad()
            m.training_step(batch)["loss"].backward()
            opt.step()
        replay = capture(step, 2, preserve=opt.state_tensors())
        for _ in range(3):
            replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            replay()
        torch.cuda.synchronize()
        print(f"C2 {prec}: {(time.perf_counter() - t0) / 5 * 1e3:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
