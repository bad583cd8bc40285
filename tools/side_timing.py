"""Diagnostics (timing only): when does each flush of the deferred weight-gradient queue run on the
side stream in the replayed headline step, without a profiler attached?  Wall-clock stamps
(mrg_debug_stamp, 1-thread kernels captured INTO the graph) at the step's start, at each flush's
fork point on the main stream, before and after every flush on its side stream, at the backward's
end and the step's end; after a replay their times from the start are printed (ms).  Env as for
bench.py (MRG_REC_STREAM, ...).

    python tools/side_timing.py            (GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import configs as C, functional as Fn  # noqa: E402
from multimodalreactiongeneration_amd.graphs import capture  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402

import ctypes  # noqa: E402
from multimodalreactiongeneration_amd import _lib  # noqa: E402

LABELS = []   # slot -> label, recorded during the capture
ON = [False]
BUF = []


def ev(label, stream):
    if ON[0]:
        _lib.check(_lib.load().mrg_debug_stamp(ctypes.c_void_p(BUF[0].data_ptr()), len(LABELS),
                                               ctypes.c_void_p(stream.cuda_stream)), "stamp")
        LABELS.append(label)


def main():
    dev = torch.device("cuda", 0)
    BUF.append(torch.zeros(4096, dtype=torch.int64, device=dev))
    orig_flush = Fn._flush_deferred

    def flush(key, device, cap=0, after=None):
        n = len(Fn._PENDING.get(key, []))
        if n == 0:
            return orig_flush(key, device, cap, after)
        ev(f"fork point (main) of a flush of {n}", torch.cuda.current_stream(device))
        orig_flush(key, device, cap, after)
        rec = Fn._REC_ON[0] and after is not None
        ev(f"  {'recurrence' if rec else 'side'}-stream end of flush of {n}", Fn._REC[key] if rec else Fn._SIDE[key])
    Fn._flush_deferred = flush
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to(dev)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=64, T=300, seed=1234, device=dev)
    one = torch.ones((), device=dev)

    def step():
        ev("step start", torch.cuda.current_stream())
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward(one)
        ev("backward end (after join)", torch.cuda.current_stream())
        opt.step()
        ev("step end", torch.cuda.current_stream())
    orig_capture_graph = torch.cuda.graph

    class marked_graph(orig_capture_graph):
        def __enter__(self):
            ON[0] = True
            return super().__enter__()

        def __exit__(self, *a):
            r = super().__exit__(*a)
            ON[0] = False
            return r
    torch.cuda.graph = marked_graph
    replay = capture(step, 2, preserve=opt.state_tensors())
    torch.cuda.graph = orig_capture_graph
    for _ in range(3):
        replay()
    torch.cuda.synchronize()
    st = BUF[0][:len(LABELS)].cpu().tolist()
    for label, v in zip(LABELS, st):
        print(f"{(v - st[0]) / 1e5:8.3f} ms  {label}", flush=True)   # 100 MHz clock


if __name__ == "__main__":
    main()
