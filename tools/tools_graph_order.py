"""Where does a HIP graph run a side-stream branch forked before a long kernel?

    python tools/tools_graph_order.py          (GPU box)

main: P (short) -> R (500 us, one 64-KB block per CU: a persistent recurrence) -> T (10 x 50 us,
one 160-KB block per CU: nothing else fits beside it).  side: S (9 x 50 us, one 16-KB block per CU,
fits beside R, not beside T), forked after P.  Ideal (S beside R): ~1.0 ms; S after T or before R: ~1.45.
Variants: where S's launches sit in capture order relative to R, and whether main joins S right after R.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib  # noqa: E402


def busy(lib, blocks, lds, us):
    _lib.check(lib.mrg_debug_busy(blocks, 64, lds, us, torch.cuda.current_stream().cuda_stream), "busy")


def body(lib, variant, side, cus):
    cur = torch.cuda.current_stream()
    busy(lib, cus, 16384, 20.0)                      # P

    def S():
        with torch.cuda.stream(side):
            for _ in range(9):
                busy(lib, cus, 16384, 50.0)
    if variant == "side-first":
        side.wait_stream(cur)
        S()
        busy(lib, cus, 65536, 500.0)                 # R
    elif variant in ("mark-after", "mark-after-join", "mark-after-newstream"):
        mark = torch.cuda.Event()
        mark.record(cur)
        busy(lib, cus, 65536, 500.0)                 # R
        s2 = torch.cuda.Stream() if variant == "mark-after-newstream" else side
        s2.wait_event(mark)
        with torch.cuda.stream(s2):
            for _ in range(9):
                busy(lib, cus, 16384, 50.0)
        if variant == "mark-after-join":
            cur.wait_stream(s2)
        if s2 is not side:
            side.wait_stream(s2)
    elif variant == "serial":
        busy(lib, cus, 65536, 500.0)
        for _ in range(9):
            busy(lib, cus, 16384, 50.0)
    for _ in range(10):
        busy(lib, cus, 160 * 1024, 50.0)             # T
    cur.wait_stream(side)


def main():
    import faulthandler
    faulthandler.enable()
    lib = _lib.load()
    dev = torch.device("cuda:0")
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    for variant in sys.argv[1:] or ("serial", "side-first", "mark-after", "mark-after-join", "mark-after-newstream"):
        side = torch.cuda.Stream(device=dev)
        for _ in range(2):
            body(lib, variant, side, cus)
        torch.cuda.synchronize()
        print(f"{variant}: eager ok", flush=True)
        t0 = time.perf_counter()
        for _ in range(5):
            body(lib, variant, side, cus)
        torch.cuda.synchronize()
        eager = (time.perf_counter() - t0) / 5 * 1e3
        g = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(device=dev)
        with torch.cuda.stream(cap):
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=cap):
                body(lib, variant, side, cus)
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        rep = (time.perf_counter() - t0) / 5 * 1e3
        print(f"{variant:22s} eager {eager:6.3f} ms   graph replay {rep:6.3f} ms", flush=True)


if __name__ == "__main__":
    main()
