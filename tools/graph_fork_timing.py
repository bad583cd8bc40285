"""Diagnostics: when does the HIP graph executor start side-stream work forked at several points of
the main stream?  Main stream: NM busy kernels of US microseconds each (mrg_debug_busy, 1 workgroup
so the side fits beside it).  Side work: after main kernel k of each fork point k in FORKS, NS busy
kernels, issued either on ONE side stream (a single chain with several incoming edges: the
production pattern of functional._flush_deferred) or on a fresh stream per fork point (each branch
one incoming and one outgoing edge).  Joined at the end.  Prints, per replay, each side kernel's
start relative to the step's start, from HIP events (eager) -- run under
`rocprofv3 --kernel-trace` for the replayed graph's real timeline.

    python tools/graph_fork_timing.py [one|many]         (on a GPU box)
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib  # noqa: E402

NM, US, NS = int(os.environ.get("NM", "12")), 200.0, 2
FORKS = tuple(int(x) for x in os.environ.get("FORKS", "1,5,9").split(","))
# REC=1: every fourth main kernel is a "recurrence" (256 workgroups x 512 threads, one per CU) and the
# side kernels are 120 workgroups x 256 threads, as in the headline step's backward
REC = os.environ.get("REC") == "1"


def main(mode):
    lib = _lib.load()
    torch.cuda.init()
    main_s = torch.cuda.Stream()
    sides = [torch.cuda.Stream() for _ in FORKS] if mode == "many" else [torch.cuda.Stream()]

    def busy(stream, us, blocks=1):
        _lib.check(lib.mrg_debug_busy(blocks, 256, 1024, us, ctypes.c_void_p(stream.cuda_stream)), "busy")

    def step():
        cur = torch.cuda.current_stream()
        used = []
        for k in range(NM):
            if REC and k % 4 == 2:
                _lib.check(lib.mrg_debug_busy(256, 512, 16384, US, ctypes.c_void_p(cur.cuda_stream)), "rec")
            else:
                busy(cur, US, 1200 if REC else 1)
            if k in FORKS:
                s = sides[FORKS.index(k)] if mode == "many" else sides[0]
                ev = torch.cuda.Event()
                ev.record(cur)
                s.wait_event(ev)
                for _ in range(NS):
                    busy(s, US / 2, 120 if REC else 1)
                if s not in used:
                    used.append(s)
        for s in used:
            cur.wait_stream(s)

    with torch.cuda.stream(main_s):
        step()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(main_s):
        with torch.cuda.graph(g, stream=main_s):
            step()
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"{mode}: {e0.elapsed_time(e1) / 5 * 1e3:.0f} us per replay; main chain alone {NM * US:.0f} us, "
          f"side work {len(FORKS) * NS * US / 2:.0f} us (forks after main kernels {FORKS})", flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "one")
