"""Does any device memory serve allocations of two different streams inside one capture of the
B=64 step (split-fork variant of DESIGN.md §4a: layer 4's weight-gradient products as separate forks,
deferral off)?  Records the caching allocator's history over the capture and reports address
ranges allocated on more than one stream, with the Python frames of both allocations.

    python tools/tools_capture_alias.py          (GPU box)
"""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd import encoder_stack as ES  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402

_orig_wg = ES._EncoderStackFn._weight_grads


def _wg(lib, ch, st, gr, l, *a):
    ES.SPLIT_FORKS = (l == 4) if SPLIT[0] else False
    return _orig_wg(lib, ch, st, gr, l, *a)


ES._EncoderStackFn._weight_grads = staticmethod(_wg)
SPLIT = [True]


def frames(ev):
    out = []
    for f in ev.get("frames", []):
        fn = f.get("filename", "")
        if "multimodalreactiongeneration_amd" in fn or "tools" in fn:
            out.append(f"{os.path.basename(fn)}:{f.get('line')}:{f.get('name')}")
    return out[:4]


def main():
    Fn.set_wgrad_defer(False)
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to("cuda:0")
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=64, T=300, ratio=1, seed=5, device="cuda:0")

    def step():
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward()
    for split in (True, False):
        SPLIT[0] = split
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        torch.cuda.memory._record_memory_history(max_entries=2_000_000, clear_history=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        torch.cuda.synchronize()
        snap = torch.cuda.memory._snapshot()
        torch.cuda.memory._record_memory_history(enabled=None)
        ev = [e for e in snap["device_traces"][0] if e["action"] == "alloc"]
        streams = defaultdict(int)
        for e in ev:
            streams[e["stream"]] += 1
        print(f"split={split}: {len(ev)} allocations in the capture, per stream {dict(streams)}", flush=True)
        # address ranges shared by allocations of different streams
        byaddr = sorted(ev, key=lambda e: e["addr"])
        hits = 0
        for i, a in enumerate(byaddr):
            for b in byaddr[i + 1:]:
                if b["addr"] >= a["addr"] + a["size"]:
                    break
                if b["stream"] != a["stream"]:
                    hits += 1
                    if hits <= 6:
                        print(f"  overlap: {a['addr']:#x}+{a['size']} stream {a['stream']:#x} {frames(a)}\n"
                              f"           {b['addr']:#x}+{b['size']} stream {b['stream']:#x} {frames(b)}", flush=True)
        print(f"  {hits} cross-stream overlapping allocation pairs", flush=True)
        del g
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
