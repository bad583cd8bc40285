"""Dump the captured B=64 lstmformer step's HIP graph (hipGraphDebugDotPrint through torch's
CUDAGraph.debug_dump) with one side-stream fork per weight-gradient product and without, deferral
off, for offline dependency analysis (tools/tools_dot_deps.py).

    python tools/tools_capture_dot.py OUTDIR          (GPU box)
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd import encoder_stack as ES  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402


def main(out):
    out = os.path.abspath(out)
    os.makedirs(out, exist_ok=True)
    Fn.set_wgrad_defer(False)
    for split in (True, False):
        ES.SPLIT_FORKS = split
        mc, oc, me = C.lstmformer_config(ratio=1)
        torch.manual_seed(0)
        m = Metaformer(mc, oc, me).to("cuda:0")
        opt = m.configure_optimizers()["optimizer"]
        batch = make_batch(B=64, T=300, ratio=1, seed=5, device="cuda:0")

        def step():
            opt.zero_grad()
            m.training_step(list(batch))["loss"].backward()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph(keep_graph=True)
        with torch.cuda.graph(g):
            step()
        torch.cuda.synchronize()
        path = os.path.join(out, f"step_split{int(split)}.dot")
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipGraphDebugDotPrint.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint]
        rc = hip.hipGraphDebugDotPrint(ctypes.c_void_p(g.raw_cuda_graph()), path.encode(), 1)
        print(f"hipGraphDebugDotPrint rc={rc}", flush=True)
        print(f"split_forks={int(split)}: {path} exists {os.path.exists(path)}", flush=True)
        del g, m, opt
        torch.cuda.synchronize()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/dot")
