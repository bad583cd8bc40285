"""Diagnostics: the captured headline step (bench.py's schedule: weight gradients deferred beside the
backward recurrences on the side stream, AdamW in the graph) dumped with hipGraphDebugDotPrint, then
for every node whose predecessors are not just the node captured before it (forks and joins), its
predecessors -- to see which main-stream node each deferred weight-gradient chain waits for.

    python tools/capture_side_deps.py OUTDIR          (GPU box)
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
from multimodalreactiongeneration_amd import configs as C, functional as Fn  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402
from tools_dot_deps import parse, short  # noqa: E402


def main(out):
    out = os.path.abspath(out)
    os.makedirs(out, exist_ok=True)
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
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    Fn.reset_fork_point()
    with torch.cuda.graph(g):
        step()
    Fn.reset_fork_point()
    torch.cuda.synchronize()
    path = os.path.join(out, "step.dot")
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipGraphDebugDotPrint.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_uint]
    rc = hip.hipGraphDebugDotPrint(ctypes.c_void_p(g.raw_cuda_graph()), path.encode(), 1)
    print(f"hipGraphDebugDotPrint rc={rc} -> {path}", flush=True)
    nodes, edges = parse(path)
    pred = {}
    for a, b in edges:
        pred.setdefault(b, []).append(a)
    print(f"{len(nodes)} nodes, {len(edges)} edges")
    for i in sorted(nodes):
        p = sorted(pred.get(i, []))
        if p != [i - 1]:
            print(f"{i:4d} {short(nodes[i][1]):28s} {nodes[i][2]:16s} <- " +
                  ", ".join(f"{j}:{short(nodes[j][1])}" for j in p), flush=True)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/side_deps")
