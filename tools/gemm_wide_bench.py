"""Per-shape timing of the k-contiguous x6 products (C = A B^T, the step's forward / input-gradient
GEMMs at M = B*T = 19200): the default LDS-DMA kernel on fp32 B (gemm_x6g_kernel), the same kernel on
pre-split B planes, and the row-owning kernel on B planes (gemm_wide.hip, configs bn / ring depth).

    python tools/gemm_wide_bench.py [cfg ...]          (on a GPU box; cfg as mrg_gemm_set_wide)
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib, functional as Fn  # noqa: E402

R = 64 * 300
SHAPES = [(R, 256, 256, 35), (R, 256, 512, 15), (R, 1024, 256, 15), (R, 512, 256, 10), (R, 256, 1024, 15),
          (R, 64, 256, 6), (R, 256, 64, 5), (6400, 1024, 256, 30), (6400, 256, 256, 30)]


def timeit(fn, iters=30):
    fn()
    torch.cuda.synchronize()
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main(cfgs):
    lib = _lib.load()
    dev = "cuda:0"
    VP, CI = ctypes.c_void_p, ctypes.c_int
    st = lambda: VP(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    print(f"{'M':>6} {'N':>5} {'K':>5} {'x6g fp32B':>10} {'x6g planes':>10} " +
          " ".join(f"{'w' + str(c):>8}" for c in cfgs) + "   (us; TF/s of the best; max rel err)")
    tot = {k: 0.0 for k in ["fp32", "pl0"] + [str(c) for c in cfgs]}
    for M, N, K, calls in SHAPES:
        g = torch.Generator().manual_seed(M + N + K)
        A = torch.randn(M, K, generator=g).to(dev)
        B = torch.randn(N, K, generator=g).to(dev)
        C = torch.zeros(M, N, device=dev)
        planes = torch.empty(3, N, K, dtype=torch.int16, device=dev)
        _lib.check(lib.mrg_split_planes_batched(1, (VP * 1)(Fn._ptr(B)), (VP * 1)(VP(planes.data_ptr())), (CI * 1)(N),
                                                (CI * 1)(K), (CI * 1)(0), st()), "split")
        ref = A.double() @ B.double().t()

        def fp32():
            Fn.gemm(M, N, K, Fn._ptr(A), 0, K, Fn._ptr(B), 1, K, Fn._ptr(C), N, device=A.device)

        def pl():
            _lib.check(lib.mrg_gemm_x6_planes(M, N, K, 1.0, Fn._ptr(A), K, 0, 0, VP(planes.data_ptr()), K, N * K,
                                              0.0, Fn._ptr(C), N, None, 0, None, 0, st()), "planes")
        res, errs = {}, {}
        res["fp32"] = timeit(fp32)
        errs["fp32"] = ((C.double() - ref).abs().max() / ref.abs().max()).item()
        prev = lib.mrg_gemm_set_wide(0)
        for key, cfg in [("pl0", 0)] + [(str(c), c) for c in cfgs]:
            lib.mrg_gemm_set_wide(cfg)
            C.zero_()
            res[key] = timeit(pl)
            errs[key] = ((C.double() - ref).abs().max() / ref.abs().max()).item()
        lib.mrg_gemm_set_wide(prev)
        for k in tot:
            tot[k] += res[k] * calls
        best = min(res.values())
        tf = 2.0 * M * N * K / (best * 1e-6) / 1e12
        print(f"{M:6d} {N:5d} {K:5d} {res['fp32']:10.1f} {res['pl0']:10.1f} " +
              " ".join(f"{res[str(c)]:8.1f}" for c in cfgs) +
              f"   {tf:6.1f} TF/s  err " + " ".join(f"{errs[k]:.1e}" for k in res), flush=True)
    print("step-weighted ms: " + "  ".join(f"{k}={v / 1e3:.3f}" for k, v in tot.items()))


if __name__ == "__main__":
    main([int(c) for c in sys.argv[1:]] or [12, 22])
