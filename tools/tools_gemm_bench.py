"""Per-shape timing of mrg_gemm_f32 on the GEMM shapes of the lstmformer step (B=64, T=300, H=256).

    python tools/tools_gemm_bench.py            (on a GPU box)

Prints TFLOP/s per shape against the 157.3 TF f32 MFMA peak, plus the step-weighted total.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402

R = 64 * 300
# (name, M, N, K, transA, transB, calls per step, wgrad)
SHAPES = [
    ("lstm Gx  X W_ih^T", R, 1024, 256, 0, 1, 15, False),
    ("lstm dX  dG W_ih", R, 256, 1024, 0, 0, 15, False),
    ("lstm dW  dG^T X", 1024, 256, R, 1, 0, 30, True),
    ("lin256 fwd", R, 256, 256, 0, 1, 35, False),
    ("lin256 dX", R, 256, 256, 0, 0, 35, False),
    ("lin256 dW", 256, 256, R, 1, 0, 35, True),
    ("kv512 fwd", R, 512, 256, 0, 1, 10, False),
    ("kv512 dX", R, 256, 512, 0, 0, 10, False),
    ("kv512 dW", 512, 256, R, 1, 0, 10, True),
    ("cat512 fwd", R, 256, 512, 0, 1, 5, False),
    ("ffn 256->64", R, 64, 256, 0, 1, 6, False),
    ("ffn 64->256", R, 256, 64, 0, 1, 5, False),
]
PROBES = [
    ("square NN 4096^3", 4096, 4096, 4096, 0, 0, 0, False),
    ("square NT 4096^3", 4096, 4096, 4096, 0, 1, 0, False),
    ("square TN 4096^3", 4096, 4096, 4096, 1, 0, 0, False),
    ("4096x4096 K=256 NT", 4096, 4096, 256, 0, 1, 0, False),
    ("19200x1024 K=1024 NT", R, 1024, 1024, 0, 1, 0, False),
    ("lstm dX as NT (W_ih^T copy)", R, 256, 1024, 0, 1, 0, False),
    ("kv512 dX as NT", R, 256, 512, 0, 1, 0, False),
    ("odd NN 1000x70x45", 1000, 70, 45, 0, 0, 0, False),
    ("odd NT 333x129x97", 333, 129, 97, 0, 1, 0, False),
    ("odd TN 130x66x1001", 130, 66, 1001, 1, 0, 0, False),
    ("odd TT 77x200x33", 77, 200, 33, 1, 1, 0, False),
    ("odd wgrad 1024x6x19200", 6, 1024, R, 1, 0, 0, True),
]


def run_shape(M, N, K, ta, tb, wgrad, iters=20):
    dev = "cuda:0"
    A = torch.randn((K, M) if ta else (M, K), device=dev)
    B = torch.randn((N, K) if tb else (K, N), device=dev)
    C = torch.zeros(M, N, device=dev)
    lda = A.shape[1]
    ldb = B.shape[1]
    splits = Fn.wgrad_splits(M, N, K) if wgrad else 1

    planes = os.environ.get("MRG_BENCH_PLANES") == "1" and not ta and tb and not wgrad
    if planes:   # B as a weight [N][K] with its bf16 planes (functional.prepare_weight_planes)
        Fn.prepare_weight_planes([B])

    def go():
        if planes:
            Fn._fwd_gemm(M, N, K, Fn._ptr(A), lda, B, Fn._ptr(C), N, device=A.device)
            return
        Fn.gemm(M, N, K, Fn._ptr(A), ta, lda, Fn._ptr(B), tb, ldb, Fn._ptr(C), N,
                beta=1.0 if wgrad else 0.0, splits=splits, device=A.device)
    go()
    torch.cuda.synchronize()
    ref = ((A.t() if ta else A).double() @ (B.t() if tb else B).double())
    err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
    for _ in range(2):
        go()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        go()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    return ms, splits, err


def main():
    from multimodalreactiongeneration_amd import _lib
    modes = [int(m) for m in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1, 0]
    for mode in modes:   # 2 = bf16 operands (mrg_gemm_bf16_ex, models' precision "bf16")
        _lib.check(_lib.load().mrg_gemm_set_mode(1 if mode == 2 else mode), "mode")
        print(f"=== GEMM mode {mode} ({ {0: 'exact f32 MFMA', 1: 'x6 bf16 split', 2: 'bf16 operands'}[mode] })")
        with Fn.precision("bf16" if mode == 2 else "32"):
            one_mode()


def one_mode():
    tot_ms = tot_fl = 0.0
    for name, M, N, K, ta, tb, calls, wgrad in SHAPES:
        ms, splits, err = run_shape(M, N, K, ta, tb, wgrad)
        fl = 2.0 * M * N * K
        tf = fl / (ms / 1e3) / 1e12
        tot_ms += ms * calls
        tot_fl += fl * calls
        print(f"{name:20s} M={M:6d} N={N:5d} K={K:6d} splits={splits:3d}  {ms*1e3:8.1f} us  "
              f"{tf:6.1f} TF/s ({tf/157.3*100:5.1f}%)  x{calls}/step  err={err:.1e}")
    print(f"step-weighted: {tot_ms:.2f} ms/step, {tot_fl/(tot_ms/1e3)/1e12:.1f} TF/s")
    for name, M, N, K, ta, tb, calls, wgrad in PROBES:
        ms, splits, err = run_shape(M, N, K, ta, tb, wgrad, iters=5)  # noqa
        tf = 2.0 * M * N * K / (ms / 1e3) / 1e12
        print(f"{name:20s} {ms*1e3:8.1f} us  {tf:6.1f} TF/s ({tf/157.3*100:5.1f}%)  err={err:.1e}")


if __name__ == "__main__":
    main()
