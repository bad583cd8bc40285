"""Per-launch timing of the fused scheduled-sampling decode kernels (decode.hip) and of the few-row
dX GEMM at the C3 shape (B = 64, H = 256, HB = 64, FO = 6), each launched back to back N times
inside one captured HIP graph (so the number is device time per launch including the in-graph
launch gap).

    python tools/tools_ssd_kernels.py            (on a GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402

P = Fn._ptr
S = Fn._stream


def timed(fn, n=200):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def main():
    lib = _lib.load()
    dev = "cuda:0"
    B, H, HB, FO, F, FM, T = 64, 256, 64, 6, 140, 6, 4
    r = lambda *s: torch.randn(*s, device=dev) * 0.1  # noqa: E731
    Pm, xf, wf = r(B, H), r(B, F), r(H, F)
    hp, rp, gm, bt = r(B, H), r(B, H), r(H) + 1, r(H)
    xout, mean, rstd = r(B, H), r(B), r(B)
    w_ih, b_ih, b_hh = r(4 * H, H), r(4 * H), r(4 * H)
    gates, c, h = r(B, 4 * H), r(B, H), r(B, H)
    w1, b1, w2, b2 = r(HB, H), r(HB), r(FO, HB), r(FO)
    u, z = r(B, H), r(B, HB)
    mask = torch.ones(T, dtype=torch.uint8, device=dev)
    ms = r(B, T, FM)
    xfn = r(B, F)
    dy, dfn = r(B, T, FO), r(B, H)
    dyt, dz, du, duo, g, dG = r(B, FO), r(B, HB), r(B, H), r(B, H), r(B, H), r(B, 4 * H)
    w_t = w_ih.t().contiguous()
    dX = r(B, H)
    out = {}
    for mode in (0, 1):
        out[f"ssd_gate_cell_fwd mode {mode}"] = timed(lambda: lib.mrg_ssd_gate_cell_fwd(
            B, H, mode, P(Pm), P(hp), P(rp), P(gm), P(bt), 1e-5, P(xout), P(mean), P(rstd),
            P(w_ih), P(b_ih), P(b_hh), P(gates), P(c), P(h), S()))
    for dbg in (1, 2, 3):
        out[f"  gate_cell mode 1 dbg {dbg}"] = timed(lambda: lib.mrg_ssd_gate_cell_fwd_dbg(
            dbg, B, H, 1, P(Pm), P(hp), P(rp), P(gm), P(bt), 1e-5, P(xout), P(mean), P(rstd),
            P(w_ih), P(b_ih), P(b_hh), P(gates), P(c), P(h), S()))
    wms_t = r(FO, H)
    yb = r(B, T, FO)
    for t in (0, 1):
        out[f"ssd_feat_gate_cell_fwd t={t}"] = timed(lambda: lib.mrg_ssd_feat_gate_cell_fwd(
            B, H, HB, FO, F, t, P(Pm), P(z) if t else None, P(w2), P(b2), P(mask), P(ms), T * FM, FM, P(wms_t),
            P(yb) if t else None, T * FO, P(xfn), P(xout), P(w_ih), P(b_ih), P(b_hh), P(gates), P(c), P(h), S()))
    out["ssd_ffn_z_fwd"] = timed(lambda: lib.mrg_ssd_ffn_z_fwd(
        B, H, HB, P(hp), P(rp), P(gm), P(bt), 1e-5, P(u), P(mean), P(rstd), P(w1), P(b1), P(z), S()))
    out["ssd_y_fwd"] = timed(lambda: lib.mrg_ssd_y_fwd(B, HB, FO, P(z), P(w2), P(b2), P(yb), T * FO, S()))
    v = r(HB, 2)
    out["ssd_ffn_bwd"] = timed(lambda: lib.mrg_ssd_ffn_bwd(
        B, H, HB, FO, 1, P(dy), T * FO, P(dfn), None, P(wms_t), P(mask), P(w1), P(w2), P(b1), P(v), P(z), P(dyt), P(dz),
        P(duo), P(hp), P(rp), P(gm), P(mean), P(rstd), P(g), P(gates), P(c), P(dG), S()))
    out["ssd_ln_cell_bwd"] = timed(lambda: lib.mrg_ssd_ln_cell_bwd(
        B, H, P(du), P(hp), P(rp), P(gm), P(mean), P(rstd), P(g), P(gates), P(c), P(dG), FM, None, None, None, S()))
    vt, dyxb = r(FM, 4 * H), r(B, FM)
    out["ssd_ln_cell_bwd + dyx"] = timed(lambda: lib.mrg_ssd_ln_cell_bwd(
        B, H, P(du), P(hp), P(rp), P(gm), P(mean), P(rstd), P(g), P(gates), P(c), P(dG), FM, P(vt), P(wms_t),
        P(dyxb), S()))
    out["ssd_dx"] = timed(lambda: lib.mrg_ssd_dx(B, H, P(dG), P(w_t), P(g), P(dX), S()))
    out["dX gemm rows TB=1 (W_ih^T)"] = timed(lambda: Fn.gemm(B, H, 4 * H, P(dG), 0, 4 * H, P(w_t), 1, 4 * H, P(dX), H,
                                                           epi=3, aux=P(g), ldaux=H, device=dev))
    out["dX gemm rows TB=0 (W_ih)"] = timed(lambda: Fn.gemm(B, H, 4 * H, P(dG), 0, 4 * H, P(w_ih), 0, H, P(dX), H,
                                                         epi=3, aux=P(g), ldaux=H, device=dev))
    empty = torch.empty(1, device=dev)
    out["torch fill_ (launch floor)"] = timed(lambda: empty.fill_(1.0))
    for k, v in out.items():
        print(f"{k:34s} {v:7.2f} us/launch")


if __name__ == "__main__":
    main()
