"""Op-level parity of the HIP kernels (libmrg.so) on a real MI355X.

Floating-point bar: max|a-b| / max|b| <= 1e-4 (fp32, BASELINE north_star),
checked against the reference's own golden vectors where they exist
(tests/golden/ops.npz, produced by torch.nn.LSTM / nn.MultiheadAttention as
the reference instantiates them) and against the CPU oracle / a plain torch
fp32 reference otherwise.
"""
import math

import numpy as np
import pytest
import torch

from tests.golden_util import load, prefixed, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _lib():
    from multimodalreactiongeneration_amd import _lib as L
    L.load()
    yield
    from multimodalreactiongeneration_amd import functional as Fn
    torch.cuda.synchronize()
    Fn.check_errors()


def _param(t):
    return torch.nn.Parameter(t.clone().to(DEV))


@pytest.fixture(params=[1, 0], ids=["x6", "exact_f32"])
def gemm_mode(request):
    """Both GEMM arithmetics: the x6 bf16 split (default) and the exact f32 MFMA."""
    from multimodalreactiongeneration_amd import _lib as L
    lib = L.load()
    old = lib.mrg_gemm_get_mode()
    L.check(lib.mrg_gemm_set_mode(request.param), "mode")
    yield request.param
    L.check(lib.mrg_gemm_set_mode(old), "mode")


@pytest.mark.parametrize("M,N,K", [(19200, 1024, 256), (600, 6, 64), (37, 45, 53), (2048, 256, 512)])
def test_linear_fwd_bwd_vs_torch_fp32(M, N, K, gemm_mode):
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(M + N)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    wd, bd = _param(w), _param(b)
    y = Fn.linear(xd, wd, bd)
    y.backward(dy.to(DEV))
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    yr = torch.nn.functional.linear(xr, wr, br)
    yr.backward(dy.double())
    assert rel_err(y, yr) < TOL
    assert rel_err(xd.grad, xr.grad) < TOL
    assert rel_err(wd.grad, wr.grad) < TOL
    assert rel_err(bd.grad, br.grad) < TOL


@pytest.mark.parametrize("M,N,K,epi,split", [
    (64, 1024, 256, 0, False), (64, 256, 1024, 3, False), (3, 70, 300, 1, False), (64, 6, 40, 0, False),
    (130, 200, 520, 0, True), (200, 128, 1024, 3, True)])
def test_few_row_gemms(M, N, K, epi, split):
    """M <= 64 (the T = 1 decode's batch rows) runs the register-fed exact-f32 MFMA kernel
    (gemm_rows_kernel); a few-tile product with K >= 512 runs split-K with the slabs combined by
    the last K slice of each tile (mrg_gemm_f32_ex counters).  Three back-to-back calls check
    that the tickets return to zero and that both are bitwise repeatable."""
    from multimodalreactiongeneration_amd import functional as Fn
    assert (Fn.act_splits(M, N, K) > 1) == split
    g = torch.Generator().manual_seed(M * N + K)
    a = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    bias = torch.randn(N, generator=g)
    c0 = torch.randn(M, N, generator=g)
    aux = torch.randn(M, N, generator=g)
    ad, wd, bd, auxd = a.to(DEV), w.to(DEV), bias.to(DEV), aux.to(DEV)
    outs = []
    for _ in range(3):
        c = c0.to(DEV)
        Fn.gemm(M, N, K, Fn._ptr(ad), 0, K, Fn._ptr(wd), 1, K, Fn._ptr(c), N, beta=0.5, bias=Fn._ptr(bd),
                epi=epi, aux=Fn._ptr(auxd) if epi >= 2 else None, ldaux=N, device=DEV)
        outs.append(c)
    torch.cuda.synchronize()
    ref = a.double() @ w.double().t() + 0.5 * c0.double() + bias.double()
    if epi == 1:
        ref = ref.clamp_min(0)
    elif epi == 3:
        ref = ref + aux.double()
    assert rel_err(outs[0], ref) < TOL
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    assert int(Fn._counters(DEV).abs().sum()) == 0


@pytest.mark.parametrize("depth,bn", [(2, 128), (3, 128), (3, 64), (4, 128)])
@pytest.mark.parametrize("M,N,K,epi,rowmap", [
    (19200, 1024, 256, 0, False), (19200, 256, 256, 3, False), (1000, 192, 96, 1, False), (300, 64, 32, 0, False),
    (64 * 300, 256, 512, 0, True)])
def test_glds_gemm_vs_fp64(M, N, K, epi, rowmap, depth, bn):
    """The LDS-DMA pipelined x6 kernel (gemm_x6g_kernel: k-contiguous A and B, DMA ring of `depth`
    k-tiles, fragments split into bf16 planes as they are read) against fp64: M and N edges
    (clamped rows, masked stores), bias / beta / ReLU / residual epilogues, and an A read through a
    RowMap ([B, T] rows of a [B, T + 12, K] view: the [:, lead:] slice).  Bitwise repeatable."""
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd import _lib as L
    lib = L.load()
    g = torch.Generator().manual_seed(M + 7 * N + K + depth)
    if rowmap:
        B_, T_ = 64, M // 64
        full = torch.randn(B_, T_ + 12, K, generator=g)
        a = full[:, 12:].reshape(M, K)
        ad = full.to(DEV)
        a_ptr, lda, a_hi, a_div = Fn._ptr(ad, 12 * K), K, (T_ + 12) * K, T_
    else:
        a = torch.randn(M, K, generator=g)
        ad = a.to(DEV)
        a_ptr, lda, a_hi, a_div = Fn._ptr(ad), K, 0, 0
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    bias = torch.randn(N, generator=g)
    c0 = torch.randn(M, N, generator=g)
    aux = torch.randn(M, N, generator=g)
    wd, bd, auxd = w.to(DEV), bias.to(DEV), aux.to(DEV)
    L.check(lib.mrg_gemm_set_glds(depth, bn), "glds")
    try:
        outs = []
        for _ in range(2):
            c = c0.to(DEV)
            Fn.gemm(M, N, K, a_ptr, 0, lda, Fn._ptr(wd), 1, K, Fn._ptr(c), N, beta=0.5, bias=Fn._ptr(bd), epi=epi,
                    aux=Fn._ptr(auxd) if epi >= 2 else None, ldaux=N, a_hi=a_hi, a_div=a_div, device=DEV)
            outs.append(c)
        torch.cuda.synchronize()
    finally:
        L.check(lib.mrg_gemm_set_glds(0, 128), "glds")
    ref = a.double() @ w.double().t() + 0.5 * c0.double() + bias.double()
    if epi == 1:
        ref = ref.clamp_min(0)
    elif epi == 3:
        ref = ref + aux.double()
    assert rel_err(outs[0], ref) < 2e-6
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("M,N,K", [(19200, 256, 256), (4096, 1024, 256), (2100, 512, 96)])
def test_weight_planes_linear_vs_fp64(M, N, K):
    """Pre-split weights (prepare_weight_planes: three bf16 planes of W and of W^T in one launch) feed
    the forward product x W^T and the input-gradient product dY W (mrg_gemm_x6_planes); the weight
    gradient stays on the fp32-operand path.  All against fp64; planes dropped after the optimizer
    would have run (invalidate) and when the weight is rewritten through torch (version check)."""
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(M + N + K)
    x = torch.randn(M, K, generator=g)
    w = torch.randn(N, K, generator=g) / math.sqrt(K)
    b = torch.randn(N, generator=g)
    dy = torch.randn(M, N, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    wd, bd = _param(w), _param(b)
    prev = Fn.set_weight_planes(True)
    try:
        Fn.prepare_weight_planes([wd])
        assert Fn._plane_operand(wd, False) is not None and Fn._plane_operand(wd, True) is not None
        y = Fn.linear(xd, wd, bd)
        y.backward(dy.to(DEV))
        torch.cuda.synchronize()
    finally:
        Fn.set_weight_planes(prev)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    yr = torch.nn.functional.linear(xr, wr, b.double())
    yr.backward(dy.double())
    assert rel_err(y, yr) < 2e-6
    assert rel_err(xd.grad, xr.grad) < 2e-6
    assert rel_err(wd.grad, wr.grad) < 2e-6
    Fn.set_weight_planes(True)
    try:
        Fn.prepare_weight_planes([wd])
        with torch.no_grad():
            wd.mul_(2.0)   # rewritten through torch: the planes are stale and must not be used
        assert Fn._plane_operand(wd, False) is None
        Fn.invalidate_weight_planes()
        assert not Fn._PLANES
    finally:
        Fn.set_weight_planes(prev)


@pytest.mark.parametrize("wg", [1, 0], ids=["glds", "regstaged"])
@pytest.mark.parametrize("rows,N,In,time_shift", [(19200, 1024, 256, False), (64 * 299, 1024, 256, True),
                                                  (19200, 256, 256, False), (2048, 100, 36, False)])
def test_weight_grad_kernels_vs_fp64(rows, N, In, time_shift, wg):
    """Weight gradients dW += dY^T X with the fused bias sums, on the LDS-DMA weight-gradient kernel
    (gemm_x6g_wgrad_kernel: k-strided operands through the DMA ring, split-K slabs) and on the
    register-staged one, against fp64; the time-shifted form (dY rows t >= 1 against X rows t - 1 of
    [B, T] tensors, dW_hh) reads both operands through RowMaps."""
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(rows + N + In + wg)
    if time_shift:
        B_, T_ = 64, 300
        dy_full = torch.randn(B_, T_, N, generator=g)
        x_full = torch.randn(B_, T_, In, generator=g)
        dy = dy_full[:, 1:].reshape(-1, N)
        x = x_full[:, :-1].reshape(-1, In)
        dyd, xd = dy_full.to(DEV), x_full.to(DEV)
        kw = dict(dy_hi=T_ * N, dy_div=T_ - 1, x_hi=T_ * In, x_div=T_ - 1)
        dyp, xp = Fn._ptr(dyd, N), Fn._ptr(xd)
    else:
        dy = torch.randn(rows, N, generator=g)
        x = torch.randn(rows, In, generator=g)
        dyd, xd = dy.to(DEV), x.to(DEV)
        kw = {}
        dyp, xp = Fn._ptr(dyd), Fn._ptr(xd)
    gw0 = torch.randn(N, In, generator=g)
    gb0 = torch.randn(N, generator=g)
    gw, gb = gw0.to(DEV), gb0.to(DEV)
    from multimodalreactiongeneration_amd import _lib as L
    lib = L.load()
    prev = Fn.set_wgrad_stream(False)
    try:
        old = lib.mrg_gemm_set_glds_wg(wg)
        Fn._wgrad(dyp, N, xp, In, dy.shape[0], N, In, gw, DEV, gb=gb, keep=(dyd, xd), **kw)
        torch.cuda.synchronize()
        lib.mrg_gemm_set_glds_wg(old)
    finally:
        Fn.set_wgrad_stream(prev)
    ref_w = gw0.double() + dy.double().t() @ x.double()
    ref_b = gb0.double() + dy.double().sum(0)
    assert rel_err(gw, ref_w) < 2e-6
    assert rel_err(gb, ref_b) < 2e-6


@pytest.mark.parametrize("rows,N,In,time_shift", [(19200, 1024, 256, False), (64 * 299, 1024, 256, True),
                                                  (19200, 256, 256, False), (19200, 256, 512, False),
                                                  (2048, 100, 36, False), (6400, 64, 256, False)])
def test_weight_grad_kernel_vs_fp64(rows, N, In, time_shift):
    """The weight-gradient product (gemm_x6g_wgrad_kernel: dW += dY^T X with the bias gradient fused)
    vs fp64: split-K slabs, ragged tiles and the time-shifted RowMap form of dW_hh included."""
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd import _lib as L
    lib = L.load()
    g = torch.Generator().manual_seed(rows + 3 * N + In)
    if time_shift:
        B_, T_ = 64, 300
        dy_full, x_full = torch.randn(B_, T_, N, generator=g), torch.randn(B_, T_, In, generator=g)
        dy, x = dy_full[:, 1:].reshape(-1, N), x_full[:, :-1].reshape(-1, In)
        dyd, xd = dy_full.to(DEV), x_full.to(DEV)
        kw = dict(dy_hi=T_ * N, dy_div=T_ - 1, x_hi=T_ * In, x_div=T_ - 1)
        dyp, xp = Fn._ptr(dyd, N), Fn._ptr(xd)
    else:
        dy, x = torch.randn(rows, N, generator=g), torch.randn(rows, In, generator=g)
        dyd, xd = dy.to(DEV), x.to(DEV)
        kw = {}
        dyp, xp = Fn._ptr(dyd), Fn._ptr(xd)
    gw0, gb0 = torch.randn(N, In, generator=g), torch.randn(N, generator=g)
    prev = Fn.set_wgrad_stream(False)
    try:
        gw, gb = gw0.to(DEV), gb0.to(DEV)
        Fn._wgrad(dyp, N, xp, In, dy.shape[0], N, In, gw, DEV, gb=gb, keep=(dyd, xd), **kw)
        torch.cuda.synchronize()
    finally:
        Fn.set_wgrad_stream(prev)
    del lib
    assert rel_err(gw, gw0.double() + dy.double().t() @ x.double()) < 2e-6
    assert rel_err(gb, gb0.double() + dy.double().sum(0)) < 2e-6


def _bf16(t):
    return t.to(torch.bfloat16).double()


@pytest.mark.parametrize("M,N,K,kind", [(19200, 1024, 256, "nt"), (19200, 256, 256, "nt"), (4800, 512, 512, "nt"),
                                        (19200, 1024, 256, "wgrad"), (19200, 256, 256, "wgrad")])
def test_bf16_gemm_kernels_are_bf16_operands(M, N, K, kind):
    """precision 'bf16' (BASELINE configs[1]): the LDS-DMA kernels' one-plane form (gemm_x6g_kernel /
    gemm_x6g_wgrad_kernel with NP = 1) rounds each operand to bf16 (RNE) and accumulates in fp32:
    equal to fp64 on the bf16-rounded operands up to fp32 accumulation, and visibly NOT the fp32
    product (the arithmetic really is bf16)."""
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(M + N + K)
    prev = Fn.set_wgrad_stream(False)
    try:
        with Fn.precision("bf16"):
            if kind == "nt":
                a = torch.randn(M, K, generator=g)
                w = torch.randn(N, K, generator=g) / math.sqrt(K)
                ad, wd = a.to(DEV), w.to(DEV)
                c = torch.empty(M, N, device=DEV)
                Fn.gemm(M, N, K, Fn._ptr(ad), 0, K, Fn._ptr(wd), 1, K, Fn._ptr(c), N, device=DEV)
                exact = a.double() @ w.double().t()
                ref = _bf16(a) @ _bf16(w).t()
                out = c
            else:
                dy = torch.randn(M, N, generator=g)
                x = torch.randn(M, K, generator=g)
                dyd, xd = dy.to(DEV), x.to(DEV)
                gw = torch.zeros(N, K, device=DEV)
                gb = torch.zeros(N, device=DEV)
                Fn._wgrad(Fn._ptr(dyd), N, Fn._ptr(xd), K, M, N, K, gw, DEV, gb=gb, keep=(dyd, xd))
                exact = dy.double().t() @ x.double()
                ref = _bf16(dy).t() @ _bf16(x)
                out = gw
                assert rel_err(gb, dy.double().sum(0)) < 2e-6   # bias sums stay fp32
            torch.cuda.synchronize()
    finally:
        Fn.set_wgrad_stream(prev)
    assert rel_err(out, ref) < 2e-6
    assert rel_err(out, exact) > 1e-4


@pytest.mark.parametrize("M,N,K,transB,a_off", [
    (64, 256, 1024, 0, 0), (64, 128, 512, 1, 0), (37, 96, 516, 0, 0), (64, 256, 1024, 1, 1), (50, 40, 64, 1, 3)])
def test_few_row_gemm_operand_layouts(M, N, K, transB, a_off):
    """gemm_rows_kernel with B row-major [K, N] (the dX form dG W) or [N, K], k-runs loaded as float4
    when aligned and element-wise otherwise (odd K per lane group, an A view offset off 16 B)."""
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(M + N + K + a_off)
    abuf = torch.randn(M * K + a_off, generator=g)
    a = abuf[a_off:].view(M, K)
    w = torch.randn((K, N) if transB == 0 else (N, K), generator=g) / math.sqrt(K)
    abd, wd = abuf.to(DEV), w.to(DEV)
    c = torch.zeros(M, N, device=DEV)
    Fn.gemm(M, N, K, Fn._ptr(abd, a_off), 0, K, Fn._ptr(wd), transB, N if transB == 0 else K, Fn._ptr(c), N,
            device=DEV)
    torch.cuda.synchronize()
    wm = w.double() if transB == 0 else w.double().t()
    assert rel_err(c, a.double() @ wm) < TOL


@pytest.mark.parametrize("rows,N,In,splits,time_shift", [
    (19200, 1024, 256, 32, False), (19200, 256, 256, 120, False), (1000, 70, 45, 1, False),
    (777, 130, 33, 5, False), (64 * 299, 1024, 256, 16, True), (64, 1024, 256, 1, False),
    (37, 130, 33, 1, False)])
def test_weight_grad_with_fused_bias_sums(rows, N, In, splits, time_shift, gemm_mode):
    """gw += dY^T X and gb (+ gb2) += colsum(dY) in one mrg_gemm_f32_ex call, incl. a RowMap'd
    (time-shifted, [:, 1:] of [64, 300, F]) operand pair as the LSTM's dW_hh uses."""
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(rows + N)
    if time_shift:
        T = 300
        dYf = torch.randn(64, T, N, generator=g)
        Xf = torch.randn(64, T, In, generator=g)
        dY, X = dYf[:, 1:].reshape(-1, N), Xf[:, :-1].reshape(-1, In)
        dYd, Xd = dYf.to(DEV), Xf.to(DEV)
        kw = dict(dy_hi=T * N, dy_div=T - 1, x_hi=T * In, x_div=T - 1)
        dy_ptr, x_ptr = Fn._ptr(dYd, N), Fn._ptr(Xd)
    else:
        dY, X = torch.randn(rows, N, generator=g), torch.randn(rows, In, generator=g)
        dYd, Xd = dY.to(DEV), X.to(DEV)
        kw = {}
        dy_ptr, x_ptr = Fn._ptr(dYd), Fn._ptr(Xd)
    gw0, gb0 = torch.randn(N, In, generator=g), torch.randn(N, generator=g)
    gw, gb, gb2 = gw0.to(DEV), gb0.to(DEV), gb0.to(DEV) * 2
    orig = Fn.wgrad_splits
    Fn.wgrad_splits = lambda *a: splits
    try:
        Fn._wgrad(dy_ptr, N, x_ptr, In, dY.shape[0], N, In, gw, torch.device(DEV), gb=gb, gb2=gb2, **kw)
    finally:
        Fn.wgrad_splits = orig
    torch.cuda.synchronize()
    ref_w = gw0.double() + dY.double().t() @ X.double()
    ref_b = gb0.double() + dY.double().sum(0)
    assert rel_err(gw, ref_w) < TOL
    assert rel_err(gb, ref_b) < TOL
    assert rel_err(gb2, gb0.double() * 2 + dY.double().sum(0)) < TOL


def test_ffn_relu_fused_vs_torch():
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(1)
    x = torch.randn(3000, 256, generator=g)
    w1, b1 = torch.randn(64, 256, generator=g) / 16, torch.randn(64, generator=g)
    w2, b2 = torch.randn(6, 64, generator=g) / 8, torch.randn(6, generator=g)
    dz = torch.randn(3000, 6, generator=g)
    ps = [_param(t) for t in (w1, b1, w2, b2)]
    xd = x.to(DEV).requires_grad_(True)
    z = Fn.ffn(xd, *ps)
    z.backward(dz.to(DEV))
    rs = [t.double().requires_grad_(True) for t in (x, w1, b1, w2, b2)]
    zr = torch.nn.functional.linear(torch.relu(torch.nn.functional.linear(rs[0], rs[1], rs[2])), rs[3], rs[4])
    zr.backward(dz.double())
    assert rel_err(z, zr) < TOL
    assert rel_err(xd.grad, rs[0].grad) < TOL
    for p, r in zip(ps, rs[1:]):
        assert rel_err(p.grad, r.grad) < TOL


@pytest.mark.parametrize("E", [6, 36, 64, 128, 256, 512, 768, 1000])
def test_residual_layernorm_vs_torch(E):
    """float4 kernels for E % 4 == 0 (partial last chunk at 36 / 768 / 1000), scalar ones otherwise;
    1001 rows leaves the backward's two-row pass ragged."""
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(E)
    a, b = torch.randn(1001, E, generator=g), torch.randn(1001, E, generator=g)
    gam, bet = 1 + 0.1 * torch.randn(E, generator=g), 0.1 * torch.randn(E, generator=g)
    dy = torch.randn(1001, E, generator=g)
    ad, bd = a.to(DEV).requires_grad_(True), b.to(DEV).requires_grad_(True)
    gd, btd = _param(gam), _param(bet)
    y = Fn.residual_layernorm(ad, bd, gd, btd)
    y.backward(dy.to(DEV))
    ar, br = a.double().requires_grad_(True), b.double().requires_grad_(True)
    gr, btr = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(ar + br, (E,), gr, btr, 1e-5)
    yr.backward(dy.double())
    assert rel_err(y, yr) < TOL
    assert rel_err(ad.grad, ar.grad) < TOL and rel_err(bd.grad, br.grad) < TOL
    assert rel_err(gd.grad, gr.grad) < TOL and rel_err(btd.grad, btr.grad) < TOL


@pytest.mark.parametrize("rows,E", [(5000, 256), (19200, 256), (19200, 1000), (70, 256), (150000, 64)])
def test_layernorm_param_reduce_row_groups(rows, E):
    """dgamma / dbeta through the 2-D ticketed parameter reduce: ragged row groups (5000 rows), the
    benchmark's 19,200 rows, E = 1000 (16 column blocks, partial last), a single group, and enough
    partial blocks that the 64 groups take several rounds of loads each; twice in a row (the tickets
    return to 0), vs torch float64."""
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(rows + E)
    a, b = torch.randn(rows, E, generator=g), torch.randn(rows, E, generator=g)
    gam, bet = 1 + 0.1 * torch.randn(E, generator=g), 0.1 * torch.randn(E, generator=g)
    dy = torch.randn(rows, E, generator=g)
    gr, btr = gam.double().requires_grad_(True), bet.double().requires_grad_(True)
    yr = torch.nn.functional.layer_norm(a.double() + b.double(), (E,), gr, btr, 1e-5)
    yr.backward(dy.double())
    for _ in range(2):
        gd, btd = _param(gam), _param(bet)
        y = Fn.residual_layernorm(a.to(DEV), b.to(DEV), gd, btd)
        y.backward(dy.to(DEV))
        torch.cuda.synchronize()
        assert rel_err(gd.grad, gr.grad) < TOL and rel_err(btd.grad, btr.grad) < TOL


def test_layernorm_param_reduce_concurrent_streams():
    """mrg_residual_layernorm_param_reduce on four streams at once, 24 launches each, streams held back
    by busy kernels so their launches overlap in any order (tickets are per (device, stream),
    not rotated over a global pool): every launch's dgamma / dbeta bitwise equals a lone reduce of the
    same partials (each launch consumes its own copy of the workspace)."""
    import ctypes
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd.functional import _ptr
    lib = _lib.load()
    rows, E = 19200, 256
    g = torch.Generator().manual_seed(77)
    a, b, dy = (torch.randn(rows, E, generator=g).to(DEV) for _ in range(3))
    gam, bet = (1 + 0.1 * torch.randn(E, generator=g)).to(DEV), (0.1 * torch.randn(E, generator=g)).to(DEV)
    y, dx = torch.empty_like(a), torch.empty_like(a)
    mean, rstd = torch.empty(rows, device=DEV), torch.empty(rows, device=DEV)
    ws = torch.empty(lib.mrg_residual_layernorm_bwd_workspace_bytes(rows, E) // 4, device=DEV)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.mrg_residual_layernorm_fwd(rows, E, _ptr(a), _ptr(b), _ptr(gam), _ptr(bet), 1e-5, _ptr(y),
                                              _ptr(mean), _ptr(rstd), st), "fwd")
    _lib.check(lib.mrg_residual_layernorm_bwd(rows, E, _ptr(dy), _ptr(a), _ptr(b), _ptr(gam), _ptr(mean),
                                              _ptr(rstd), _ptr(dx), None, None, 0, _ptr(ws), st), "bwd")
    ref = torch.empty(2, E, device=DEV)
    w0 = ws.clone()
    _lib.check(lib.mrg_residual_layernorm_param_reduce(rows, E, _ptr(w0), _ptr(ref[0]), _ptr(ref[1]), 0, st), "ref")
    n_str, per = 4, 24
    copies = [ws.clone() for _ in range(n_str * per)]
    outs = torch.full((n_str * per, 2, E), float("nan"), device=DEV)
    streams = [torch.cuda.Stream(device=DEV) for _ in range(n_str)]
    torch.cuda.synchronize()
    for j in range(per):
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                if j % 6 == i:
                    _lib.check(lib.mrg_debug_busy(1, 64, 256, 200.0, ctypes.c_void_p(s.cuda_stream)), "busy")
                k = j * n_str + i
                _lib.check(lib.mrg_residual_layernorm_param_reduce(rows, E, _ptr(copies[k]), _ptr(outs[k, 0]),
                                                                   _ptr(outs[k, 1]), 0,
                                                                   ctypes.c_void_p(s.cuda_stream)), "reduce")
    torch.cuda.synchronize()
    for k in range(n_str * per):
        assert torch.equal(outs[k], ref), k


@pytest.mark.parametrize("loss_type", ["huber", "mse", "mae", "smoothl1"])
def test_masked_loss_vs_oracle(loss_type):
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    g = torch.Generator().manual_seed(3)
    y = torch.randn(4, 12, 6, generator=g) * 2
    t = torch.randn(4, 9, 6, generator=g) * 2
    t[1, 6:] = -100.0
    yd = y.to(DEV).requires_grad_(True)
    loss = Fn.masked_loss(yd, t.to(DEV), lead=3, loss_type=loss_type)
    loss.backward()
    yr = y.clone().requires_grad_(True)
    lr = O.masked_regression_loss(yr[:, 3:], t, loss_type)
    lr.backward()
    assert abs(loss.item() - lr.item()) <= 1e-5 * max(1.0, abs(lr.item()))
    assert rel_err(yd.grad, yr.grad) < TOL


def test_lstm_layer_matches_nn_lstm_golden():
    from multimodalreactiongeneration_amd import functional as Fn
    d = load("ops")
    p = {k: _param(v) for k, v in prefixed(d, "lstm1/param/").items()}
    x = torch.from_numpy(d["lstm1/x"]).to(DEV).requires_grad_(True)
    h0 = torch.from_numpy(d["lstm1/h0"])[0].to(DEV).requires_grad_(True)
    c0 = torch.from_numpy(d["lstm1/c0"])[0].to(DEV).requires_grad_(True)
    y, hT, cT = Fn.lstm_layer(x, p["weight_ih_l0"], p["weight_hh_l0"], p["bias_ih_l0"], p["bias_hh_l0"], h0, c0)
    assert rel_err(y, d["lstm1/y"]) < TOL
    assert rel_err(hT, d["lstm1/hT"][0]) < TOL
    assert rel_err(cT, d["lstm1/cT"][0]) < TOL
    loss = (y * torch.from_numpy(d["lstm1/dy"]).to(DEV)).sum() \
        + (hT * torch.from_numpy(d["lstm1/dhT"])[0].to(DEV)).sum() \
        + (cT * torch.from_numpy(d["lstm1/dcT"])[0].to(DEV)).sum()
    loss.backward()
    torch.cuda.synchronize()
    assert rel_err(x.grad, d["lstm1/dx"]) < TOL
    assert rel_err(h0.grad, d["lstm1/dh0"][0]) < TOL
    assert rel_err(c0.grad, d["lstm1/dc0"][0]) < TOL
    for k in p:
        assert rel_err(p[k].grad, d[f"lstm1/grad/{k}"]) < TOL, k


def test_bidirectional_two_layer_lstm_golden():
    from multimodalreactiongeneration_amd.model.layers import LSTM
    d = load("ops")
    lstm = LSTM(16, 16, num_layers=2, bidirectional=True)
    lstm.load_state_dict(prefixed(d, "lstm2/param/"))
    lstm = lstm.to(DEV)
    x = torch.from_numpy(d["lstm2/x"]).to(DEV).requires_grad_(True)
    y, (hT, cT) = lstm(x)
    assert rel_err(y, d["lstm2/y"]) < TOL
    assert rel_err(hT, d["lstm2/hT"]) < TOL
    assert rel_err(cT, d["lstm2/cT"]) < TOL
    y.backward(torch.from_numpy(d["lstm2/dy"]).to(DEV))
    torch.cuda.synchronize()
    assert rel_err(x.grad, d["lstm2/dx"]) < TOL
    for k, prm in lstm.named_parameters():
        assert rel_err(prm.grad, d[f"lstm2/grad/{k}"]) < TOL, k


def test_unsupported_hidden_size_fails_loudly():
    from multimodalreactiongeneration_amd.model.layers import LSTM
    lstm = LSTM(8, 12).to(DEV)
    with pytest.raises(RuntimeError):
        lstm(torch.randn(2, 3, 8, device=DEV))


@pytest.mark.parametrize("H,In,B,T,rev", [(256, 256, 64, 300, False), (128, 128, 64, 300, True),
                                          (64, 40, 5, 50, False), (32, 16, 3, 20, True), (16, 8, 2, 9, False)])
def test_lstm_layer_vs_oracle(H, In, B, T, rev):
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    g = torch.Generator().manual_seed(H + T)
    k = 1 / math.sqrt(H)
    w_ih = (torch.rand(4 * H, In, generator=g) * 2 - 1) * k
    w_hh = (torch.rand(4 * H, H, generator=g) * 2 - 1) * k
    b_ih = (torch.rand(4 * H, generator=g) * 2 - 1) * k
    b_hh = (torch.rand(4 * H, generator=g) * 2 - 1) * k
    x = torch.randn(B, T, In, generator=g)
    dy = torch.randn(B, T, H, generator=g)
    ps = [_param(t) for t in (w_ih, w_hh, b_ih, b_hh)]
    xd = x.to(DEV).requires_grad_(True)
    y, hT, cT = Fn.lstm_layer(xd, *ps, reverse=rev)
    y.backward(dy.to(DEV))
    torch.cuda.synchronize()
    rs = [t.clone().requires_grad_(True) for t in (w_ih, w_hh, b_ih, b_hh)]
    xr = x.clone().requires_grad_(True)
    yr, hr, cr = O.lstm_layer(xr, *rs, reverse=rev)
    yr.backward(dy)
    assert rel_err(y, yr) < TOL
    assert rel_err(cT, cr) < TOL
    assert rel_err(xd.grad, xr.grad) < TOL
    for p, r in zip(ps, rs):
        assert rel_err(p.grad, r.grad) < TOL


@pytest.mark.parametrize("H,In,B", [(256, 256, 64), (64, 40, 5), (16, 8, 3)])
def test_lstm_single_step_chain_vs_oracle(H, In, B):
    """T = 1 steps (the scheduled-sampling decode, lstm_with_sample.py:410-433) go through the cell
    kernels; four chained steps carry (h, c) and their gradients from step to step."""
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    g = torch.Generator().manual_seed(H + In)
    k = 1 / math.sqrt(H)
    w = [(torch.rand(4 * H, n, generator=g) * 2 - 1) * k for n in (In, H)]
    bb = [(torch.rand(4 * H, generator=g) * 2 - 1) * k for _ in range(2)]
    xs = [torch.randn(B, 1, In, generator=g) for _ in range(4)]
    dys = [torch.randn(B, 1, H, generator=g) for _ in range(4)]
    ps = [_param(t) for t in (*w, *bb)]
    rs = [t.clone().requires_grad_(True) for t in (*w, *bb)]
    xd = [x.to(DEV).requires_grad_(True) for x in xs]
    xr = [x.clone().requires_grad_(True) for x in xs]
    h = c = hr = cr = None
    loss = loss_r = 0
    for i in range(4):
        y, h, c = Fn.lstm_layer(xd[i], *ps, h, c)
        yr, hr, cr = O.lstm_layer(xr[i], *rs, hr, cr)
        assert y.shape == (B, 1, H)
        assert rel_err(y, yr) < TOL
        loss = loss + (y * dys[i].to(DEV)).sum()
        loss_r = loss_r + (yr * dys[i]).sum()
    (loss + c.sum()).backward()
    (loss_r + cr.sum()).backward()
    torch.cuda.synchronize()
    assert rel_err(c, cr) < TOL
    for a, r in zip(xd, xr):
        assert rel_err(a.grad, r.grad) < TOL
    for p, r in zip(ps, rs):
        assert rel_err(p.grad, r.grad) < TOL


@pytest.mark.parametrize("bs,group", [(1, 8), (2, 8), (4, 8), (8, 8), (16, 8), (8, 16), (16, 16)])
def test_lstm_batched_problems_and_forced_tiling(bs, group):
    """3 independent recurrences in one launch, every batch-tile size and group size, vs the oracle
    (outputs and input / weight gradients; batch tile 16 runs the backward's self-io form)."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    lib = _lib.load()
    H, B, T = 256, 20, 40   # 3 x 20 rows at batch tile 1 = 480 workgroups (fits 512); ragged last tiles
    g = torch.Generator().manual_seed(bs)
    probs, refs = [], []
    for _ in range(3):
        w = [torch.randn(4 * H, H, generator=g) * 0.06 for _ in range(2)]
        bb = [torch.randn(4 * H, generator=g) * 0.06 for _ in range(2)]
        x = torch.randn(B, T, H, generator=g)
        probs.append((x.to(DEV).requires_grad_(True), _param(w[0]), _param(w[1]), _param(bb[0]), _param(bb[1])))
        xr = x.clone().requires_grad_(True)
        rw = [t.clone().requires_grad_(True) for t in (w[0], w[1], bb[0], bb[1])]
        yr = O.lstm_layer(xr, *rw)[0]
        yr.square().sum().backward()
        refs.append((yr, xr, rw))
    try:
        _lib.check(lib.mrg_lstm_config(group), "group")
        ys = Fn.lstm_layers_batched(probs, force_bs=bs)
        sum(y.square().sum() for y in ys).backward()
        torch.cuda.synchronize()
        Fn.check_errors()
    finally:
        lib.mrg_lstm_config(8)
    for y, p, (yr, xr, rw) in zip(ys, probs, refs):
        assert rel_err(y, yr) < TOL
        assert rel_err(p[0].grad, xr.grad) < TOL
        for a, r in zip(p[1:], rw):
            assert rel_err(a.grad, r.grad) < TOL


@pytest.mark.parametrize("nprob,B,T,state", [(1, 37, 29, True), (5, 64, 40, False), (8, 64, 12, False),
                                             (2, 16, 300, True)])
def test_lstm_mfma_form_vs_oracle(nprob, B, T, state):
    """The MFMA form of the H = 256 recurrence (lstm_mx.hip: batch tiles of 16 rows, x6 bf16 split on
    v_mfma_f32_16x16x32_bf16), forced on: outputs, final states and every gradient (input, weights,
    biases, initial state) vs the oracle, ragged last batch tiles (B = 37) and up to 8 problems."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    lib = _lib.load()
    H = 256
    g = torch.Generator().manual_seed(nprob * 1000 + B + T)
    cases = []
    for _ in range(nprob):
        k = 1 / math.sqrt(H)
        w = [(torch.rand(4 * H, H, generator=g) * 2 - 1) * k for _ in range(2)]
        bb = [(torch.rand(4 * H, generator=g) * 2 - 1) * k for _ in range(2)]
        x = torch.randn(B, T, H, generator=g)
        h0 = torch.randn(B, H, generator=g) * 0.5 if state else None
        c0 = torch.randn(B, H, generator=g) * 0.5 if state else None
        dy = torch.randn(B, T, H, generator=g)
        cases.append((w, bb, x, h0, c0, dy))
    prev = lib.mrg_lstm_set_mx(2, 0)
    try:
        outs = []
        if nprob == 1 or state:
            for w, bb, x, h0, c0, dy in cases:
                ps = [_param(t) for t in (*w, *bb)]
                xd = x.to(DEV).requires_grad_(True)
                hd = None if h0 is None else h0.to(DEV).requires_grad_(True)
                cd = None if c0 is None else c0.to(DEV).requires_grad_(True)
                y, hT, cT = Fn.lstm_layer(xd, *ps, hd, cd)
                (y * dy.to(DEV)).sum().add(hT.sum()).add(cT.square().sum()).backward()
                outs.append((y, hT, cT, xd, ps, hd, cd))
        else:
            probs = [(x.to(DEV).requires_grad_(True), *[_param(t) for t in (*w, *bb)]) for w, bb, x, _, _, _ in cases]
            ys = Fn.lstm_layers_batched(probs)
            sum((y * c[5].to(DEV)).sum() for y, c in zip(ys, cases)).backward()
            outs = [(y, None, None, p[0], list(p[1:]), None, None) for y, p in zip(ys, probs)]
        torch.cuda.synchronize()
        Fn.check_errors()
    finally:
        lib.mrg_lstm_set_mx(prev, 0)
    for (w, bb, x, h0, c0, dy), (y, hT, cT, xd, ps, hd, cd) in zip(cases, outs):
        rs = [t.clone().requires_grad_(True) for t in (*w, *bb)]
        xr = x.clone().requires_grad_(True)
        hr = None if h0 is None else h0.clone().requires_grad_(True)
        cr = None if c0 is None else c0.clone().requires_grad_(True)
        yr, hTr, cTr = O.lstm_layer(xr, *rs, h0=hr, c0=cr)
        loss = (yr * dy).sum()
        if hT is not None:
            loss = loss + hTr.sum() + cTr.square().sum()
        loss.backward()
        assert rel_err(y, yr) < TOL
        if hT is not None:
            assert rel_err(hT, hTr) < TOL and rel_err(cT, cTr) < TOL
            assert rel_err(hd.grad, hr.grad) < TOL and rel_err(cd.grad, cr.grad) < TOL
        assert rel_err(xd.grad, xr.grad) < TOL
        for p, r in zip(ps, rs):
            assert rel_err(p.grad, r.grad) < TOL


@pytest.mark.parametrize("H,B", [(256, 64), (256, 24), (128, 16), (32, 5)])
def test_lstm_local_handoff_is_bitwise_the_agent_one(H, B):
    """The hand-off store flavour (workgroup scope for groups verified on one XCD, agent scope
    otherwise; lstm.hip put_granule / group_on_one_xcd) changes no arithmetic: forward outputs,
    final states and every gradient are bitwise those of the agent-scope hand-offs."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd import functional as Fn
    lib = _lib.load()
    T = 37
    g = torch.Generator().manual_seed(H + B)
    w = [torch.randn(4 * H, H, generator=g) * 0.06 for _ in range(2)]
    bb = [torch.randn(4 * H, generator=g) * 0.06 for _ in range(2)]
    x = torch.randn(B, T, H, generator=g)
    h0, c0 = torch.randn(B, H, generator=g), torch.randn(B, H, generator=g)
    outs = []
    prev_solo = lib.mrg_lstm_set_solo(0)   # the hand-off rings (solo groups at H <= 128 have none)
    try:
        for local in (1, 0):
            _lib.check(lib.mrg_lstm_set_local_handoff(local), "local")
            ps = [_param(t) for t in (w[0], w[1], bb[0], bb[1])]
            xx = x.to(DEV).requires_grad_(True)
            y, hT, cT = Fn.lstm_layer(xx, *ps, h0.to(DEV), c0.to(DEV))
            (y.square().sum() + hT.sum() + cT.sum()).backward()
            torch.cuda.synchronize()
            Fn.check_errors()
            outs.append([y.detach(), hT.detach(), cT.detach(), xx.grad] + [p.grad for p in ps])
    finally:
        lib.mrg_lstm_set_local_handoff(1)
        lib.mrg_lstm_set_solo(prev_solo)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("H,nprob,B,T,rev,state", [(128, 2, 64, 40, True, True), (128, 1, 37, 29, False, False),
                                                   (64, 3, 20, 33, False, True), (32, 2, 5, 17, True, False),
                                                   (128, 1, 2100, 3, False, True)])
def test_lstm_solo_groups_vs_oracle(H, nprob, B, T, rev, state):
    """Solo recurrence groups (one workgroup holds W_hh, h / dh exchanged through its LDS; the default
    at H <= 128) vs the oracle, and vs the multi-member hand-off groups: outputs, final states and
    every gradient.  B = 2100 at H = 128 is a grid larger than the GPU holds at once (its workgroups
    never wait on each other, so it completes)."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    lib = _lib.load()
    g = torch.Generator().manual_seed(H * 7 + B)
    s = 1.0 / math.sqrt(H)
    data = []
    for _ in range(nprob):
        w = [torch.randn(4 * H, H, generator=g) * s for _ in range(2)]
        bb = [torch.randn(4 * H, generator=g) * s for _ in range(2)]
        x = torch.randn(B, T, H, generator=g)
        h0 = torch.randn(B, H, generator=g) * 0.5 if state else None
        c0 = torch.randn(B, H, generator=g) * 0.5 if state else None
        data.append((x, w, bb, h0, c0))
    outs = {}
    for solo in ((1, 0) if B <= 64 else (1,)):   # (the ring groups' persistent grid cannot hold B = 2100)
        prev = lib.mrg_lstm_set_solo(solo)
        try:
            res = []
            for x, w, bb, h0, c0 in data:
                ps = [_param(t) for t in (w[0], w[1], bb[0], bb[1])]
                xx = x.to(DEV).requires_grad_(True)
                hd = h0.to(DEV).requires_grad_(True) if state else None
                cd = c0.to(DEV).requires_grad_(True) if state else None
                y, hT, cT = Fn.lstm_layer(xx, *ps, hd, cd, reverse=rev)
                (y.square().sum() + hT.square().sum() + cT.sum()).backward()
                torch.cuda.synchronize()
                Fn.check_errors()
                res.append([y.detach(), hT.detach(), cT.detach(), xx.grad] + [p.grad for p in ps] +
                           ([hd.grad, cd.grad] if state else []))
            outs[solo] = res
        finally:
            lib.mrg_lstm_set_solo(prev)
    if B <= 64:   # the oracle at small sizes
        for (x, w, bb, h0, c0), got in zip(data, outs[1]):
            xr = x.clone().requires_grad_(True)
            rw = [t.clone().requires_grad_(True) for t in (w[0], w[1], bb[0], bb[1])]
            hr = h0.clone().requires_grad_(True) if state else None
            cr = c0.clone().requires_grad_(True) if state else None
            yr, hTr, cTr = O.lstm_layer(xr, *rw, hr, cr, reverse=rev)
            (yr.square().sum() + hTr.square().sum() + cTr.sum()).backward()
            ref = [yr, hTr, cTr, xr.grad] + [t.grad for t in rw] + ([hr.grad, cr.grad] if state else [])
            for a, r in zip(got, ref):
                assert rel_err(a, r.detach()) < TOL
    for a_list, b_list in zip(outs[1], outs.get(0, [])):
        for a, b in zip(a_list, b_list):
            assert rel_err(a, b) < TOL
    for a in outs[1][0]:
        assert torch.isfinite(a).all()


@pytest.mark.parametrize("resln,masked", [(False, False), (True, False), (True, True)])
def test_mha_one_key_shortcut_matches_attention_kernel(resln, masked):
    """Tq = Tk = 1 (a generation frame attending to one frame): the value-projection shortcut
    (functional._MHAOneKeyFn) against the full attention path (_MHAFn) on the same inputs,
    forward and backward; masked: one row hidden by the padding AND rule (NaN in both paths)."""
    from multimodalreactiongeneration_amd import functional as Fn
    B, E, heads = 64, 256, 4
    g = torch.Generator().manual_seed(11)
    q = torch.randn(B, 1, E, generator=g)
    kv = torch.randn(B, 1, E, generator=g)
    dy = torch.randn(B, 1, E, generator=g)
    ws = [torch.randn(3 * E, E, generator=g) * 0.05, torch.randn(3 * E, generator=g) * 0.05,
          torch.randn(E, E, generator=g) * 0.05, torch.randn(E, generator=g) * 0.05,
          1 + torch.randn(E, generator=g) * 0.1, torch.randn(E, generator=g) * 0.1]
    qpad = kpad = None
    keep = torch.ones(B, dtype=torch.bool)
    if masked:
        qpad = torch.zeros(B, 1, dtype=torch.uint8)
        kpad = torch.zeros(B, 1, dtype=torch.uint8)
        qpad[3] = kpad[3] = 1      # hidden row
        qpad[5] = 1                # query padding alone hides nothing
        keep[3] = False
        qpad, kpad = qpad.to(DEV), kpad.to(DEV)
    outs = []
    for one_key in (True, False):
        ps = [_param(w) for w in ws]
        qq, kk = q.to(DEV).requires_grad_(True), kv.to(DEV).requires_grad_(True)
        extra = (ps[4], ps[5]) if resln else ()
        eps = 1e-5 if resln else None
        if one_key:
            y = Fn._MHAOneKeyFn.apply(eps, qq, kk, *ps[:4], qpad, kpad, *extra)
        else:
            y = Fn._MHAFn.apply((heads, True, eps), qq, kk, *ps[:4], qpad, kpad, *extra)
        (y[keep] * dy.to(DEV)[keep]).sum().backward()
        torch.cuda.synchronize()
        outs.append((y.detach(), qq.grad, kk.grad, [None if p.grad is None else p.grad.clone() for p in ps]))
    (y1, dq1, dk1, g1), (y0, dq0, dk0, g0) = outs
    if masked:
        assert torch.isnan(y1[3]).all() and torch.isnan(y0[3]).all()
    assert rel_err(y1[keep], y0[keep]) < 1e-6
    assert rel_err(dk1[keep], dk0[keep]) < 1e-5
    if resln:
        assert rel_err(dq1[keep], dq0[keep]) < 1e-5
    else:
        assert dq1 is None or float(dq1.abs().max()) == 0.0
        assert float(dq0.abs().max()) <= 1e-5 * float(dk0.abs().max())
    if masked:
        return  # the hidden row's NaN reaches every parameter gradient in both paths
    # V rows of in_proj, its bias, out_proj, LN: same gradients; Q / K rows: none vs ~0
    assert rel_err(g1[0][2 * E:], g0[0][2 * E:]) < 1e-5
    assert rel_err(g1[1][2 * E:], g0[1][2 * E:]) < 1e-5
    assert float(g1[0][:2 * E].abs().max()) == 0.0
    assert float(g0[0][:2 * E].abs().max()) <= 1e-5 * float(g0[0].abs().max())
    for a_, b_ in zip(g1[2:], g0[2:]):
        if b_ is not None:
            assert rel_err(a_, b_) < 1e-5


@pytest.mark.parametrize("case", [0, 1, 2])
def test_mha_with_reference_mask_golden(case):
    from multimodalreactiongeneration_amd.model.layers import MultiheadAttention
    from multimodalreactiongeneration_amd.model.masks import gen_attention_mask
    d = load("ops")
    p = f"mha{case}/"
    heads = int(d[p + "heads"])
    q = torch.from_numpy(d[p + "q"])
    kv = torch.from_numpy(d[p + "kv"])
    E = q.shape[-1]
    mha = MultiheadAttention(E, heads, batch_first=True, kdim=E, vdim=E)
    mha.load_state_dict(prefixed(d, p + "param/"))
    mha = mha.to(DEV)
    mq, mk = q.clone(), kv.clone()
    mq[1, q.shape[1] - 2:] = -100
    mk[1, kv.shape[1] - 3:] = -100
    mask = gen_attention_mask(mq.to(DEV), mk.to(DEV), heads)
    assert torch.equal(mask.dense().reshape(-1, q.shape[1], kv.shape[1]).cpu(), torch.from_numpy(d[p + "mask"]))
    qd = q.to(DEV).requires_grad_(True)
    kvd = kv.to(DEV).requires_grad_(True)
    o, _ = mha(qd, kvd, kvd, None, False, mask, False, False)
    o.backward(torch.from_numpy(d[p + "do"]).to(DEV))
    torch.cuda.synchronize()
    assert rel_err(o, d[p + "o"]) < TOL
    assert rel_err(qd.grad, d[p + "dq"]) < TOL
    assert rel_err(kvd.grad, d[p + "dkv"]) < TOL
    for k, prm in mha.named_parameters():
        assert rel_err(prm.grad, d[p + f"grad/{k}"]) < TOL, k


@pytest.mark.parametrize("Tq,Tk,E,heads,causal", [(300, 300, 256, 4, True), (300, 2400, 256, 4, True),
                                                  (100, 100, 256, 8, False), (37, 74, 64, 2, True),
                                                  (40, 20, 128, 4, True)])
def test_attention_vs_oracle(Tq, Tk, E, heads, causal):
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    B = 3
    g = torch.Generator().manual_seed(Tq + Tk)
    q, kv = torch.randn(B, Tq, E, generator=g), torch.randn(B, Tk, E, generator=g)
    sd = {"in_proj_weight": torch.randn(3 * E, E, generator=g) / math.sqrt(E),
          "in_proj_bias": torch.randn(3 * E, generator=g) * 0.1,
          "out_proj.weight": torch.randn(E, E, generator=g) / math.sqrt(E),
          "out_proj.bias": torch.randn(E, generator=g) * 0.1}
    do = torch.randn(B, Tq, E, generator=g)
    ps = {k: _param(v) for k, v in sd.items()}
    qd, kvd = q.to(DEV).requires_grad_(True), kv.to(DEV).requires_grad_(True)
    qpad = torch.zeros(B, Tq, dtype=torch.uint8, device=DEV) if causal else None
    kpad = torch.zeros(B, Tk, dtype=torch.uint8, device=DEV) if causal else None
    o = Fn.mha(qd, kvd, ps["in_proj_weight"], ps["in_proj_bias"], ps["out_proj.weight"], ps["out_proj.bias"],
               heads, causal, qpad, kpad)
    o.backward(do.to(DEV))
    torch.cuda.synchronize()
    rs = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    qr, kvr = q.clone().requires_grad_(True), kv.clone().requires_grad_(True)
    mask = O.gen_attention_mask(qr, kvr, heads).reshape(-1, Tq, Tk) if causal else None
    orf = O.mha(qr, kvr, rs, "", heads, mask)
    orf.backward(do)
    assert rel_err(o, orf) < TOL
    assert rel_err(qd.grad, qr.grad) < TOL
    assert rel_err(kvd.grad, kvr.grad) < TOL
    for k in sd:
        assert rel_err(ps[k].grad, rs[k].grad) < TOL, k


@pytest.mark.parametrize("Tq,Tk,E,heads", [(64, 128, 64, 4), (150, 75, 128, 2), (90, 90, 32, 4)])
def test_attention_ragged_padding_vs_oracle(Tq, Tk, E, heads):
    """Block-causal mask + the padding AND rule with ragged lengths (eval-mode padding flows through)."""
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    B = 3
    g = torch.Generator().manual_seed(Tq * 7 + Tk)
    q, kv = torch.randn(B, Tq, E, generator=g), torch.randn(B, Tk, E, generator=g)
    for bi, (lq, lk) in enumerate([(Tq, Tk), (Tq * 2 // 3, Tk * 2 // 3), (Tq // 3, Tk // 2)]):
        q[bi, lq:] = -100.0
        kv[bi, lk:] = -100.0
    sd = {"in_proj_weight": torch.randn(3 * E, E, generator=g) / math.sqrt(E) * 0.1,
          "in_proj_bias": torch.randn(3 * E, generator=g) * 0.1,
          "out_proj.weight": torch.randn(E, E, generator=g) / math.sqrt(E),
          "out_proj.bias": torch.randn(E, generator=g) * 0.1}
    do = torch.randn(B, Tq, E, generator=g)
    ps = {k: _param(v) for k, v in sd.items()}
    qd, kvd = q.to(DEV).requires_grad_(True), kv.to(DEV).requires_grad_(True)
    o = Fn.mha(qd, kvd, ps["in_proj_weight"], ps["in_proj_bias"], ps["out_proj.weight"], ps["out_proj.bias"],
               heads, True, Fn.padding_flags(q.to(DEV)), Fn.padding_flags(kv.to(DEV)))
    o.backward(do.to(DEV))
    torch.cuda.synchronize()
    rs = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    qr, kvr = q.clone().requires_grad_(True), kv.clone().requires_grad_(True)
    orf = O.mha(qr, kvr, rs, "", heads, O.gen_attention_mask(qr, kvr, heads).reshape(-1, Tq, Tk))
    orf.backward(do)
    assert not torch.isnan(orf).any()
    assert rel_err(o, orf) < TOL
    assert rel_err(qd.grad, qr.grad) < TOL
    assert rel_err(kvd.grad, kvr.grad) < TOL
    for k in sd:
        assert rel_err(ps[k].grad, rs[k].grad) < TOL, k


def test_attention_fully_masked_row_is_nan_like_reference():
    """A query row whose every visible key is padding (AND rule) -> NaN, as softmax(-inf row)."""
    from multimodalreactiongeneration_amd import functional as Fn
    from oracle import mrg_oracle as O
    B, T, E, heads = 1, 4, 16, 2
    q = torch.randn(B, T, E)
    kv = torch.randn(B, T, E)
    q[0, 0] = -100
    kv[0, 0] = -100   # query 0 sees only key 0, both padded -> masked
    sd = {"in_proj_weight": torch.randn(3 * E, E) * 0.2, "in_proj_bias": torch.zeros(3 * E),
          "out_proj.weight": torch.randn(E, E) * 0.2, "out_proj.bias": torch.zeros(E)}
    ps = {k: _param(v) for k, v in sd.items()}
    o = Fn.mha(q.to(DEV), kv.to(DEV), ps["in_proj_weight"], ps["in_proj_bias"], ps["out_proj.weight"],
               ps["out_proj.bias"], heads, True, Fn.padding_flags(q.to(DEV)), Fn.padding_flags(kv.to(DEV)))
    ref = O.mha(q, kv, sd, "", heads, O.gen_attention_mask(q, kv, heads).reshape(-1, T, T))
    assert torch.isnan(ref[0, 0]).all() and torch.isnan(o[0, 0].cpu()).all()
    assert rel_err(o[0, 1:], ref[0, 1:]) < TOL


def test_adamw_matches_oracle_over_three_steps():
    from multimodalreactiongeneration_amd.optim import FusedAdamW
    from oracle import mrg_oracle as O
    g = torch.Generator().manual_seed(9)
    p0 = [torch.randn(300, 7, generator=g), torch.randn(1000, generator=g)]
    params = [torch.nn.Parameter(t.clone().to(DEV)) for t in p0]
    opt = FusedAdamW(params, lr=1e-3, weight_decay=1e-2)
    ref = {str(i): t.clone() for i, t in enumerate(p0)}
    state = {}
    for step in range(3):
        grads = [torch.randn(t.shape, generator=g) for t in p0]
        for p, gr in zip(params, grads):
            p.grad.copy_(gr.to(DEV))
        opt.step()
        O.adamw_step(ref, {str(i): gr for i, gr in enumerate(grads)}, state, 1e-3, 1e-2)
    for i, p in enumerate(params):
        assert rel_err(p.detach(), ref[str(i)]) < 1e-6


@pytest.mark.parametrize("In,H,B,T,bidir,state", [(16, 32, 4, 20, False, False), (24, 32, 3, 9, True, True),
                                                  (256, 256, 64, 40, False, True), (256, 256, 37, 25, True, False),
                                                  (128, 128, 64, 30, True, True), (40, 64, 9, 17, False, True)])
def test_gru_vs_torch_fp64(In, H, B, T, bidir, state):
    """layers.GRU (persistent recurrences, gru_rec.hip: ring groups at H = 256, solo groups below) vs
    torch.nn.GRU in fp64: outputs, final states, input / state / every parameter gradient (SURVEY 8f
    rank 4)."""
    from multimodalreactiongeneration_amd.model.layers import GRU
    torch.manual_seed(In + H + T)
    ref = torch.nn.GRU(In, H, num_layers=2, batch_first=True, bidirectional=bidir).double()
    g = GRU(In, H, num_layers=2, batch_first=True, bidirectional=bidir)
    g.load_state_dict({k: v.float() for k, v in ref.state_dict().items()})
    g = g.to(DEV)
    D = 2 if bidir else 1
    x = torch.randn(B, T, In, dtype=torch.float64)
    h0 = torch.randn(2 * D, B, H, dtype=torch.float64) if state else None
    dy = torch.randn(B, T, D * H, dtype=torch.float64)
    dh = torch.randn(2 * D, B, H, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    hr = None if h0 is None else h0.clone().requires_grad_(True)
    yr, hnr = ref(xr, hr)
    ((yr * dy).sum() + (hnr * dh).sum()).backward()
    xd = x.float().to(DEV).requires_grad_(True)
    hd = None if h0 is None else h0.float().to(DEV).requires_grad_(True)
    y, hn = g(xd, hd)
    ((y * dy.float().to(DEV)).sum() + (hn * dh.float().to(DEV)).sum()).backward()
    torch.cuda.synchronize()
    assert rel_err(y, yr) < TOL
    assert rel_err(hn, hnr) < TOL
    assert rel_err(xd.grad, xr.grad) < TOL
    if state:
        assert rel_err(hd.grad, hr.grad) < TOL
    gp = dict(g.named_parameters())
    for k, p in ref.named_parameters():
        assert rel_err(gp[k].grad, p.grad) < TOL, k


@pytest.mark.parametrize("H,B,T,reverse,group", [(256, 64, 300, False, 4), (256, 64, 300, True, 8),
                                                 (128, 64, 300, True, 1)])
def test_gru_persistent_matches_per_step(H, B, T, reverse, group):
    """The persistent GRU recurrence (one launch per layer direction) vs the per-step products + cell
    kernels at the GRU config's width (B = 64, T = 300): outputs, final state and every gradient, for
    both ring sizes at H = 256 (mrg_gru_config)."""
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd import _lib as L
    lib = L.load()
    prev_group = lib.mrg_gru_config(group) if H == 256 else None
    g = torch.Generator().manual_seed(H + T)
    s = 1.0 / math.sqrt(H)
    w = [torch.randn(3 * H, H, generator=g) * s for _ in range(2)]
    bb = [torch.randn(3 * H, generator=g) * s for _ in range(2)]
    x = torch.randn(B, T, H, generator=g)
    h0 = torch.randn(B, H, generator=g) * 0.5
    dy = torch.randn(B, T, H, generator=g)
    outs = []
    prev = Fn._GRU_PERSIST[0]
    try:
        for persist in (True, False):
            Fn._GRU_PERSIST[0] = persist
            ps = [_param(t) for t in (w[0], w[1], bb[0], bb[1])]
            xx = x.to(DEV).requires_grad_(True)
            hh = h0.to(DEV).requires_grad_(True)
            y, hT = Fn.gru_layer(xx, *ps, hh, reverse=reverse)
            ((y * dy.to(DEV)).sum() + hT.square().sum()).backward()
            torch.cuda.synchronize()
            Fn.check_errors()
            outs.append([y.detach(), hT.detach(), xx.grad, hh.grad] + [p.grad for p in ps])
    finally:
        Fn._GRU_PERSIST[0] = prev
        if prev_group is not None:
            lib.mrg_gru_config(prev_group)
    for a, b in zip(*outs):
        assert rel_err(a, b) < TOL


def test_adamw_graph_replay_follows_lr_scheduler():
    """A replayed graph holding opt.step() uses the LR the CosineAnnealingLR scheduler sets between
    replays (the device-side LR follows param_groups[0]['lr']), and capture(preserve=...) leaves
    no warm-up update behind: three replays == three torch.optim.AdamW steps."""
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.optim import FusedAdamW
    g = torch.Generator().manual_seed(4)
    p0 = [torch.randn(64, 33, generator=g), torch.randn(517, generator=g)]
    grads = [torch.randn(t.shape, generator=g) for t in p0]
    params = [torch.nn.Parameter(t.clone().to(DEV)) for t in p0]
    opt = FusedAdamW(params, lr=1e-2, weight_decay=1e-2)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=4)
    for p, gr in zip(params, grads):
        p.grad.copy_(gr.to(DEV))
    replay = capture(opt.step, 2, preserve=opt.state_tensors())
    ref = [torch.nn.Parameter(t.clone()) for t in p0]
    ropt = torch.optim.AdamW(ref, lr=1e-2, weight_decay=1e-2)
    rsched = torch.optim.lr_scheduler.CosineAnnealingLR(ropt, T_max=4)
    for _ in range(3):
        replay()
        for p, gr in zip(ref, grads):
            p.grad = gr.clone()
        ropt.step()
        sched.step()
        rsched.step()
    torch.cuda.synchronize()
    for p, r in zip(params, ref):
        assert rel_err(p.detach(), r.detach()) < 1e-6


def test_lstm_handoff_timeout_skips_adamw_and_raises():
    """A persistent-LSTM hand-off timeout (forced with mrg_lstm_debug_inject) must not train on its
    garbage gradients: the AdamW kernel skips the update, FusedAdamW.step raises at the next step
    and check_errors() raises."""
    from multimodalreactiongeneration_amd import _lib as L
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.optim import FusedAdamW
    torch.manual_seed(3)
    H, B, T = 64, 4, 12
    ws = [torch.nn.Parameter((torch.randn(4 * H, H) * 0.1).to(DEV)) for _ in range(2)]
    bs = [torch.nn.Parameter(torch.zeros(4 * H).to(DEV)) for _ in range(2)]
    opt = FusedAdamW(ws + bs, lr=1e-3)
    x = torch.randn(B, T, H, device=DEV)
    before = opt.flat.clone()
    prev_solo = L.load().mrg_lstm_set_solo(0)   # a hand-off ring to drop (solo groups have none)
    L.check(L.load().mrg_lstm_debug_inject(1), "inject")
    y, _, _ = Fn.lstm_layer(x, ws[0], ws[1], bs[0], bs[1])
    y.square().sum().backward()
    opt.step()
    torch.cuda.synchronize()
    assert torch.equal(opt.flat, before)          # update skipped on the device
    assert float(opt.step_lr[0]) == 0.0           # and not counted
    with pytest.raises(RuntimeError, match="timed out"):
        opt.step()                                # the next host-visible point raises
    Fn.check_errors()                             # flag cleared by the raise above
    y, _, _ = Fn.lstm_layer(x, ws[0], ws[1], bs[0], bs[1])   # a clean launch works again
    y.square().sum().backward()
    opt.step()
    torch.cuda.synchronize()
    Fn.check_errors()
    L.load().mrg_lstm_set_solo(prev_solo)
    assert not torch.equal(opt.flat, before)


@pytest.mark.parametrize("mode,mx", [(1, 2), (2, 2), (2, 0)])
def test_lstm_handoff_timeout_reports_and_returns(mode, mx):
    """The hand-off timeout path of the MFMA recurrence (lstm_mx.hip pair granules, forward: mode 1) and
    of the backward recurrences (mode 2; MFMA and VALU forms): member 0 drops its first hand-off, the
    waiting members time out, OR the device error flag (which DDP agrees on across ranks) and the
    launch returns; a clean launch afterwards matches a clean launch before."""
    from multimodalreactiongeneration_amd import _lib as L
    from multimodalreactiongeneration_amd import functional as Fn
    lib = L.load()
    torch.manual_seed(5)
    H, B, T = 256, 16, 4
    w = [torch.nn.Parameter((torch.randn(4 * H, H) * 0.05).to(DEV)) for _ in range(2)]
    b = [torch.nn.Parameter(torch.zeros(4 * H).to(DEV)) for _ in range(2)]
    x = torch.randn(B, T, H, device=DEV)
    err = Fn._err_flag(DEV)
    prev = lib.mrg_lstm_set_mx(mx, 0)

    def run():
        for p in w + b:
            p.grad = None
        y, _, _ = Fn.lstm_layer(x, w[0], w[1], b[0], b[1])
        y.square().sum().backward()
        torch.cuda.synchronize()
        return y.detach().clone(), w[1].grad.detach().clone()
    try:
        y0, g0 = run()
        assert int(err.item()) == 0
        L.check(lib.mrg_lstm_debug_inject(mode), "inject")
        run()
        assert int(err.item()) != 0
        err.zero_()
        y1, g1 = run()
        assert int(err.item()) == 0
        assert torch.equal(y1, y0) and torch.equal(g1, g0)
    finally:
        lib.mrg_lstm_debug_inject(0)
        lib.mrg_lstm_set_mx(prev, 0)
        err.zero_()


@pytest.mark.parametrize("M,N,K,epi,n", [(3840, 1024, 256, 0, 11), (3840, 256, 256, 3, 5), (3840, 256, 1024, 3, 16),
                                         (300, 256, 64, 0, 3), (100, 96, 40, 1, 2)])
def test_batched_gemm_matches_single_products(M, N, K, epi, n, gemm_mode):
    """mrg_gemm_x6g_batched (the encoder stack's per-diagonal products): every problem bitwise equal to
    the same product launched alone (shapes outside the LDS-DMA kernel run one by one)."""
    import ctypes
    from multimodalreactiongeneration_amd import _lib as L
    from multimodalreactiongeneration_amd import functional as Fn
    lib = L.load()
    g = torch.Generator().manual_seed(M + N + K + n)
    As = [torch.randn(M, K, generator=g).to(DEV) for _ in range(n)]
    Ws = [(torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV) for _ in range(n)]
    bs = [torch.randn(N, generator=g).to(DEV) for _ in range(n)]
    aux = [torch.randn(M, N, generator=g).to(DEV) for _ in range(n)] if epi >= 2 else None
    Cs = [torch.empty(M, N, device=DEV) for _ in range(n)]
    VP = ctypes.c_void_p
    arr = lambda v: (VP * n)(*[VP(t.data_ptr()) for t in v])  # noqa: E731
    L.check(lib.mrg_gemm_x6g_batched(n, M, N, K, 1.0, arr(As), K, arr(Ws), K, 0.0, arr(Cs), N, arr(bs), epi,
                                     None if aux is None else arr(aux), N, 0, Fn._stream()), "batched")
    for i in range(n):
        ref = torch.empty(M, N, device=DEV)
        L.check(lib.mrg_gemm_f32_ex(M, N, K, 1.0, VP(As[i].data_ptr()), 0, K, 0, 0, VP(Ws[i].data_ptr()), 1, K, 0, 0,
                                    0.0, VP(ref.data_ptr()), N, VP(bs[i].data_ptr()), epi,
                                    None if aux is None else VP(aux[i].data_ptr()), N, None, 1, None, None, 0.0, None,
                                    Fn._stream()), "single")
        torch.cuda.synchronize()
        assert torch.equal(Cs[i], ref), i
        exact = As[i].double() @ Ws[i].double().T + bs[i].double()
        if epi == 1:
            exact = exact.clamp_min(0)
        elif epi == 3:
            exact = exact + aux[i].double()
        assert rel_err(Cs[i], exact) < TOL


@pytest.mark.parametrize("M,N,K,epi,beta", [(19200, 1024, 256, 0, 0.0), (19200, 256, 256, 3, 0.0),
                                            (19200, 512, 256, 1, 0.0), (19200, 256, 1024, 3, 1.0),
                                            (2100, 256, 512, 2, 0.0), (6400, 1024, 256, 0, 0.0),
                                            (6400, 256, 128, 3, 1.0), (1000, 200, 256, 1, 0.0)])
def test_weight_plane_products_every_kernel(M, N, K, epi, beta):
    """C = epi(A W^T + beta C + bias) on W's pre-split bf16 planes (mrg_gemm_x6_planes) through each kernel
    mrg_gemm_set_wide selects: the LDS-DMA tile kernel (0) and the row-owning ring kernel (gemm_x6w_kernel,
    64 / 128 columns), vs fp64: every epilogue, accumulation into C, ragged M and N."""
    import ctypes
    from multimodalreactiongeneration_amd import _lib as L
    from multimodalreactiongeneration_amd import functional as Fn
    lib = L.load()
    g = torch.Generator().manual_seed(M + N + K + epi)
    A = torch.randn(M, K, generator=g).to(DEV)
    W = (torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV)
    b = torch.randn(N, generator=g).to(DEV)
    aux = torch.randn(M, N, generator=g).to(DEV) if epi >= 2 else None
    C0 = torch.randn(M, N, generator=g).to(DEV)
    VP, CI = ctypes.c_void_p, ctypes.c_int
    planes = torch.empty(3, N, K, dtype=torch.int16, device=DEV)
    L.check(lib.mrg_split_planes_batched(1, (VP * 1)(VP(W.data_ptr())), (VP * 1)(VP(planes.data_ptr())), (CI * 1)(N),
                                         (CI * 1)(K), (CI * 1)(0), Fn._stream()), "split")
    exact = A.double() @ W.double().T + b.double() + beta * C0.double()
    if epi == 1:
        exact = exact.clamp_min(0)
    elif epi == 2:
        exact = exact * (aux.double() > 0)
    elif epi == 3:
        exact = exact + aux.double()
    prev = lib.mrg_gemm_set_wide(0)
    try:
        for cfg in (0, 12, 22):
            lib.mrg_gemm_set_wide(cfg)
            C = C0.clone()
            L.check(lib.mrg_gemm_x6_planes(M, N, K, 1.0, VP(A.data_ptr()), K, 0, 0, VP(planes.data_ptr()), K, N * K,
                                           beta, VP(C.data_ptr()), N, VP(b.data_ptr()), epi,
                                           None if aux is None else VP(aux.data_ptr()), N, Fn._stream()), "planes")
            torch.cuda.synchronize()
            # x6 is fp32-class: ~6e-7 of the output's scale, so a dropped or mis-split product (~1e-5) fails
            assert ((C.double() - exact).abs().max() / exact.abs().max()).item() < 3e-6, cfg
    finally:
        lib.mrg_gemm_set_wide(prev)


@pytest.mark.parametrize("n,M,N,K,epi,beta", [(5, 19200, 256, 256, 3, 0.0), (3, 6400, 1024, 256, 1, 1.0),
                                              (2, 2100, 64, 512, 2, 0.0)])
def test_batched_plane_products_match_single(n, M, N, K, epi, beta):
    """mrg_gemm_x6_planes_batched (the encoder stack's and fused integrators' projections): each problem
    bitwise equal to its own mrg_gemm_x6_planes launch on the same row-owning kernel configuration."""
    import ctypes
    from multimodalreactiongeneration_amd import _lib as L
    from multimodalreactiongeneration_amd import functional as Fn
    lib = L.load()
    g = torch.Generator().manual_seed(n * M + N + K)
    VP, CI = ctypes.c_void_p, ctypes.c_int
    As = [torch.randn(M, K, generator=g).to(DEV) for _ in range(n)]
    Ws = [(torch.randn(N, K, generator=g) / math.sqrt(K)).to(DEV) for _ in range(n)]
    bs = [torch.randn(N, generator=g).to(DEV) for _ in range(n)]
    aux = [torch.randn(M, N, generator=g).to(DEV) for _ in range(n)] if epi >= 2 else None
    C0 = [torch.randn(M, N, generator=g).to(DEV) for _ in range(n)]
    planes = [torch.empty(3, N, K, dtype=torch.int16, device=DEV) for _ in range(n)]
    arr = lambda xs: (VP * n)(*[VP(x.data_ptr()) for x in xs])  # noqa: E731
    L.check(lib.mrg_split_planes_batched(n, arr(Ws), arr(planes), (CI * n)(*[N] * n), (CI * n)(*[K] * n),
                                         (CI * n)(*[0] * n), Fn._stream()), "split")
    Cb = [c.clone() for c in C0]
    L.check(lib.mrg_gemm_x6_planes_batched(n, M, N, K, 1.0, arr(As), K, arr(planes), K, N * K, beta, arr(Cb), N,
                                           arr(bs), epi, None if aux is None else arr(aux), N, Fn._stream()),
            "batched")
    prev = lib.mrg_gemm_set_wide(12)
    try:
        for i in range(n):
            C = C0[i].clone()
            L.check(lib.mrg_gemm_x6_planes(M, N, K, 1.0, VP(As[i].data_ptr()), K, 0, 0, VP(planes[i].data_ptr()), K,
                                           N * K, beta, VP(C.data_ptr()), N, VP(bs[i].data_ptr()), epi,
                                           None if aux is None else VP(aux[i].data_ptr()), N, Fn._stream()), "single")
            torch.cuda.synchronize()
            assert torch.equal(Cb[i], C), i
    finally:
        lib.mrg_gemm_set_wide(prev)


@pytest.mark.parametrize("n,rows,E", [(11, 3840, 256), (3, 70, 512), (16, 32, 36)])
def test_batched_layernorm_matches_single(n, rows, E):
    """mrg_residual_layernorm_{fwd,bwd}_batched: each problem bitwise equal to the row-mapped single
    launch, output / incoming-gradient rows through per-problem maps (time-major <-> batch-major)."""
    import ctypes
    from multimodalreactiongeneration_amd import _lib as L
    from multimodalreactiongeneration_amd import functional as Fn
    lib = L.load()
    g = torch.Generator().manual_seed(n * rows + E)
    VP, CL, CI = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
    Bm = 2 if rows % 2 == 0 else 1
    Tm = rows // Bm
    r = lambda *s: torch.randn(*s, generator=g).to(DEV)  # noqa: E731
    a, b, dy = [r(rows, E) for _ in range(n)], [r(rows, E) for _ in range(n)], [r(Bm, Tm, E) for _ in range(n)]
    gam, bet = [1 + 0.1 * r(E) for _ in range(n)], [0.1 * r(E) for _ in range(n)]
    maps = [(Tm * E, E, Bm) if i % 2 else (E, 0, 0) for i in range(n)]   # odd problems: time-major -> [B, T, E]
    nblk = (rows + 31) // 32
    outs = {k: [torch.zeros(Bm, Tm, E, device=DEV) if k in ("y", "y1") else
                torch.zeros(rows, E, device=DEV) if k in ("dx", "dx1") else
                torch.zeros(nblk * 2 * E, device=DEV) if k in ("ws", "ws1") else torch.zeros(rows, device=DEV)
                for _ in range(n)] for k in ("y", "m", "s", "dx", "ws", "y1", "m1", "s1", "dx1", "ws1")}
    P = lambda v: (VP * n)(*[VP(t.data_ptr()) for t in v])  # noqa: E731
    L.check(lib.mrg_residual_layernorm_fwd_batched(
        n, rows, E, P(a), P(b), P(gam), P(bet), 1e-5, P(outs["y"]), (CL * n)(*[m[0] for m in maps]),
        (CL * n)(*[m[1] for m in maps]), (CI * n)(*[m[2] for m in maps]), P(outs["m"]), P(outs["s"]), Fn._stream()),
        "fwd batched")
    L.check(lib.mrg_residual_layernorm_bwd_batched(
        n, rows, E, P(dy), (CL * n)(*[m[0] for m in maps]), (CL * n)(*[m[1] for m in maps]),
        (CI * n)(*[m[2] for m in maps]), P(a), P(b), P(gam), P(outs["m"]), P(outs["s"]), P(outs["dx"]),
        P(outs["ws"]), Fn._stream()), "bwd batched")
    for i in range(n):
        lo, hi, dv = maps[i]
        L.check(lib.mrg_residual_layernorm_fwd_map(rows, E, VP(a[i].data_ptr()), VP(b[i].data_ptr()),
                                                   VP(gam[i].data_ptr()), VP(bet[i].data_ptr()), 1e-5,
                                                   VP(outs["y1"][i].data_ptr()), lo, hi, dv,
                                                   VP(outs["m1"][i].data_ptr()), VP(outs["s1"][i].data_ptr()),
                                                   Fn._stream()), "fwd")
        L.check(lib.mrg_residual_layernorm_bwd_map(rows, E, VP(dy[i].data_ptr()), lo, hi, dv, VP(a[i].data_ptr()),
                                                   VP(b[i].data_ptr()), VP(gam[i].data_ptr()),
                                                   VP(outs["m1"][i].data_ptr()), VP(outs["s1"][i].data_ptr()),
                                                   VP(outs["dx1"][i].data_ptr()), VP(outs["ws1"][i].data_ptr()),
                                                   Fn._stream()), "bwd")
    torch.cuda.synchronize()
    for i in range(n):
        for k in ("y", "m", "s", "dx", "ws"):
            assert torch.equal(outs[k][i], outs[k + "1"][i]), (i, k)
    # and the math: problem 1 (batch-major output) vs torch fp64
    x = (a[1] + b[1]).double()
    ref = torch.nn.functional.layer_norm(x, (E,), gam[1].double(), bet[1].double(), 1e-5)
    lo, hi, dv = maps[1]
    got = outs["y"][1].reshape(Bm, Tm, E).permute(1, 0, 2).reshape(rows, E) if dv else outs["y"][1].reshape(rows, E)
    assert rel_err(got, ref) < TOL


@pytest.mark.parametrize("lds", [64 * 1024, 160 * 1024])
def test_recurrence_behind_cu_occupying_kernel_does_not_time_out(lds):
    """A persistent recurrence launched while another stream's kernel holds every CU (the RCCL
    all-reduce of an overlapped DDP bucket, ddp.GradReducer(overlap=True)) waits for CUs and then
    runs; its hand-offs do not time out and the result is bitwise the one run alone."""
    from multimodalreactiongeneration_amd import _lib as L
    from multimodalreactiongeneration_amd import functional as Fn
    lib = L.load()
    torch.manual_seed(5)
    H, B, T = 256, 64, 300
    k = 1 / math.sqrt(H)
    ps = [_param((torch.rand(*s) * 2 - 1) * k) for s in ((4 * H, H), (4 * H, H), (4 * H,), (4 * H,))]
    x = torch.randn(B, T, H, device=DEV)
    with torch.no_grad():
        ref = Fn.lstm_layer(x, *ps)[0].clone()
    torch.cuda.synchronize()
    cus = L.cu_count(0)
    other = torch.cuda.Stream(device=DEV)
    start = torch.cuda.Event()
    start.record()
    other.wait_event(start)
    with torch.cuda.stream(other):   # 4 workgroups of 1024 lanes per CU for 30 ms
        L.check(lib.mrg_debug_busy(4 * cus, 1024, lds, 30000.0, Fn._stream()), "busy")
    with torch.no_grad():
        y = Fn.lstm_layer(x, *ps)[0]
    torch.cuda.synchronize()
    Fn.check_errors()
    assert torch.equal(y, ref)


def test_kernel_bound_probe_times_the_kernels():
    """functional.probe_start(kernel=True) (mrg_probe_*: hipExtLaunchKernelGGL events bound to each
    kernel) reports every launch of a probed call, no more than the stream-event bracket of the same
    call and most of it for a large GEMM; untagged launches are not timed."""
    from multimodalreactiongeneration_amd import functional as Fn
    g = torch.Generator().manual_seed(1)
    x = torch.randn(19200, 256, generator=g).to(DEV)
    w = torch.randn(1024, 256, generator=g).to(DEV) / 16
    b = torch.zeros(1024, device=DEV)
    Fn.linear(x, w, b)
    torch.cuda.synchronize()
    res = {}
    for kernel in (False, True):
        Fn.probe_start("gemm", kernel=kernel)
        for _ in range(5):
            Fn.linear(x, w, b)
        Fn.residual_layernorm(x, x, torch.ones(256, device=DEV), torch.zeros(256, device=DEV))  # not probed
        res[kernel] = Fn.probe_stop(with_work=True)["gemm"]
    assert len(res[True]) == len(res[False]) == 5
    for (tk, wk), (te, we) in zip(res[True], res[False]):
        assert wk == we == 2.0 * 19200 * 1024 * 256
        assert 0.0 < tk <= te * 1.02
    assert sum(t for t, _ in res[True]) >= 0.5 * sum(t for t, _ in res[False])


def test_fill_zero_any_alignment_and_size():
    """mrg_fill_zero clears exactly [p, p + bytes) at every byte alignment (16-B body, byte ends)."""
    from multimodalreactiongeneration_amd import _lib as L
    from multimodalreactiongeneration_amd import functional as Fn
    lib = L.load()
    buf = torch.empty(70000, dtype=torch.uint8, device=DEV)
    for off in (0, 1, 3, 8, 15, 16, 17):
        for n in (0, 1, 5, 15, 16, 17, 31, 33, 4096, 65537):
            buf.fill_(0xAB)
            L.check(lib.mrg_fill_zero(Fn._ptr(buf, off), n, Fn._stream()), "fill")
            host = buf.cpu()
            assert int(host[off:off + n].sum()) == 0, (off, n)
            assert bool((host[:off] == 0xAB).all()) and bool((host[off + n:] == 0xAB).all()), (off, n)
    z = Fn.zeros(3, 5, dtype=torch.int64, device=DEV)
    assert z.dtype == torch.int64 and int(z.abs().sum()) == 0


@pytest.mark.parametrize("Tq,Tk,causal,cuts", [(300, 300, True, (0, 100, 200, 300)), (150, 300, True, (0, 37, 64, 150)),
                                                (300, 150, True, (0, 150, 300)), (100, 100, False, (0, 50, 100))])
def test_attention_query_chunks_match_whole(Tq, Tk, causal, cuts):
    """mrg_attention_{fwd,bwd}_chunk over query chunks (the block wavefront's form) vs one whole call:
    outputs, log-sum-exp and dQ bitwise (every query's arithmetic is the same); dK / dV either
    accumulated chunk by chunk (passes 3, kv_accumulate) within fp32 reordering, or from one pass-2
    call over the whole sequence after the chunks' dQ passes (bitwise); ragged padding flags included."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd.functional import _ptr, _stream
    lib = _lib.load()
    B, Hh, D = 3, 4, 64
    E = Hh * D
    g = torch.Generator().manual_seed(Tq + 3 * Tk)
    q, k, v, do = (torch.randn(B, T, E, generator=g).to(DEV) for T in (Tq, Tk, Tk, Tq))
    qpad = torch.zeros(B, Tq, dtype=torch.uint8)
    kpad = torch.zeros(B, Tk, dtype=torch.uint8)
    qpad[1, Tq * 2 // 3:] = 1
    kpad[1, Tk * 2 // 3:] = 1
    qpad, kpad = qpad.to(DEV), kpad.to(DEV)
    sc = 1.0 / math.sqrt(D)
    f = dict(device=DEV, dtype=torch.float32)

    def bwd_args(qq, oo, lse, dd, dq, dk, dv):
        return (_ptr(qq), Tq * E, E, _ptr(k), Tk * E, E, _ptr(v), Tk * E, E, _ptr(oo), Tq * E, E, _ptr(lse),
                _ptr(qpad), _ptr(kpad), int(causal), sc, _ptr(dd), Tq * E, E, _ptr(dq), Tq * E, E, _ptr(dk), Tk * E, E,
                _ptr(dv), Tk * E, E)
    o, lse = torch.empty(B, Tq, E, **f), torch.empty(B, Hh, Tq, **f)
    assert lib.mrg_attention_fwd(B, Hh, Tq, Tk, D, _ptr(q), Tq * E, E, _ptr(k), Tk * E, E, _ptr(v), Tk * E, E, _ptr(o),
                                 Tq * E, E, _ptr(lse), _ptr(qpad), _ptr(kpad), int(causal), sc, _stream()) == 0
    dq, dk, dv = torch.empty(B, Tq, E, **f), torch.empty(B, Tk, E, **f), torch.empty(B, Tk, E, **f)
    ws = torch.empty(B * Hh * Tq, **f)
    prev = lib.mrg_attention_set_fused(0)   # the chunk forms are the two-pass kernels: compare like with like
    try:
        assert lib.mrg_attention_bwd(B, Hh, Tq, Tk, D, *bwd_args(q, o, lse, do, dq, dk, dv), _ptr(ws), _stream()) == 0
    finally:
        lib.mrg_attention_set_fused(prev)
    oc, dqc, dqs = torch.full_like(o, 7.0), torch.full_like(dq, 7.0), torch.full_like(dq, 7.0)
    dkc, dvc = torch.zeros_like(dk), torch.zeros_like(dv)
    dks, dvs = torch.full_like(dk, 7.0), torch.full_like(dv, 7.0)
    lc = torch.full_like(lse, 7.0)
    wsc, wss = torch.empty(B * Hh * Tq, **f), torch.empty(B * Hh * Tq, **f)

    def chunk_bwd(q0, n, dqx, dkx, dvx, passes, acc, wsx):
        return lib.mrg_attention_bwd_chunk(
            B, Hh, n, Tk, D, q0, Tq, _ptr(q, q0 * E), Tq * E, E, _ptr(k), Tk * E, E, _ptr(v), Tk * E, E,
            _ptr(oc, q0 * E), Tq * E, E, _ptr(lc), _ptr(qpad), _ptr(kpad), int(causal), sc, _ptr(do, q0 * E),
            Tq * E, E, _ptr(dqx, q0 * E), Tq * E, E, _ptr(dkx), Tk * E, E, _ptr(dvx), Tk * E, E, passes, acc,
            _ptr(wsx), _stream())
    for q0, q1 in zip(cuts[:-1], cuts[1:]):
        n = q1 - q0
        assert lib.mrg_attention_fwd_chunk(B, Hh, n, Tk, D, q0, Tq, _ptr(q, q0 * E), Tq * E, E, _ptr(k), Tk * E, E,
                                           _ptr(v), Tk * E, E, _ptr(oc, q0 * E), Tq * E, E, _ptr(lc), _ptr(qpad),
                                           _ptr(kpad), int(causal), sc, _stream()) == 0
        assert chunk_bwd(q0, n, dqc, dkc, dvc, 3, 1, wsc) == 0
        assert chunk_bwd(q0, n, dqs, dks, dvs, 1, 0, wss) == 0
    assert chunk_bwd(0, Tq, dqs, dks, dvs, 2, 0, wss) == 0
    torch.cuda.synchronize()
    assert torch.equal(lc, lse)
    assert torch.equal(oc, o) and torch.equal(dqc, dq) and torch.equal(dqs, dq)
    assert torch.equal(dks, dk) and torch.equal(dvs, dv)
    assert rel_err(dkc, dk) < 1e-5 and rel_err(dvc, dv) < 1e-5


@pytest.mark.parametrize("B,Tq,Tk,causal,ragged", [(64, 300, 300, True, True), (3, 300, 2400, True, True),
                                                   (3, 37, 74, True, False), (2, 320, 320, False, True),
                                                   (3, 40, 20, True, True), (3, 100, 100, False, False),
                                                   (2, 321, 321, True, True)])
def test_attention_single_pass_backward_matches_two_pass(B, Tq, Tk, causal, ragged):
    """attn_bwd_fused_kernel (one workgroup per (sample, head), dQ shares accumulated in LDS) against the
    two-pass dQ, dK / dV kernels on the same forward: dK and dV bitwise (same products, same order,
    same delta), dQ within fp32 reordering, and dQ against a float64 reference on two samples.
    Tq = 321 is past the single-pass limit (the two-pass form runs: bitwise)."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd.functional import _ptr, _stream
    lib = _lib.load()
    Hh, D = 4, 64
    E = Hh * D
    g = torch.Generator().manual_seed(Tq * 5 + Tk)
    q, do = torch.randn(B, Tq, E, generator=g), torch.randn(B, Tq, E, generator=g)
    kv = torch.randn(B, Tk, 2 * E, generator=g)
    qpad = torch.zeros(B, Tq, dtype=torch.uint8)
    kpad = torch.zeros(B, Tk, dtype=torch.uint8)
    if ragged:
        for b in range(1, B):
            qpad[b, Tq - (b * 37) % (Tq // 2 + 1) - 1:] = 1
            kpad[b, Tk - (b * 53) % (Tk // 2 + 1) - 1:] = 1
    q, do, kv, qpad, kpad = (t.to(DEV) for t in (q, do, kv, qpad, kpad))
    f = dict(device=DEV, dtype=torch.float32)
    sc = 1.0 / math.sqrt(D)
    o, lse = torch.empty(B, Tq, E, **f), torch.empty(B, Hh, Tq, **f)
    assert lib.mrg_attention_fwd(B, Hh, Tq, Tk, D, _ptr(q), Tq * E, E, _ptr(kv), Tk * 2 * E, 2 * E, _ptr(kv, E),
                                 Tk * 2 * E, 2 * E, _ptr(o), Tq * E, E, _ptr(lse), _ptr(qpad), _ptr(kpad), int(causal),
                                 sc, _stream()) == 0
    outs = {}
    for fused in (1, 0):
        dq, dkv = torch.full((B, Tq, E), 7.0, **f), torch.full((B, Tk, 2 * E), 7.0, **f)
        ws = torch.empty(B * Hh * Tq, **f)
        prev = lib.mrg_attention_set_fused(fused)
        try:
            assert lib.mrg_attention_bwd(
                B, Hh, Tq, Tk, D, _ptr(q), Tq * E, E, _ptr(kv), Tk * 2 * E, 2 * E, _ptr(kv, E), Tk * 2 * E, 2 * E,
                _ptr(o), Tq * E, E, _ptr(lse), _ptr(qpad), _ptr(kpad), int(causal), sc, _ptr(do), Tq * E, E,
                _ptr(dq), Tq * E, E, _ptr(dkv), Tk * 2 * E, 2 * E, _ptr(dkv, E), Tk * 2 * E, 2 * E, _ptr(ws),
                _stream()) == 0
        finally:
            lib.mrg_attention_set_fused(prev)
        torch.cuda.synchronize()
        outs[fused] = (dq, dkv)
    (dq1, dkv1), (dq0, dkv0) = outs[1], outs[0]
    assert torch.equal(dkv1, dkv0)
    if Tq > 320:
        assert torch.equal(dq1, dq0)
    else:
        assert rel_err(dq1, dq0) < 1e-5
    # float64 reference of dQ on two samples (the reference's mask rules: block-causal, AND padding)
    for b in (0, B - 1):
        qq = q[b].double().view(Tq, Hh, D).transpose(0, 1).requires_grad_(True)
        kk = kv[b, :, :E].double().view(Tk, Hh, D).transpose(0, 1)
        vv = kv[b, :, E:].double().view(Tk, Hh, D).transpose(0, 1)
        i, j = torch.arange(Tq, device=DEV)[:, None], torch.arange(Tk, device=DEV)[None, :]
        vis = torch.ones(Tq, Tk, dtype=torch.bool, device=DEV)
        if causal:
            vis = (j < (i + 1) * (Tk // Tq)) if Tk >= Tq else (j <= i // (Tq // Tk))
        vis = vis & ~(qpad[b].bool()[:, None] & kpad[b].bool()[None, :])
        s = (qq @ kk.transpose(1, 2)) * sc
        s = s.masked_fill(~vis, float("-inf"))
        oo = torch.softmax(s, -1) @ vv
        oo.backward(do[b].double().view(Tq, Hh, D).transpose(0, 1))
        ref = qq.grad.transpose(0, 1).reshape(Tq, E)
        assert rel_err(dq1[b], ref) < 1e-4
