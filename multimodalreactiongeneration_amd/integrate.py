"""One fused op for a metaformer block's integrator: every cross-attention mixer of the main
modality, the concat and ``cat_linear`` (IntegrateModalBlock, multi_modal_metaformer.py:128-217).

Reference, per other modality i (MHAMixerLayerd with one MHAMixerBlock, mixer_block.py:567-603,
931-963; ResidualConnection residual_connection.py:20-37; FeedForward with nonlinearity none,
mixer_block.py:37-87):

    a_i = MHA_i(q, kv_i, kv_i, block-causal mask)        (nn.MultiheadAttention, for_sequential.py:42-51)
    u_i = LN1_i(a_i + q)
    y_i = LN2_i(u_i W_ff_i^T + b_ff_i + u_i)
    out = cat(y_0, y_1, ...) W_cat^T + b_cat             (multi_modal_metaformer.py:214-215)

As autograd composes it, every block pays a concat in the forward, a contiguous copy of each
integrator's slice of the concat gradient and an add of the query's two gradients in the backward
(at::native kernels between the library's).  Here the integrators' same-shape products run as
batched launches (mrg_gemm_x6g_batched: the query / output / FeedForward projections of every
integrator in one grid each; mrg_residual_layernorm_*_batched), the last LayerNorm of integrator i
writes its rows straight into columns [iE, (i+1)E) of the concat buffer (row-mapped output, row
stride nE), its backward reads its incoming gradient from there in place, and the query's
gradient accumulates both integrators' dQ W_q (+ residual) in the epilogues of two GEMMs on one
buffer (beta = 1 for the second).  The arithmetic per element is that of the per-module path.
"""
from __future__ import annotations

import ctypes
import math
from typing import List, Sequence

import torch
from torch.autograd import Function

from . import _lib
from . import functional as Fn
from .functional import _ptr, _stream, gemm, _dx_gemm, _wt_note, _gbuf, _on_side

VP, CL, CI = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
_PER = 10   # in_w, in_b, out_w, out_b, ln1 w, ln1 b, ff w, ff b, ln2 w, ln2 b


def _arr(ct, v):
    return (ct * len(v))(*v)


def _p(t, off=0):
    return VP(t.data_ptr() + 4 * off)


def _bgemm(M, N, K, items, lda, ldc, *, epi=0, ldaux=0, transposed=False, beta=0.0, dev=None):
    """Same-shape products in one launch: items = [(A ptr, w, C ptr, bias ptr | None, aux ptr | None)];
    transposed: input-gradient products dY w through w's [in][out] copy (functional._wt), one by one
    when a copy is missing."""
    lib = _lib.load()
    if Fn.planes_batched(M, N, K, items, lda, ldc, epi=epi, ldaux=ldaux, beta=beta, transposed=transposed):
        return
    bs = []
    for a_p, w, c_p, b_p, x_p in items:
        wt = Fn._wt(w) if (transposed and M >= Fn._WT_MIN_ROWS) else (None if transposed else w)
        if wt is None:
            for a2, w2, c2, b2, x2 in items:
                _dx_gemm(M, N, K, a2, lda, w2, c2, ldc, bias=b2, epi=epi, aux=x2, ldaux=ldaux, beta=beta, device=dev)
            return
        bs.append(_ptr(wt))
    n = len(items)
    with Fn._probe("gemm", 2.0 * M * N * K * n):
        rc = lib.mrg_gemm_x6g_batched(
            n, M, N, K, 1.0, _arr(VP, [it[0] for it in items]), lda, _arr(VP, bs), K, beta,
            _arr(VP, [it[2] for it in items]), ldc,
            None if all(it[3] is None for it in items) else _arr(VP, [it[3] for it in items]), epi,
            None if all(it[4] is None for it in items) else _arr(VP, [it[4] for it in items]), ldaux,
            1 if Fn._ARITH[0] == "bf16" else 0, _stream())
    _lib.check(rc, "batched gemm (integrator)")


class KVSink:
    """The input gradient of one key / value source shared by several integrators (block 0's encoder
    outputs, attended by every block, multi_modal_metaformer.py:440-462), summed in place: each
    consumer's backward adds its dKV_i W_kv_i into ONE buffer in its GEMM epilogue (beta = 1 after the
    first) and returns no gradient for the source; the source's PRODUCER drains the buffer at the start
    of its own backward (encoder_stack._EncoderStackFn), which autograd runs only after every consumer
    that received a gradient has run its backward.  So the sum is never formed by autograd's separate
    adds, and it is right in any consumer order, for several forwards over one source, for a source
    passed twice to one op and when some consumers' backward never runs.  A source whose producer does
    not drain (no ``_mrg_kv_sink`` attribute) gets per-consumer gradients that autograd sums.

    Limitation: the consumers return None for a sinked source, so the summed gradient
    reaches the source tensor only inside its producer's backward.  ``torch.autograd.grad(...,
    inputs=[encoder_output])``, tensor hooks and ``retain_grad()`` on an encoder output therefore see
    a gradient without the integrators' share.  A backward pass that ends before the producer drains
    (e.g. one stopped at the encoder outputs) would leave a stale sum behind: the next pass's first
    write detects it (the autograd graph task that wrote it is recorded) and raises instead of adding
    onto it."""
    __slots__ = ("written", "buf", "task")

    def __init__(self):
        self.written, self.buf, self.task = 0, None, None

    def begin_write(self):
        """Called by a consumer before it adds its share: True when it is the first write of this pass."""
        task = torch._C._current_graph_task_id()
        if self.written and self.task != task:
            raise RuntimeError("integrate.KVSink: a key / value gradient sum from an earlier backward pass was "
                               "never drained by its producer (a backward stopped at the encoder outputs?); "
                               "refusing to add this pass's gradient onto it")
        self.task = task
        return self.written == 0

    def drain(self):
        buf = self.buf if self.written else None
        self.written, self.buf, self.task = 0, None, None
        return buf


class _IntegrateFn(Function):
    """spec = (n, heads, causal, eps); tensors = q, kv_0..kv_{n-1}, qpad_0..qpad_{n-1},
    kpad_0..kpad_{n-1}, 10 per integrator, cat_w, cat_b (pads: uint8 [B, T] flags or None)."""

    @staticmethod
    @Fn._keeps_precision
    def forward(ctx, spec, *t):
        n, heads, causal, eps = spec
        q_in = t[0]
        kvs = list(t[1:1 + n])
        qpads = list(t[1 + n:1 + 2 * n])
        kpads = list(t[1 + 2 * n:1 + 3 * n])
        P = [t[1 + 3 * n + _PER * i:1 + 3 * n + _PER * (i + 1)] for i in range(n)]
        cat_w, cat_b = t[1 + 3 * n + _PER * n:]
        _lib.require_device(q_in)
        dev = q_in.device
        lib = _lib.load()
        B, Tq, E = q_in.shape
        D = E // heads
        N = B * Tq
        f32 = dict(device=dev, dtype=torch.float32)
        q2 = q_in.contiguous()
        kv2 = [kv.contiguous() for kv in kvs]
        Q = torch.empty(n, N, E, **f32)
        _bgemm(N, E, E, [(_ptr(q2), P[i][0][:E], _ptr(Q[i]), _ptr(P[i][1]), None) for i in range(n)], E, E, dev=dev)
        KV = []
        for i in range(n):
            Tk = kv2[i].shape[1]
            KV.append(torch.empty(B, Tk, 2 * E, **f32))
        same_k = len({kv.shape[1] for kv in kv2}) == 1
        groups = [list(range(n))] if same_k else [[i] for i in range(n)]
        for g in groups:
            Nk = B * kv2[g[0]].shape[1]
            _bgemm(Nk, 2 * E, E, [(_ptr(kv2[i]), P[i][0][E:], _ptr(KV[i]), _p(P[i][1], E), None) for i in g],
                   E, 2 * E, dev=dev)
        O = torch.empty(n, N, E, **f32)
        lse = torch.empty(n, B, heads, Tq, **f32)
        scale = 1.0 / math.sqrt(D)
        for i in range(n):
            Tk = kv2[i].shape[1]
            with Fn._probe("attn_fwd", 4.0 * D * B * heads * Fn.visible_pairs(Tq, Tk, causal)):
                rc = lib.mrg_attention_fwd(B, heads, Tq, Tk, D, _ptr(Q[i]), Tq * E, E, _ptr(KV[i]), Tk * 2 * E,
                                           2 * E, _p(KV[i], E), Tk * 2 * E, 2 * E, _ptr(O[i]), Tq * E, E,
                                           _ptr(lse[i]), _ptr(qpads[i]), _ptr(kpads[i]), int(causal), scale, _stream())
            _lib.check(rc, "attention fwd (integrator)")
        A = torch.empty(n, N, E, **f32)    # attention outputs after out_proj
        _bgemm(N, E, E, [(_ptr(O[i]), P[i][2], _ptr(A[i]), _ptr(P[i][3]), None) for i in range(n)], E, E, dev=dev)
        U = torch.empty(n, N, E, **f32)
        m1, r1 = torch.empty(n, N, **f32), torch.empty(n, N, **f32)
        _bln_fwd(N, E, eps, [(_ptr(A[i]), _ptr(q2), _ptr(P[i][4]), _ptr(P[i][5]), _ptr(U[i]), (E, 0, 0),
                              _ptr(m1[i]), _ptr(r1[i])) for i in range(n)])
        Z = torch.empty(n, N, E, **f32)
        _bgemm(N, E, E, [(_ptr(U[i]), P[i][6], _ptr(Z[i]), _ptr(P[i][7]), None) for i in range(n)], E, E, dev=dev)
        cat = torch.empty(N, n * E, **f32)
        m2, r2 = torch.empty(n, N, **f32), torch.empty(n, N, **f32)
        _bln_fwd(N, E, eps, [(_ptr(Z[i]), _ptr(U[i]), _ptr(P[i][8]), _ptr(P[i][9]), _p(cat, i * E), (n * E, 0, 0),
                              _ptr(m2[i]), _ptr(r2[i])) for i in range(n)])
        out = torch.empty(B, Tq, E, **f32)
        gemm(N, E, n * E, _ptr(cat), 0, n * E, _ptr(cat_w), 1, n * E, _ptr(out), E, bias=_ptr(cat_b), device=dev)
        _wt_note(cat_w, N)
        for i in range(n):
            for w, rows in ((P[i][0][:E], N), (P[i][2], N), (P[i][6], N), (P[i][0][E:], B * kv2[i].shape[1])):
                _wt_note(w, rows)
        ctx.save_for_backward(q2, Q, O, lse, A, U, m1, r1, Z, m2, r2, cat, *qpads, *kv2, *KV, *kpads)
        ctx.params = (P, cat_w, cat_b)
        ctx.spec = (n, heads, causal, scale)
        ctx.kv_need = [ctx.needs_input_grad[2 + i] for i in range(n)]
        ctx.sinks = [getattr(kvs[i], "_mrg_kv_sink", None) if ctx.kv_need[i] else None for i in range(n)]
        ctx.q_need = ctx.needs_input_grad[1]
        return out

    @staticmethod
    @Fn._keeps_precision
    def backward(ctx, dout):
        n, heads, causal, scale = ctx.spec
        s = ctx.saved_tensors
        q2, Q, O, lse, A, U, m1, r1, Z, m2, r2, cat = s[:12]
        qpads, kv2 = list(s[12:12 + n]), list(s[12 + n:12 + 2 * n])
        KV, kpads = list(s[12 + 2 * n:12 + 3 * n]), list(s[12 + 3 * n:12 + 4 * n])
        P, cat_w, cat_b = ctx.params
        B, Tq, E = q2.shape
        D = E // heads
        N = B * Tq
        dev = dout.device
        lib = _lib.load()
        f32 = dict(device=dev, dtype=torch.float32)
        do2 = dout.reshape(N, E).contiguous()
        dcat = torch.empty(N, n * E, **f32)
        _dx_gemm(N, n * E, E, _ptr(do2), E, cat_w, _ptr(dcat), n * E, device=dev)
        wsb = lib.mrg_residual_layernorm_bwd_workspace_bytes(N, E) // 4
        ws2, ws1 = torch.empty(n, wsb, **f32), torch.empty(n, wsb, **f32)
        G2 = torch.empty(n, N, E, **f32)
        _bln_bwd(N, E, [(_p(dcat, i * E), (n * E, 0, 0), _ptr(Z[i]), _ptr(U[i]), _ptr(P[i][8]), _ptr(m2[i]),
                         _ptr(r2[i]), _ptr(G2[i]), _ptr(ws2[i])) for i in range(n)])
        dU = torch.empty(n, N, E, **f32)      # g2 W_ff + g2 (residual branch in the epilogue)
        _bgemm(N, E, E, [(_ptr(G2[i]), P[i][6], _ptr(dU[i]), None, _ptr(G2[i])) for i in range(n)], E, E,
               epi=3, ldaux=E, transposed=True, dev=dev)
        G1 = torch.empty(n, N, E, **f32)
        _bln_bwd(N, E, [(_ptr(dU[i]), (E, 0, 0), _ptr(A[i]), _ptr(q2), _ptr(P[i][4]), _ptr(m1[i]), _ptr(r1[i]),
                         _ptr(G1[i]), _ptr(ws1[i])) for i in range(n)])
        dO = torch.empty(n, N, E, **f32)
        _bgemm(N, E, E, [(_ptr(G1[i]), P[i][2], _ptr(dO[i]), None, None) for i in range(n)], E, E,
               transposed=True, dev=dev)
        dQ = torch.empty(n, N, E, **f32)
        dKV = [torch.empty(B, kv.shape[1], 2 * E, **f32) for kv in kv2]
        for i in range(n):
            Tk = kv2[i].shape[1]
            ws = Fn._ws(lib.mrg_attention_bwd_workspace_bytes(B, heads, Tq), dev)
            with Fn._probe("attn_bwd", 10.0 * D * B * heads * Fn.visible_pairs(Tq, Tk, causal)):
                rc = lib.mrg_attention_bwd(
                    B, heads, Tq, Tk, D, _ptr(Q[i]), Tq * E, E, _ptr(KV[i]), Tk * 2 * E, 2 * E, _p(KV[i], E),
                    Tk * 2 * E, 2 * E, _ptr(O[i]), Tq * E, E, _ptr(lse[i]), _ptr(qpads[i]), _ptr(kpads[i]), int(causal),
                    scale, _ptr(dO[i]), Tq * E, E, _ptr(dQ[i]), Tq * E, E, _ptr(dKV[i]), Tk * 2 * E, 2 * E,
                    _p(dKV[i], E), Tk * 2 * E, 2 * E, _ptr(ws), _stream())
            _lib.check(rc, "attention bwd (integrator)")
        dq = None
        if ctx.q_need:   # dq = sum_i (dQ_i W_q_i + g1_i): two epilogue-3 GEMMs into one buffer
            dq = torch.empty(B, Tq, E, **f32)
            for i in range(n):
                _dx_gemm(N, E, E, _ptr(dQ[i]), E, P[i][0][:E], _ptr(dq), E, epi=3, aux=_ptr(G1[i]), ldaux=E,
                         beta=0.0 if i == 0 else 1.0, device=dev)
        dkv = []
        for i in range(n):
            if not ctx.kv_need[i]:
                dkv.append(None)
                continue
            Tk = kv2[i].shape[1]
            sink = ctx.sinks[i]
            if sink is None:   # no draining producer: this consumer's own part, summed by autograd
                g = torch.empty(B, Tk, E, **f32)
                _dx_gemm(B * Tk, E, 2 * E, _ptr(dKV[i]), 2 * E, P[i][0][E:], _ptr(g), E, device=dev)
                dkv.append(g)
                continue
            first = sink.begin_write()
            if first:
                sink.buf = torch.empty(B, Tk, E, **f32)
            _dx_gemm(B * Tk, E, 2 * E, _ptr(dKV[i]), 2 * E, P[i][0][E:], _ptr(sink.buf), E,
                     beta=0.0 if first else 1.0, device=dev)
            sink.written += 1
            dkv.append(None)   # the producer drains the sum (KVSink)
        _IntegrateFn._param_grads(lib, ctx, dev, do2, cat, G2, U, G1, O, dQ, q2, dKV, kv2, ws1, ws2, N, E, n)
        return (None, dq, *dkv) + (None,) * (len(ctx.needs_input_grad) - 2 - n)

    @staticmethod
    def _param_grads(lib, ctx, dev, do2, cat, G2, U, G1, O, dQ, q2, dKV, kv2, ws1, ws2, N, E, n):
        """Every parameter gradient of the integrator as ONE fork onto the weight-gradient stream."""
        P, cat_w, cat_b = ctx.params
        gcw, gcb = _gbuf(cat_w), _gbuf(cat_b)
        per = []
        for i in range(n):
            gw, gb = _gbuf(P[i][0]), _gbuf(P[i][1])
            per.append(dict(in_w=gw, in_b=gb, out_w=_gbuf(P[i][2]), out_b=_gbuf(P[i][3]), g1=_gbuf(P[i][4]),
                            b1=_gbuf(P[i][5]), ff_w=_gbuf(P[i][6]), ff_b=_gbuf(P[i][7]), g2=_gbuf(P[i][8]),
                            b2=_gbuf(P[i][9])))
        keep = (do2, cat, G2, U, G1, O, dQ, q2, ws1, ws2, *dKV, *kv2)

        def wg(dY, ldy, X, ldx, rows, Nout, Nin, gw, gb=None):
            if gw is None:
                if gb is not None:
                    Fn.colsum(rows, Nout, dY, ldy, _ptr(gb), device=dev)
                return
            gemm(Nout, Nin, rows, dY, 1, ldy, X, 0, ldx, _ptr(gw), Nin, beta=1.0,
                 splits=Fn.wgrad_splits(Nout, Nin, rows), device=dev, asum_out=_ptr(gb))

        def reduce(ws, gg, gb):
            if gg is None and gb is None:
                return
            scratch = Fn._ws(2 * E * 4, dev).view(2, E) if (gg is None or gb is None) else None
            _lib.check(lib.mrg_residual_layernorm_param_reduce(
                N, E, _ptr(ws), _ptr(gg if gg is not None else scratch[0]), _ptr(gb if gb is not None else scratch[1]),
                1, _stream()), "layernorm param reduce")

        def issue():
            wg(_ptr(do2), E, _ptr(cat), n * E, N, E, n * E, gcw, gcb)
            for i, g in enumerate(per):
                wg(_ptr(G2[i]), E, _ptr(U[i]), E, N, E, E, g["ff_w"], g["ff_b"])
                reduce(ws2[i], g["g2"], g["b2"])
                reduce(ws1[i], g["g1"], g["b1"])
                wg(_ptr(G1[i]), E, _ptr(O[i]), E, N, E, E, g["out_w"], g["out_b"])
                wg(_ptr(dQ[i]), E, _ptr(q2), E, N, E, E, None if g["in_w"] is None else g["in_w"][:E],
                   None if g["in_b"] is None else g["in_b"][:E])
                Nk = kv2[i].shape[0] * kv2[i].shape[1]
                wg(_ptr(dKV[i]), 2 * E, _ptr(kv2[i]), E, Nk, 2 * E, E, None if g["in_w"] is None else g["in_w"][E:],
                   None if g["in_b"] is None else g["in_b"][E:])
        _on_side(dev, N, keep, issue, writes=(gcw, gcb, *[t for g in per for t in g.values()]))


def _bln_fwd(rows, E, eps, items):
    col = list(zip(*items))
    rc = _lib.load().mrg_residual_layernorm_fwd_batched(
        len(items), rows, E, _arr(VP, col[0]), _arr(VP, col[1]), _arr(VP, col[2]), _arr(VP, col[3]), eps,
        _arr(VP, col[4]), _arr(CL, [m[0] for m in col[5]]), _arr(CL, [m[1] for m in col[5]]),
        _arr(CI, [m[2] for m in col[5]]), _arr(VP, col[6]), _arr(VP, col[7]), _stream())
    _lib.check(rc, "batched layernorm fwd (integrator)")


def _bln_bwd(rows, E, items):
    col = list(zip(*items))
    rc = _lib.load().mrg_residual_layernorm_bwd_batched(
        len(items), rows, E, _arr(VP, col[0]), _arr(CL, [m[0] for m in col[1]]), _arr(CL, [m[1] for m in col[1]]),
        _arr(CI, [m[2] for m in col[1]]), _arr(VP, col[2]), _arr(VP, col[3]), _arr(VP, col[4]), _arr(VP, col[5]),
        _arr(VP, col[6]), _arr(VP, col[7]), _arr(VP, col[8]), _stream())
    _lib.check(rc, "batched layernorm bwd (integrator)")


def integrate(q: torch.Tensor, kvs: Sequence[torch.Tensor], qpads, kpads, params: Sequence[Sequence[torch.Tensor]],
              cat_w, cat_b, heads: int, causal: bool, eps: float) -> torch.Tensor:
    """cat_linear(cat_i LN2_i(FF_i(LN1_i(MHA_i(q, kv_i) + q)) + ...)): see the module docstring.
    params[i] = (in_proj_weight, in_proj_bias, out_proj.weight, out_proj.bias, ln1.weight, ln1.bias,
    ff.weight, ff.bias, ln2.weight, ln2.bias)."""
    n = len(kvs)
    flat = [q, *kvs, *qpads, *kpads]
    for p in params:
        flat += list(p)
    flat += [cat_w, cat_b]
    return _IntegrateFn.apply((n, int(heads), bool(causal), float(eps)), *flat)
