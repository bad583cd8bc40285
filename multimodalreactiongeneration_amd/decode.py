"""Fused scheduled-sampling decode of LSTMwithSample (BASELINE configs[2]).

Reference: LSTMwithSample.prediction / head_motion_generation / generate_one_step
(mr_gen/model/lstm_with_sampling/lstm_with_sample.py:339-433): a Python loop of T single-frame
forwards.  Only the chain  feat(t) -> layered LSTMs (zero state, Q2) -> FFN -> y(t) -> ms_in(t+1)
is sequential across frames (ms_in(0) = ms[0], ms_in(t+1) = mask[t] ? y(t) : ms[t], Q10), so:

* the sampler, whose state the reference carries from frame to frame, runs ONCE over the whole
  audio sequence [lead audio | frames] (the caller, LSTMwithSample._fused_prediction): frame t's
  output is the same LSTM state the reference reaches after its warm-up and t frames;
* the feature projection of [sampler | partner motion] for every frame is one GEMM (P); per frame
  only the ms_in columns are added (W_f = [W_a | W_mp | W_ms], one Linear in the reference);
* the frame loop runs L + 1 launches forward and 2L backward (decode.hip): per layer the gates +
  zero-state cell with the layer input built in the prologue (layer 1: the previous frame's FFN
  output Linear, the sampling select and the ms columns of the feature projection; layer l > 1:
  the previous LayerNorm), then the last LayerNorm + the FFN's first Linear; in backward per layer
  the [FFN /] LayerNorm / cell backward kernel and the dX kernel;
* every weight gradient (W_ih, biases, LayerNorms, FFN, feature projection) and the sampler-output
  gradient is one GEMM / reduction over all T*B rows after the loop.

Same numbers as the reference up to fp32 reassociation (tests/test_gpu_models.py pins it to the
reference's golden and to the oracle at benchmark width).
"""
from __future__ import annotations


import ctypes
import os

import torch
from torch.autograd import Function

from . import _lib
from .functional import _err_flag, _gbuf, _keeps_precision, _probe, _ptr, _resln_bwd, _stream, _wgrad, _side, gemm

F32 = torch.float32
# the forward frame loop as ONE persistent launch (ssd_loop.hip) when H = 256, HB = 64, FO <= 16,
# nl <= 4 and its grid fits; MRG_SSD_LOOP=0 keeps the L + 1 launches per frame
_LOOP = [os.environ.get("MRG_SSD_LOOP", "1") == "1"]
# the backward frame loop likewise (ssd_loop.hip ssd_loop_bwd_kernel; nl >= 2); MRG_SSD_LOOP_BWD=0
# keeps the 2L launches per frame
_LOOP_BWD = [os.environ.get("MRG_SSD_LOOP_BWD", "1") == "1"]


class _SSDecodeFn(Function):
    """y [B, T, FO] of the scheduled-sampling decode; see the module docstring.

    tensors: a_s [B, T, SA] sampler outputs of the frames, mp [B, T, FMp] partner motion,
    ms [B, T, FM] teacher self motion, mask [T] (device uint8), w_f [H, SA+FMp+FM], b_f [H],
    then per layer (w_ih [4H, H], w_hh, b_ih, b_hh, ln_w, ln_b), then w1 [HB, H], b1, w2 [FO, HB], b2.
    """

    @staticmethod
    @_keeps_precision
    def forward(ctx, spec, a_s, mp, ms, mask, w_f, b_f, *params):
        nl, eps = spec
        _lib.require_device(a_s)
        lib = _lib.load()
        dev = a_s.device
        B, T, SA = a_s.shape
        FMp, FM = mp.shape[2], ms.shape[2]
        H, F = w_f.shape
        if F != SA + FMp + FM:
            raise RuntimeError(f"feature_projection [{H}, {F}] vs inputs {SA} + {FMp} + {FM}")
        layers = [params[6 * i:6 * i + 6] for i in range(nl)]
        w1, b1, w2, b2 = params[6 * nl:6 * nl + 4]
        HB, FO = w1.shape[0], w2.shape[0]
        if FO != FM:
            raise RuntimeError("the prediction feeds back as motion_self: output size must equal its features")
        # X_f [T, B, F] = [sampler | partner | ms_in], time-major so a frame is one slab; the ms_in
        # columns are written by the layer-1 kernel of each frame (the sampling select)
        xf = torch.empty(T, B, F, device=dev, dtype=F32)
        xf[:, :, :SA].copy_(a_s.transpose(0, 1))
        xf[:, :, SA:SA + FMp].copy_(mp.transpose(0, 1))
        P = torch.empty(T, B, H, device=dev, dtype=F32)
        gemm(T * B, H, SA + FMp, _ptr(xf), 0, F, _ptr(w_f), 1, F, _ptr(P), H, bias=_ptr(b_f), device=dev)
        wms_t = w_f[:, SA + FMp:].t().contiguous()  # W_ms^T [FM, H]
        X = [torch.empty(T, B, H, device=dev, dtype=F32) for _ in range(nl)]
        G = [torch.empty(T, B, 4 * H, device=dev, dtype=F32) for _ in range(nl)]
        C = [torch.empty(T, B, H, device=dev, dtype=F32) for _ in range(nl)]
        Hs = [torch.empty(T, B, H, device=dev, dtype=F32) for _ in range(nl)]
        stats = [torch.empty(2, T, B, device=dev, dtype=F32) for _ in range(nl)]
        U = torch.empty(T, B, H, device=dev, dtype=F32)
        Z = torch.empty(T, B, HB, device=dev, dtype=F32)
        y = torch.empty(B, T, FO, device=dev, dtype=F32)
        msc = ms.contiguous()
        slab, gslab, zslab = B * H, B * 4 * H, B * HB
        lw, lb = layers[-1][4], layers[-1][5]
        if _LOOP[0] and H == 256 and HB == 64 and FO <= 16 and nl <= 4 and lib.mrg_ssd_loop_fits(B, 0) == 1:
            # the loop stores the gates, c, h and X_0; the LayerNorm outputs (X_i, U) and statistics,
            # Z, y and X_f's ms columns are formed after it (below): stored inside the loop they fell on
            # one member, which then ran ~1.2 us behind its group at every stage (ssd_loop.hip)
            lp = []
            for i, (w_ih, _w_hh, b_ih, b_hh, g_, b_) in enumerate(layers):
                lp += [w_ih, b_ih, b_hh, g_, b_, X[i] if i == 0 else None, G[i], C[i], Hs[i]]
            lpa = (ctypes.c_void_p * len(lp))(*[_ptr(q) for q in lp])
            ring = torch.zeros(max(1, lib.mrg_ssd_loop_ring_bytes(B, nl) // 8), dtype=torch.int64, device=dev)
            # algorithmic FLOPs (bench's "ssd" family): gates 8H^2 per row and layer, FFN, the ms columns
            flop = 2.0 * T * B * (4 * H * H * nl + H * HB + HB * FO + FO * H)
            with _probe("ssd", flop):
                _lib.check(lib.mrg_ssd_loop_fwd(
                    B, T, H, HB, FO, nl, eps, lpa, len(lp), _ptr(P), _ptr(wms_t), _ptr(w1), _ptr(b1), _ptr(w2),
                    _ptr(b2), _ptr(msc), msc.stride(0), msc.stride(1), _ptr(mask), _ptr(ring),
                    _ptr(_err_flag(dev)), _stream()), "ssd loop fwd")
            rows = T * B
            for i, (_w_ih, _w_hh, _b_ih, _b_hh, g_, b_) in enumerate(layers):
                # X_{i+1} (U after the last layer) = LN(h_i + X_i) with its statistics
                out = X[i + 1] if i + 1 < nl else U
                _lib.check(lib.mrg_residual_layernorm_fwd(rows, H, _ptr(Hs[i]), _ptr(X[i]), _ptr(g_), _ptr(b_), eps,
                                                          _ptr(out), _ptr(stats[i][0]), _ptr(stats[i][1]),
                                                          _stream()), "ssd layernorm")
            gemm(rows, HB, H, _ptr(U), 0, H, _ptr(w1), 1, H, _ptr(Z), HB, bias=_ptr(b1), epi=1, device=dev)
            y_tb = torch.empty(T, B, FO, device=dev, dtype=F32)
            gemm(rows, FO, HB, _ptr(Z), 0, HB, _ptr(w2), 1, HB, _ptr(y_tb), FO, bias=_ptr(b2), device=dev)
            y.copy_(y_tb.transpose(0, 1))
            # X_f's ms columns: ms_in(0) = ms[:, 0], ms_in(t + 1) = mask[t] ? y(t) : ms[:, t]
            xms = xf[:, :, SA + FMp:]
            xms[0].copy_(msc[:, 0])
            if T > 1:
                xms[1:].copy_(torch.where(mask[:-1].bool()[:, None, None], y_tb[:-1], msc[:, :-1].transpose(0, 1)))
            T_launch = 0
        else:
            T_launch = T
        for t in range(T_launch):
            for i, (w_ih, _w_hh, b_ih, b_hh, _g, _b) in enumerate(layers):
                cell = (_ptr(w_ih), _ptr(b_ih), _ptr(b_hh), _ptr(G[i], t * gslab), _ptr(C[i], t * slab),
                        _ptr(Hs[i], t * slab), _stream())
                if i == 0:
                    # X = P(t) + ms_in(t) W_ms^T, ms_in(t) = mask[t-1] ? y(t-1) : ms[t-1] (y(t-1) from z(t-1))
                    _lib.check(lib.mrg_ssd_feat_gate_cell_fwd(
                        B, H, HB, FO, F, t, _ptr(P, t * slab), _ptr(Z, (t - 1) * zslab) if t else None, _ptr(w2),
                        _ptr(b2), _ptr(mask), _ptr(msc), msc.stride(0), msc.stride(1), _ptr(wms_t),
                        _ptr(y, (t - 1) * FO) if t else None, T * FO, _ptr(xf, t * B * F + SA + FMp),
                        _ptr(X[0], t * slab), *cell), "ssd feat/gate/cell fwd")
                else:
                    pw, pb = layers[i - 1][4], layers[i - 1][5]
                    _lib.check(lib.mrg_ssd_gate_cell_fwd(
                        B, H, 1, None, _ptr(Hs[i - 1], t * slab), _ptr(X[i - 1], t * slab), _ptr(pw), _ptr(pb), eps,
                        _ptr(X[i], t * slab), _ptr(stats[i - 1][0], t * B), _ptr(stats[i - 1][1], t * B), *cell),
                        "ssd gate/cell fwd")
            _lib.check(lib.mrg_ssd_ffn_z_fwd(
                B, H, HB, _ptr(Hs[-1], t * slab), _ptr(X[-1], t * slab), _ptr(lw), _ptr(lb), eps, _ptr(U, t * slab),
                _ptr(stats[-1][0], t * B), _ptr(stats[-1][1], t * B), _ptr(w1), _ptr(b1), _ptr(Z, t * zslab),
                _stream()), "ssd ffn z fwd")
        if T_launch:
            _lib.check(lib.mrg_ssd_y_fwd(B, HB, FO, _ptr(Z, (T - 1) * zslab), _ptr(w2), _ptr(b2),
                                         _ptr(y, (T - 1) * FO), T * FO, _stream()), "ssd y fwd")
        ctx.spec = (nl, eps, B, T, SA, FMp, FM, H, F, HB, FO)
        ctx.save_for_backward(mask, w_f, b_f, *params, xf, U, Z, wms_t, *X, *G, *C, *Hs, *stats)
        ctx.set_materialize_grads(False)
        return y

    @staticmethod
    @_keeps_precision
    def backward(ctx, dy):
        nl, eps, B, T, SA, FMp, FM, H, F, HB, FO = ctx.spec
        sv = ctx.saved_tensors
        mask, w_f, b_f = sv[:3]
        params = sv[3:3 + 6 * nl + 4]
        layers = [params[6 * i:6 * i + 6] for i in range(nl)]
        w1, b1, w2, b2 = params[6 * nl:6 * nl + 4]
        rest = sv[3 + 6 * nl + 4:]
        xf, U, Z, wms_t = rest[:4]
        X, G, C, Hs, stats = (list(rest[4 + k * nl:4 + (k + 1) * nl]) for k in range(5))
        dev = xf.device
        lib = _lib.load()
        if dy is None:
            return (None,) * (7 + len(params))
        dy = dy.contiguous()
        rows = T * B
        dyt = torch.empty(T, B, FO, device=dev, dtype=F32)
        dz = torch.empty(T, B, HB, device=dev, dtype=F32)
        duL = torch.empty(T, B, H, device=dev, dtype=F32)
        gs = [torch.empty(T, B, H, device=dev, dtype=F32) for _ in range(nl)]
        dG = [torch.empty(T, B, 4 * H, device=dev, dtype=F32) for _ in range(nl)]
        dX = [torch.empty(T, B, H, device=dev, dtype=F32) for _ in range(nl)]  # dX[0] = dfeat
        slab, gslab, zslab = B * H, B * 4 * H, B * HB
        ext = nl >= 2
        loop = (ext and _LOOP_BWD[0] and H == 256 and HB == 64 and FO <= 16 and nl <= 4
                and lib.mrg_ssd_loop_bwd_fits(B, 0) == 1)
        # W_ih^T copies: the per-frame dX = dG W_ih reads both operands k-contiguous (float4)
        w_t = [None if (loop or (ext and i == 0)) else lay[0].t().contiguous() for i, lay in enumerate(layers)]
        # v = [W1 gamma | W1 beta] [HB, 2] of the last LayerNorm: its row sums through W1 (decode.hip)
        lw, lb = layers[-1][4], layers[-1][5]
        gb = torch.stack([lw.detach(), lb.detach()])
        v = torch.empty(HB, 2, device=dev, dtype=F32)
        gemm(HB, 2, H, _ptr(w1), 0, H, _ptr(gb), 1, H, _ptr(v), 2, device=dev)
        # the bottom layer forms each frame's y gradient through the select itself (dyx = dfeat W_ms
        # with vt = W_ms^T W_ih0), so its dX (dfeat) is one GEMM over all frames after the loop
        if ext:
            vt = torch.empty(FM, 4 * H, device=dev, dtype=F32)
            gemm(FM, 4 * H, H, _ptr(wms_t), 0, H, _ptr(layers[0][0]), 1, H, _ptr(vt), 4 * H, device=dev)
            dyx = None if loop else torch.empty(T, B, FM, device=dev, dtype=F32)
        if loop:
            lp = []
            for i, lay in enumerate(layers):
                lp += [lay[0] if i else None, lay[4], lay[5], X[i], G[i], C[i], Hs[i], stats[i][0], stats[i][1],
                       gs[i], dG[i], dX[i] if i else None]
            lpa = (ctypes.c_void_p * len(lp))(*[_ptr(q) for q in lp])
            ring = torch.zeros(max(1, lib.mrg_ssd_loop_bwd_ring_bytes(B) // 8), dtype=torch.int64, device=dev)
            # dX = dG W_ih over the 3 nonzero gate blocks per lower layer, FFN backward, the dyx products
            flop = 2.0 * T * B * (3 * H * H * (nl - 1) + HB * (H + FO) + FO * 4 * H)
            with _probe("ssd", flop):
                _lib.check(lib.mrg_ssd_loop_bwd(
                    B, T, H, HB, FO, nl, lpa, len(lp), _ptr(dy), _ptr(mask), _ptr(w1), _ptr(w2), _ptr(b1), _ptr(v),
                    _ptr(Z), _ptr(vt), _ptr(wms_t), _ptr(duL), _ptr(ring), _ptr(_err_flag(dev)), _stream()),
                    "ssd loop bwd")
        for t in (range(T - 1, -1, -1) if not loop else ()):
            for i in range(nl - 1, -1, -1):
                cell = (_ptr(gs[i], t * slab), _ptr(G[i], t * gslab), _ptr(C[i], t * slab), _ptr(dG[i], t * gslab))
                if i == nl - 1:
                    nxt = t + 1 < T
                    _lib.check(lib.mrg_ssd_ffn_bwd(
                        B, H, HB, FO, t, _ptr(dy, t * FO), T * FO,
                        _ptr(dX[0], (t + 1) * slab) if (nxt and not ext) else None,
                        _ptr(dyx, (t + 1) * B * FM) if (nxt and ext) else None,
                        _ptr(wms_t), _ptr(mask), _ptr(w1), _ptr(w2), _ptr(b1), _ptr(v), _ptr(Z, t * zslab),
                        _ptr(dyt, t * B * FO), _ptr(dz, t * zslab), _ptr(duL, t * slab), _ptr(Hs[i], t * slab),
                        _ptr(X[i], t * slab), _ptr(lw), _ptr(stats[i][0], t * B), _ptr(stats[i][1], t * B), *cell,
                        _stream()), "ssd ffn bwd")
                else:
                    bottom = ext and i == 0
                    _lib.check(lib.mrg_ssd_ln_cell_bwd(
                        B, H, _ptr(dX[i + 1], t * slab), _ptr(Hs[i], t * slab), _ptr(X[i], t * slab),
                        _ptr(layers[i][4]), _ptr(stats[i][0], t * B), _ptr(stats[i][1], t * B), *cell, FM,
                        _ptr(vt) if bottom else None, _ptr(wms_t) if bottom else None,
                        _ptr(dyx, t * B * FM) if bottom else None, _stream()), "ssd ln/cell bwd")
                    if bottom:
                        continue
                # dX = dG W_ih + g (g: the LayerNorm's residual branch)
                _lib.check(lib.mrg_ssd_dx(B, H, _ptr(dG[i], t * gslab), _ptr(w_t[i]), _ptr(gs[i], t * slab),
                                          _ptr(dX[i], t * slab), _stream()), "ssd dx")
        if ext:  # every frame's dfeat = dG0 W_ih0 + g0 in one GEMM
            gemm(T * B, H, 4 * H, _ptr(dG[0]), 0, 4 * H, _ptr(layers[0][0]), 0, H, _ptr(dX[0]), H, epi=3,
                 aux=_ptr(gs[0]), ldaux=H, device=dev)
        if loop:
            # dy_total(t) = dy(t) + mask[t] dfeat(t+1) W_ms and dz = relu'(z) (dy_total W2), formed here
            # from dX_0 (the loop keeps them in registers: stored by one member they held it back)
            dyx = torch.empty(T, B, FM, device=dev, dtype=F32)
            gemm(rows, FM, H, _ptr(dX[0]), 0, H, _ptr(wms_t), 1, H, _ptr(dyx), FM, device=dev)
            dyt.copy_(dy.transpose(0, 1))
            if T > 1:
                dyt[:-1].add_(dyx[1:] * mask[:-1].to(F32)[:, None, None])
            gemm(rows, HB, FO, _ptr(dyt), 0, FO, _ptr(w2), 0, HB, _ptr(dz), HB, device=dev)
            dz.mul_(Z > 0)
        # weight gradients over all T * B rows
        for i, (w_ih, w_hh, b_ih, b_hh, lw, lb) in enumerate(layers):
            _wgrad(_ptr(dG[i]), 4 * H, _ptr(X[i]), H, rows, 4 * H, H, _gbuf(w_ih), dev, gb=_gbuf(b_ih),
                   gb2=_gbuf(b_hh), keep=(dG[i], X[i]))
            _gbuf(w_hh)  # zero state: its gradient is exactly zero, as nn.LSTM's is
            du = duL if i == nl - 1 else dX[i + 1]
            _resln_bwd(du.view(rows, H), Hs[i].view(rows, H), X[i].view(rows, H), lw, lb,
                       stats[i][0].reshape(rows), stats[i][1].reshape(rows))
        _wgrad(_ptr(dyt), FO, _ptr(Z), HB, rows, FO, HB, _gbuf(w2), dev, gb=_gbuf(b2), keep=(dyt, Z))
        _wgrad(_ptr(dz), HB, _ptr(U), H, rows, HB, H, _gbuf(w1), dev, gb=_gbuf(b1), keep=(dz, U))
        _wgrad(_ptr(dX[0]), H, _ptr(xf), F, rows, H, F, _gbuf(w_f), dev, gb=_gbuf(b_f), keep=(dX[0], xf))
        da = None
        if ctx.needs_input_grad[1]:
            da_t = torch.empty(T, B, SA, device=dev, dtype=F32)
            gemm(rows, SA, H, _ptr(dX[0]), 0, H, _ptr(w_f), 0, F, _ptr(da_t), SA, device=dev)
            da = da_t.transpose(0, 1)
        return (None, da, None, None, None, None, None) + (None,) * len(params)


def scheduled_sampling_decode(a_s, mp, ms, mask, w_f, b_f, layers, ffn, eps=1e-5):
    """y [B, T, FO] of head_motion_generation given the sampler outputs a_s [B, T, SA].

    layers: [(w_ih, w_hh, b_ih, b_hh, ln_weight, ln_bias)] of the layered LSTM (zero state each
    frame); ffn: (w1, b1, w2, b2) of Linear -> ReLU -> Linear; mask: [T] bool (device or host)."""
    dev = a_s.device
    m = mask.to(device=dev, dtype=torch.uint8)
    flat = [p for lay in layers for p in lay] + list(ffn)
    return _SSDecodeFn.apply((len(layers), float(eps)), a_s, mp.to(dev), ms.to(dev), m, w_f, b_f, *flat)
