"""Layer-wavefront schedule of the first metaformer block's LSTM encoder stacks.

Reference: ``MultiModalMetaformerBlock`` block 0 embeds every modality
(multi_modal_metaformer.py:102-125) with an ``LSTMMixerLayerd`` per modality: the main
modality through 1 ``LSTMMixerBlock``, audio and partner through ``encoder_num_layer`` = 5
(lstmformer.py:165-170, mixer_block.py:833-843).  Each block is

    y = LSTM(x)                       (mixer_block.py:479-507, zero initial state)
    u = LN1(y + x)                    (ResidualConnection, residual_connection.py:20-37)
    v = LN2(u W_ff^T + b_ff + u)      (FeedForward, nonlinearity none: one Linear, :37-87)

and the modality's features enter through ``feature_embedding`` (Linear F -> H,
multi_modal_metaformer.py:433-435,486-490).

Every op above is causal in time, so layer l's time chunk c needs only layer l-1's chunk c
and its own chunk c-1 (carried h, c).  The stacks therefore run as a wavefront over
(layer, time chunk): diagonal d holds every (modality, layer l, chunk d - l), and all of
them are ONE persistent recurrence launch (lstm.hip, up to 12 problems, the (h, c) state
of chunk c-1 read in place as chunk c's h0 / c0).  Fifteen layers x 300 steps of latency-
bound recurrence become (chunks + layers - 1) launches of one chunk each: the hand-off
latencies of the layers in flight overlap instead of adding up.  The backward runs the
same diagonals in reverse with (dh, dc) carried from chunk c+1 to c.

Layout: everything inside the stack is time-major ([T, B, .] rows t*B + b), so a time
chunk is a contiguous block of rows for the chunked GEMMs and LayerNorms; the embedding
GEMM reads the batch-major features through a row map, and the last LayerNorm writes the
batch-major output the integrators consume (mrg_residual_layernorm_fwd_map).  The
arithmetic per element is the per-layer path's (same kernels, same fp32 math); only the
launch granularity changes.
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence

import torch
from torch.autograd import Function

from . import _lib
from . import functional as Fn
from .functional import _ptr, _stream, gemm, _dx_gemm, _wt_note, _gbuf, _on_side

# time steps per chunk (the diagonal width); MRG_STACK_CHUNK overrides.  100 since the deferred weight
# gradients run beside the backward recurrences (longer recurrences leave them more room): A/B on one
# box 50 / 60 / 75 / 100 / 150 / 300 -> 21.80 / 21.68 / 21.53 / 21.29 / 21.55 / 23.05 ms/step (r03)
# Weight gradients are issued per layer once its chunk 0 is done.  Per (layer, chunk) as each chunk's
# backward completed (three times as many, smaller products, starting diagonals earlier) measured
# 22.47 vs 21.15 ms/step (r04) and 22.14 vs 20.38 (r05, with the recurrence stream): removed.
# one side-stream fork per weight-gradient product instead of one per layer (a capture regression case:
# tests/test_gpu_capture.py)
SPLIT_FORKS = os.environ.get("MRG_STACK_SPLIT_FORKS", "0") == "1"
CHUNK = int(os.environ.get("MRG_STACK_CHUNK", "100"))
# problems per recurrence launch (lstm.hip: <= 12); 0 = as many as the MFMA form's grid keeps resident
# (8 workgroups of 16 rows per problem, one per CU: 8 problems at B = 64 on 256 CUs; a wider launch
# falls back to the VALU form at batch tiles of 16, measured 3x slower per step)
MAXP = int(os.environ.get("MRG_STACK_MAXP", "0"))


def _maxp(B, dev):
    if MAXP > 0:
        return MAXP
    per = 8 * ((B + 15) // 16)
    return max(1, min(12, _lib.cu_count(dev.index or 0) // per))


def _split(v, cap):
    """v into ceil(len / cap) launches of balanced size."""
    k = (len(v) + cap - 1) // cap
    q = (len(v) + k - 1) // k
    return [v[s:s + q] for s in range(0, len(v), q)]
VP, CL, CI = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
_PER_LAYER = 10   # w_ih, w_hh, b_ih, b_hh, ln1 gamma, ln1 beta, w_ff, b_ff, ln2 gamma, ln2 beta


def _chunks(T, tc):
    return [(t0, min(T, t0 + tc)) for t0 in range(0, T, tc)]


def _p(t, off=0):
    return VP(t.data_ptr() + 4 * off)


class _Chain:
    """One modality: features [B, T, F] -> embedding -> L layers (tensors are time-major)."""

    def __init__(self, feat, emb_w, emb_b, layers):
        self.feat, self.emb_w, self.emb_b, self.layers = feat, emb_w, emb_b, layers
        self.B, self.T, self.F = feat.shape
        self.H = emb_w.shape[0]
        self.L = len(layers)


class _RingPool:
    """Hand-off rings of every recurrence launch of one pass, zeroed by ONE fill up front (each launch
    needs its rings zero at its start; a fill per launch was one more kernel on the critical path)."""

    def __init__(self, n, elems, dev):
        self.buf = Fn.zeros(max(1, n), elems, dtype=torch.int64, device=dev)
        self.next = 0

    def take(self, n):
        if self.next + n > self.buf.shape[0]:
            raise RuntimeError("encoder stack: ring pool exhausted")
        out = self.buf[self.next:self.next + n]
        self.next += n
        return out


def _launch_fwd(lib, items, B, Tc, H, dev, pool=None):
    """One persistent forward launch over `items` = [(chain, layer state dict, t0)]."""
    n = len(items)
    xb = pool.take(n) if pool is not None else \
        Fn.zeros(n, lib.mrg_lstm_fwd_xbuf_bytes(B, H) // 8, dtype=torch.int64, device=dev)
    gx, gbs, gts, whh, bhh, h0, c0, y, ybs, yts, gates, cs, lay, rev = ([] for _ in range(14))
    for ch, st, t0 in items:
        r0 = t0 * B
        gx.append(_p(st["gx"], r0 * 4 * H)); gbs.append(4 * H); gts.append(B * 4 * H)
        whh.append(_p(st["w_hh"])); bhh.append(_p(st["b_hh"]))
        h0.append(None if t0 == 0 else _p(st["y"], (r0 - B) * H))
        c0.append(None if t0 == 0 else _p(st["cs"], (r0 - B) * H))
        y.append(_p(st["y"], r0 * H)); ybs.append(H); yts.append(B * H)
        gates.append(_p(st["gates"], r0 * 4 * H)); cs.append(_p(st["cs"], r0 * H))
        lay += [4 * H, B * 4 * H, H, B * H, H, H, 0, 0]
        rev.append(0)
    A = lambda ct, v: (ct * n)(*v)  # noqa: E731
    with Fn._probe("lstm_fwd", 8.0 * H * H * B * Tc * n):
        rc = lib.mrg_lstm_fwd(n, B, Tc, H, A(VP, gx), A(CL, gbs), A(CL, gts), A(VP, whh), A(VP, bhh),
                              A(VP, h0), A(VP, c0), A(VP, y), A(CL, ybs), A(CL, yts), A(VP, gates), A(VP, cs),
                              None, None, A(CI, rev), A(VP, [_p(xb[i]) for i in range(n)]),
                              (CL * (8 * n))(*lay), _ptr(Fn._err_flag(dev)), _lib.cu_count(dev.index or 0), 0,
                              _stream())
    _lib.check(rc, "lstm fwd (encoder stack)")


def _launch_bwd(lib, items, B, Tc, H, dev, pool=None):
    """One persistent backward launch over `items` = [(chain, state, grads, t0, dhT, dcT, dh0, dc0)]."""
    n = len(items)
    xb = pool.take(n) if pool is not None else \
        Fn.zeros(n, lib.mrg_lstm_bwd_xbuf_bytes(B, H) // 8, dtype=torch.int64, device=dev)
    whh, gates, cs, c0, dy, dybs, dyts, dhT, dcT, dG, dh0, dc0, lay, rev = ([] for _ in range(14))
    for ch, st, gr, t0, dh_in, dc_in, dh_out, dc_out in items:
        r0 = t0 * B
        whh.append(_p(st["w_hh"])); gates.append(_p(st["gates"], r0 * 4 * H)); cs.append(_p(st["cs"], r0 * H))
        c0.append(None if t0 == 0 else _p(st["cs"], (r0 - B) * H))
        dy.append(_p(gr["g1"], r0 * H)); dybs.append(H); dyts.append(B * H)
        dhT.append(None if dh_in is None else _p(dh_in)); dcT.append(None if dc_in is None else _p(dc_in))
        dG.append(_p(gr["dG"], r0 * 4 * H))
        dh0.append(None if dh_out is None else _p(dh_out)); dc0.append(None if dc_out is None else _p(dc_out))
        lay += [4 * H, B * 4 * H, H, B * H, H, 4 * H, B * 4 * H, 0]
        rev.append(0)
    A = lambda ct, v: (ct * n)(*v)  # noqa: E731
    # deferred weight gradients (functional._DEFER) run beside this recurrence, as in _LSTMFn.backward
    cap, mark = Fn.fork_beside_recurrence(dev)
    lib.mrg_lstm_set_blocks_per_cu(cap)
    with Fn._probe("lstm_bwd", 8.0 * H * H * B * Tc * n):
        rc = lib.mrg_lstm_bwd(n, B, Tc, H, A(VP, whh), A(VP, gates), A(VP, cs), A(VP, c0), A(VP, dy),
                              A(CL, dybs), A(CL, dyts), A(VP, dhT), A(VP, dcT), A(VP, dG), A(VP, dh0), A(VP, dc0),
                              A(CI, rev), A(VP, [_p(xb[i]) for i in range(n)]), (CL * (8 * n))(*lay),
                              _ptr(Fn._err_flag(dev)), _lib.cu_count(dev.index or 0), 0, _stream())
    _lib.check(rc, "lstm bwd (encoder stack)")
    Fn.flush_beside_recurrence(dev, mark)


_BMAX = 16   # problems per batched GEMM / LayerNorm launch (mrg_gemm_x6g_batched, mrg_residual_layernorm_*_batched)
VPP = ctypes.POINTER(ctypes.c_void_p)


def _arr(ct, v):
    return (ct * len(v))(*v)


def _bgemm(lib, M, N, K, items, lda, ldc, *, epi=0, ldaux=0, transposed=False, dev=None):
    """Same-shape products C_p = A_p w_p^T + bias_p (+ aux_p) in one launch; items = [(A ptr, w, C ptr,
    bias ptr | None, aux ptr | None)].  transposed: the products are dY w (input gradients), run as
    dY (w^T)^T through the [in][out] copies (functional._wt); per product when a copy is missing."""
    if not items:
        return
    if Fn.planes_batched(M, N, K, items, lda, ldc, epi=epi, ldaux=ldaux, transposed=transposed):
        return
    bs = []
    for a_p, w, c_p, b_p, x_p in items:
        if transposed:
            wt = Fn._wt(w) if M >= Fn._WT_MIN_ROWS else None
            if wt is None:   # no [in][out] copy: the per-product path
                for a_p2, w2, c_p2, b_p2, x_p2 in items:
                    _dx_gemm(M, N, K, a_p2, lda, w2, c_p2, ldc, bias=b_p2, epi=epi, aux=x_p2, ldaux=ldaux, device=dev)
                return
            bs.append(_ptr(wt))
        else:
            bs.append(_ptr(w))
    n = len(items)
    with Fn._probe("gemm", 2.0 * M * N * K * n):
        rc = lib.mrg_gemm_x6g_batched(
            n, M, N, K, 1.0, _arr(VP, [it[0] for it in items]), lda, _arr(VP, bs), K, 0.0,
            _arr(VP, [it[2] for it in items]), ldc,
            None if all(it[3] is None for it in items) else _arr(VP, [it[3] for it in items]), epi,
            None if all(it[4] is None for it in items) else _arr(VP, [it[4] for it in items]), ldaux,
            1 if Fn._ARITH[0] == "bf16" else 0, _stream())
    _lib.check(rc, "batched gemm (encoder stack)")


def _bln_fwd(lib, rows, H, eps, items):
    """items = [(a, b, gamma, beta, y, (lo, hi, div), mean, rstd)] pointers: one batched launch."""
    if not items:
        return
    col = list(zip(*items))
    rc = lib.mrg_residual_layernorm_fwd_batched(
        len(items), rows, H, _arr(VP, col[0]), _arr(VP, col[1]), _arr(VP, col[2]), _arr(VP, col[3]), eps,
        _arr(VP, col[4]), _arr(CL, [m[0] for m in col[5]]), _arr(CL, [m[1] for m in col[5]]),
        _arr(CI, [m[2] for m in col[5]]), _arr(VP, col[6]), _arr(VP, col[7]), _stream())
    _lib.check(rc, "batched layernorm fwd (encoder stack)")


def _bln_bwd(lib, rows, H, items):
    """items = [(dy, (lo, hi, div), a, b, gamma, mean, rstd, dx, ws)] pointers: one batched launch."""
    if not items:
        return
    col = list(zip(*items))
    rc = lib.mrg_residual_layernorm_bwd_batched(
        len(items), rows, H, _arr(VP, col[0]), _arr(CL, [m[0] for m in col[1]]), _arr(CL, [m[1] for m in col[1]]),
        _arr(CI, [m[2] for m in col[1]]), _arr(VP, col[2]), _arr(VP, col[3]), _arr(VP, col[4]), _arr(VP, col[5]),
        _arr(VP, col[6]), _arr(VP, col[7]), _arr(VP, col[8]), _stream())
    _lib.check(rc, "batched layernorm bwd (encoder stack)")


def _bgroups(probs):
    """Problems of one diagonal by chunk length, at most _BMAX per batched launch."""
    by = {}
    for pr in probs:
        by.setdefault(pr[4] - pr[3], []).append(pr)
    return [(k, v[s:s + _BMAX]) for k, v in by.items() for s in range(0, len(v), _BMAX)]


def _diagonals(chains, tc):
    """[(d, [(m, l, c, t0, t1)])]: every (chain, layer, chunk) with l + c = d."""
    out = []
    D = max(ch.L + len(_chunks(ch.T, tc)) - 1 for ch in chains)
    for d in range(D):
        probs = []
        for m, ch in enumerate(chains):
            ck = _chunks(ch.T, tc)
            for l in range(ch.L):
                c = d - l
                if 0 <= c < len(ck):
                    probs.append((m, l, c, ck[c][0], ck[c][1]))
        out.append(probs)
    return out


def _groups(items, key, cap):
    """Split into launches: same key (chunk length), at most cap problems each."""
    by = {}
    for it in items:
        by.setdefault(key(it), []).append(it)
    return [(k, part) for k, v in by.items() for part in _split(v, cap)]


class _EncoderStackFn(Function):
    """spec = (layers per chain, chunk length, eps); tensors = per chain [feat, emb_w, emb_b,
    10 per layer]; returns the last layer's output of every chain, batch-major [B, T, H]."""

    @staticmethod
    @Fn._keeps_precision
    def forward(ctx, spec, *tensors):
        nls, tc, eps, sinks = spec
        ctx.sinks = sinks
        ctx.set_materialize_grads(False)   # a source whose gradient comes through its KVSink gets None
        lib = _lib.load()
        chains, k = [], 0
        for L in nls:
            feat, ew, eb = tensors[k:k + 3]
            k += 3
            layers = [tensors[k + _PER_LAYER * i:k + _PER_LAYER * (i + 1)] for i in range(L)]
            k += _PER_LAYER * L
            chains.append(_Chain(feat.contiguous(), ew, eb, layers))
        _lib.require_device(chains[0].feat)
        dev = chains[0].feat.device
        B, H = chains[0].B, chains[0].H
        f32 = dict(device=dev, dtype=torch.float32)
        states, outs = [], []
        for ch in chains:
            T, F = ch.T, ch.F
            rows = T * B
            # embedding, time-major output: A rows read in (t, b) order from the [B, T, F] features
            x0 = torch.empty(T, B, H, **f32)
            gemm(rows, H, F, _ptr(ch.feat), 0, T * F, _ptr(ch.emb_w), 1, F, _ptr(x0), H, bias=_ptr(ch.emb_b),
                 a_hi=F, a_div=B, device=dev)
            sts = []
            for l, (w_ih, w_hh, b_ih, b_hh, g1, be1, w_ff, b_ff, g2, be2) in enumerate(ch.layers):
                st = dict(w_ih=w_ih, w_hh=w_hh, b_ih=b_ih, b_hh=b_hh, g1=g1, be1=be1, w_ff=w_ff, b_ff=b_ff, g2=g2,
                          be2=be2, x=x0 if l == 0 else sts[-1]["v"],
                          gx=torch.empty(T, B, 4 * H, **f32), y=torch.empty(T, B, H, **f32),
                          gates=torch.empty(T, B, 4 * H, **f32), cs=torch.empty(T, B, H, **f32),
                          u=torch.empty(T, B, H, **f32), z=torch.empty(T, B, H, **f32),
                          v=torch.empty(T, B, H, **f32) if l + 1 < ch.L else None,
                          m1=torch.empty(rows, **f32), r1=torch.empty(rows, **f32),
                          m2=torch.empty(rows, **f32), r2=torch.empty(rows, **f32))
                _wt_note(w_ih, rows)
                _wt_note(w_ff, rows)
                sts.append(st)
            states.append(sts)
            outs.append(torch.empty(B, T, H, **f32))

        # per diagonal: the chunks' input projections (one batched GEMM), ONE recurrence launch, then
        # residual LN, FeedForward Linear, residual LN of every chunk (batched LayerNorm / GEMM launches)
        diags = _diagonals(chains, tc)
        pool = _RingPool(sum(len(p) for p in diags), lib.mrg_lstm_fwd_xbuf_bytes(B, H) // 8, dev)
        for probs in diags:
            bg = _bgroups(probs)
            for tlen, grp in bg:
                items = []
                for m, l, c, t0, t1 in grp:
                    st, r0 = states[m][l], t0 * B
                    items.append((_p(st["x"], r0 * H), st["w_ih"], _p(st["gx"], r0 * 4 * H), _ptr(st["b_ih"]), None))
                _bgemm(lib, tlen * B, 4 * H, H, items, H, 4 * H, dev=dev)
            for tlen, grp in _groups(probs, lambda p: p[4] - p[3], _maxp(B, dev)):
                _launch_fwd(lib, [(chains[m], states[m][l], t0) for m, l, c, t0, t1 in grp], B, tlen, H, dev, pool)
            for tlen, grp in bg:
                n = tlen * B
                ln1, ff, ln2 = [], [], []
                for m, l, c, t0, t1 in grp:
                    ch, st, r0 = chains[m], states[m][l], t0 * B
                    ln1.append((_p(st["y"], r0 * H), _p(st["x"], r0 * H), _ptr(st["g1"]), _ptr(st["be1"]),
                                _p(st["u"], r0 * H), (H, 0, 0), _p(st["m1"], r0), _p(st["r1"], r0)))
                    ff.append((_p(st["u"], r0 * H), st["w_ff"], _p(st["z"], r0 * H), _ptr(st["b_ff"]), None))
                    if st["v"] is not None:
                        out, omap = _p(st["v"], r0 * H), (H, 0, 0)
                    else:   # last layer: rows (t, b) land in the batch-major output [B, T, H]
                        out, omap = _p(outs[m], t0 * H), (ch.T * H, H, B)
                    ln2.append((_p(st["z"], r0 * H), _p(st["u"], r0 * H), _ptr(st["g2"]), _ptr(st["be2"]), out, omap,
                                _p(st["m2"], r0), _p(st["r2"], r0)))
                _bln_fwd(lib, n, H, eps, ln1)
                _bgemm(lib, n, H, H, ff, H, H, dev=dev)
                _bln_fwd(lib, n, H, eps, ln2)

        ctx.chains, ctx.tc, ctx.B, ctx.H = chains, tc, B, H
        save = []
        for sts in states:
            for st in sts:
                st.pop("gx")   # not needed by the backward
                for key in ("x", "y", "gates", "cs", "u", "z", "m1", "r1", "m2", "r2"):
                    save.append(st[key])
        ctx.save_for_backward(*save)
        ctx.keys = ("x", "y", "gates", "cs", "u", "z", "m1", "r1", "m2", "r2")
        ctx.params = [[{k2: st[k2] for k2 in ("w_ih", "w_hh", "b_ih", "b_hh", "g1", "be1", "w_ff", "b_ff", "g2",
                                               "be2")} for st in sts] for sts in states]
        return tuple(outs)

    @staticmethod
    @Fn._keeps_precision
    def backward(ctx, *douts):
        chains, tc, B, H = ctx.chains, ctx.tc, ctx.B, ctx.H
        lib = _lib.load()
        saved = list(ctx.saved_tensors)
        dev = saved[0].device
        f32 = dict(device=dev, dtype=torch.float32)
        states, k = [], 0
        for m, ch in enumerate(chains):
            sts = []
            for l in range(ch.L):
                st = dict(zip(ctx.keys, saved[k:k + len(ctx.keys)]))
                k += len(ctx.keys)
                st.update(ctx.params[m][l])
                sts.append(st)
            states.append(sts)
        douts = list(douts)
        for m, sink in enumerate(ctx.sinks):   # the fused integrators' summed key / value gradients
            g = sink.drain()
            if g is not None:
                douts[m] = g if douts[m] is None else douts[m] + g
        grads, carry = [], {}
        wsb = lib.mrg_residual_layernorm_bwd_workspace_bytes
        for m, ch in enumerate(chains):
            T, rows = ch.T, ch.T * B
            nblk = sum(_ln_blocks(lib, (c1 - c0) * B, H) for c0, c1 in _chunks(T, tc))
            gl = []
            for l in range(ch.L):
                gl.append(dict(dG=torch.empty(T, B, 4 * H, **f32), g1=torch.empty(T, B, H, **f32),
                               g2=torch.empty(T, B, H, **f32),
                               dv=torch.empty(T, B, H, **f32),   # gradient of this layer's input x
                               ws1=torch.empty(nblk * 2 * H, **f32), ws2=torch.empty(nblk * 2 * H, **f32),
                               nblk=nblk))
                carry[(m, l)] = [torch.empty(B, H, **f32) for _ in range(4)]   # dh, dc of two chunks
            grads.append(gl)
            if douts[m] is None:
                douts = list(douts)
                douts[m] = Fn.zeros(B, T, H, **f32)
        douts = [d.contiguous() for d in douts]

        def block_off(T, c):
            return sum(_ln_blocks(lib, (c1 - c0) * B, H) for c0, c1 in _chunks(T, tc)[:c])

        diags = _diagonals(chains, tc)
        # backward: diagonals in reverse, within one the chunk index of every chain's top layer first
        rdiag = []
        D = max(ch.L + len(_chunks(ch.T, tc)) - 1 for ch in chains)
        for rd in range(D):
            probs = []
            for m, ch in enumerate(chains):
                ck = _chunks(ch.T, tc)
                for l in range(ch.L - 1, -1, -1):
                    c = len(ck) - 1 - (rd - (ch.L - 1 - l))
                    if 0 <= c < len(ck):
                        probs.append((m, l, c, ck[c][0], ck[c][1]))
            rdiag.append(probs)
        del diags

        pool = _RingPool(sum(len(p) for p in rdiag), lib.mrg_lstm_bwd_xbuf_bytes(B, H) // 8, dev)
        for probs in rdiag:
            bg = _bgroups(probs)
            for tlen, grp in bg:   # LN2, FeedForward, LN1 backward of the chunks (batched launches)
                n = tlen * B
                du = torch.empty(len(grp), n, H, **f32)   # d(u) = g2 W_ff + g2 (residual branch in the epilogue)
                ln2, ff, ln1 = [], [], []
                for i, (m, l, c, t0, t1) in enumerate(grp):
                    ch, st, gr = chains[m], states[m][l], grads[m][l]
                    r0 = t0 * B
                    bo = block_off(ch.T, c) * 2 * H
                    if l == ch.L - 1:   # the stack's output gradient, batch-major
                        dy, dmap = _p(douts[m], t0 * H), (ch.T * H, H, B)
                    else:
                        dy, dmap = _p(grads[m][l + 1]["dv"], r0 * H), (H, 0, 0)
                    ln2.append((dy, dmap, _p(st["z"], r0 * H), _p(st["u"], r0 * H), _ptr(st["g2"]), _p(st["m2"], r0),
                                _p(st["r2"], r0), _p(gr["g2"], r0 * H), _p(gr["ws2"], bo)))
                    ff.append((_p(gr["g2"], r0 * H), st["w_ff"], _ptr(du[i]), None, _p(gr["g2"], r0 * H)))
                    ln1.append((_ptr(du[i]), (H, 0, 0), _p(st["y"], r0 * H), _p(st["x"], r0 * H), _ptr(st["g1"]),
                                _p(st["m1"], r0), _p(st["r1"], r0), _p(gr["g1"], r0 * H), _p(gr["ws1"], bo)))
                _bln_bwd(lib, n, H, ln2)
                _bgemm(lib, n, H, H, ff, H, H, epi=3, ldaux=H, transposed=True, dev=dev)
                _bln_bwd(lib, n, H, ln1)
            items = {}
            for m, l, c, t0, t1 in probs:
                ch = chains[m]
                nc = len(_chunks(ch.T, tc))
                cb = carry[(m, l)]
                cur, nxt = (cb[0], cb[1]) if c % 2 == 0 else (cb[2], cb[3])   # this chunk's dh0 / dc0 out
                prv = (cb[2], cb[3]) if c % 2 == 0 else (cb[0], cb[1])        # chunk c+1's dh0 / dc0
                dh_in, dc_in = (None, None) if c == nc - 1 else prv
                dh_out, dc_out = (None, None) if c == 0 else (cur, nxt)
                items.setdefault(t1 - t0, []).append(
                    (ch, states[m][l], grads[m][l], t0, dh_in, dc_in, dh_out, dc_out))
            for tlen, grp in items.items():
                for part in _split(grp, _maxp(B, dev)):
                    _launch_bwd(lib, part, B, tlen, H, dev, pool)
            for tlen, grp in bg:   # input gradients of the chunks: dG W_ih + g1 (residual), batched
                items = []
                for m, l, c, t0, t1 in grp:
                    st, gr, r0 = states[m][l], grads[m][l], t0 * B
                    items.append((_p(gr["dG"], r0 * 4 * H), st["w_ih"], _p(gr["dv"], r0 * H), None,
                                  _p(gr["g1"], r0 * H)))
                _bgemm(lib, tlen * B, H, 4 * H, items, 4 * H, H, epi=3, ldaux=H, transposed=True, dev=dev)
            for m, l, c, t0, t1 in probs:
                if c == 0:
                    _EncoderStackFn._weight_grads(lib, chains[m], states[m][l], grads[m][l], l, B, H, dev,
                                                  0, chains[m].T, 0)
        return (None,) + tuple(_EncoderStackFn._input_grads(chains, ctx.needs_input_grad))

    @staticmethod
    def _weight_grads(lib, ch, st, gr, l, B, H, dev, t0, t1, bo):
        """Layer l's parameter gradients over time steps [t0, t1) (one chunk, or the whole sequence once
        its last chunk is done), accumulated into the gradient buffers and issued as ONE fork onto the
        weight-gradient side stream (functional._side); bo = the chunk's first LayerNorm partial block.
        Rows are time-major, so a chunk is one contiguous row range."""
        T = ch.T
        r0, rows = t0 * B, (t1 - t0) * B
        dG, g2, g1, dx0 = gr["dG"], gr["g2"], gr["g1"], gr["dv"]
        gbi, gbh = _gbuf(st["b_ih"]), _gbuf(st["b_hh"])
        first = gbi if gbi is not None else gbh
        gw_ih, gw_hh, gw_ff, gb_ff = _gbuf(st["w_ih"]), _gbuf(st["w_hh"]), _gbuf(st["w_ff"]), _gbuf(st["b_ff"])
        lns = [(gr["ws1"], _gbuf(st["g1"]), _gbuf(st["be1"])), (gr["ws2"], _gbuf(st["g2"]), _gbuf(st["be2"]))]
        emb = (_gbuf(ch.emb_w), _gbuf(ch.emb_b)) if l == 0 else (None, None)
        keep = (dG, g2, g1, dx0, st["x"], st["y"], st["u"], gr["ws1"], gr["ws2"], ch.feat)
        th = max(t0, 1)   # dW_hh pairs dG_t with y_{t-1}: t >= 1

        def wg(dY, ldy, X, ldx, n, Nout, Nin, gw, **kw):
            if gw is None:
                gb = kw.get("gb")
                if gb is not None:
                    Fn.colsum(n, Nout, dY, ldy, _ptr(gb), out2=_ptr(kw.get("gb2")), device=dev)
                return
            gemm(Nout, Nin, n, dY, 1, ldy, X, 0, ldx, _ptr(gw), Nin, beta=1.0, b_hi=kw.get("x_hi", 0),
                 b_div=kw.get("x_div", 0), splits=Fn.wgrad_splits(Nout, Nin, n), device=dev,
                 asum_out=_ptr(kw.get("gb")), asum_out2=_ptr(kw.get("gb2")))

        # the partial blocks to reduce: one chunk's (starting at block bo), or every chunk's
        nb = gr["nblk"] if (t0 == 0 and t1 == T) else _ln_blocks(lib, rows, H)

        def ln_reduce(ws, gg, gb):
            scratch = Fn._ws(2 * H * 4, dev).view(2, H) if (gg is None or gb is None) else None
            _lib.check(lib.mrg_residual_layernorm_param_reduce(
                _ln_rows(lib, nb, H), H, _p(ws, bo * 2 * H), _ptr(gg if gg is not None else scratch[0]),
                _ptr(gb if gb is not None else scratch[1]), 1, _stream()), "layernorm param reduce")

        parts = [lambda: wg(_p(dG, r0 * 4 * H), 4 * H, _p(st["x"], r0 * H), H, rows, 4 * H, H, gw_ih, gb=first,
                            gb2=gbh if gbi is not None else None)]
        if gw_hh is not None and t1 > th:   # sum_t dG_t^T y_{t-1}: time-major rows shifted by one step
            parts.append(lambda: wg(_p(dG, th * B * 4 * H), 4 * H, _p(st["y"], (th - 1) * B * H), H, (t1 - th) * B,
                                    4 * H, H, gw_hh))
        parts.append(lambda: wg(_p(g2, r0 * H), H, _p(st["u"], r0 * H), H, rows, H, H, gw_ff, gb=gb_ff))
        for ws, gg, gb in lns:
            if gg is not None or gb is not None:
                parts.append(lambda ws=ws, gg=gg, gb=gb: ln_reduce(ws, gg, gb))
        if l == 0:   # the embedding: dW_emb = sum dx0^T feat (features read time-major through a row map)
            parts.append(lambda: wg(_p(dx0, r0 * H), H, _p(ch.feat, t0 * ch.F), T * ch.F, rows, H, ch.F, emb[0],
                                    x_hi=ch.F, x_div=B, gb=emb[1]))
        writes = (gw_ih, first, gbh, gw_hh, gw_ff, gb_ff, *emb, *[t for _, gg, gb in lns for t in (gg, gb)])
        if SPLIT_FORKS:   # one fork per product (the round-3 pattern, kept as a capture regression case)
            for f in parts:
                _on_side(dev, rows, keep, f, writes=writes)
            return

        def issue():
            for f in parts:
                f()
        _on_side(dev, rows, keep, issue, writes=writes)

    @staticmethod
    def _input_grads(chains, need):
        # the features are data (no gradient), parameters get theirs in place through _gbuf
        return [None] * (len(need) - 1)


def _ln_blocks(lib, rows, H) -> int:
    """LayerNorm-backward partial blocks of `rows` rows (from the C ABI's workspace size, so the row
    count per block is never restated here)."""
    return int(lib.mrg_residual_layernorm_bwd_workspace_bytes(rows, H)) // (2 * H * 4)


def _ln_rows(lib, nblk, H) -> int:
    """A row count whose parameter reduce covers exactly `nblk` partial blocks: chunks of a length that
    is not a multiple of the block rows leave a partial block each, so the sum of the chunks' blocks
    can exceed the blocks of their total rows (B = 4, 100-step chunks: 3 x 13 blocks, not 38)."""
    rpb = 4096 // _ln_blocks(lib, 4096, H)
    return nblk * rpb


def stack_eligible(H, B) -> bool:
    lib = _lib.load()
    return bool(lib.mrg_lstm_supported_hidden(H)) and H % 4 == 0 and Fn._ARITH[0] is None


def encoder_stack(chains: Sequence[Sequence], eps: float, chunk: int = 0) -> List[torch.Tensor]:
    """chains: [(feat [B, T, F], emb_w, emb_b, [(w_ih, w_hh, b_ih, b_hh, ln1_w, ln1_b, ff_w, ff_b, ln2_w,
    ln2_b)] per layer)]; returns the last layer's output of every chain ([B, T, H], batch-major)."""
    flat, nls = [], []
    for feat, ew, eb, layers in chains:
        flat += [feat, ew, eb]
        for lay in layers:
            flat += list(lay)
        nls.append(len(layers))
    from .integrate import KVSink
    sinks = [KVSink() for _ in chains]
    outs = list(_EncoderStackFn.apply((tuple(nls), int(chunk or CHUNK), float(eps), sinks), *flat))
    for o, sink in zip(outs, sinks):
        o._mrg_kv_sink = sink   # consumers (integrate._IntegrateFn) sum their dKV into it; backward drains
    return outs
