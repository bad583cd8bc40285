"""(block, time-chunk) wavefront of the metaformer blocks after the first.

Reference: ``MultiModalMetaformer.forward`` runs its blocks one after the other
(multi_modal_metaformer.py:476-509); every block after the first
(``MultiModalMetaformerBlock``, :220-338, ``encode_other_modal`` False) is

    e   = LSTMMixerBlock(x)                 LN2(LN1(LSTM(x) + x) W_ff^T + b + LN1(..))   (mixer_block.py:479-507)
    c_i = IntegrateModal_i(e, kv_i)         LN2_i(FF_i(LN1_i(MHA_i(e, kv_i) + e)) + ..)  (:128-217, for_sequential.py:42-51)
    f   = cat(c_0, c_1) W_cat^T + b_cat     (:214-215)
    out = LN(relu(f W_in^T + b_in) W_out^T + b_out + f)                                  (FeedForward, mixer_block.py:37-87)

with kv_i the first block's encoder outputs (complete before block 1 starts) and the
integrators' block-causal mask (query t sees keys j < (t + 1) Tk / T, gen_attention_mask,
:32-79).  Every op is causal in time, so block k's time chunk c needs only block k-1's chunk
c and its own chunk c-1 (the carried LSTM h, c): the blocks run as a wavefront over
(block, chunk) diagonals, like the encoder stacks (encoder_stack.py).  Per diagonal, ONE
recurrence launch holds every (block, chunk) in flight, and each of the other ops is one
batched launch over them; round 3 ran four single-problem 300-step recurrences (about 465 us
forward and 530-580 us backward each) strictly one after another.

Layout: time-major inside ([T, B, .] rows t * B + b) so a chunk is a contiguous row range;
the batch-major block input / output are permuted once at the edges (mrg_swap01).  The
key / value projections of every block are one batched GEMM up front (they read only the
encoder outputs); attention runs per query chunk (mrg_attention_*_chunk: global mask indices,
dK / dV of the chunks accumulated in a fixed order).  The backward walks the diagonals in
reverse with (dh, dc) carried from chunk c+1 to c; each block's parameter gradients go as ONE
fork onto the weight-gradient side stream once its chunk 0 is done, and its key / value input
gradients into the encoder outputs' KVSink (integrate.py).  Arithmetic per element is the
per-block path's (same kernels); only the launch granularity and fp32 summation orders of the
weight gradients change.
"""
from __future__ import annotations

import math
import os
from typing import List, Sequence

import torch
from torch.autograd import Function

from . import _lib
from . import functional as Fn
from .encoder_stack import (VP, CL, CI, _arr, _bln_fwd, _bln_bwd, _chunks, _groups, _maxp, _RingPool,
                            _launch_fwd, _launch_bwd, _ln_blocks, _ln_rows, _p)
from .functional import _ptr, _stream, gemm, _dx_gemm, _wt_note, _gbuf, _on_side

# time steps per chunk; MRG_BLOCK_CHUNK overrides (0 turns the wavefront off: per-block schedule)
CHUNK = int(os.environ.get("MRG_BLOCK_CHUNK", "100"))
_BMAX = 16
RUNS = [0]   # forward passes through the wavefront (tests check the schedule they compare really ran)

# per block: LSTM block (w_ih, w_hh, b_ih, b_hh, ln1 w, ln1 b, ff w, ff b, ln2 w, ln2 b),
# per integrator (in_w, in_b, out_w, out_b, ln1 w, ln1 b, ff w, ff b, ln2 w, ln2 b),
# cat_w, cat_b, FeedForward (in_w, in_b, out_w, out_b, ln w, ln b)
_PL, _PI, _PF = 10, 10, 6


def _bgemm(lib, M, N, K, items, lda, ldc, *, epi=0, ldaux=0, transposed=False, beta=0.0, dev=None):
    """Same-shape products in one launch; items = [(A ptr, w, C ptr, bias ptr | None, aux ptr | None)];
    transposed: dY w products through w's [in][out] copy (one by one when a copy is missing)."""
    if not items:
        return
    bs = []
    for it in items:
        w = it[1]
        if transposed:
            wt = Fn._wt(w) if M >= Fn._WT_MIN_ROWS else None
            if wt is None:
                for a2, w2, c2, b2, x2 in items:
                    _dx_gemm(M, N, K, a2, lda, w2, c2, ldc, bias=b2, epi=epi, aux=x2, ldaux=ldaux, beta=beta,
                             device=dev)
                return
            bs.append(_ptr(wt))
        else:
            bs.append(_ptr(w))
    for s in range(0, len(items), _BMAX):
        part, bp = items[s:s + _BMAX], bs[s:s + _BMAX]
        with Fn._probe("gemm", 2.0 * M * N * K * len(part)):
            rc = lib.mrg_gemm_x6g_batched(
                len(part), M, N, K, 1.0, _arr(VP, [it[0] for it in part]), lda, _arr(VP, bp), K, beta,
                _arr(VP, [it[2] for it in part]), ldc,
                None if all(it[3] is None for it in part) else _arr(VP, [it[3] for it in part]), epi,
                None if all(it[4] is None for it in part) else _arr(VP, [it[4] for it in part]), ldaux,
                1 if Fn._ARITH[0] == "bf16" else 0, _stream())
        _lib.check(rc, "batched gemm (block stack)")


def _by_len(probs):
    """[(chunk rows length, [problems])] of one diagonal (ragged last chunks form their own group)."""
    out = {}
    for pr in probs:
        out.setdefault(pr[3] - pr[2], []).append(pr)
    return list(out.items())


class _Block:
    """One block's parameters (views into the flat parameter buffer) and activations."""

    def __init__(self, params, n):
        self.lstm = params[:_PL]
        self.integ = [params[_PL + _PI * i:_PL + _PI * (i + 1)] for i in range(n)]
        self.cat_w, self.cat_b = params[_PL + _PI * n:_PL + _PI * n + 2]
        self.ffn = params[_PL + _PI * n + 2:]


class _BlockStackFn(Function):
    """spec = (nblocks, n integrators, heads, causal, eps, chunk, sinks); tensors = x [B, T, E],
    kv_0..kv_{n-1}, qpad_0..qpad_{n-1}, kpad_0..kpad_{n-1} (uint8 or None, one mask per integrator),
    then per block 10 + 10 n + 2 + 6 parameters.  Returns the last block's output [B, T, E]."""

    @staticmethod
    @Fn._keeps_precision
    def forward(ctx, spec, x, *t):
        nb, n, heads, causal, eps, tc, sinks = spec
        RUNS[0] += 1
        kvs = list(t[:n])
        qpads = list(t[n:2 * n])
        kpads = list(t[2 * n:3 * n])
        per = _PL + _PI * n + 2 + _PF
        pr = t[3 * n:]
        blocks = [_Block(pr[per * k:per * (k + 1)], n) for k in range(nb)]
        _lib.require_device(x)
        lib = _lib.load()
        dev = x.device
        B, T, E = x.shape
        D = E // heads
        Hb = blocks[0].ffn[0].shape[0]
        rows = T * B
        f32 = dict(device=dev, dtype=torch.float32)
        kv2 = [kv.contiguous() for kv in kvs]
        Tks = [kv.shape[1] for kv in kv2]
        scale = 1.0 / math.sqrt(D)

        xt = torch.empty(T, B, E, **f32)
        _lib.check(lib.mrg_swap01(B, T, E, _ptr(x.contiguous()), _ptr(xt), 0.0, _stream()), "swap01")

        # every block's key / value projections (they read only the encoder outputs): one launch per Tk
        KV = [[torch.empty(B, Tks[i], 2 * E, **f32) for i in range(n)] for _ in range(nb)]
        for Tk in sorted(set(Tks)):
            items = [(_ptr(kv2[i]), blocks[k].integ[i][0][E:], _ptr(KV[k][i]), _p(blocks[k].integ[i][1], E), None)
                     for k in range(nb) for i in range(n) if Tks[i] == Tk]
            _bgemm(lib, B * Tk, 2 * E, E, items, E, 2 * E, dev=dev)

        S = []   # per block: activation buffers (time-major)
        for k, bl in enumerate(blocks):
            st = dict(x=xt if k == 0 else S[k - 1]["out"],
                      gx=torch.empty(T, B, 4 * E, **f32), y=torch.empty(T, B, E, **f32),
                      gates=torch.empty(T, B, 4 * E, **f32), cs=torch.empty(T, B, E, **f32),
                      u=torch.empty(T, B, E, **f32), z=torch.empty(T, B, E, **f32), e=torch.empty(T, B, E, **f32),
                      m1=torch.empty(rows, **f32), r1=torch.empty(rows, **f32),
                      m2=torch.empty(rows, **f32), r2=torch.empty(rows, **f32),
                      Q=torch.empty(n, T, B, E, **f32), O=torch.empty(n, T, B, E, **f32),
                      A=torch.empty(n, T, B, E, **f32), U=torch.empty(n, T, B, E, **f32),
                      Z=torch.empty(n, T, B, E, **f32), mi1=torch.empty(n, rows, **f32),
                      ri1=torch.empty(n, rows, **f32), mi2=torch.empty(n, rows, **f32),
                      ri2=torch.empty(n, rows, **f32), cat=torch.empty(T, B, n * E, **f32),
                      f=torch.empty(T, B, E, **f32), h1=torch.empty(T, B, Hb, **f32), h2=torch.empty(T, B, E, **f32),
                      out=torch.empty(T, B, E, **f32), m3=torch.empty(rows, **f32), r3=torch.empty(rows, **f32),
                      lse=torch.empty(n, B, heads, T, **f32))
            st.update(w_hh=bl.lstm[1], b_hh=bl.lstm[3])
            S.append(st)
            w_ih, _, _, _, _, _, w_ff = bl.lstm[:7]
            for w in (w_ih, w_ff, bl.cat_w, bl.ffn[0], *[bl.integ[i][0][:E] for i in range(n)],
                      *[bl.integ[i][2] for i in range(n)], *[bl.integ[i][6] for i in range(n)]):
                _wt_note(w, rows)
            for i in range(n):
                _wt_note(bl.integ[i][0][E:], B * Tks[i])

        ck = _chunks(T, tc)
        pool = _RingPool(sum(1 for _ in ck) * nb, lib.mrg_lstm_fwd_xbuf_bytes(B, E) // 8, dev)
        pads = [(_ptr(qp) if causal else None, _ptr(kp) if causal else None) for qp, kp in zip(qpads, kpads)]
        for d in range(nb + len(ck) - 1):
            probs = [(k, c, ck[c][0], ck[c][1]) for k in range(nb) for c in [d - k] if 0 <= c < len(ck)]
            _BlockStackFn._fwd_diagonal(lib, probs, blocks, S, KV, Tks, pads, B, T, E, n, heads, causal, scale, eps,
                                        dev, pool)

        y = torch.empty(B, T, E, **f32)
        _lib.check(lib.mrg_swap01(T, B, E, _ptr(S[-1]["out"]), _ptr(y), 0.0, _stream()), "swap01")
        ctx.save_for_backward(x, *kv2, *qpads, *kpads)
        ctx.blocks, ctx.S, ctx.KV, ctx.Tks, ctx.pads = blocks, S, KV, Tks, pads
        ctx.spec = (nb, n, heads, causal, eps, tc, sinks, B, T, E, Hb, scale)
        ctx.kv_need = [ctx.needs_input_grad[2 + i] for i in range(n)]
        ctx.x_need = ctx.needs_input_grad[1]
        return y

    @staticmethod
    def _fwd_diagonal(lib, probs, blocks, S, KV, Tks, pads, B, T, E, n, heads, causal, scale, eps, dev, pool):
        D = E // heads
        Hb = blocks[0].ffn[0].shape[0]
        groups = _by_len(probs)
        for tl, grp in groups:   # LSTM input projections
            items = [(_p(S[k]["x"], t0 * B * E), blocks[k].lstm[0], _p(S[k]["gx"], t0 * B * 4 * E),
                      _ptr(blocks[k].lstm[2]), None) for k, c, t0, t1 in grp]
            _bgemm(lib, tl * B, 4 * E, E, items, E, 4 * E, dev=dev)
        for tl, grp in _groups(probs, lambda p: p[3] - p[2], _maxp(B, dev)):
            _launch_fwd(lib, [(None, S[k], t0) for k, c, t0, t1 in grp], B, tl, E, dev, pool)
        for tl, grp in groups:
            N = tl * B
            lst = [(k, t0 * B) for k, c, t0, t1 in grp]
            _bln_fwd(lib, N, E, eps, [(_p(S[k]["y"], r0 * E), _p(S[k]["x"], r0 * E), _ptr(blocks[k].lstm[4]),
                                       _ptr(blocks[k].lstm[5]), _p(S[k]["u"], r0 * E), (E, 0, 0), _p(S[k]["m1"], r0),
                                       _p(S[k]["r1"], r0)) for k, r0 in lst])
            _bgemm(lib, N, E, E, [(_p(S[k]["u"], r0 * E), blocks[k].lstm[6], _p(S[k]["z"], r0 * E),
                                   _ptr(blocks[k].lstm[7]), None) for k, r0 in lst], E, E, dev=dev)
            _bln_fwd(lib, N, E, eps, [(_p(S[k]["z"], r0 * E), _p(S[k]["u"], r0 * E), _ptr(blocks[k].lstm[8]),
                                       _ptr(blocks[k].lstm[9]), _p(S[k]["e"], r0 * E), (E, 0, 0), _p(S[k]["m2"], r0),
                                       _p(S[k]["r2"], r0)) for k, r0 in lst])
            # integrators: query projections, attention per chunk, out projection, LN, FF, LN -> concat
            _bgemm(lib, N, E, E, [(_p(S[k]["e"], r0 * E), blocks[k].integ[i][0][:E], _p(S[k]["Q"][i], r0 * E),
                                   _ptr(blocks[k].integ[i][1]), None) for k, r0 in lst for i in range(n)], E, E, dev=dev)
            for k, c, t0, t1 in grp:
                for i in range(n):
                    Tk = Tks[i]
                    with Fn._probe("attn_fwd", 4.0 * D * B * heads * _chunk_pairs(t0, t1, T, Tk, causal)):
                        rc = lib.mrg_attention_fwd_chunk(
                            B, heads, t1 - t0, Tk, D, t0, T, _p(S[k]["Q"][i], t0 * B * E), E, B * E,
                            _ptr(KV[k][i]), Tk * 2 * E, 2 * E, _p(KV[k][i], E), Tk * 2 * E, 2 * E,
                            _p(S[k]["O"][i], t0 * B * E), E, B * E, _ptr(S[k]["lse"][i]), pads[i][0], pads[i][1],
                            int(causal), scale, _stream())
                    _lib.check(rc, "attention fwd chunk (block stack)")
            _bgemm(lib, N, E, E, [(_p(S[k]["O"][i], r0 * E), blocks[k].integ[i][2], _p(S[k]["A"][i], r0 * E),
                                   _ptr(blocks[k].integ[i][3]), None) for k, r0 in lst for i in range(n)], E, E, dev=dev)
            _bln_fwd(lib, N, E, eps, [(_p(S[k]["A"][i], r0 * E), _p(S[k]["e"], r0 * E), _ptr(blocks[k].integ[i][4]),
                                       _ptr(blocks[k].integ[i][5]), _p(S[k]["U"][i], r0 * E), (E, 0, 0),
                                       _p(S[k]["mi1"][i], r0), _p(S[k]["ri1"][i], r0)) for k, r0 in lst for i in range(n)])
            _bgemm(lib, N, E, E, [(_p(S[k]["U"][i], r0 * E), blocks[k].integ[i][6], _p(S[k]["Z"][i], r0 * E),
                                   _ptr(blocks[k].integ[i][7]), None) for k, r0 in lst for i in range(n)], E, E, dev=dev)
            _bln_fwd(lib, N, E, eps, [(_p(S[k]["Z"][i], r0 * E), _p(S[k]["U"][i], r0 * E), _ptr(blocks[k].integ[i][8]),
                                       _ptr(blocks[k].integ[i][9]), _p(S[k]["cat"], r0 * n * E + i * E), (n * E, 0, 0),
                                       _p(S[k]["mi2"][i], r0), _p(S[k]["ri2"][i], r0)) for k, r0 in lst for i in range(n)])
            _bgemm(lib, N, E, n * E, [(_p(S[k]["cat"], r0 * n * E), blocks[k].cat_w, _p(S[k]["f"], r0 * E),
                                       _ptr(blocks[k].cat_b), None) for k, r0 in lst], n * E, E, dev=dev)
            # the block's FeedForward: relu(f W_in^T + b_in) W_out^T + b_out, residual LN
            _bgemm(lib, N, Hb, E, [(_p(S[k]["f"], r0 * E), blocks[k].ffn[0], _p(S[k]["h1"], r0 * Hb),
                                    _ptr(blocks[k].ffn[1]), None) for k, r0 in lst], E, Hb, epi=1, dev=dev)
            _bgemm(lib, N, E, Hb, [(_p(S[k]["h1"], r0 * Hb), blocks[k].ffn[2], _p(S[k]["h2"], r0 * E),
                                    _ptr(blocks[k].ffn[3]), None) for k, r0 in lst], Hb, E, dev=dev)
            _bln_fwd(lib, N, E, eps, [(_p(S[k]["h2"], r0 * E), _p(S[k]["f"], r0 * E), _ptr(blocks[k].ffn[4]),
                                       _ptr(blocks[k].ffn[5]), _p(S[k]["out"], r0 * E), (E, 0, 0), _p(S[k]["m3"], r0),
                                       _p(S[k]["r3"], r0)) for k, r0 in lst])

    @staticmethod
    @Fn._keeps_precision
    def backward(ctx, dy):
        nb, n, heads, causal, eps, tc, sinks, B, T, E, Hb, scale = ctx.spec
        saved = ctx.saved_tensors
        x, kv2 = saved[0], list(saved[1:1 + n])
        blocks, S, KV, Tks, pads = ctx.blocks, ctx.S, ctx.KV, ctx.Tks, ctx.pads
        lib = _lib.load()
        dev = dy.device
        D = E // heads
        rows = T * B
        f32 = dict(device=dev, dtype=torch.float32)
        ck = _chunks(T, tc)
        nblk = sum(_ln_blocks(lib, (c1 - c0) * B, E) for c0, c1 in ck)

        def boff(c):
            return sum(_ln_blocks(lib, (c1 - c0) * B, E) for c0, c1 in ck[:c]) * 2 * E

        G = []   # per block: gradient buffers (time-major)
        for k in range(nb):
            G.append(dict(dout=torch.empty(T, B, E, **f32), g3=torch.empty(T, B, E, **f32),
                          dh1=torch.empty(T, B, Hb, **f32), df=torch.empty(T, B, E, **f32),
                          dcat=torch.empty(T, B, n * E, **f32), G2=torch.empty(n, T, B, E, **f32),
                          dU=torch.empty(n, T, B, E, **f32), G1=torch.empty(n, T, B, E, **f32),
                          dO=torch.empty(n, T, B, E, **f32), dQ=torch.empty(n, T, B, E, **f32),
                          dKV=[torch.empty(B, Tks[i], 2 * E, **f32) for i in range(n)],
                          de=torch.empty(T, B, E, **f32), g2=torch.empty(T, B, E, **f32),
                          du=torch.empty(T, B, E, **f32), g1=torch.empty(T, B, E, **f32),
                          dG=torch.empty(T, B, 4 * E, **f32), dlt=torch.empty(n, B, heads, T, **f32),
                          ws1=torch.empty(nblk * 2 * E, **f32), ws2=torch.empty(nblk * 2 * E, **f32),
                          wsi1=torch.empty(n, nblk * 2 * E, **f32), wsi2=torch.empty(n, nblk * 2 * E, **f32),
                          ws3=torch.empty(nblk * 2 * E, **f32),
                          carry=[torch.empty(B, E, **f32) for _ in range(4)]))
        dxt = torch.empty(T, B, E, **f32)
        _lib.check(lib.mrg_swap01(B, T, E, _ptr(dy.contiguous()), _ptr(G[-1]["dout"]), 0.0, _stream()), "swap01")

        pool = _RingPool(len(ck) * nb, lib.mrg_lstm_bwd_xbuf_bytes(B, E) // 8, dev)
        own = [None] * n
        nd = nb + len(ck) - 1
        for d in range(nd - 1, -1, -1):
            probs = [(k, c, ck[c][0], ck[c][1]) for k in range(nb) for c in [d - k] if 0 <= c < len(ck)]
            _BlockStackFn._bwd_diagonal(lib, probs, blocks, S, G, KV, Tks, pads, dxt, B, T, E, Hb, n, heads, causal,
                                        scale, len(ck), boff, dev, pool)
            for k, c, t0, t1 in probs:
                if c == 0:   # block k is done: its parameter gradients, its key / value input gradients
                    _BlockStackFn._weight_grads(lib, blocks[k], S[k], G[k], kv2, Tks, nblk, B, T, E, Hb, n, dev)
                    for i in range(n):
                        if ctx.kv_need[i]:
                            own[i] = _BlockStackFn._kv_input_grad(sinks[i], G[k]["dKV"][i], blocks[k].integ[i][0][E:],
                                                                  B, Tks[i], E, dev, own[i])
        dx = None
        if ctx.x_need:
            dx = torch.empty(B, T, E, **f32)
            _lib.check(lib.mrg_swap01(T, B, E, _ptr(dxt), _ptr(dx), 0.0, _stream()), "swap01")
        # key / value sources without a draining producer get this op's own summed gradient
        return (None, dx, *own) + (None,) * (len(ctx.needs_input_grad) - 2 - n)

    @staticmethod
    def _kv_input_grad(sink, dKV, w_kv, B, Tk, E, dev, own):
        """dkv += dKV W_kv: into the encoder output's KVSink (drained by the encoder stack's backward), or
        into this op's own gradient `own` for a source without one; returns `own`."""
        if sink is None:
            first = own is None
            if first:
                own = torch.empty(B, Tk, E, device=dev, dtype=torch.float32)
            _dx_gemm(B * Tk, E, 2 * E, _ptr(dKV), 2 * E, w_kv, _ptr(own), E, beta=0.0 if first else 1.0, device=dev)
            return own
        if sink.written == 0:
            sink.buf = torch.empty(B, Tk, E, device=dev, dtype=torch.float32)
        _dx_gemm(B * Tk, E, 2 * E, _ptr(dKV), 2 * E, w_kv, _ptr(sink.buf), E,
                 beta=0.0 if sink.written == 0 else 1.0, device=dev)
        sink.written += 1
        return own

    @staticmethod
    def _bwd_diagonal(lib, probs, blocks, S, G, KV, Tks, pads, dxt, B, T, E, Hb, n, heads, causal, scale, nck,
                      boff, dev, pool):
        D = E // heads
        groups = _by_len(probs)
        for tl, grp in groups:
            N = tl * B
            lst = [(k, c, t0 * B) for k, c, t0, t1 in grp]
            # block FeedForward: LN backward, relu'd output product, input product (+ residual)
            _bln_bwd(lib, N, E, [(_p(G[k]["dout"], r0 * E), (E, 0, 0), _p(S[k]["h2"], r0 * E), _p(S[k]["f"], r0 * E),
                                  _ptr(blocks[k].ffn[4]), _p(S[k]["m3"], r0), _p(S[k]["r3"], r0),
                                  _p(G[k]["g3"], r0 * E), _p(G[k]["ws3"], boff(c))) for k, c, r0 in lst])
            _bgemm(lib, N, Hb, E, [(_p(G[k]["g3"], r0 * E), blocks[k].ffn[2], _p(G[k]["dh1"], r0 * Hb), None,
                                    _p(S[k]["h1"], r0 * Hb)) for k, c, r0 in lst], E, Hb, epi=2, ldaux=Hb,
                   transposed=True, dev=dev)
            _bgemm(lib, N, E, Hb, [(_p(G[k]["dh1"], r0 * Hb), blocks[k].ffn[0], _p(G[k]["df"], r0 * E), None,
                                    _p(G[k]["g3"], r0 * E)) for k, c, r0 in lst], Hb, E, epi=3, ldaux=E,
                   transposed=True, dev=dev)
            _bgemm(lib, N, n * E, E, [(_p(G[k]["df"], r0 * E), blocks[k].cat_w, _p(G[k]["dcat"], r0 * n * E), None,
                                       None) for k, c, r0 in lst], E, n * E, transposed=True, dev=dev)
            # integrators, in reverse
            _bln_bwd(lib, N, E, [(_p(G[k]["dcat"], r0 * n * E + i * E), (n * E, 0, 0), _p(S[k]["Z"][i], r0 * E),
                                  _p(S[k]["U"][i], r0 * E), _ptr(blocks[k].integ[i][8]), _p(S[k]["mi2"][i], r0),
                                  _p(S[k]["ri2"][i], r0), _p(G[k]["G2"][i], r0 * E), _p(G[k]["wsi2"][i], boff(c)))
                                 for k, c, r0 in lst for i in range(n)])
            _bgemm(lib, N, E, E, [(_p(G[k]["G2"][i], r0 * E), blocks[k].integ[i][6], _p(G[k]["dU"][i], r0 * E), None,
                                   _p(G[k]["G2"][i], r0 * E)) for k, c, r0 in lst for i in range(n)], E, E, epi=3,
                   ldaux=E, transposed=True, dev=dev)
            _bln_bwd(lib, N, E, [(_p(G[k]["dU"][i], r0 * E), (E, 0, 0), _p(S[k]["A"][i], r0 * E), _p(S[k]["e"], r0 * E),
                                  _ptr(blocks[k].integ[i][4]), _p(S[k]["mi1"][i], r0), _p(S[k]["ri1"][i], r0),
                                  _p(G[k]["G1"][i], r0 * E), _p(G[k]["wsi1"][i], boff(c)))
                                 for k, c, r0 in lst for i in range(n)])
            _bgemm(lib, N, E, E, [(_p(G[k]["G1"][i], r0 * E), blocks[k].integ[i][2], _p(G[k]["dO"][i], r0 * E), None,
                                   None) for k, c, r0 in lst for i in range(n)], E, E, transposed=True, dev=dev)
            # attention: each chunk's dQ pass (+ its delta rows); after a block's last chunk (c == 0 here)
            # one dK / dV pass over the whole sequence from the stored log-sum-exp / delta rows
            for k, c, t0, t1 in grp:
                for i in range(n):
                    Tk = Tks[i]
                    args = [_ptr(KV[k][i]), Tk * 2 * E, 2 * E, _p(KV[k][i], E), Tk * 2 * E, 2 * E]
                    with Fn._probe("attn_bwd", 10.0 * D * B * heads * _chunk_pairs(t0, t1, T, Tk, causal)):
                        for q0, q1, passes in ((t0, t1, 1),) + (((0, T, 2),) if c == 0 else ()):
                            rc = lib.mrg_attention_bwd_chunk(
                                B, heads, q1 - q0, Tk, D, q0, T, _p(S[k]["Q"][i], q0 * B * E), E, B * E, *args,
                                _p(S[k]["O"][i], q0 * B * E), E, B * E, _ptr(S[k]["lse"][i]), pads[i][0], pads[i][1],
                                int(causal), scale, _p(G[k]["dO"][i], q0 * B * E), E, B * E,
                                _p(G[k]["dQ"][i], q0 * B * E), E, B * E, _ptr(G[k]["dKV"][i]), Tk * 2 * E, 2 * E,
                                _p(G[k]["dKV"][i], E), Tk * 2 * E, 2 * E, passes, 0, _ptr(G[k]["dlt"][i]), _stream())
                            _lib.check(rc, "attention bwd chunk (block stack)")
            # de = sum_i (dQ_i W_q_i + G1_i): the first integrator's product stores, the others add
            for i in range(n):
                _bgemm(lib, N, E, E, [(_p(G[k]["dQ"][i], r0 * E), blocks[k].integ[i][0][:E], _p(G[k]["de"], r0 * E),
                                       None, _p(G[k]["G1"][i], r0 * E)) for k, c, r0 in lst], E, E, epi=3, ldaux=E,
                       transposed=True, beta=0.0 if i == 0 else 1.0, dev=dev)
            # the LSTM block: LN2, FeedForward (+ residual), LN1
            _bln_bwd(lib, N, E, [(_p(G[k]["de"], r0 * E), (E, 0, 0), _p(S[k]["z"], r0 * E), _p(S[k]["u"], r0 * E),
                                  _ptr(blocks[k].lstm[8]), _p(S[k]["m2"], r0), _p(S[k]["r2"], r0),
                                  _p(G[k]["g2"], r0 * E), _p(G[k]["ws2"], boff(c))) for k, c, r0 in lst])
            _bgemm(lib, N, E, E, [(_p(G[k]["g2"], r0 * E), blocks[k].lstm[6], _p(G[k]["du"], r0 * E), None,
                                   _p(G[k]["g2"], r0 * E)) for k, c, r0 in lst], E, E, epi=3, ldaux=E, transposed=True,
                   dev=dev)
            _bln_bwd(lib, N, E, [(_p(G[k]["du"], r0 * E), (E, 0, 0), _p(S[k]["y"], r0 * E), _p(S[k]["x"], r0 * E),
                                  _ptr(blocks[k].lstm[4]), _p(S[k]["m1"], r0), _p(S[k]["r1"], r0),
                                  _p(G[k]["g1"], r0 * E), _p(G[k]["ws1"], boff(c))) for k, c, r0 in lst])
        # the recurrences of the diagonal, (dh, dc) carried from chunk c + 1
        items = []
        for k, c, t0, t1 in probs:
            cb = G[k]["carry"]
            cur, nxt = (cb[0], cb[1]) if c % 2 == 0 else (cb[2], cb[3])
            prv = (cb[2], cb[3]) if c % 2 == 0 else (cb[0], cb[1])
            dh_in, dc_in = (None, None) if c == nck - 1 else prv
            dh_out, dc_out = (None, None) if c == 0 else (cur, nxt)
            items.append((t1 - t0, (None, S[k], G[k], t0, dh_in, dc_in, dh_out, dc_out)))
        for tl, grp in _groups(items, lambda it: it[0], _maxp(B, dev)):
            _launch_bwd(lib, [it[1] for it in grp], B, tl, E, dev, pool)
        # input gradients dG W_ih + g1 (residual) -> the previous block's output gradient (or the input's)
        for tl, grp in groups:
            N = tl * B
            _bgemm(lib, N, E, 4 * E, [(_p(G[k]["dG"], t0 * B * 4 * E), blocks[k].lstm[0],
                                       _p(G[k - 1]["dout"] if k > 0 else dxt, t0 * B * E), None,
                                       _p(G[k]["g1"], t0 * B * E)) for k, c, t0, t1 in grp], 4 * E, E, epi=3,
                   ldaux=E, transposed=True, dev=dev)

    @staticmethod
    def _weight_grads(lib, bl, st, gr, kv2, Tks, nblk, B, T, E, Hb, n, dev):
        """Every parameter gradient of one block over all T * B rows, as ONE fork onto the weight-gradient
        side stream (functional._on_side)."""
        rows = T * B
        w_ih, w_hh, b_ih, b_hh, g1, be1, w_ff, b_ff, g2, be2 = bl.lstm
        gbi, gbh = _gbuf(b_ih), _gbuf(b_hh)
        keep = [st["x"], st["y"], st["u"], st["e"], st["O"], st["U"], st["cat"], st["f"], st["h1"], *kv2,
                gr["dG"], gr["g2"], gr["G2"], gr["G1"], gr["dQ"], *gr["dKV"], gr["df"], gr["dh1"], gr["g3"],
                gr["ws1"], gr["ws2"], gr["wsi1"], gr["wsi2"], gr["ws3"]]

        def wg(dY, ldy, X, ldx, m, Nout, Nin, gw, gb=None, gb2=None):
            if gw is None:
                if gb is not None:
                    Fn.colsum(m, Nout, dY, ldy, _ptr(gb), out2=_ptr(gb2), device=dev)
                return
            gemm(Nout, Nin, m, dY, 1, ldy, X, 0, ldx, _ptr(gw), Nin, beta=1.0, splits=Fn.wgrad_splits(Nout, Nin, m),
                 device=dev, asum_out=_ptr(gb), asum_out2=_ptr(gb2))

        def reduce(ws, gg, gb):
            gg, gb = _gbuf(gg), _gbuf(gb)
            if gg is None and gb is None:
                return
            scratch = Fn._ws(2 * E * 4, dev).view(2, E) if (gg is None or gb is None) else None
            _lib.check(lib.mrg_residual_layernorm_param_reduce(
                _ln_rows(lib, nblk, E), E, _ptr(ws), _ptr(gg if gg is not None else scratch[0]),
                _ptr(gb if gb is not None else scratch[1]), 1, _stream()), "layernorm param reduce")

        def sl(p, a, b):
            g = _gbuf(p)
            return None if g is None else g[a:b]

        def issue():
            # the LSTM block
            wg(_ptr(gr["dG"]), 4 * E, _ptr(st["x"]), E, rows, 4 * E, E, _gbuf(w_ih),
               gb=gbi if gbi is not None else gbh, gb2=gbh if gbi is not None else None)
            if T > 1:   # sum_t dG_t^T y_{t-1}: time-major rows shifted by one step
                wg(_p(gr["dG"], B * 4 * E), 4 * E, _ptr(st["y"]), E, (T - 1) * B, 4 * E, E, _gbuf(w_hh))
            wg(_ptr(gr["g2"]), E, _ptr(st["u"]), E, rows, E, E, _gbuf(w_ff), gb=_gbuf(b_ff))
            reduce(gr["ws1"], g1, be1)
            reduce(gr["ws2"], g2, be2)
            # the integrators
            for i in range(n):
                P = bl.integ[i]
                wg(_ptr(gr["G2"][i]), E, _ptr(st["U"][i]), E, rows, E, E, _gbuf(P[6]), gb=_gbuf(P[7]))
                reduce(gr["wsi2"][i], P[8], P[9])
                reduce(gr["wsi1"][i], P[4], P[5])
                wg(_ptr(gr["G1"][i]), E, _ptr(st["O"][i]), E, rows, E, E, _gbuf(P[2]), gb=_gbuf(P[3]))
                wg(_ptr(gr["dQ"][i]), E, _ptr(st["e"]), E, rows, E, E, sl(P[0], 0, E), gb=sl(P[1], 0, E))
                wg(_ptr(gr["dKV"][i]), 2 * E, _ptr(kv2[i]), E, B * Tks[i], 2 * E, E, sl(P[0], E, 3 * E),
                   gb=sl(P[1], E, 3 * E))
            wg(_ptr(gr["df"]), E, _ptr(st["cat"]), n * E, rows, E, n * E, _gbuf(bl.cat_w), gb=_gbuf(bl.cat_b))
            # the FeedForward
            wg(_ptr(gr["g3"]), E, _ptr(st["h1"]), Hb, rows, E, Hb, _gbuf(bl.ffn[2]), gb=_gbuf(bl.ffn[3]))
            wg(_ptr(gr["dh1"]), Hb, _ptr(st["f"]), E, rows, Hb, E, _gbuf(bl.ffn[0]), gb=_gbuf(bl.ffn[1]))
            reduce(gr["ws3"], bl.ffn[4], bl.ffn[5])
        _on_side(dev, rows, keep, issue)


def _chunk_pairs(t0, t1, T, Tk, causal):
    """Visible (query, key) pairs of queries [t0, t1) per (sample, head) under the block-causal rule."""
    if not causal:
        return (t1 - t0) * Tk
    if Tk >= T:
        r = Tk // T
        return sum(min((i + 1) * r, Tk) for i in range(t0, t1))
    r = T // Tk
    return sum(i // r + 1 for i in range(t0, t1))


def block_stack(x, kvs, qpads, kpads, blocks: Sequence[Sequence[torch.Tensor]], heads, causal, eps, sinks,
                chunk: int = 0) -> torch.Tensor:
    """Blocks 1.. of the metaformer as one (block, chunk) wavefront op; see the module docstring.
    blocks[k] = the 10 + 10 n + 2 + 6 parameters of block k (_Block order); qpads / kpads: each
    integrator's padding flags (gen_attention_mask's per-modality masks)."""
    n = len(kvs)
    flat = [x, *kvs, *qpads, *kpads]
    for b in blocks:
        flat += list(b)
    return _BlockStackFn.apply((len(blocks), n, int(heads), bool(causal), float(eps), int(chunk or CHUNK),
                                list(sinks)), *flat)
