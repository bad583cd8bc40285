"""lstmformer generation with the frame loop on the fused per-frame kernels (gen.hip).

Reference: Metaformer.prediction -> head_motion_generation -> generate_one_step
(mr_gen/model/lstmformer/lstmformer.py:426-521, form_generation_init :523-547).  Every frame is a
T = 1 forward of the whole model with zero recurrent state and empty lead inputs; the
frame's self-motion input is the previous prediction (mask true) or motion_s one frame late.

What this module hoists out of the frame loop (inference only, no autograd), because it does not
depend on the previous frame:

* the other modalities' block-0 encoders (feature Linear + every LSTM mixer block of the audio and
  partner-motion stacks), as [T * B]-row GEMMs, zero-state LSTM cells and LayerNorms;
* with one audio frame per prediction frame (ratio 1), each block's integrator attention output:
  the query sees exactly one key (generation zeroes the -100 padding, so no key is ever masked, and
  the block-causal rule admits key 0 for query 0), so the softmax weight is exactly 1 and
  MHA(q, kv) = out_proj(V(kv)) for any q -- two more [T * B]-row GEMMs per integrator.

The frame loop then runs the main chain only: five gen.hip launches per block and one for the
output FeedForward with the sampling select (6 x 5 + 1 = 26 per frame instead of ~145), every
LayerNorm computed in the prologue of the launch that consumes it.  Forms outside this plan (ratio
> 1, widths other than E = 256 / bottleneck 64, GRU mixers, grad enabled) return None and the caller
runs the per-frame module forward.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch
from torch import nn

from . import _lib
from . import functional as Fn
from .functional import _ptr, _stream

F32 = torch.float32
E_GEN, HB_GEN = 256, 64
# the whole frame loop as ONE persistent launch (gen.hip gen_loop_kernel) when its grid fits;
# MRG_GEN_LOOP=0 keeps the 26 launches per frame
_LOOP = [os.environ.get("MRG_GEN_LOOP", "1") == "1"]


def _arr(*ts):
    return (ctypes.c_void_p * len(ts))(*[t if isinstance(t, ctypes.c_void_p) else _ptr(t) for t in ts])


def _ffn_parts(ff, residual: bool):
    """(w1, b1, w2, b2[, ln]) of a FeedForward Linear -> ReLU -> Linear (with its residual LayerNorm)."""
    seq = ff.feed_forward
    ln = None
    if residual:
        from .model.layers import ResidualConnection
        if not isinstance(seq, ResidualConnection) or seq.layer_norm is None:
            return None
        ln, seq = seq.layer_norm, seq.module
    mods = list(seq.children())
    if len(mods) != 3 or not isinstance(mods[1], nn.ReLU) or any(m.bias is None for m in (mods[0], mods[2])):
        return None
    return mods[0].weight, mods[0].bias, mods[2].weight, mods[2].bias, ln


class GenPlan:
    """The parameters of Metaformer.metaformer arranged for the fused frame loop, or ``ok = False``."""

    def __init__(self, mf, ratio: int):
        self.ok = False
        if ratio != 1 or mf.interlayer_residual or mf.repeat_with_encoder or mf.hidden_dim != E_GEN:
            return
        if not mf._fast_eligible():
            return
        blocks = list(mf.metaformer_blocks)
        first = mf._stack_layers(blocks[0])
        if first is None or len(first[0]) != 3:
            return
        layers0, eps = first
        self.eps = eps
        self.enc = layers0[1:]                   # block 0's audio / partner-motion stacks
        self.fe = list(mf.feature_embedding)
        if any(e.bias is None for e in self.fe):
            return
        self.blocks = []
        dummy = torch.empty(1, 1, E_GEN, device=self.fe[0].weight.device)
        for bi, blk in enumerate(blocks):
            got = mf._stack_layers(blk) if bi else first
            if got is None or len(got[0][0]) != 1 or got[1] != eps or any(v is None for v in got[0][0][0]):
                return
            args = blk.integrator.fused_args(dummy, [dummy, dummy], [None, None], [None, None])
            if args is None or len(args[0]) != 2 or args[5] != eps:
                return
            ffn = _ffn_parts(blk.feedforward, True)
            if ffn is None or ffn[0].shape[0] != HB_GEN or ffn[4].eps != eps:
                return
            self.blocks.append({"lstm": got[0][0][0], "integ": args[0], "cat": (args[1], args[2]), "ffn": ffn})
        out = _ffn_parts(mf.output_feedforward, False)
        if out is None or out[0].shape[0] != HB_GEN or out[2].shape[0] > 16:
            return
        self.out = out
        self.fm = out[2].shape[0]
        if self.fe[0].weight.shape[1] != self.fm:
            return
        self.ok = True

    # ---- frame-independent work over all T frames ([T * B] rows, time-major)
    def _encoder(self, x, layers):
        lib = _lib.load()
        N, H = x.shape[0], E_GEN
        gates = torch.empty(N, 4 * H, device=x.device, dtype=F32)
        c = torch.empty(N, H, device=x.device, dtype=F32)
        for w_ih, _w_hh, b_ih, b_hh, l1w, l1b, fw, fb, l2w, l2b in layers:
            g = Fn.linear(x, w_ih, b_ih)
            h = torch.empty(N, H, device=x.device, dtype=F32)
            _lib.check(lib.mrg_lstm_cell_fwd(N, H, _ptr(g), 4 * H, _ptr(b_hh), None, _ptr(gates), _ptr(c), _ptr(h),
                                             H, None, _stream()), "gen encoder cell")
            y = Fn.residual_layernorm(h, x, l1w, l1b, self.eps)
            x = Fn.residual_layernorm(Fn.linear(y, fw, fb), y, l2w, l2b, self.eps)
        return x

    def generate(self, fb, mp, ms, mask):
        """fb [T][B][1][Fa], mp / ms [T][B][1][fm] (time-major, padding zeroed), mask [T] bool ->
        prediction [B, T, fm]."""
        lib = _lib.load()
        T, B = ms.shape[0], ms.shape[1]
        dev = ms.device
        E, eps = E_GEN, self.eps
        others = [self._encoder(Fn.linear(x.reshape(T * B, -1), e.weight, e.bias), layers)
                  for x, e, layers in zip((fb, mp), self.fe[1:], self.enc)]
        # per block and integrator: out_proj(V(kv)), the attention output at one visible key
        att = []
        for blk in self.blocks:
            att.append([Fn.linear(Fn.linear(kv, iw[2 * E:], ib[2 * E:]), ow, ob)
                        for kv, (iw, ib, ow, ob, *_r) in zip(others, blk["integ"])])
        msc = ms.reshape(T, B, self.fm).contiguous()
        # the kernel reads one byte per frame (a device bool tensor as it is: refreshed per graph replay)
        mask_u8 = mask if (mask.device == dev and mask.dtype in (torch.bool, torch.uint8)) \
            else mask.to(device=dev, dtype=torch.uint8)
        pred = torch.empty(B, T, self.fm, device=dev, dtype=F32)
        ms_in = torch.empty(B, self.fm, device=dev, dtype=F32)
        xb, hh, y, z, m3, zf = (torch.empty(B, E, device=dev, dtype=F32) for _ in range(6))
        y01, z01 = (torch.empty(B, 2 * E, device=dev, dtype=F32) for _ in range(2))
        st = _stream()
        fe0 = self.fe[0]
        if _LOOP[0] and lib.mrg_gen_loop_fits(B, _lib.cu_count(dev.index or 0)) == 1:
            return self._generate_loop(lib, B, T, att, msc, mask_u8, pred, st)
        # argument tuples made once (the frame loop only varies the frame pointers)
        calls = []
        for bi, blk in enumerate(self.blocks):
            w_ih, _w_hh, b_ih, b_hh, l1w, l1b, fw, fbias, l2w, l2b = blk["lstm"]
            i0, i1 = blk["integ"]
            cw, cb = blk["cat"]
            w1, b1, w2, b2, fln = blk["ffn"]
            prev = self.blocks[bi - 1]["ffn"][4] if bi else None
            calls.append(dict(
                lstm=(w_ih, b_ih, b_hh, prev),
                lin0=(_arr(hh), _arr(xb), _arr(l1w), _arr(l1b), _arr(fw), _arr(fbias)),
                lin1=(_arr(z), _arr(y), _arr(l2w), _arr(l2b), _arr(i0[4], i1[4]), _arr(i0[5], i1[5]),
                      _arr(i0[6], i1[6]), _arr(i0[7], i1[7])),
                lin2=(_arr(_ptr(z01), _ptr(z01, E)), _arr(_ptr(y01), _ptr(y01, E)), _arr(i0[8], i1[8]),
                      _arr(i0[9], i1[9]), _arr(cw), _arr(cb)),
                ffn=(w1, b1, w2, b2)))
        ow1, ob1, ow2, ob2, _ = self.out
        lastln = self.blocks[-1]["ffn"][4]
        # algorithmic FLOPs of each launch (2 x rows x outputs x K; the LayerNorms are O(rows x E))
        f_lstm, f_lin0 = 2.0 * B * 4 * E * E, 2.0 * B * E * E
        f_lin1, f_lin2 = 2.0 * B * 2 * E * E, 2.0 * B * E * 2 * E
        f_ffn, f_out = 2.0 * B * HB_GEN * (E + E), 2.0 * B * HB_GEN * (E + self.fm)
        for t in range(T):
            for bi, c in enumerate(calls):
                w_ih, b_ih, b_hh, prev = c["lstm"]
                if bi == 0:
                    src = msc[0] if t == 0 else ms_in
                    with Fn._probe("gen", f_lstm + 2.0 * B * E * self.fm):
                        _lib.check(lib.mrg_gen_lstm(B, self.fm, _ptr(src), _ptr(fe0.weight), _ptr(fe0.bias), None, None,
                                                    None, None, eps, _ptr(xb), _ptr(w_ih), _ptr(b_ih), _ptr(b_hh),
                                                    _ptr(hh), st), "gen lstm")
                else:
                    with Fn._probe("gen", f_lstm):
                        _lib.check(lib.mrg_gen_lstm(B, self.fm, None, None, None, _ptr(zf), _ptr(m3),
                                                    _ptr(prev.weight), _ptr(prev.bias), eps, _ptr(xb), _ptr(w_ih),
                                                    _ptr(b_ih), _ptr(b_hh), _ptr(hh), st), "gen lstm")
                a, r, ga, be, w, bias = c["lin0"]
                with Fn._probe("gen", f_lin0):
                    _lib.check(lib.mrg_gen_linear(0, B, a, r, ga, be, E, None, None, None, eps, _ptr(y), E, w, bias,
                                                  _ptr(z), E, st), "gen mixer linear")
                a, r, ga, be, ga2, be2, w, bias = c["lin1"]
                a2 = _arr(_ptr(att[bi][0], t * B * E), _ptr(att[bi][1], t * B * E))
                with Fn._probe("gen", f_lin1):
                    _lib.check(lib.mrg_gen_linear(1, B, a, r, ga, be, E, a2, ga2, be2, eps, _ptr(y01), 2 * E, w,
                                                  bias, _ptr(z01), 2 * E, st), "gen integrators")
                a, r, ga, be, w, bias = c["lin2"]
                with Fn._probe("gen", f_lin2):
                    _lib.check(lib.mrg_gen_linear(2, B, a, r, ga, be, 2 * E, None, None, None, eps, None, 0, w, bias,
                                                  _ptr(m3), E, st), "gen cat_linear")
                w1, b1, w2, b2 = c["ffn"]
                with Fn._probe("gen", f_ffn):
                    _lib.check(lib.mrg_gen_ffn(B, E, _ptr(m3), None, None, None, eps, _ptr(w1), _ptr(b1), _ptr(w2),
                                               _ptr(b2), _ptr(zf), None, 0, None, None, None, t, st), "gen ffn")
            with Fn._probe("gen", f_out):
                _lib.check(lib.mrg_gen_ffn(B, self.fm, _ptr(zf), _ptr(m3), _ptr(lastln.weight), _ptr(lastln.bias),
                                           eps, _ptr(ow1), _ptr(ob1), _ptr(ow2), _ptr(ob2), None, _ptr(pred),
                                           T * self.fm, _ptr(ms_in), _ptr(msc[t]), _ptr(mask_u8), t, st),
                           "gen output")
        return pred

    def _generate_loop(self, lib, B, T, att, msc, mask_u8, pred, st):
        """The frame loop in one persistent launch (mrg_gen_loop; pointer table order in include/mrg.h)."""
        ptrs = []
        for bi, blk in enumerate(self.blocks):
            w_ih, _w_hh, b_ih, b_hh, l1w, l1b, fw, fbias, l2w, l2b = blk["lstm"]
            i0, i1 = blk["integ"]
            cw, cb = blk["cat"]
            w1, b1, w2, b2, fln = blk["ffn"]
            ptrs += [w_ih, b_ih, b_hh, l1w, l1b, fw, fbias, l2w, l2b]
            for ip in (i0, i1):
                ptrs += [ip[4], ip[5], ip[6], ip[7], ip[8], ip[9]]
            ptrs += [cw, cb, w1, b1, w2, b2, fln.weight, fln.bias, att[bi][0], att[bi][1]]
        ow1, ob1, ow2, ob2, _ = self.out
        fe0 = self.fe[0]
        ptrs += [fe0.weight, fe0.bias, ow1, ob1, ow2, ob2]
        ring = Fn.zeros(max(1, lib.mrg_gen_loop_ring_bytes(B) // 8), dtype=torch.int64, device=msc.device)
        E = E_GEN
        flop = T * (len(self.blocks) * 2.0 * B * (4 * E * E + E * E + 2 * E * E + 2 * E * E + 2 * HB_GEN * E)
                    + 2.0 * B * HB_GEN * (E + self.fm))
        with Fn._probe("gen", flop):
            _lib.check(lib.mrg_gen_loop(B, T, self.fm, len(self.blocks), self.eps, _arr(*ptrs), len(ptrs), _ptr(msc),
                                        _ptr(mask_u8), _ptr(pred), _ptr(ring), _ptr(Fn._err_flag(msc.device)), st),
                       "gen loop")
        return pred


_PLANS = {}


def plan_for(model) -> Optional[GenPlan]:
    """The model's GenPlan (cached per module identity and parameter storage), or None outside it."""
    mf = model.metaformer
    key = (id(mf), mf.feature_embedding[0].weight.data_ptr(), model.ratio)
    p = _PLANS.get(key)
    if p is None:
        p = GenPlan(mf, model.ratio)
        _PLANS.clear()
        _PLANS[key] = p
    return p if p.ok else None
