"""Multi-modal metaformer (reference: mr_gen/model/utils/multi_modal_metaformer.py).

Module tree, constructor arguments and state_dict names follow the reference
(MultiModalEmbedding / IntegrateModalBlock / MultiModalMetaformerBlock /
MultiModalMetaformer).  ``MultiModalMetaformer.forward`` has one MI355X-
specific schedule: in the first block the per-modality LSTM encoders advance
layer by layer and every group of same-shape layers runs as ONE persistent
recurrence launch (main + audio + partner at layer 0, audio + partner above),
which is legal because the reference's recurrent state is never carried
 and the encoders are independent until the integrator.
"""
from __future__ import annotations

import os
from typing import Any, List, Tuple

import torch
from torch import nn

from .. import functional as Fn
from .layers import Linear, FeedForward, ResidualConnection
from .masks import gen_attention_mask  # noqa: F401  (re-export, reference location)
from .mixers import (MixerLayerdFactory, LSTMMixerLayerd, MHAMixerLayerd, LSTMMixerBlock,
                     split_state)


def check_form_modal_num(modal_num: int, sameone, msg: str = None) -> list:
    if not isinstance(sameone, (list, tuple)):
        raise TypeError(f"must be list or tuple. but got {type(sameone)}")
    if modal_num != len(sameone):
        if len(sameone) != 1:
            raise ValueError("" if msg is None else msg)
        sameone = list(sameone) * modal_num
    return sameone



# the fused integrator also serves the T = 1 frames of autoregressive generation (one launch per
# batched projection / LayerNorm instead of per-integrator modules, no mask or concat glue);
# MRG_FUSED_T1=0 keeps those frames on the per-module path
_FUSED_MIN_T = 1 if os.environ.get("MRG_FUSED_T1", "1") == "1" else 2

class MultiModalEmbedding(nn.Module):
    def __init__(self, modal_num: int, mixer_configs):
        super().__init__()
        self.modal_num = modal_num
        self.mixer_configs = check_form_modal_num(modal_num, mixer_configs,
                                                  "modal_num must be equal to the length of mixer_configs.")
        factory = MixerLayerdFactory()
        self.modal_embeddings = nn.ModuleList([factory.build(*c) for c in self.mixer_configs])

    def forward(self, x, hx=None, other=None):
        x = check_form_modal_num(self.modal_num, x, "The length of x must be equal to modal_num.")
        hx = [None] * self.modal_num if hx is None else hx
        other = [(None,)] * self.modal_num if other is None else other
        ys, states = [], []
        for i, emb in enumerate(self.modal_embeddings):
            out = emb(x[i], hx[i], other[i])
            ys.append(out[0])
            states.append(out[1])
        return (ys, states)


class IntegrateModalBlock(nn.Module):
    """Cross-attend the main modality to each other modality, concat, cat_linear (:128-217)."""

    def __init__(self, modal_num: int, mixer_configs, output_dim: int):
        super().__init__()
        self.modal_num = modal_num
        self.mixer_configs = check_form_modal_num(modal_num - 1, mixer_configs,
                                                  "modal_num must be equal to the length + 1 of mixer_configs.")
        factory = MixerLayerdFactory()
        self.integrators = nn.ModuleList()
        width = 0
        for kind, cfg in self.mixer_configs:
            if kind != "mha":
                raise TypeError("IntegrateModalBlock only supports mha mixer.")
            self.integrators.append(factory.build(kind, cfg))
            width += cfg["output_projection_size"] if cfg.get("output_projection") else cfg["hidden_size"]
        self.cat_linear = Linear(width, output_dim)

    def check_form_input(self, other_modals, attn_mask, hx=None):
        other_modals = [other_modals] if isinstance(other_modals, torch.Tensor) else other_modals
        other_modals = check_form_modal_num(self.modal_num - 1, other_modals,
                                            "The length of other_modals must be equal to modal_num - 1.")
        attn_mask = [None] * (self.modal_num - 1) if attn_mask is None else attn_mask
        attn_mask = [attn_mask] if not isinstance(attn_mask, (list, tuple)) else attn_mask
        attn_mask = check_form_modal_num(self.modal_num - 1, attn_mask,
                                         "The length of attn_mask must be equal to modal_num - 1.")
        hx = [None] * (self.modal_num - 1) if hx is None else hx
        return other_modals, attn_mask, hx

    # ---- MI355X schedule: every integrator + the concat + cat_linear as one fused op (integrate.py)
    use_fused = os.environ.get("MRG_FUSED_INTEGRATOR", "1") == "1"

    def _fused(self, main_modal, other_modals, attn_mask, hxs):
        """integrate.integrate(...) when the block is inside its form (single-block MHA layerds with
        residual LN, one-Linear residual-LN FeedForward, block-causal or no mask, no state), else None."""
        from ..integrate import integrate
        args = self.fused_args(main_modal, other_modals, attn_mask, hxs)
        if args is None:
            return None
        params, cw, cb, heads, causal, eps, qpads, kpads = args
        return integrate(main_modal, list(other_modals), qpads, kpads, params, cw, cb, heads, causal, eps)

    def fused_args(self, main_modal, other_modals, attn_mask, hxs):
        """(per-integrator parameter tuples, cat_w, cat_b, heads, causal, eps, qpads, kpads) of the fused
        form (integrate.py), or None when the block is outside it."""
        from .masks import BlockCausalMask
        if not (self.use_fused and isinstance(main_modal, torch.Tensor) and main_modal.is_cuda
                and main_modal.dim() == 3 and main_modal.shape[1] >= _FUSED_MIN_T and all(h is None for h in hxs)):
            return None
        B, T, E = main_modal.shape
        n = len(self.integrators)
        cw = self.cat_linear.weight
        if self.cat_linear.bias is None or tuple(cw.shape) != (E, n * E):
            return None
        params, heads, eps, masks = [], set(), set(), []
        for integ, kv, m in zip(self.integrators, other_modals, attn_mask):
            if (integ.input_projection is not None or integ.output_projection is not None or integ.self_attention
                    or len(integ.mixer) != 1):
                return None
            blk = integ.mixer[0]
            res, ffw = blk.mixer, getattr(blk.feed_forward, "feed_forward", None)
            if not (isinstance(res, ResidualConnection) and res.layer_norm is not None and len(res.module.mixer) == 1):
                return None
            mha = res.module.mixer[0].mha
            if (not mha.batch_first or (mha.dropout and mha.training) or mha.in_proj_bias is None
                    or tuple(mha.in_proj_weight.shape) != (3 * E, E) or mha.out_proj.bias is None
                    or getattr(mha, "bias_k", None) is not None):
                return None
            if not (isinstance(ffw, ResidualConnection) and ffw.layer_norm is not None):
                return None
            mods = list(ffw.module.children())
            if len(mods) != 1 or not isinstance(mods[0], nn.Linear) or mods[0].bias is None:
                return None
            if not (isinstance(kv, torch.Tensor) and kv.dim() == 3 and kv.shape[0] == B and kv.shape[2] == E
                    and kv.is_cuda):
                return None
            if m is not None and not isinstance(m, BlockCausalMask):
                return None
            heads.add(mha.num_heads)
            eps.update((res.layer_norm.eps, ffw.layer_norm.eps))
            masks.append(m)
            params.append((mha.in_proj_weight, mha.in_proj_bias, mha.out_proj.weight, mha.out_proj.bias,
                           res.layer_norm.weight, res.layer_norm.bias, mods[0].weight, mods[0].bias,
                           ffw.layer_norm.weight, ffw.layer_norm.bias))
        if len(heads) != 1 or len(eps) != 1 or E % next(iter(heads)) != 0:
            return None
        causal = masks[0] is not None
        if any((m is not None) != causal for m in masks):
            return None
        qpads = [m.main_pad if causal else None for m in masks]
        kpads = [m.other_pad if causal else None for m in masks]
        return params, cw, self.cat_linear.bias, heads.pop(), causal, eps.pop(), qpads, kpads

    def forward(self, main_modal, other_modals, attn_mask=None, hxs=None):
        other_modals, attn_mask, hxs = self.check_form_input(other_modals, attn_mask, hxs)
        out = self._fused(main_modal, other_modals, attn_mask, hxs)
        if out is not None:
            return (out, [None] * (self.modal_num - 1))
        ys, states = [], []
        for i, integ in enumerate(self.integrators):
            y, st, _ = integ(main_modal, hxs[i], other_modals[i], other_modals[i], attn_mask[i])
            ys.append(y)
            states.append(st)
        return (self.cat_linear(torch.cat(ys, dim=-1)), states)


class MultiModalMetaformerBlock(nn.Module):
    """embedding -> integrator -> FeedForward (:220-338)."""

    def __init__(self, num_modal: int, main_modal_embedding_config, integrate_configs, feedforward_configs: dict,
                 encode_other_modal: bool = False, other_modal_embedding_config=None):
        super().__init__()
        if not encode_other_modal or other_modal_embedding_config is None:
            other_modal_embedding_config = []
        if isinstance(main_modal_embedding_config, tuple):
            main_modal_embedding_config = [main_modal_embedding_config]
        if encode_other_modal:
            other_modal_embedding_config = check_form_modal_num(
                num_modal - 1, other_modal_embedding_config,
                "The length of other_modal_embedding_config must be equal to num_modal - 1.")
        integrate_configs = check_form_modal_num(num_modal - 1, integrate_configs,
                                                 "The length of integrate_configs must be equal to num_modal - 1.")
        self.num_modal = num_modal
        self.emb_num_modal = num_modal if encode_other_modal else 1
        self.encode_other_modal = encode_other_modal
        self.embedding_configs = list(main_modal_embedding_config) + list(other_modal_embedding_config)
        self.emb_mixer_type = [c[0] for c in self.embedding_configs]
        self.embedding = MultiModalEmbedding(self.emb_num_modal, self.embedding_configs)
        self.integrator = IntegrateModalBlock(num_modal, integrate_configs, feedforward_configs["hidden_size"])
        self.feedforward = FeedForward(**feedforward_configs)

    def forward(self, main_modal, other_modals=None, hx=None, prev_hx=None, main_modal_others=None,
                other_modals_others=None, integrate_attn_mask=None):
        if isinstance(main_modal, tuple):
            (main_modal, other_modals, hx, prev_hx, main_modal_others, other_modals_others,
             integrate_attn_mask) = main_modal
        first, hx, prev_hx = split_state(hx, prev_hx)
        if first is None:
            first = {"emb": None, "crm": None}
        other_modals_others = other_modals_others if other_modals_others else [None]
        other_modals_others = check_form_modal_num(self.num_modal - 1, other_modals_others,
                                                   "The length of other_modals_others must be equal to num_modal - 1.")
        mods = [main_modal] + (list(other_modals) if self.encode_other_modal else [])
        others = [main_modal_others] + list(other_modals_others)
        mods, emb_states = self.embedding(mods, first["emb"], others)
        main_modal = mods[0]
        if self.encode_other_modal:
            other_modals = mods[1:]
        main_modal, crm = self.integrator(main_modal, other_modals, integrate_attn_mask, first["crm"])
        prev_hx.append({"emb": emb_states, "crm": crm})
        main_modal = self.feedforward(main_modal)
        return (main_modal, other_modals, hx, prev_hx, main_modal_others, other_modals_others,
                integrate_attn_mask)


def _lstm_block_tail(block: LSTMMixerBlock, y, x):
    """Residual LN of the LSTM output, then the block's FeedForward."""
    y = block.mixer.combine(y, x)
    return block.feed_forward(y)


class MultiModalMetaformer(nn.Module):
    """Feature projections, metaformer blocks, output FFN (:341-509)."""

    def __init__(self, modal_num: int, hidden_dim: int, num_layer: int, main_modal_feature_dim,
                 main_mixer_type, main_mixer_configs, integrate_mixer_configs, feedforward_configs: dict,
                 output_feedforward_configs: dict, other_modal_feature_dim=None, other_mixer_type="mha",
                 other_mixer_configs=None, repeat_with_encoder: bool = False,
                 interlayer_residual: bool = False, interlayer_residual_norm: bool = True):
        super().__init__()
        if isinstance(main_modal_feature_dim, (list, tuple)):
            main_modal_feature_dim = main_modal_feature_dim[0]
        if isinstance(main_mixer_type, (list, tuple)):
            main_mixer_type = main_mixer_type[0]
        if isinstance(main_mixer_configs, (list, tuple)):
            main_mixer_configs = main_mixer_configs[0]
        main_cfgs = [(main_mixer_type, main_mixer_configs)]
        if isinstance(integrate_mixer_configs, dict):
            integrate_mixer_configs = [integrate_mixer_configs]
        integrate_mixer_configs = check_form_modal_num(modal_num - 1, integrate_mixer_configs,
                                                       "The length of integrate_mixer_configs must be equal to modal_num - 1.")
        integ_cfgs = [("mha", c) for c in integrate_mixer_configs]
        if isinstance(other_modal_feature_dim, int):
            other_modal_feature_dim = [other_modal_feature_dim]
        other_modal_feature_dim = check_form_modal_num(modal_num - 1, other_modal_feature_dim,
                                                       "The length of other_modal_feature_dim must be equal to modal_num - 1.")
        if isinstance(other_mixer_type, str):
            other_mixer_type = [other_mixer_type]
        other_mixer_type = check_form_modal_num(modal_num - 1, other_mixer_type,
                                                "The length of other_mixer_type must be equal to modal_num - 1.")
        if isinstance(other_mixer_configs, dict):
            other_mixer_configs = [other_mixer_configs]
        other_mixer_configs = check_form_modal_num(modal_num - 1, other_mixer_configs,
                                                   "The length of other_mixer_configs must be equal to modal_num - 1.")
        other_cfgs = [(other_mixer_type[i], other_mixer_configs[i]) for i in range(modal_num - 1)]
        self.modal_num, self.hidden_dim, self.num_layer = modal_num, hidden_dim, num_layer
        self.repeat_with_encoder, self.interlayer_residual = repeat_with_encoder, interlayer_residual
        self.embedding_mixer_type = [main_mixer_type] + list(other_mixer_type)
        self.feature_embedding = nn.ModuleList(
            [Linear(d, hidden_dim) for d in [main_modal_feature_dim] + list(other_modal_feature_dim)])
        blocks = [MultiModalMetaformerBlock(modal_num, main_cfgs, integ_cfgs, feedforward_configs,
                                            encode_other_modal=True, other_modal_embedding_config=other_cfgs)]
        for _ in range(num_layer - 1):
            blocks.append(MultiModalMetaformerBlock(modal_num, main_cfgs, integ_cfgs, feedforward_configs,
                                                    encode_other_modal=repeat_with_encoder,
                                                    other_modal_embedding_config=other_cfgs if repeat_with_encoder else None))
        self.metaformer_blocks = nn.ModuleList(
            [ResidualConnection(b, interlayer_residual_norm, hidden_dim) if interlayer_residual else b
             for b in blocks])
        self.output_feedforward = FeedForward(**output_feedforward_configs)

    # ---- MI355X schedule for the first block's embedding (batched recurrences)
    def _fast_first_embedding(self, block: MultiModalMetaformerBlock, mods: List[torch.Tensor]):
        layerds = list(block.embedding.modal_embeddings)
        if not all(isinstance(l, LSTMMixerLayerd) and l.input_projection is None and l.output_projection is None
                   for l in layerds):
            return None
        chains = [list(l.mixer) for l in layerds]
        if not all(isinstance(m, LSTMMixerBlock) and isinstance(m.mixer, ResidualConnection) for c in chains for m in c):
            return None
        xs = list(mods)
        depth = max(len(c) for c in chains)
        for layer in range(depth):
            active = [i for i, c in enumerate(chains) if layer < len(c)]
            groups = {}
            for i in active:
                groups.setdefault((tuple(xs[i].shape), chains[i][layer].lstm_params()[1].shape[1]), []).append(i)
            for idxs in groups.values():
                # at most two recurrences per launch: two batch-tile-2 problems fill the chip's
                # 512 resident workgroups; three would need batch tiles of 4 (longer GEMV per step)
                for start in range(0, len(idxs), 2):
                    part = idxs[start:start + 2]
                    # LN(LSTM(x) + x) fused per problem, then each block's FeedForward (fused too)
                    probs = []
                    for i in part:
                        ln = chains[i][layer].mixer.layer_norm
                        probs.append((xs[i], *chains[i][layer].lstm_params(), ln.weight, ln.bias, ln.eps))
                    us = Fn.lstm_layers_batched(probs)
                    for i, u in zip(part, us):
                        xs[i] = chains[i][layer].feed_forward(u)
        return xs

    # ---- MI355X schedule: block 0's embedding stacks as one layer-wavefront (encoder_stack.py: one
    # recurrence launch and batched GEMM / LayerNorm launches per (layer, time chunk) diagonal); on by
    # default (measured 27.6 -> 26.0 ms/step), MRG_ENCODER_STACK=0 keeps the per-layer schedule
    use_encoder_stack = os.environ.get("MRG_ENCODER_STACK", "1") == "1"

    def _stack_layers(self, block: MultiModalMetaformerBlock):
        """Per modality the (w_ih, w_hh, b_ih, b_hh, ln1, ff, ln2) tensors of block 0's LSTM blocks, or
        None when a block is outside the stack's form (LSTM 1-layer unidirectional H -> H, residual LN,
        FeedForward = one Linear + residual LN, one LayerNorm eps)."""
        from torch import nn as _nn
        out, eps = [], set()
        for lay in block.embedding.modal_embeddings:
            layers = []
            for mb in lay.mixer:
                lstm = mb.mixer.module.mixer if isinstance(mb.mixer, ResidualConnection) else None
                ff = getattr(mb.feed_forward, "feed_forward", None)
                if lstm is None or lstm.num_layers != 1 or lstm.bidirectional or mb.mixer.layer_norm is None:
                    return None
                if lstm.input_size != lstm.hidden_size or not isinstance(ff, ResidualConnection) or ff.layer_norm is None:
                    return None
                mods = list(ff.module.children())
                if len(mods) != 1 or not isinstance(mods[0], _nn.Linear) or mods[0].bias is None:
                    return None
                ln1, ln2 = mb.mixer.layer_norm, ff.layer_norm
                eps.update((ln1.eps, ln2.eps))
                layers.append((*lstm.direction_params(0), ln1.weight, ln1.bias, mods[0].weight, mods[0].bias,
                               ln2.weight, ln2.bias))
            out.append(layers)
        if len(eps) != 1:
            return None
        return out, eps.pop()

    def _stack_first_block(self, block, feats):
        """Block 0's embeddings (feature Linear + every LSTM block of every modality) as one wavefront, or
        None when outside it (the per-layer schedule below then runs)."""
        from ..encoder_stack import encoder_stack, stack_eligible
        if not (self.use_encoder_stack and block.encode_other_modal and len(feats) == self.modal_num):
            return None
        got = self._stack_layers(block)
        if got is None:
            return None
        layers, eps = got
        H = self.hidden_dim
        if not (stack_eligible(H, feats[0].shape[0]) and all(f.dim() == 3 and f.is_cuda and f.shape[1] >= 8
                                                             and f.shape[0] == feats[0].shape[0] for f in feats)):
            return None
        if any(f.requires_grad for f in feats):   # the stack returns no feature gradient (features are data)
            return None
        embs = list(self.feature_embedding)
        if any(e.bias is None for e in embs):
            return None
        return encoder_stack([(f, e.weight, e.bias, l) for f, e, l in zip(feats, embs, layers)], eps)

    def _fast_eligible(self) -> bool:
        if self.interlayer_residual:
            return False
        for block in self.metaformer_blocks:
            for lay in block.embedding.modal_embeddings:
                if not (isinstance(lay, LSTMMixerLayerd) and lay.input_projection is None
                        and lay.output_projection is None):
                    return False
                for m in lay.mixer:
                    if not (isinstance(m, LSTMMixerBlock) and isinstance(m.mixer, ResidualConnection)
                            and m.mixer.layer_norm is not None):
                        return False
        return True

    def forward(self, main_modal, other_modals, hx=None, main_modal_others=None, other_modals_others=None,
                integrate_attn_mask=None):
        """Returns (main, other_modals, per-block state record) like the reference (:476-509).

        The record the reference returns holds only None leaves (states are never
        produced), and feeding it back is stateless; both are mirrored.
        """
        fast = _none_leaves(hx) and _none_leaves(main_modal_others) and _none_leaves(other_modals_others) \
            and self._fast_eligible()
        stacked = self._stack_first_block(self.metaformer_blocks[0], [main_modal] + list(other_modals)) \
            if fast else None
        if stacked is None:
            main_modal = self.feature_embedding[0](main_modal)
            other_modals = [self.feature_embedding[i + 1](o) for i, o in enumerate(other_modals)]
        if fast:
            record = []
            for bi, block in enumerate(self.metaformer_blocks):
                mods = [main_modal] + (list(other_modals) if block.encode_other_modal else [])
                enc = stacked if (bi == 0 and stacked is not None) else self._fast_first_embedding(block, mods)
                main_modal = enc[0]
                if block.encode_other_modal:
                    other_modals = enc[1:]
                main_modal, _ = block.integrator(main_modal, other_modals, integrate_attn_mask, None)
                main_modal = block.feedforward(main_modal)
                record.append({"emb": [None] * block.emb_num_modal, "crm": [None] * (self.modal_num - 1)})
            return self.output_feedforward(main_modal), other_modals, record
        args = [other_modals, hx, None, main_modal_others, other_modals_others, integrate_attn_mask]
        for block in self.metaformer_blocks:
            main_modal, *args = block(main_modal, *args)
        main_modal = self.output_feedforward(main_modal)
        return main_modal, args[0], args[2]


def _none_leaves(x) -> bool:
    if x is None:
        return True
    if isinstance(x, dict):
        return all(_none_leaves(v) for v in x.values())
    if isinstance(x, (list, tuple)):
        return all(_none_leaves(v) for v in x)
    return False
