"""Token mixers, mixer blocks and layered mixers (reference: mr_gen/model/utils/mixer_block.py).

Same constructor arguments, module attribute names and forward tuple
conventions as the reference (nn.Sequential-friendly tuples, the
``split_state`` state plumbing), so configs and checkpoints carry over.
LSTM, GRU and MHA mixers run on libmrg.so.  The MLP mixer is outside the
benchmarked path (unused by the BASELINE configs) and raises.
"""
from __future__ import annotations

import inspect
from typing import Any, List, Tuple

import torch
from torch import nn

from .. import functional as Fn
from .layers import GRU, LSTM, MHAforSequentail, ResidualConnection, FeedForward


def split_state(state, prev_state):
    """Peel the first entry of a layered state list (mixer_block.py:21-30), quirks included."""
    first, rest = (None, None) if state is None else (state[:1], state[1:])
    if first is not None:
        first = None if (first == [] and first) else first[0]
    if rest is not None:
        rest = None if (rest == [] and rest) else rest
    return first, rest, ([] if prev_state is None else prev_state)


class Mixer(nn.Module):
    pass


class MixerBlock(nn.Module):
    pass


class MixerLayerd(nn.Module):
    pass


class LSTMMixer(Mixer):
    """nn.LSTM token mixer (mixer_block.py:211-252)."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int = 1, bias: bool = True,
                 batch_first: bool = True, dropout: float = 0.0, bidirectional: bool = False,
                 proj_size: int = 0, device=None, dtype=None):
        super().__init__()
        if num_layers < 1:
            raise ValueError("num_layers must be greater than 0.")
        if bidirectional:
            if hidden_size % 2:
                raise ValueError("hidden_size must be even number when bidirectional is True.")
            hidden_size //= 2
        self.mixer = LSTM(input_size, hidden_size, num_layers=num_layers, bias=bias,
                          batch_first=batch_first, dropout=dropout, bidirectional=bidirectional,
                          proj_size=proj_size, device=device, dtype=dtype)

    def forward(self, x, hn=None):
        return self.mixer(x, hn)

    def fused_residual_ln(self, ln, x, hn=None):
        """LN(LSTM(x) + x) in one op when the LSTM is one unidirectional layer from a zero state."""
        m = self.mixer
        if hn is not None or m.num_layers != 1 or m.bidirectional or not isinstance(x, torch.Tensor):
            return None
        u, hT, cT = Fn.lstm_residual_layernorm(x, *m.direction_params(0), ln.weight, ln.bias, ln.eps)
        return u, (hT.unsqueeze(0), cT.unsqueeze(0))


class MHAMixer(Mixer):
    """Stack of MultiheadAttention layers; returns the last output tensor (mixer_block.py:255-305)."""

    def __init__(self, input_size: int, num_heads: int, num_layers: int = 1, dropout: float = 0.0,
                 add_bias_kv: bool = False, add_zero_attn: bool = False, kdim: int = None,
                 vdim: int = None, batch_first: bool = False, nonlinearity=None, bias: bool = True,
                 device=None, dtype=None):
        super().__init__()
        if num_layers < 1:
            raise ValueError("num_layers must be greater than 0.")
        self.mixer = nn.ModuleList([
            MHAforSequentail(input_size, num_heads, dropout, bias, add_bias_kv, add_zero_attn, kdim, vdim,
                             batch_first, nonlinearity, device=device, dtype=dtype)
            for _ in range(num_layers)])

    def fused_residual_ln(self, ln, q, k, v, attn_mask=None):
        """LN(MHA(q, k, v) + q) in one op (single layer, batch_first, k is v, reference mask)."""
        from .masks import BlockCausalMask
        if len(self.mixer) != 1 or k is not v:
            return None
        mha = self.mixer[0].mha
        if not mha.batch_first or (mha.dropout and mha.training):
            return None
        if attn_mask is not None and not isinstance(attn_mask, BlockCausalMask):
            return None
        causal, qpad, kpad = False, None, None
        if attn_mask is not None:
            causal, qpad, kpad = True, attn_mask.main_pad, attn_mask.other_pad
        return Fn.mha_residual_layernorm(q, k, mha.in_proj_weight, mha.in_proj_bias, mha.out_proj.weight,
                                         mha.out_proj.bias, mha.num_heads, ln.weight, ln.bias, ln.eps,
                                         causal, qpad, kpad)

    def forward(self, q, k, v, attn_mask=None):
        if len(self.mixer) > 1:
            raise NotImplementedError("MHAMixer num_layers > 1 (reference feeds a tuple into layer 2)")
        x = (q, k, v, None, False, attn_mask, False, False)
        return self.mixer[0](x)[0]


class MLPMixer(Mixer):
    def __init__(self, *a, **k):
        raise NotImplementedError("MLP mixer is outside the MI355X path (not in the BASELINE configs)")


class GRUMixer(Mixer):
    """nn.GRU token mixer (mixer_block.py:169-208)."""

    def __init__(self, input_size: int, hidden_size: int, num_layers: int = 1, batch_first: bool = True,
                 dropout: float = 0.0, bidirectional: bool = False, bias: bool = True, device=None, dtype=None):
        super().__init__()
        if num_layers < 1:
            raise ValueError("num_layers must be greater than 0.")
        if bidirectional:
            if hidden_size % 2 != 0:
                raise ValueError("hidden_size must be even number when bidirectional is True.")
            hidden_size //= 2
        self.mixer = GRU(input_size, hidden_size, num_layers=num_layers, bias=bias, batch_first=batch_first,
                         dropout=dropout, bidirectional=bidirectional, device=device, dtype=dtype)

    def forward(self, x, hn=None):
        return self.mixer(x, hn)


class LSTMMixerBlock(MixerBlock):
    """Residual LSTM mixer + FeedForward (mixer_block.py:431-507)."""

    def __init__(self, hidden_size: int, num_layers: int = 1, dropout: float = 0.0,
                 batch_first: bool = True, bidirectional: bool = False, proj_size: int = 0,
                 nonlinearity=None, residual: bool = False, residual_layer_norm: bool = False,
                 bottleneck_size: int = None, bias: bool = True, device=None, dtype=None):
        super().__init__()
        self.mixer = LSTMMixer(hidden_size, hidden_size, num_layers, bias, batch_first, dropout,
                               bidirectional, proj_size, device, dtype)
        if residual:
            self.mixer = ResidualConnection(self.mixer, residual_layer_norm, hidden_size)
        self.feed_forward = FeedForward(hidden_size, bottleneck_size, None, nonlinearity, residual,
                                        residual_layer_norm, bias, device, dtype)

    def lstm_params(self):
        m = self.mixer.module if isinstance(self.mixer, ResidualConnection) else self.mixer
        return m.mixer.direction_params(0)

    def forward(self, x, hx=None, prev_hx=None):
        if isinstance(x, (tuple, list)):
            x, hx, prev_hx = x
        elif not isinstance(x, torch.Tensor):
            raise TypeError(f"x must be torch.Tensor or tuple or list, but got {type(x)}.")
        first, hx, prev_hx = split_state(hx, prev_hx)
        y, first = self.mixer(x, first)
        y = self.feed_forward(y)
        prev_hx.append(first)
        return (y, hx, prev_hx)


class GRUMixerBlock(MixerBlock):
    """Residual GRU mixer + FeedForward (mixer_block.py:355-428)."""

    def __init__(self, hidden_size: int, num_layers: int = 1, dropout: float = 0.0, batch_first: bool = True,
                 bidirectional: bool = False, nonlinearity=None, residual: bool = False,
                 residual_layer_norm: bool = False, bottleneck_size: int = None, bias: bool = True,
                 device=None, dtype=None):
        super().__init__()
        self.mixer = GRUMixer(hidden_size, hidden_size, num_layers, batch_first, dropout, bidirectional, bias,
                              device, dtype)
        if residual:
            self.mixer = ResidualConnection(self.mixer, residual_layer_norm, hidden_size)
        self.feed_forward = FeedForward(hidden_size, bottleneck_size, None, nonlinearity, residual,
                                        residual_layer_norm, bias, device, dtype)

    def forward(self, x, hx=None, prev_hx=None):
        if isinstance(x, (tuple, list)):
            x, hx, prev_hx = x
        elif not isinstance(x, torch.Tensor):
            raise TypeError(f"x must be torch.Tensor or tuple or list, but got {type(x)}.")
        first, hx, prev_hx = split_state(hx, prev_hx)
        y, first = self.mixer(x, first)
        y = self.feed_forward(y)
        prev_hx.append(first)
        return (y, hx, prev_hx)


class MHAMixerBlock(MixerBlock):
    """Residual MHA mixer + FeedForward (mixer_block.py:510-603)."""

    def __init__(self, hidden_size: int, num_layers: int = 1, num_heads: int = 1, dropout: float = 0.0,
                 batch_first: bool = True, add_bias_kv: bool = False, add_zero_attn: bool = False,
                 kdim: int = None, vdim: int = None, max_context_len: int = 125, nonlinearity=None,
                 residual: bool = False, residual_layer_norm: bool = False, bottleneck_size: int = None,
                 bias: bool = True, device=None, dtype=None):
        super().__init__()
        self.mixer = MHAMixer(hidden_size, num_heads, num_layers, dropout, add_bias_kv, add_zero_attn,
                              kdim, vdim, batch_first, nonlinearity, bias, device, dtype)
        if residual:
            self.mixer = ResidualConnection(self.mixer, residual_layer_norm, hidden_size)
        self.feed_forward = FeedForward(hidden_size, bottleneck_size, None, nonlinearity, residual,
                                        residual_layer_norm, bias, device, dtype)
        self.max_context_len = max_context_len

    def mha_module(self):
        m = self.mixer.module if isinstance(self.mixer, ResidualConnection) else self.mixer
        return m.mixer[0].mha

    def forward(self, query, key=None, value=None, attn_mask=None, hx=None, prev_hx=None):
        if isinstance(query, (tuple, list)):
            query, key, value, attn_mask, hx, prev_hx = query
        elif not isinstance(query, torch.Tensor):
            raise TypeError(f"query must be torch.Tensor or tuple or list, but got {type(query)}.")
        first, hx, prev_hx = split_state(hx, prev_hx)
        if isinstance(first, (tuple, list)) and not self.training:
            # KV-cache concat of the reference (dead in practice: states are never produced, Q1/Q5)
            key = torch.cat([first[0], key], dim=1)[-self.max_context_len:]
            value = torch.cat([first[1], value], dim=1)[-self.max_context_len:]
        x = self.mixer(query, key, value, attn_mask)
        x = self.feed_forward(x)
        prev_hx.append((key, value))
        return (x, key, value, attn_mask, hx, prev_hx)


class _Layerd(MixerLayerd):
    def _projections(self, hidden_size, input_projection, input_projection_size, output_projection,
                     output_projection_size, bias):
        from .layers import Linear
        self.input_projection = None
        if input_projection and input_projection_size is None:
            raise ValueError("input_projection_size must be specified when input_projection is True.")
        if input_projection:
            self.input_projection = Linear(input_projection_size, hidden_size, bias=bias)
        self.output_projection = None
        if output_projection and output_projection_size is None:
            raise ValueError("output_projection_size must be specified when output_projection is True.")
        if output_projection:
            self.output_projection = Linear(output_projection_size, hidden_size, bias=bias)


class LSTMMixerLayerd(_Layerd):
    """num_layerd LSTMMixerBlocks; returns the REST hx, not the produced state (Q1, mixer_block.py:833-843)."""

    def __init__(self, hidden_size: int, input_projection: bool = False, input_projection_size: int = None,
                 output_projection: bool = False, output_projection_size: int = None, num_layerd: int = 1,
                 num_internal_layer: int = 1, dropout: float = 0.0, batch_first: bool = True,
                 bidirectional: bool = False, proj_size: int = 0, nonlinearity=None, residual: bool = False,
                 residual_layer_norm: bool = False, bottleneck_size: int = None, bias: bool = True,
                 device=None, dtype=None):
        super().__init__()
        self._projections(hidden_size, input_projection, input_projection_size, output_projection,
                          output_projection_size, bias)
        self.mixer = nn.ModuleList([
            LSTMMixerBlock(hidden_size, num_internal_layer, dropout, batch_first, bidirectional, proj_size,
                           nonlinearity, residual, residual_layer_norm, bottleneck_size, bias, device, dtype)
            for _ in range(num_layerd)])

    def forward(self, x, hx=None, other=(None,)):
        if self.input_projection is not None:
            x = self.input_projection(x)
        phx = None
        for block in self.mixer:
            x, hx, phx = block(x, hx, phx)
        if self.output_projection is not None:
            x = self.output_projection(x)
        return (x, hx, other)


class MHAMixerLayerd(_Layerd):
    """num_layerd MHAMixerBlocks over (query, key, value, attn_mask) (mixer_block.py:846-963)."""

    def __init__(self, hidden_size: int, input_projection: bool = False, input_projection_size: int = None,
                 self_attention: bool = False, output_projection: bool = False,
                 output_projection_size: int = None, num_heads: int = 1, dropout: float = 0.0,
                 batch_first: bool = True, add_bias_kv: bool = False, add_zero_attn: bool = False,
                 kdim: int = None, vdim: int = None, max_context_len: int = 125, num_layerd: int = 1,
                 num_internal_layer: int = 1, nonlinearity=None, residual: bool = False,
                 residual_layer_norm: bool = False, bottleneck_size: int = None, bias: bool = True,
                 device=None, dtype=None):
        super().__init__()
        self._projections(hidden_size, input_projection, input_projection_size, output_projection,
                          output_projection_size, bias)
        self.self_attention = self_attention
        self.mixer = nn.ModuleList([
            MHAMixerBlock(hidden_size, num_internal_layer, num_heads, dropout, batch_first, add_bias_kv,
                          add_zero_attn, kdim, vdim, max_context_len, nonlinearity, residual,
                          residual_layer_norm, bottleneck_size, bias, device, dtype)
            for _ in range(num_layerd)])
        self.max_context_len = max_context_len

    def forward(self, x, hx=None, key=None, value=None, attn_mask=None):
        if isinstance(key, (tuple, list)):
            key, value, attn_mask = key
        elif not isinstance(key, torch.Tensor):
            raise TypeError(f"key must be torch.Tensor or tuple or list, but got {type(key)}.")
        query = x if self.input_projection is None else self.input_projection(x)
        if self.self_attention:
            key, value = query, query
        if key is None or value is None:
            raise ValueError("key and value must be specified when self_attention is False.")
        phx = None
        for block in self.mixer:
            query, *_, hx, phx = block(query, key, value, attn_mask, hx, phx)
        if self.output_projection is not None:
            query = self.output_projection(query)
        return (query, hx, (key, value, attn_mask))


class MLPMixerLayerd(MixerLayerd):
    def __init__(self, *a, **k):
        raise NotImplementedError("MLP mixer is outside the MI355X path (not in the BASELINE configs)")


class GRUMixerLayerd(_Layerd):
    """num_layerd GRUMixerBlocks; returns the REST hx, like the LSTM layerd (mixer_block.py:679-761)."""

    def __init__(self, hidden_size: int, input_projection: bool = False, input_projection_size: int = None,
                 output_projection: bool = False, output_projection_size: int = None, num_layerd: int = 1,
                 num_internal_layer: int = 1, dropout: float = 0.0, batch_first: bool = True,
                 bidirectional: bool = False, nonlinearity=None, residual: bool = False,
                 residual_layer_norm: bool = False, bottleneck_size: int = None, bias: bool = True,
                 device=None, dtype=None):
        super().__init__()
        self._projections(hidden_size, input_projection, input_projection_size, output_projection,
                          output_projection_size, bias)
        self.mixer = nn.ModuleList([
            GRUMixerBlock(hidden_size, num_internal_layer, dropout, batch_first, bidirectional, nonlinearity,
                          residual, residual_layer_norm, bottleneck_size, bias, device, dtype)
            for _ in range(num_layerd)])

    def forward(self, x, hx=None, other=(None,)):
        if self.input_projection is not None:
            x = self.input_projection(x)
        phx = None
        for block in self.mixer:
            x, hx, phx = block(x, hx, phx)
        if self.output_projection is not None:
            x = self.output_projection(x)
        return (x, hx, other)


_BLOCKS = {"mlp": None, "gru": GRUMixerBlock, "lstm": LSTMMixerBlock, "mha": MHAMixerBlock}
_LAYERDS = {"mlp": MLPMixerLayerd, "gru": GRUMixerLayerd, "lstm": LSTMMixerLayerd, "mha": MHAMixerLayerd}


class MixerBlockFactory:
    def build(self, mixer_type, configs):
        if mixer_type not in _BLOCKS:
            raise ValueError(f"mixer_type must be in {list(_BLOCKS)}.")
        cls = _BLOCKS[mixer_type]
        if cls is None:
            raise NotImplementedError(f"{mixer_type} mixer is outside the MI355X path")
        return cls(**configs)


class MixerLayerdFactory:
    def build(self, mixer_type, configs):
        if mixer_type not in _LAYERDS:
            raise ValueError(f"mixer_type must be in {list(_LAYERDS)}.")
        return _LAYERDS[mixer_type](**configs)


def _accepted(cls):
    return [p for p in inspect.signature(cls.__init__).parameters if p != "self"]


_LAYERD_ARGS = {
    "lstm": _accepted(LSTMMixerLayerd), "mha": _accepted(MHAMixerLayerd),
    "gru": _accepted(GRUMixerLayerd),
    "mlp": ["hidden_size", "input_projection", "input_projection_size", "output_projection",
            "output_projection_size", "num_layerd", "num_internal_layer", "nonlinearity", "residual",
            "residual_layer_norm", "bottleneck_size", "bias", "device", "dtype"],
}


def mixer_layerd_argments_select(mixer_type: str, hidden_size: int, **kw) -> dict:
    """The kwargs each *MixerLayerd accepts, defaults filled (argparser.py:382-435)."""
    if mixer_type not in _LAYERD_ARGS:
        raise ValueError(f"mixer_type must be in {list(_LAYERD_ARGS)}")
    cls = _LAYERDS[mixer_type]
    defaults = {}
    if mixer_type in ("lstm", "mha", "gru"):
        defaults = {k: v.default for k, v in inspect.signature(cls.__init__).parameters.items()
                    if k != "self" and v.default is not inspect.Parameter.empty}
    out = {k: defaults.get(k) for k in _LAYERD_ARGS[mixer_type]}
    out["hidden_size"] = hidden_size
    for k, v in kw.items():
        if k in out:
            out[k] = v
    return out


def feedforward_block_argments(hidden_size: int, bottleneck_size: int = None, output_size: int = None,
                               nonlinearity=None, residual: bool = False, residual_layer_norm: bool = False,
                               bias: bool = True, device=None, dtype=None) -> dict:
    return dict(hidden_size=hidden_size, bottleneck_size=bottleneck_size, output_size=output_size,
                nonlinearity=nonlinearity, residual=residual, residual_layer_norm=residual_layer_norm,
                bias=bias, device=device, dtype=dtype)
