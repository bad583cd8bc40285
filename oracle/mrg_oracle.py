"""ORACLE — CPU fp32 restatement of the reference's training path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module, and only as the checker / the timed CPU baseline.
The product path (``multimodalreactiongeneration_amd``) never imports it and
fails loudly when its HIP library is missing.

Pinned against the golden vectors produced by running the reference itself
(``tests/golden/make_golden.py``; checked by ``tests/test_oracle_golden.py``).

The restatement is functional: weights are passed as a ``state_dict`` keyed by
the reference's own parameter names, so the same dict loads into the reference,
into this oracle and into the MI355X build.  Each function cites the reference
code it restates.  Scope: the benchmark configuration family (LSTM embedding
mixers, MHA integrators, residual + LayerNorm everywhere, dropout 0).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

PADDING_VALUE = -100.0
# False (default): the explicit per-step restatement below (parity checks).  True: the fused ATen
# LSTM op the reference's nn.LSTM runs on CPU (bench.py times the CPU baseline with it).
ATEN_LSTM = False
Tensor = torch.Tensor
SD = Dict[str, Tensor]
# ReLU masks of a GPU forward to evaluate the restatement AT (tests only): {weight prefix of the
# Linear before the ReLU: bool tensor of its output's shape (True = the GPU's pre-activation > 0)}.
# A pre-activation within fp32 rounding of 0 can take either side of the kink under a different
# summation order; with the GPU's side injected the float64 answer is the GPU's own function of
# its inputs, so the comparison holds 1e-4 everywhere (tests/test_gpu_models.py).
RELU_MASKS: Optional[Dict[str, Tensor]] = None


# --------------------------------------------------------------------------- ops
def linear(x: Tensor, sd: SD, prefix: str) -> Tensor:
    """nn.Linear: y = x W^T + b."""
    return F.linear(x, sd[prefix + "weight"], sd.get(prefix + "bias"))


def relu(x: Tensor, prefix: str) -> Tensor:
    """torch.relu (mixer_block.py:37-87 FeedForward), or x * mask when RELU_MASKS holds this layer."""
    m = None if RELU_MASKS is None else RELU_MASKS.get(prefix)
    if m is None:
        return torch.relu(x)
    if m.shape != x.shape:
        raise ValueError(f"oracle.relu: mask {tuple(m.shape)} for {prefix} but pre-activation {tuple(x.shape)}")
    return x * m.to(x.dtype)


def residual_ln(y: Tensor, x: Tensor, sd: SD, prefix: str) -> Tensor:
    """ResidualConnection: LN(module(x) + x), dropout 0 (residual_connection.py:20-37)."""
    return F.layer_norm(y + x, (y.shape[-1],), sd[prefix + "weight"], sd[prefix + "bias"], 1e-5)


def lstm_layer(x: Tensor, w_ih: Tensor, w_hh: Tensor, b_ih: Tensor, b_hh: Tensor,
               h0: Optional[Tensor] = None, c0: Optional[Tensor] = None,
               reverse: bool = False) -> Tuple[Tensor, Tensor, Tensor]:
    """One direction of one torch.nn.LSTM layer (gate order i, f, g, o), batch_first.

    Restates the op the reference calls in LSTMMixer (mixer_block.py:237-252),
    LSTMModule (lstm_block.py:21-46) and LSTMSampler (lstm_sampler.py:16-34).
    """
    B, T, _ = x.shape
    H = w_hh.shape[1]
    if ATEN_LSTM and T > 0:
        # the fused ATen LSTM op nn.LSTM itself dispatches to on CPU (oneDNN); same math as the
        # loop below, used only to time the reference's own CPU path (bench.py cpu_baseline)
        h = x.new_zeros(1, B, H) if h0 is None else h0.unsqueeze(0)
        c = x.new_zeros(1, B, H) if c0 is None else c0.unsqueeze(0)
        xi = x.flip(1) if reverse else x
        y, hT, cT = torch.lstm(xi, (h, c), [w_ih, w_hh, b_ih, b_hh], True, 1, 0.0, True, False, True)
        return (y.flip(1) if reverse else y), hT[0], cT[0]
    gx = F.linear(x, w_ih, b_ih)
    h = x.new_zeros(B, H) if h0 is None else h0
    c = x.new_zeros(B, H) if c0 is None else c0
    ys: List[Optional[Tensor]] = [None] * T
    steps = range(T - 1, -1, -1) if reverse else range(T)
    for t in steps:
        g = gx[:, t] + F.linear(h, w_hh, b_hh)
        i, f, gg, o = g.chunk(4, dim=-1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
        h = torch.sigmoid(o) * torch.tanh(c)
        ys[t] = h
    if T == 0:
        return x.new_zeros(B, 0, H), h, c
    return torch.stack(ys, dim=1), h, c


def gru_layer(x: Tensor, w_ih: Tensor, w_hh: Tensor, b_ih: Tensor, b_hh: Tensor,
              h0: Optional[Tensor] = None, reverse: bool = False) -> Tuple[Tensor, Tensor]:
    """One direction of one torch.nn.GRU layer (gate order r, z, n), batch_first: the op GRUMixer
    calls (mixer_block.py:169-208).  n = tanh(W_in x + b_in + r * (W_hn h + b_hn))."""
    B, T, _ = x.shape
    H = w_hh.shape[1]
    if ATEN_LSTM and T > 0:
        # the fused ATen GRU op nn.GRU dispatches to on CPU (timing of the reference's own path only)
        h = x.new_zeros(1, B, H) if h0 is None else h0.unsqueeze(0)
        xi = x.flip(1) if reverse else x
        y, hT = torch.gru(xi, h, [w_ih, w_hh, b_ih, b_hh], True, 1, 0.0, True, False, True)
        return (y.flip(1) if reverse else y), hT[0]
    gx = F.linear(x, w_ih, b_ih)
    h = x.new_zeros(B, H) if h0 is None else h0
    ys: List[Optional[Tensor]] = [None] * T
    for t in (range(T - 1, -1, -1) if reverse else range(T)):
        gh = F.linear(h, w_hh, b_hh)
        xr, xz, xn = gx[:, t].chunk(3, dim=-1)
        hr, hz, hn = gh.chunk(3, dim=-1)
        r = torch.sigmoid(xr + hr)
        z = torch.sigmoid(xz + hz)
        n = torch.tanh(xn + r * hn)
        h = (1 - z) * n + z * h
        ys[t] = h
    if T == 0:
        return x.new_zeros(B, 0, H), h
    return torch.stack(ys, dim=1), h


def lstm_stack(x: Tensor, sd: SD, prefix: str, num_layers: int, bidirectional: bool,
               hx: Optional[Tuple[Tensor, Tensor]] = None):
    """torch.nn.LSTM(num_layers, bidirectional, batch_first) over ``{prefix}weight_ih_l{k}[_reverse]``."""
    D = 2 if bidirectional else 1
    hs, cs = [], []
    for layer in range(num_layers):
        outs = []
        for d in range(D):
            sfx = f"l{layer}" + ("_reverse" if d else "")
            idx = layer * D + d
            h0 = None if hx is None else hx[0][idx]
            c0 = None if hx is None else hx[1][idx]
            y, hT, cT = lstm_layer(x, sd[prefix + "weight_ih_" + sfx], sd[prefix + "weight_hh_" + sfx],
                                   sd[prefix + "bias_ih_" + sfx], sd[prefix + "bias_hh_" + sfx],
                                   h0, c0, reverse=bool(d))
            outs.append(y)
            hs.append(hT)
            cs.append(cT)
        x = torch.cat(outs, dim=-1) if D == 2 else outs[0]
    return x, (torch.stack(hs), torch.stack(cs))


def gen_attention_mask(main: Tensor, other: Tensor, heads: int,
                       padding_value: float = PADDING_VALUE) -> Tensor:
    """Block-causal rectangular mask OR (query-pad AND key-pad) (multi_modal_metaformer.py:32-79).

    True = masked.  Tk = r*Tq: query i sees key j iff j // r <= i;  Tq = r*Tk:
    query i sees key j iff j <= i // r.  Shape [B, heads, Tq, Tk].
    """
    tq, tk = main.shape[1], other.shape[1]
    if tk % tq != 0 and tq % tk != 0:
        raise ValueError(f"other_modal_len must be divisible by main_modal_len. "
                         f"main_modal_len: {tq}, other_modal_len: {tk}")
    i = torch.arange(tq).unsqueeze(1)
    j = torch.arange(tk).unsqueeze(0)
    if tk % tq == 0:
        causal = (j // (tk // tq)) > i
    else:
        causal = j > (i // (tq // tk))
    qp = main[:, :, 0] == padding_value
    kp = other[:, :, 0] == padding_value
    pad = qp.unsqueeze(2) & kp.unsqueeze(1)
    m = causal.unsqueeze(0) | pad
    return m.unsqueeze(1).expand(-1, heads, -1, -1).to(main.device)


def mha(q: Tensor, kv: Tensor, sd: SD, prefix: str, heads: int,
        mask: Optional[Tensor] = None) -> Tensor:
    """nn.MultiheadAttention(batch_first, kdim=vdim=E) forward, need_weights=False.

    Called from MHAforSequentail (for_sequential.py:42-51) with a 3-D bool
    ``attn_mask`` [B*heads, Tq, Tk] (True = masked), and from
    MultiModalAttentionBlockSequential (multi_modal_att.py:22-31) with none.
    """
    B, Tq, E = q.shape
    Tk = kv.shape[1]
    D = E // heads
    w, b = sd[prefix + "in_proj_weight"], sd[prefix + "in_proj_bias"]
    Q = F.linear(q, w[:E], b[:E]).view(B, Tq, heads, D).transpose(1, 2)
    K = F.linear(kv, w[E:2 * E], b[E:2 * E]).view(B, Tk, heads, D).transpose(1, 2)
    V = F.linear(kv, w[2 * E:], b[2 * E:]).view(B, Tk, heads, D).transpose(1, 2)
    s = torch.matmul(Q, K.transpose(-1, -2)) / math.sqrt(D)
    if mask is not None:
        s = s.masked_fill(mask.view(B, heads, Tq, Tk), float("-inf"))
    p = torch.softmax(s, dim=-1)
    o = torch.matmul(p, V).transpose(1, 2).reshape(B, Tq, E)
    return F.linear(o, sd[prefix + "out_proj.weight"], sd[prefix + "out_proj.bias"])


def masked_regression_loss(y: Tensor, target: Tensor, loss_type: str = "huber",
                           delta: float = 1.0, beta: float = 1.0, delta_order: int = 0,
                           delta_loss_scale: float = 1.0, mask_padding: bool = True) -> Tensor:
    """training_step loss (lstmformer.py:372-380, lstm_with_sample.py:288-296, simple_lstm.py:239-252).

    mask = target != -100 (int); y*mask, target*mask; feature scaler sqrt(delta_loss_scale)
    from delta_start = F // (delta_order + 1); reduction mean over every element.
    """
    if mask_padding:
        m = (target != PADDING_VALUE).int()
        y = y * m
        target = target * m
    s = torch.ones_like(y)
    s[:, :, y.shape[2] // (delta_order + 1):] = math.sqrt(delta_loss_scale)
    a, b = y * s, target * s
    if loss_type == "huber":
        return F.huber_loss(a, b, delta=delta)
    if loss_type == "mse":
        return F.mse_loss(a, b)
    if loss_type == "mae":
        return F.l1_loss(a, b)
    if loss_type == "smoothl1":
        return F.smooth_l1_loss(a, b, beta=beta)
    raise ValueError("invalid loss type")


@torch.no_grad()
def adamw_step(params: Dict[str, Tensor], grads: Dict[str, Tensor], state: Dict[str, dict],
               lr: float, weight_decay: float, betas=(0.9, 0.999), eps=1e-8):
    """torch.optim.AdamW step (configure_optimizers, lstmformer.py:327-333)."""
    b1, b2 = betas
    for k, p in params.items():
        g = grads[k]
        st = state.setdefault(k, {"step": 0, "m": torch.zeros_like(p), "v": torch.zeros_like(p)})
        st["step"] += 1
        t = st["step"]
        p.mul_(1 - lr * weight_decay)
        st["m"].mul_(b1).add_(g, alpha=1 - b1)
        st["v"].mul_(b2).addcmul_(g, g, value=1 - b2)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        denom = (st["v"].sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(st["m"], denom, value=-lr / bc1)


# ------------------------------------------------------------------ lstmformer
def _cat_inputs(inputs):
    (a, _), (mp, _), (ms, _), (la, _), (lmp, _), (lms, _) = inputs[:6]
    return torch.cat([la, a], 1), torch.cat([lmp, mp], 1), torch.cat([lms, ms], 1)


def _lstm_mixer_block(x, sd, p, kind="lstm"):
    """LSTMMixerBlock (mixer_block.py:479-507): LN(LSTM(x)+x) then LN(Linear(y)+y); with kind "gru"
    the GRUMixerBlock of config_gru.yaml (mixer_block.py:169-208,355-428: nn.GRU under the same
    parameter names)."""
    w = [sd[p + "mixer.module.mixer." + n] for n in ("weight_ih_l0", "weight_hh_l0", "bias_ih_l0", "bias_hh_l0")]
    y = gru_layer(x, *w)[0] if kind == "gru" else lstm_layer(x, *w)[0]
    y = residual_ln(y, x, sd, p + "mixer.layer_norm.")
    z = linear(y, sd, p + "feed_forward.feed_forward.module.feedforward.")
    return residual_ln(z, y, sd, p + "feed_forward.feed_forward.layer_norm.")


def _mha_mixer_block(q, kv, mask, sd, p, heads):
    """MHAMixerBlock (mixer_block.py:567-603): LN(MHA(q,kv)+q) then LN(Linear(y)+y)."""
    a = mha(q, kv, sd, p + "mixer.module.mixer.0.mha.", heads, mask)
    y = residual_ln(a, q, sd, p + "mixer.layer_norm.")
    z = linear(y, sd, p + "feed_forward.feed_forward.module.feedforward.")
    return residual_ln(z, y, sd, p + "feed_forward.feed_forward.layer_norm.")


def metaformer_forward(sd: SD, cfg, inputs) -> Tensor:
    """Metaformer.forward (lstmformer.py:236-311) -> MultiModalMetaformer.forward (multi_modal_metaformer.py:476-509).

    Recurrent state is never carried: every LSTM starts from zero.
    """
    heads, nb, enc = cfg["num_heads"], cfg["num_block"], cfg["encoder_num_layer"]
    kinds = set(cfg.get("emb_mixers", ["lstm"] * 3))
    if len(kinds) != 1 or not kinds <= {"lstm", "gru"}:
        raise ValueError(f"oracle: uniform lstm or gru emb_mixers only (config.yaml / config_gru.yaml), got {kinds}")
    kind = kinds.pop()
    a, mp, ms = _cat_inputs(inputs)
    T = mp.shape[1]
    mm_mask = gen_attention_mask(ms, mp, heads).reshape(-1, T, T)
    ma_mask = gen_attention_mask(ms, a, heads).reshape(-1, T, a.shape[1])
    P = "metaformer."
    main = linear(ms, sd, P + "feature_embedding.0.")
    others = [linear(a, sd, P + "feature_embedding.1."), linear(mp, sd, P + "feature_embedding.2.")]
    for blk in range(nb):
        bp = P + f"metaformer_blocks.{blk}."
        mods = [main] + (others if blk == 0 else [])
        for mi in range(len(mods)):
            x = mods[mi]
            for layer in range(1 if mi == 0 else enc):
                x = _lstm_mixer_block(x, sd, bp + f"embedding.modal_embeddings.{mi}.mixer.{layer}.", kind)
            mods[mi] = x
        main = mods[0]
        if blk == 0:
            others = mods[1:]
        ys = [_mha_mixer_block(main, kv, mk, sd, bp + f"integrator.integrators.{ii}.mixer.0.", heads)
              for ii, (kv, mk) in enumerate(zip(others, [ma_mask, mm_mask]))]
        main = linear(torch.cat(ys, -1), sd, bp + "integrator.cat_linear.")
        fp = bp + "feedforward.feed_forward."
        u = relu(linear(main, sd, fp + "module.input."), fp + "module.input.")
        z = linear(u, sd, fp + "module.output.")
        main = residual_ln(z, main, sd, fp + "layer_norm.")
    op = P + "output_feedforward.feed_forward."
    return linear(relu(linear(main, sd, op + "input."), op + "input."), sd, op + "output.")


def metaformer_training_loss(sd: SD, cfg, batch) -> Tuple[Tensor, Tensor]:
    """Metaformer.training_step without scheduled sampling (lstmformer.py:357-385)."""
    lead = batch[4][0].shape[1]
    target = batch[-1][0]
    ms = batch[2][0]
    ms = ms * (ms != PADDING_VALUE).int()
    inputs = list(batch[:-1])
    inputs[2] = (ms, batch[2][1])
    y = metaformer_forward(sd, cfg, inputs)[:, lead:]
    loss = masked_regression_loss(y, target, cfg["loss_type"], cfg.get("huber_delta", 1.0),
                                  cfg.get("smoothl1_beta", 1.0), cfg["delta_order"],
                                  cfg.get("delta_loss_scale", 1.0))
    return loss, y


def metaformer_prediction(sd: SD, cfg, batch, sampling_mask: Tensor) -> Tensor:
    """Metaformer.prediction (lstmformer.py:426-547): stateless single-step generation.

    form_generation_init (:523-547) zeroes the -100 padding of audio / partner / self
    motion and cuts them into per-step slices ([B, r, F] audio, [B, 1, F] pose); each step
    runs the full forward on that step with empty lead inputs (gen_dummy_input, :549-559)
    and feeds back its own output (mask true) or motion_s[step] (teacher forcing, the
    one-step lag of :492).  The warm-up forward (:461-464) only produces a state the
    forward never reads, so it is not restated.  Returns the prediction [B, T, F].
    """
    (fb, lf), (mp, lp), (ms, ls) = batch[0], batch[1], batch[2]
    T, B = mp.shape[1], mp.shape[0]
    r = fb.shape[1] // T
    fb = fb.reshape(B, T, r, fb.shape[-1]).transpose(0, 1)
    mp = mp.transpose(0, 1).unsqueeze(2)
    ms = ms.transpose(0, 1).unsqueeze(2)
    fb = fb * (fb != PADDING_VALUE).int()
    mp = mp * (mp != PADDING_VALUE).int()
    ms = ms * (ms != PADDING_VALUE).int()
    empty = [(x.new_zeros(x.shape[0], 0, x.shape[2]), n) for x, n in batch]
    y = ms[0]
    preds = []
    ones = torch.ones(B, dtype=torch.long)
    for step in range(T):
        y = metaformer_forward(sd, cfg, [(fb[step], lf), (mp[step], lp), (y, ones)] + empty[3:6])
        preds.append(y)
        y = y if bool(sampling_mask[step]) else ms[step]
    return torch.cat(preds, 1)


def metaformer_prediction_target(batch) -> Tensor:
    """The target Metaformer.prediction returns (lstmformer.py:434-435): target [B, T, F] times
    motion_s_mask [T', B, 1, F] (form_generation_init, :536-547), which BROADCASTS to
    [T', B, T, F]."""
    ms = batch[2][0].transpose(0, 1).unsqueeze(2)
    return batch[-1][0] * (ms != PADDING_VALUE).int()


def broadcast_regression_loss(pred: Tensor, target4: Tensor, loss_type: str = "huber", delta: float = 1.0,
                              beta: float = 1.0, delta_order: int = 0, delta_loss_scale: float = 1.0,
                              scaler: bool = True) -> Tensor:
    """The loss lines of training_step (lstmformer.py:372-380) and generation_step (:413-418)
    applied, as the reference applies them, to prediction [B, T, F] and the broadcast target
    [T', B, T, F]: the padding mask broadcasts y too, and the scaler's slice ``[:, :, start:]``
    lands on the T axis of the 4-d tensor (start = T // (delta_order + 1)).  generation_step has
    no scaler (``scaler=False``)."""
    m = (target4 != PADDING_VALUE).int()
    y = pred * m
    t = target4 * m
    if scaler:
        s = torch.ones_like(y)
        s[:, :, y.shape[2] // (delta_order + 1):] = math.sqrt(delta_loss_scale)
        y, t = y * s, t * s
    if loss_type == "huber":
        return F.huber_loss(y, t, delta=delta)
    if loss_type == "mse":
        return F.mse_loss(y, t)
    if loss_type == "mae":
        return F.l1_loss(y, t)
    if loss_type == "smoothl1":
        return F.smooth_l1_loss(y, t, beta=beta)
    raise ValueError("invalid loss type")


def metaformer_genrt_loss(sd: SD, cfg, batch) -> Tensor:
    """Metaformer.generation_step (lstmformer.py:410-424): teacher-forced prediction, loss on the
    broadcast target (Q9), no scaler."""
    T = batch[1][0].shape[1]
    pred = metaformer_prediction(sd, cfg, batch, torch.zeros(T, dtype=torch.bool))
    return broadcast_regression_loss(pred, metaformer_prediction_target(batch), cfg["loss_type"],
                                     cfg.get("huber_delta", 1.0), cfg.get("smoothl1_beta", 1.0), scaler=False)


def metaformer_ss_training_loss(sd: SD, cfg, batch, sampling_mask: Tensor) -> Tuple[Tensor, Tensor]:
    """Metaformer.training_step with use_scheduled_sampling (lstmformer.py:357-385): the AR
    prediction under ``sampling_mask`` (the draw of :476), loss on the broadcast target (Q9)."""
    pred = metaformer_prediction(sd, cfg, batch, sampling_mask)
    loss = broadcast_regression_loss(pred, metaformer_prediction_target(batch), cfg["loss_type"],
                                     cfg.get("huber_delta", 1.0), cfg.get("smoothl1_beta", 1.0),
                                     cfg["delta_order"], cfg.get("delta_loss_scale", 1.0))
    return loss, pred


# ---------------------------------------------------------- lstm_with_sampling
def lstm_with_sample_forward(sd: SD, cfg, inputs, hx_sampler=None):
    """LSTMwithSample.forward (lstm_with_sample.py:151-232); returns (y, hx_sampler)."""
    ratio = int(cfg["sampling_rate"] / cfg["shift"] / cfg["pred_fps"])
    a, mp, ms = _cat_inputs(inputs)
    a = linear(a, sd, "acoustic_projection.")
    h, hx_sampler = lstm_stack(a, sd, "sampling_lstm.sampler.", cfg["sampler_num_layers"], False, hx_sampler)
    a = h[:, ratio - 1::ratio, :].contiguous()
    if not (a.shape[1] == mp.shape[1] == ms.shape[1]):
        raise RuntimeError("sequence length mismatch")
    f = linear(torch.cat([a, mp, ms], -1), sd, "feature_projection.")
    for layer in range(cfg["num_layers"]):
        p = f"layerd_lstm.lstm_layered.{layer}.lstm_module."
        y, _ = lstm_stack(f, sd, p + "module.lstm_module.", 1, False)
        f = residual_ln(y, f, sd, p + "layer_norm.")
    y = linear(relu(linear(f, sd, "feed_forward.input."), "feed_forward.input."), sd, "feed_forward.mapping.")
    return y, hx_sampler


def lstm_with_sample_prediction(sd: SD, cfg, batch, sampling_mask: Tensor) -> Tuple[Tensor, Tensor]:
    """prediction(use_scheduled_sampling) (lstm_with_sample.py:339-433) with an explicit mask.

    Warm-up over the lead frames carries only the sampler state; the layered
    LSTM restarts from zero every step; teacher forcing feeds
    motion_s[step] (one-step lag, Q10).
    """
    ratio = int(cfg["sampling_rate"] / cfg["shift"] / cfg["pred_fps"])
    (fb, lf), (mp, lp), (ms, ls) = batch[0], batch[1], batch[2]
    T, B = mp.shape[1], mp.shape[0]
    fb = fb.view(B, T, ratio, fb.shape[-1]).transpose(0, 1)
    mp = mp.transpose(0, 1).unsqueeze(2)
    ms = ms.transpose(0, 1).unsqueeze(2)
    empty = [(x.new_zeros(x.shape[0], 0, x.shape[2]), n) for x, n in batch]
    _, hx = lstm_with_sample_forward(sd, cfg, empty[:3] + list(batch[3:6]))
    y = ms[0]
    preds = []
    ones = torch.ones(B, dtype=torch.long)
    for step in range(T):
        y, hx = lstm_with_sample_forward(sd, cfg, [(fb[step], lf), (mp[step], lp), (y, ones)] + empty[3:6], hx)
        preds.append(y)
        y = y if bool(sampling_mask[step]) else ms[step]
    return torch.cat(preds, 1), batch[-1][0]


def lstm_with_sample_training_loss(sd: SD, cfg, batch, sampling_mask=None):
    if sampling_mask is not None:
        y, target = lstm_with_sample_prediction(sd, cfg, batch, sampling_mask)
    else:
        lead = batch[4][0].shape[1]
        y, _ = lstm_with_sample_forward(sd, cfg, batch[:-1])
        y = y[:, lead:]
        target = batch[-1][0]
    loss = masked_regression_loss(y, target, cfg["loss_type"], cfg.get("huber_delta", 1.0),
                                  cfg.get("smoothl1_beta", 1.0), cfg["delta_order"],
                                  cfg.get("delta_loss_scale", 1.0))
    return loss, y


# ------------------------------------------------------------------ simple_lstm
def _lstm_layerd(x, sd, p, num_layers, use_ff=True, use_mixing=True, bidirectional=True):
    """LSTMLayerd -> LSTMBlock -> LSTMModule (lstm_block.py:9-169), residual + LN."""
    for layer in range(num_layers):
        bp = f"{p}lstm_layered.{layer}."
        hs, _ = lstm_stack(x, sd, bp + "lstm_module.module.lstm_module.", 1, bidirectional)
        y = linear(hs, sd, bp + "lstm_module.module.mixer.") if use_mixing else hs
        y = residual_ln(y, x, sd, bp + "lstm_module.layer_norm.")
        if use_ff:
            fp = bp + "feed_forward_module."
            u = relu(linear(y, sd, fp + "module.input."), fp + "module.input.")
            z = linear(u, sd, fp + "module.mapping.")
            y = residual_ln(z, y, sd, fp + "layer_norm.")
        x = y
    return x


def simple_lstm_forward(sd: SD, cfg, audio: Tensor, motion: Tensor) -> Tensor:
    """SimpleLSTM.forward with the Q3 tuple unwrap (simple_lstm.py:181-188)."""
    ae = _lstm_layerd(linear(audio, sd, "acoustic_encoder.embed_layer."), sd,
                      "acoustic_encoder.acostic_lstm.", cfg["acostic_num_layers"])
    me = _lstm_layerd(linear(motion, sd, "motion_encoder.embed_layer."), sd,
                      "motion_encoder.motion_lstm.", cfg["motion_num_layers"])
    x = me
    for layer in range(cfg["att_num_layers"]):
        p = f"multimodal_att.att_layers.{layer}.att_module."
        o = mha(x, ae, sd, p + "module.cross_modal_att.", cfg["att_heads"])
        o = linear(o, sd, p + "module.projection.")
        x = residual_ln(o, x, sd, p + "layer_norm.")
    d = _lstm_layerd(x, sd, "motion_decoder.decoder_lstm.", cfg["decoder_num_layers"])
    d = d[:, -1:, :]
    return linear(relu(linear(d, sd, "motion_decoder.mapping.input."), "motion_decoder.mapping.input."), sd,
                  "motion_decoder.mapping.output.")


def simple_lstm_training_loss(sd: SD, cfg, audio, motion, target):
    y = simple_lstm_forward(sd, cfg, audio, motion)
    return masked_regression_loss(y, target, "mse", mask_padding=False,
                                  delta_loss_scale=cfg.get("delta_loss_scale", 1.0)), y


# ------------------------------------------------------------------ helpers
def run_train_step(loss_fn, sd: SD, optim_cfg, *args, **kw):
    """loss, output, grads, params-after-AdamW for a functional loss over ``sd``."""
    params = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
    loss, y = loss_fn(params, *args, **kw)
    loss.backward()
    grads = {k: (p.grad if p.grad is not None else torch.zeros_like(p)) for k, p in params.items()}
    after = {k: p.detach().clone() for k, p in params.items()}
    adamw_step(after, grads, {}, optim_cfg["lr"], optim_cfg["weight_decay"])
    return loss.detach(), y.detach(), grads, after


# ---------------------------------------------------------- data-loader features
def melscale_fbanks_htk(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int) -> Tensor:
    """Triangular mel filterbank [n_freqs, n_mels] as torchaudio.functional.melscale_fbanks
    (norm=None, mel_scale="htk") builds it for transforms.MelSpectrogram (audio.py:16-22).

    torchaudio is a third-party dependency the reference does not pin (its Docker base,
    pytorch 23.04, ships torchaudio 2.1) and it is absent here, so this restates its published
    algorithm: linear frequency grid, n_mels + 2 points equally spaced in HTK mel
    (2595 log10(1 + f / 700)), and min(down, up) slopes clamped at 0; float32 throughout.
    Parity of this part is UNPINNED (no fixture can be produced without torchaudio).
    """
    all_freqs = torch.linspace(0, sample_rate // 2, n_freqs)
    m_min = 2595.0 * math.log10(1.0 + f_min / 700.0)
    m_max = 2595.0 * math.log10(1.0 + f_max / 700.0)
    m_pts = torch.linspace(m_min, m_max, n_mels + 2)
    f_pts = 700.0 * (10 ** (m_pts / 2595.0) - 1.0)
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts.unsqueeze(0) - all_freqs.unsqueeze(1)
    down = (-1.0 * slopes[:, :-2]) / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return torch.clamp(torch.min(down, up), min=0.0)


def compute_log_power(wave: Tensor, nfft: int, shift: int) -> Tensor:
    """AudioPreprocessor.compute_log_power (audio.py:43-56): per-frame log of the raw frame's
    energy, frame by frame as the reference loops."""
    num_frames = (len(wave) - nfft) // shift + 1
    out = torch.zeros(num_frames)
    for f in range(num_frames):
        s = torch.sum(torch.pow(wave[f * shift:f * shift + nfft], 2))
        out[f] = torch.log(torch.clamp(s, 1e-10))
    return out


def compute_delta(x: Tensor, delta_order: int) -> Tensor:
    """compute_delta (audio.py:58-67, motion_nx.py:49-58)."""
    if delta_order == 0:
        return x
    d1 = x[1:] - x[:-1]
    if delta_order == 1:
        return torch.cat([x[1:], d1], dim=1)
    d2 = d1[1:] - d1[:-1]
    if delta_order == 2:
        return torch.cat([x[2:], d1[1:], d2], dim=1)
    raise ValueError("delta_order must be 0, 1 or 2")


def audio_features(wave: Tensor, sample_rate: int, nfft: int, shift: int, nmels: int, delta_order: int) -> Tensor:
    """AudioPreprocessor.__call__ after the file read (audio.py:25-41): MelSpectrogram(n_fft,
    hop, n_mels, center=False) = |STFT|^2 with a periodic Hann window, mel projection, log with
    the two clamps, the log power as an extra row, transpose, deltas."""
    spec = torch.stft(wave, n_fft=nfft, hop_length=shift, win_length=nfft, window=torch.hann_window(nfft),
                      center=False, normalized=False, onesided=True, return_complex=True).abs().pow(2.0)
    fb = melscale_fbanks_htk(nfft // 2 + 1, 0.0, float(sample_rate // 2), nmels, sample_rate)
    mel = torch.matmul(spec.transpose(-1, -2), fb).transpose(-1, -2)
    fbank = torch.log(torch.clamp(torch.clamp(mel, 1e-10), 1e-6) * 1)
    power = compute_log_power(wave, nfft, shift)
    fbank = torch.cat([fbank, power.unsqueeze(0)], dim=0).T.to(torch.float32)
    return compute_delta(fbank, delta_order)
