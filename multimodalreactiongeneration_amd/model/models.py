"""The three trainable models with the reference's LightningModule surface.

  Metaformer      mr_gen/model/lstmformer/lstmformer.py:70-559
  LSTMwithSample  mr_gen/model/lstm_with_sampling/lstm_with_sample.py:59-463
  SimpleLSTM      mr_gen/model/simple_lstm/simple_lstm.py:146-269

Constructors take the same ``(model, optim, metrics)`` mappings (any object
with attribute access and ``.get``: OmegaConf DictConfig, configs.AttrDict,
or a plain dict).  ``forward`` / ``training_step`` / ``validation_step`` /
``lossfun`` / ``configure_optimizers`` / ``prediction`` keep their reference
signatures and return conventions.  pytorch_lightning is not a dependency:
``LightningSurface`` provides ``log`` / ``log_dict`` / ``current_epoch`` /
``device`` so a Lightning ``Trainer`` or a plain loop can drive the models.
torchmetrics logging is out of scope (no effect on loss or grads).

Precision switch: ``model.precision`` ("32" default; "bf16" / "bf16-mixed" as Lightning's
Trainer(precision=...) names it, or the config key ``precision``) selects the arithmetic of every
op the model runs: bf16 = GEMM operands rounded to bf16 on the bf16 matrix cores with fp32
accumulation; LayerNorm, softmax, the recurrent cell state c, the loss and the optimizer stay fp32,
and parameters / gradients stay fp32 masters (BASELINE configs[1], SURVEY §8c bf16 gate).
"""
from __future__ import annotations

import functools
import math
import os
from collections import OrderedDict
from typing import Any, Dict, List, Tuple

import torch
from torch import nn

from .. import functional as Fn
from ..configs import as_attr
from ..optim import FusedAdamW
from .layers import (Linear, LSTMSampler, LSTMLayerd, MultimodalAttention, ResidualConnection, paired_lstm_layerd,
                     run_sequential_ffn)
from .masks import gen_attention_mask
from .metaformer import MultiModalMetaformer
from .mixers import mixer_layerd_argments_select, feedforward_block_argments

PADDING_VALUE = -100


def _in_precision(fn):
    """Run a model entry point under the model's compute precision (functional.precision)."""
    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        with Fn.precision(self.precision):
            return fn(self, *args, **kwargs)
    return wrapper


class LightningSurface(nn.Module):
    """The slice of pl.LightningModule the reference models use."""

    current_epoch = 0
    precision = "32"

    def set_precision(self, precision):
        """'32' (fp32 arithmetic) or 'bf16' / 'bf16-mixed' (bf16 GEMM operands, fp32 accumulation)."""
        if precision not in Fn.PRECISIONS:
            raise ValueError(f"unsupported precision {precision!r}")
        self.precision = precision
        return self

    def log(self, name, value, **kw):
        pass

    def log_dict(self, *a, **kw):
        pass

    @property
    def device(self):
        return next(self.parameters()).device

    def _loss_spec(self, cfg):
        return dict(loss_type=cfg.loss_type, delta=cfg.get("huber_delta", 1.0),
                    beta=cfg.get("smoothl1_beta", 1.0))

    def _optimizers(self, optim):
        if optim.use_optimizer == "adam":
            opt = FusedAdamW(self.parameters(), lr=optim.lr, weight_decay=optim.weight_decay)
        elif optim.use_optimizer == "sgd":
            # off the benchmarked path (SURVEY §8a13 uses AdamW); plain torch optimizer
            opt = torch.optim.SGD(self.parameters(), lr=optim.lr, momentum=optim.momentum,
                                  weight_decay=optim.weight_decay)
        else:
            raise ValueError("invalid optimizer type")
        self.optimizer = opt
        if optim.use_lr_sched:
            self.lr_scheduler = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=optim.max_epochs)
            return {"optimizer": opt, "lr_scheduler": {"scheduler": self.lr_scheduler, "monitor": "val_loss"}}
        return {"optimizer": opt}


def gen_target_dict(cfg) -> Dict[str, Tuple[int, int]]:
    """Metric slices (lstmformer.py:37-67); [angle, centroid] naming quirk Q8 kept."""
    out = {"centroid": (0, 3), "angle": (3, 6)}
    tail = 6
    if not cfg.use_centroid:
        out.pop("centroid")
        out["angle"] = (0, 3)
        tail = 3
    elif not cfg.use_angle:
        out.pop("angle")
        tail = 3
    for order in (1, 2):
        if cfg.delta_order >= order:
            for name in ("centroid", "angle"):
                if getattr(cfg, "use_" + name):
                    out[f"delta{order}-{name}"] = (tail, tail + 3)
                    tail += 3
    return out


def _cat_lead(lead, x):
    return x if lead.shape[1] == 0 else torch.cat([lead, x], dim=1)


def _loss_type_of(cfg):
    if cfg.loss_type not in ("mse", "mae", "huber", "smoothl1"):
        raise ValueError("invalid loss type")
    return cfg.loss_type


class _TorchLoss(nn.Module):
    """What ``lossfun()`` returns: a callable loss module backed by the fused kernel."""

    def __init__(self, loss_type, reduction, delta, beta):
        super().__init__()
        if reduction != "mean":
            raise NotImplementedError("only reduction='mean' (the reference configs)")
        self.loss_type, self.delta, self.beta = loss_type, delta, beta

    def forward(self, y, target):
        return Fn.masked_loss(y, target, 0, self.loss_type, self.delta, self.beta, mask_padding=False)


class Metaformer(LightningSurface):
    """LSTM + cross-modal attention metaformer (lstmformer.py:70-559)."""

    def __init__(self, model, optim, metrics):
        super().__init__()
        model, optim, metrics = as_attr(model), as_attr(optim), as_attr(metrics)
        self.model, self.optim, self.metrics = model, optim, metrics
        self.set_precision(model.get("precision", "32"))
        self.max_epochs = model.max_epochs
        self.use_scheduled_sampling = model.use_scheduled_sampling
        _loss_type_of(model)
        self.huber_delta = model.get("huber_delta", 1.0)
        self.smoothl1_beta = model.get("smoothl1_beta", 1.0)
        acoustic_fps = model.sampling_rate / model.shift
        ratio = acoustic_fps / model.pred_fps
        if ratio != int(ratio):
            raise ValueError("pred_fps must be a divisor of acoustic_fps",
                             f"pred_fps: {model.pred_fps}, acoustic_fps: {acoustic_fps}, ratio: {ratio}")
        self.ratio = int(ratio)
        self.modalities = list(model.modalities)
        self.other_modalities = [m for i, m in enumerate(self.modalities) if i != model.main_modal_idx]
        self.max_context_len = model.max_context_len
        self.context_len = []
        for m in self.other_modalities:
            if m == "audio":
                self.context_len.append(self.max_context_len * acoustic_fps)
            elif m == "motion":
                self.context_len.append(self.max_context_len * model.pred_fps)
            else:
                raise ValueError("invalid modality")
        self.acoustic_input_size = (model.nmels + 1) * (model.delta_order + 1)
        self.motion_base_size = (model.use_centroid + model.use_angle) * 3
        self.motion_input_size = self.motion_base_size * (model.delta_order + 1)
        self.modal_num = len(self.modalities)
        self.hidden_dim, self.num_block, self.num_heads = model.hidden_size, model.num_block, model.num_heads
        mixers = list(model.emb_mixers)
        self.main_mixer_type = mixers[model.main_modal_idx]
        self.other_mixer_type = [m for i, m in enumerate(mixers) if i != model.main_modal_idx]
        self.repeat_with_encoder = model.repeat_with_encoder
        self.interlayer_residual = model.interlayer_residual
        self.interlayer_residual_norm = model.interlayer_residual_norm

        common = dict(hidden_size=self.hidden_dim, input_projection=False, output_projection=False,
                      self_attention=True, num_heads=model.num_heads, dropout=model.dropout,
                      batch_first=True, bidirectional=False, proj_size=model.proj_size,
                      add_bias_kv=model.add_bias_kv, add_zero_attn=model.add_zero_attn,
                      kdim=self.hidden_dim, vdim=self.hidden_dim, max_context_len=125,
                      num_layerd=model.num_layerd, num_internal_layer=model.num_internal_layer,
                      nonlinearity=model.nonlinearity, bottleneck_size=model.bottleneck_size,
                      residual=model.residual, residual_layer_norm=model.residual_layer_norm,
                      bias=model.bias)
        self.common_configs = common
        self.main_mixer_configs = mixer_layerd_argments_select(self.main_mixer_type, **common)
        enc = dict(common, num_layerd=model.encoder_num_layer)
        self.other_mixer_configs = [mixer_layerd_argments_select(t, **enc) for t in self.other_mixer_type]
        # the reference aliases ONE dict for every integrator, so the last context length wins (Q4)
        shared = mixer_layerd_argments_select("mha", **dict(common, self_attention=False))
        self.integrate_mixer_configs = [shared] * (self.modal_num - 1)
        for c in self.context_len:
            shared["max_context_len"] = c
        self.feedforward_configs = feedforward_block_argments(
            self.hidden_dim, model.bottleneck_size, nonlinearity=model.ffn_nonlinearity,
            residual=model.residual, residual_layer_norm=model.residual_layer_norm, bias=model.bias)
        self.output_feedforward_configs = feedforward_block_argments(
            self.hidden_dim, model.bottleneck_size, output_size=self.motion_input_size,
            nonlinearity=model.ffn_nonlinearity, residual=False, bias=model.bias)
        self.metaformer = MultiModalMetaformer(
            modal_num=self.modal_num, hidden_dim=self.hidden_dim, num_layer=self.num_block,
            main_modal_feature_dim=self.motion_input_size, main_mixer_type=self.main_mixer_type,
            main_mixer_configs=self.main_mixer_configs, integrate_mixer_configs=self.integrate_mixer_configs,
            feedforward_configs=self.feedforward_configs,
            output_feedforward_configs=self.output_feedforward_configs,
            other_modal_feature_dim=[self.acoustic_input_size, self.motion_input_size],
            other_mixer_type=self.other_mixer_type, other_mixer_configs=self.other_mixer_configs,
            repeat_with_encoder=self.repeat_with_encoder, interlayer_residual=self.interlayer_residual,
            interlayer_residual_norm=self.interlayer_residual_norm)
        self.optimizer = None
        self.lr_scheduler = None
        self.delta_loss_scale = model.get("delta_loss_scale", 1.0)
        self.delta_order = metrics.delta_order
        self.target_dict = gen_target_dict(metrics)

    @_in_precision
    def forward(self, acoustic_partner, motion_partner, motion_self, leading_acoustic_partner,
                leading_motion_partner, leading_motion_self, hxs=None):
        dev = self.device
        a = _cat_lead(leading_acoustic_partner[0].to(dev), acoustic_partner[0].to(dev))
        mp = _cat_lead(leading_motion_partner[0].to(dev), motion_partner[0].to(dev))
        ms = _cat_lead(leading_motion_self[0].to(dev), motion_self[0].to(dev))
        T = mp.shape[1]
        if torch.is_grad_enabled() and mp.shape[0] * T >= 2048:
            # a training forward over whole sequences: the bf16 planes of every weight, once per step
            # (functional.prepare_weight_planes; per-frame decode forwards keep the step's planes)
            Fn.prepare_weight_planes(self.parameters())
        mm = gen_attention_mask(ms, mp, self.num_heads, PADDING_VALUE).view(-1, T, T)
        ma = gen_attention_mask(ms, a, self.num_heads, PADDING_VALUE).view(-1, T, a.shape[1])
        self_masks = [gen_attention_mask(x, x, self.num_heads, PADDING_VALUE) if t == "mha" else None
                      for x, t in ((a, self.other_mixer_type[0]), (mp, self.other_mixer_type[1]))]
        ms_mask = gen_attention_mask(ms, ms, self.num_heads, PADDING_VALUE) if self.main_mixer_type == "mha" else None
        y, _, hxs = self.metaformer(ms, [a, mp], hxs, (None, None, ms_mask),
                                    [(None, None, self_masks[0]), (None, None, self_masks[1])], [ma, mm])
        return y, hxs

    def lossfun(self):
        return _TorchLoss(self.model.loss_type, self.model.loss_reduction, self.huber_delta, self.smoothl1_beta)

    def configure_optimizers(self):
        return self._optimizers(self.optim)

    def _masked_loss(self, y, target, lead):
        return Fn.masked_loss(y, target.to(y.device), lead, self.model.loss_type, self.huber_delta,
                              self.smoothl1_beta, True, self.delta_order, self.delta_loss_scale)

    @_in_precision
    def training_step(self, batch: List, *args, sampling_mask=None):
        if self.use_scheduled_sampling:
            self.log("scheduled_sampling_rate", self.current_epoch / self.max_epochs, logger=True)
            pred = self._generate(batch, use_scheduled_sampling=True, sampling_mask=sampling_mask)
            # the reference's loss over the [T, B, T, F] broadcast target (Q9, lstmformer.py:372-380)
            loss = Fn.broadcast_masked_loss(pred, batch[-1][0].to(pred.device), batch[2][0].to(pred.device),
                                            self.model.loss_type, self.huber_delta, self.smoothl1_beta, True,
                                            self.delta_order, self.delta_loss_scale)
        else:
            lead = batch[4][0].shape[1]
            target = batch[-1][0]
            ms = batch[2][0].to(self.device)
            batch[2] = (Fn.zero_padding(ms, PADDING_VALUE), batch[2][1])
            y, _ = self.forward(*batch[:-1])
            loss = self._masked_loss(y, target, lead)
        self.log("train_loss", loss, prog_bar=True, logger=True)
        return {"loss": loss}

    @_in_precision
    def validation_step(self, batch: List, *args):
        lead = batch[4][0].shape[1]
        y, _ = self.forward(*batch[:-1])
        loss = Fn.masked_loss(y, batch[-1][0].to(y.device), lead, self.model.loss_type, self.huber_delta,
                              self.smoothl1_beta, True)
        self.log("val_loss", loss, prog_bar=True, logger=True)
        gen_loss = self.generation_step(batch)["loss"]
        return {"loss": loss, "gen_loss": gen_loss}

    @_in_precision
    def generation_step(self, batch: List, sampling_mask=None):
        """genrt_loss (lstmformer.py:410-424): teacher-forced generation, loss over the broadcast
        [T, B, T, F] target of prediction (Q9), no scaler."""
        pred = self._generate(batch, sampling_mask=sampling_mask)
        loss = Fn.broadcast_masked_loss(pred, batch[-1][0].to(pred.device), batch[2][0].to(pred.device),
                                        self.model.loss_type, self.huber_delta, self.smoothl1_beta, scaler=False)
        self.log("genrt_loss", loss, prog_bar=False, logger=True)
        return {"loss": loss}

    # ---------------- autoregressive generation (lstmformer.py:426-559)
    @_in_precision
    def prediction(self, batch: List, use_scheduled_sampling: bool = False, full_generation: bool = False,
                   sampling_mask=None):
        """Stateless step-by-step generation (the reference never carries state, Q1).

        Returns (prediction [B, T, F], target) with the reference's target: batch target [B, T, F]
        times motion_s_mask [T, B, 1, F], i.e. the BROADCAST [T, B, T, F] tensor of
        lstmformer.py:434-435 (Q9).  The training / generation losses never form it
        (``Fn.broadcast_masked_loss``).  ``sampling_mask`` ([T] bool) overrides the mask drawn from
        the flags; on the GPU it selects on the device, so the whole generation can be captured as
        one HIP graph (``graphs.capture``).
        """
        pred = self._generate(batch, use_scheduled_sampling, full_generation, sampling_mask)
        ms = batch[2][0].to(pred.device)
        target = batch[-1][0].to(pred.device) * (ms.transpose(0, 1).unsqueeze(2) != PADDING_VALUE).to(ms.dtype)
        return pred, target

    def _generate(self, batch: List, use_scheduled_sampling: bool = False, full_generation: bool = False,
                  sampling_mask=None):
        """head_motion_generation (lstmformer.py:466-521) after form_generation_init (:523-547)."""
        dev = self.device
        (fb, lf), (mp, lp), (ms, ls) = batch[0], batch[1], batch[2]
        T, B = mp.shape[1], mp.shape[0]
        # time-major copies made once: every per-frame slice below is then contiguous, so the
        # ops of the T single-frame forwards run on it in place (no per-frame layout copies)
        fb = fb.to(dev).view(B, T, self.ratio, fb.shape[-1]).transpose(0, 1).contiguous()
        mp = mp.to(dev).transpose(0, 1).unsqueeze(2).contiguous()
        ms = ms.to(dev).transpose(0, 1).unsqueeze(2).contiguous()
        fb = fb * (fb != PADDING_VALUE).to(fb.dtype)
        mp = mp * (mp != PADDING_VALUE).to(mp.dtype)
        ms = ms * (ms != PADDING_VALUE).to(ms.dtype)
        if sampling_mask is not None:
            mask = sampling_mask
        elif use_scheduled_sampling:
            mask = torch.rand(T) < (self.current_epoch / self.max_epochs)
        else:
            mask = torch.ones(T, dtype=torch.bool) if full_generation else torch.zeros(T, dtype=torch.bool)
        if not torch.is_grad_enabled():
            # inference: the frame loop on the fused per-frame kernels (generate.py); the warm-up
            # forward below only makes a state no frame reads, so it is skipped there
            from ..generate import plan_for
            plan = plan_for(self)
            if plan is not None:
                return plan.generate(fb, mp, ms, mask)
        empty = [(torch.empty(x.shape[0], 0, x.shape[2], device=dev), n) for x, n in batch]
        _, cell = self.forward(*empty[:3], *batch[3:6], hxs=None)
        on_device = mask.device.type != "cpu"
        y = ms[0]
        preds = []
        ones = torch.ones(B, dtype=torch.long)
        for step in range(T):
            y, cell = self.forward((fb[step], lf), (mp[step], lp), (y, ones), *empty[3:6], cell)
            preds.append(y)
            if on_device:
                y = torch.where(mask[step], y, ms[step])
            else:
                y = y if bool(mask[step]) else ms[step]
        return torch.cat(preds, dim=1)


class LSTMwithSample(LightningSurface):
    """Sampled-audio LSTM predictor with scheduled sampling (lstm_with_sample.py:59-463)."""

    def __init__(self, model, optim, metrics):
        super().__init__()
        model, optim, metrics = as_attr(model), as_attr(optim), as_attr(metrics)
        self.model, self.optim, self.metrics = model, optim, metrics
        self.set_precision(model.get("precision", "32"))
        self.max_epochs = model.max_epochs
        self.use_scheduled_sampling = model.use_scheduled_sampling
        _loss_type_of(model)
        self.huber_delta = model.get("huber_delta", 1.0)
        self.smoothl1_beta = model.get("smoothl1_beta", 1.0)
        self.ratio = int(model.sampling_rate / model.shift / model.pred_fps)
        motion = (model.use_centroid + model.use_angle) * 3 * (model.delta_order + 1) * 2
        acoustic = (model.nmels + 1) * (model.delta_order + 1)
        self.acoustic_projection = Linear(acoustic, model.sampler_hidden_size)
        self.sampling_lstm = LSTMSampler(model.sampler_hidden_size, model.sampler_num_layers,
                                         model.sampler_dropout_rate, self.ratio, bidirectional=False)
        self.feature_projection = Linear(motion + model.sampler_hidden_size, model.hidden_size)
        self.layerd_lstm = LSTMLayerd(
            input_size=model.hidden_size, lstm_hidden_size=model.hidden_size,
            affine_hidden_size=model.hidden_size, bottleneck_size=model.bottleneck_size,
            num_layers=model.num_layers, num_layers_per_block=model.num_lstm, output_size=model.hidden_size,
            dropout=model.dropout_rate, bidirectional=False, use_layer_norm=model.use_layer_norm,
            use_mixing=model.use_mixing, use_residual=model.use_residual, use_feed_forward=False)
        ff = OrderedDict()
        ff["input"] = Linear(model.hidden_size, model.bottleneck_size)
        if model.use_relu:
            ff["relu"] = nn.ReLU()
        ff["mapping"] = Linear(model.bottleneck_size, motion // 2)
        self.feed_forward = nn.Sequential(ff)
        self.optimizer = None
        self.lr_scheduler = None
        self.delta_loss_scale = model.get("delta_loss_scale", 1.0)
        self.all_static = model.get("all_static", False)
        self.delta_order = metrics.delta_order
        self.target_dict = gen_target_dict(metrics)

    @_in_precision
    def forward(self, acoustic_partner, motion_partner, motion_self, leading_acoustic_partner,
                leading_motion_partner, leading_motion_self, cell_state=None):
        dev = self.device
        ms_len = motion_self[1]
        hx_sampler, hxs = (None, None) if cell_state is None else cell_state
        la, lmp = leading_acoustic_partner[0].to(dev), leading_motion_partner[0].to(dev)
        a = _cat_lead(la, acoustic_partner[0].to(dev))
        mp = _cat_lead(lmp, motion_partner[0].to(dev))
        ms = _cat_lead(leading_motion_self[0].to(dev), motion_self[0].to(dev))
        lead_len, motion_len = lmp.shape[1], mp.shape[1]
        a = self.acoustic_projection(a)
        a, hx_sampler = self.sampling_lstm(a, hx_sampler)
        if not (a.shape[1] == mp.shape[1] == ms.shape[1]):
            raise RuntimeError(f"acoustic: {a.shape} motion_p: {mp.shape} motion_s: {ms.shape} ratio: {self.ratio}")
        features = self.feature_projection(torch.cat([a, mp, ms], dim=-1))
        h, hxs = self.layerd_lstm(features, hxs)
        y = run_sequential_ffn(self.feed_forward, h)
        return y, (lead_len, motion_len, ms_len), (hx_sampler, hxs)

    def lossfun(self):
        return _TorchLoss(self.model.loss_type, self.model.loss_reduction, self.huber_delta, self.smoothl1_beta)

    def configure_optimizers(self):
        return self._optimizers(self.optim)

    @_in_precision
    def training_step(self, batch: List, *args, sampling_mask=None):
        if self.use_scheduled_sampling:
            self.log("scheduled_sampling_rate", self.current_epoch / self.max_epochs, logger=True)
            y, target = self.prediction(batch, use_scheduled_sampling=True, sampling_mask=sampling_mask)
            lead = 0
        else:
            y, (lead, _, _), _ = self.forward(*batch[:-1])
            target = batch[-1][0]
        loss = Fn.masked_loss(y, target.to(y.device), lead, self.model.loss_type, self.huber_delta,
                              self.smoothl1_beta, True, self.delta_order, self.delta_loss_scale)
        self.log("train_loss", loss, prog_bar=True, logger=True)
        return {"loss": loss}

    @_in_precision
    def validation_step(self, batch: List, *args):
        y, (lead, _, _), _ = self.forward(*batch[:-1])
        loss = Fn.masked_loss(y, batch[-1][0].to(y.device), lead, self.model.loss_type, self.huber_delta,
                              self.smoothl1_beta, True)
        self.log("val_loss", loss, prog_bar=True, logger=True)
        pred, target = self.prediction(batch)
        gen_loss = Fn.masked_loss(pred, target, 0, self.model.loss_type, self.huber_delta, self.smoothl1_beta, True)
        return {"loss": loss, "gen_loss": gen_loss}

    @_in_precision
    def prediction(self, batch: List, use_scheduled_sampling: bool = False, full_generation: bool = False,
                   sampling_mask=None):
        """Autoregressive decode (lstm_with_sample.py:339-433).

        The sampler state is carried across steps; the layered LSTM restarts
        from zero every step (Q2); teacher forcing feeds motion_s[step] (Q10).
        ``sampling_mask`` overrides the global-RNG draw (tests pin it); on the GPU it makes the
        step graph-capturable (``graphs.capture``).
        """
        dev = self.device
        (fb, lf), (mp, lp), (ms, ls) = batch[0], batch[1], batch[2]
        T, B = mp.shape[1], mp.shape[0]
        target = batch[-1][0].to(dev)
        if sampling_mask is None:
            if use_scheduled_sampling:
                sampling_mask = torch.rand(T) < (self.current_epoch / self.max_epochs)
            else:
                sampling_mask = (torch.ones if full_generation else torch.zeros)(T, dtype=torch.bool)
        # the fused decode computes in fp32 only: under precision='bf16' the per-frame path runs, so
        # every product of the step follows the selected arithmetic (as _LSTMCellFn's fused step does)
        if self.use_fused_decode and Fn._ARITH[0] is None and self._fused_params() is not None:
            return self._fused_prediction(batch, sampling_mask), target
        # time-major copies made once: every per-frame slice below is then contiguous, so the
        # ops of the T single-frame forwards run on it in place (no per-frame layout copies)
        fb = fb.to(dev).view(B, T, self.ratio, fb.shape[-1]).transpose(0, 1).contiguous()
        mp = mp.to(dev).transpose(0, 1).unsqueeze(2).contiguous()
        ms = ms.to(dev).transpose(0, 1).unsqueeze(2).contiguous()
        empty = [(torch.empty(x.shape[0], 0, x.shape[2], device=dev), n) for x, n in batch]
        _, _, cell = self.forward(*empty[:3], *batch[3:6], cell_state=None)
        y = ms[0]
        preds = []
        ones = torch.ones(B, dtype=torch.long)
        # a device-resident mask selects on the GPU (same values and gradients as the host branch):
        # no host read per frame, so the whole decode + backward can be captured in one HIP graph
        on_device = torch.is_tensor(sampling_mask) and sampling_mask.device.type != "cpu"
        for step in range(T):
            y, _, cell = self.forward((fb[step], lf), (mp[step], lp), (y, ones), *empty[3:6], cell)
            preds.append(y)
            if on_device:
                y = torch.where(sampling_mask[step], y, ms[step])
            else:
                y = y if bool(sampling_mask[step]) else ms[step]
        return torch.cat(preds, dim=1), target

    # ---------------- fused decode (decode.py / decode.hip)
    use_fused_decode = True

    def _fused_params(self):
        """Parameters of the fused decode, or None when this configuration is outside it (the
        per-frame path above then runs): layered blocks = residual LN around a 1-layer
        unidirectional LSTM without mixing or feed-forward, FFN = Linear -> ReLU -> Linear."""
        try:
            layers = []
            for blk in self.layerd_lstm.lstm_layered:
                rc = blk.lstm_module
                if blk.use_feed_forward or not isinstance(rc, ResidualConnection) or rc.layer_norm is None:
                    return None
                mod = rc.module
                if mod.mixer is not None:
                    return None
                lstm = mod.lstm_module
                if lstm.num_layers != 1 or lstm.bidirectional:
                    return None
                ln = rc.layer_norm
                layers.append((*lstm.direction_params(0), ln.weight, ln.bias))
            ff = list(self.feed_forward.children())
            if len(ff) != 3 or not isinstance(ff[1], nn.ReLU):
                return None
            H = self.feature_projection.weight.shape[0]
            if not (4 <= H <= 256 and H % 4 == 0 and ff[0].weight.shape[0] <= 64 and ff[2].weight.shape[0] <= 8):
                return None
            if any(p[4].shape[0] != H or abs(rc.layer_norm.eps - 1e-5) > 0 for p in layers):
                return None
            return layers, (ff[0].weight, ff[0].bias, ff[2].weight, ff[2].bias)
        except AttributeError:
            return None

    def _fused_prediction(self, batch, sampling_mask):
        """head_motion_generation with the sampler over the whole audio sequence in one pass and the
        per-frame chain in the fused kernels (decode.py).  Equivalent to the per-frame path: the
        sampler state the reference carries (warm-up over the lead, then frame by frame) is the
        state of one LSTM pass over [lead audio | frame audio]."""
        from ..decode import scheduled_sampling_decode
        dev = self.device
        a = _cat_lead(batch[3][0].to(dev), batch[0][0].to(dev))
        a, _ = self.sampling_lstm(self.acoustic_projection(a), None)
        lead, T = batch[4][0].shape[1], batch[1][0].shape[1]
        if a.shape[1] != lead + T:
            raise RuntimeError(f"acoustic: {a.shape} motion frames: {lead} + {T} ratio: {self.ratio}")
        layers, ffn = self._fused_params()
        return scheduled_sampling_decode(a[:, lead:], batch[1][0], batch[2][0], sampling_mask,
                                         self.feature_projection.weight, self.feature_projection.bias,
                                         layers, ffn, eps=self.layerd_lstm.lstm_layered[0].lstm_module.layer_norm.eps)


class AcousticEncoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.embed_layer = Linear(cfg.acostic_feat_size, cfg.acostic_affine_size)
        self.acostic_lstm = LSTMLayerd(
            input_size=cfg.acostic_affine_size, lstm_hidden_size=cfg.acostic_lstm_size,
            affine_hidden_size=cfg.acostic_affine_size, num_layers=cfg.acostic_num_layers,
            num_layers_per_block=cfg.acostic_num_lstm, output_size=cfg.acostic_output_size,
            dropout=cfg.dropout_rate, bidirectional=cfg.bidirectional, use_layer_norm=cfg.use_layer_norm,
            use_relu=cfg.use_relu, use_mixing=cfg.use_mixing, use_residual=cfg.use_residual)

    def forward(self, acoustic_feature):
        # the reference returns LSTMLayerd's (tensor, hxs) tuple and crashes downstream (Q3);
        # the tensor is the only runnable reading
        return self.acostic_lstm(self.embed_layer(acoustic_feature))[0]


class MotionEncoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.embed_layer = Linear(cfg.motion_feat_size, cfg.motion_affine_size)
        self.motion_lstm = LSTMLayerd(
            input_size=cfg.motion_affine_size, lstm_hidden_size=cfg.motion_lstm_size,
            affine_hidden_size=cfg.motion_affine_size, num_layers=cfg.motion_num_layers,
            num_layers_per_block=cfg.motion_num_lstm, output_size=cfg.motion_output_size,
            dropout=cfg.dropout_rate, bidirectional=cfg.bidirectional, use_layer_norm=cfg.use_layer_norm,
            use_relu=cfg.use_relu, use_mixing=cfg.use_mixing, use_residual=cfg.use_residual)

    def forward(self, head_feature):
        return self.motion_lstm(self.embed_layer(head_feature))[0]


class MotionDecoder(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.decoder_lstm = LSTMLayerd(
            input_size=cfg.motion_output_size, lstm_hidden_size=cfg.decoder_lstm_size,
            affine_hidden_size=cfg.decoder_affine_size, bottleneck_size=cfg.decoder_bottleneck_size,
            num_layers=cfg.decoder_num_layers, num_layers_per_block=cfg.decoder_num_lstm,
            output_size=cfg.decoder_output_size, dropout=cfg.dropout_rate,
            bidirectional=cfg.decoder_bidirectional, use_layer_norm=cfg.decoder_use_layer_norm,
            use_relu=cfg.decoder_use_relu, use_mixing=cfg.decoder_use_mixing,
            use_residual=cfg.decoder_use_residual)
        ff = OrderedDict()
        ff["input"] = Linear(cfg.decoder_output_size, cfg.decoder_mapping_size)
        if cfg.decoder_use_relu:
            ff["relu"] = nn.ReLU()
        ff["output"] = Linear(cfg.decoder_mapping_size, cfg.output_size)
        self.mapping = nn.Sequential(ff)

    def seq_reshape(self, x):
        shape = list(x.shape)
        x = x.reshape(-1, x.shape[-2], x.shape[-1])[:, -1:, :]
        shape[-2] = 1
        return x.reshape(shape)

    def forward(self, att_embedded):
        y = self.decoder_lstm(att_embedded)[0]
        return run_sequential_ffn(self.mapping, self.seq_reshape(y))


class SimpleLSTM(LightningSurface):
    """Bi-LSTM encoders + cross-attention + bi-LSTM decoder (simple_lstm.py:146-269)."""

    def __init__(self, cfg, optim, metrics):
        super().__init__()
        cfg, optim, metrics = as_attr(cfg), as_attr(optim), as_attr(metrics)
        self.cfg, self.optim, self.metrics = cfg, optim, metrics
        self.set_precision(cfg.get("precision", "32"))
        self.acoustic_encoder = AcousticEncoder(cfg)
        self.motion_encoder = MotionEncoder(cfg)
        self.multimodal_att = MultimodalAttention(
            modal1_feat_size=cfg.acostic_output_size, modal2_feat_size=cfg.motion_output_size,
            num_head=cfg.att_heads, num_layers=cfg.att_num_layers, dropout=cfg.dropout_rate,
            use_residual=cfg.att_use_residual, use_layer_norm=cfg.att_use_layer_norm)
        self.motion_decoder = MotionDecoder(cfg)
        self.optimizer = None
        self.lr_scheduler = None
        self.delta_loss_scale = cfg.get("delta_loss_scale", 1.0)
        self.all_static = cfg.get("all_static", False)
        self.delta_order = metrics.delta_order

    # MI355X schedule: the acoustic and motion encoders' block-i recurrences share one launch
    # (layers.paired_lstm_layerd); MRG_PAIR_ENCODERS=0 runs the encoders one after the other
    pair_encoders = os.environ.get("MRG_PAIR_ENCODERS", "1") == "1"

    @_in_precision
    def forward(self, acoustic_feature, motion_feature):
        enc_a, enc_m = self.acoustic_encoder, self.motion_encoder
        xa, xm = enc_a.embed_layer(acoustic_feature), enc_m.embed_layer(motion_feature)
        out = paired_lstm_layerd([enc_a.acostic_lstm, enc_m.motion_lstm], [xa, xm]) if self.pair_encoders \
            else None
        ae, me = out if out is not None else (enc_a.acostic_lstm(xa)[0], enc_m.motion_lstm(xm)[0])
        return self.motion_decoder(self.multimodal_att(me, ae))

    def lossfun(self):
        return _TorchLoss("mse", "mean", 1.0, 1.0)

    def configure_optimizers(self):
        return self._optimizers(self.optim)

    def split_and_form(self, x, y):
        if self.delta_order == 0:
            return y
        size = (self.metrics.use_centroid + self.metrics.use_angle) * 3
        _y = y.split(size, dim=-1)[0]
        _x = x[:, -1:, :].split(size, dim=-1)[0]
        v = _y - _x
        if self.delta_order == 1:
            return torch.cat([_y, v], dim=-1)
        return torch.cat([_y, v, v - x[:, -1:, :].split(size, dim=-1)[1]], dim=-1)

    @_in_precision
    def training_step(self, batch, *args):
        a, m, target = batch
        dev = self.device
        y = self.forward(a.to(dev), m.to(dev))
        if self.all_static:
            y = self.split_and_form(m.to(dev), y)
        loss = Fn.masked_loss(y, target.to(dev), 0, "mse", mask_padding=False,
                              delta_order=self.delta_order, delta_loss_scale=self.delta_loss_scale)
        self.log("train_loss", loss, prog_bar=True, logger=True)
        return {"loss": loss}

    @_in_precision
    def validation_step(self, batch, *args):
        a, m, target = batch
        dev = self.device
        y = self.forward(a.to(dev), m.to(dev))
        if self.all_static:
            y = self.split_and_form(m.to(dev), y)
        loss = Fn.masked_loss(y, target.to(dev), 0, "mse", mask_padding=False)
        self.log("val_loss", loss, prog_bar=True, logger=True)
        return {"loss": loss}


MODEL_TYPE = ["simple_lstm", "lstmformer", "lstm_with_sampling"]


def load_model(model_type: str, model_path: str, cfg):
    """model_loader.load_model (model_loader.py:13-26) with a pickle-free checkpoint load."""
    cls = {"simple_lstm": SimpleLSTM, "lstmformer": Metaformer, "lstm_with_sampling": LSTMwithSample}
    if model_type not in cls:
        raise ValueError(f"model_type must be one of {MODEL_TYPE}")
    cfg = as_attr(cfg)
    model = cls[model_type](as_attr(cfg.model), as_attr(cfg.optim), as_attr(cfg.metrics))
    state = torch.load(model_path, map_location="cpu", weights_only=True)
    model.load_state_dict(state["state_dict"] if "state_dict" in state else state)
    return model
