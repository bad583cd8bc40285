"""Synthetic batches in the reference's batch format.

Reference format (mr_gen/model/lstmformer/dataloader.py:91-99,114-121): a
``list`` of 7 ``(Tensor[B, T_i, F_i] float32, Tensor[B] int64 lengths)`` pairs,
ordered audio_partner, motion_partner, motion_self, lead_audio,
lead_motion_partner, lead_motion_self, target, each padded with -100
(``PADDING_VALUE``, dataloader.py:17).  Inputs are drawn from NumPy's legacy
``RandomState`` whose stream is frozen by NumPy policy, so the build container
and the GPU box regenerate identical tensors from a seed.
"""
from __future__ import annotations

import numpy as np
import torch

PADDING_VALUE = -100.0


def _pad(rs, B, T, F, lengths):
    x = rs.standard_normal((B, T, F)).astype(np.float32)
    if lengths is not None:
        for b, n in enumerate(lengths):
            x[b, n:] = PADDING_VALUE
    return x


def make_batch(B=64, T=300, lead=0, ratio=1, feat_audio=40, feat_motion=6, seed=1234,
               lengths=None, device="cpu"):
    """Return the 7-pair list of the lstmformer / lstm_with_sampling loaders.

    ``lengths`` (per batch element, in prediction frames) makes the batch ragged:
    frames past the length are set to -100 in every modality (audio scaled by ratio).
    """
    rs = np.random.RandomState(seed)
    a_len = None if lengths is None else [n * ratio for n in lengths]
    audio = _pad(rs, B, T * ratio, feat_audio, a_len)
    mp = _pad(rs, B, T, feat_motion, lengths)
    ms = _pad(rs, B, T, feat_motion, lengths)
    la = rs.standard_normal((B, lead * ratio, feat_audio)).astype(np.float32)
    lmp = rs.standard_normal((B, lead, feat_motion)).astype(np.float32)
    lms = rs.standard_normal((B, lead, feat_motion)).astype(np.float32)
    tgt = _pad(rs, B, T, feat_motion, lengths)
    full = [T] * B if lengths is None else list(lengths)

    def pair(arr, ln):
        return (torch.from_numpy(arr).to(device), torch.tensor(ln, dtype=torch.long))

    return [pair(audio, [n * ratio for n in full]), pair(mp, full), pair(ms, full),
            pair(la, [lead * ratio] * B), pair(lmp, [lead] * B), pair(lms, [lead] * B),
            pair(tgt, full)]


def make_simple_batch(B=4, T=100, feat_audio=40, feat_motion=6, out=6, seed=1234,
                      device="cpu"):
    """SimpleLSTM batch: (audio[B,T,Fa], motion[B,T,Fm], target[B,1,out]) (simple_lstm/dataloader.py:56-61)."""
    rs = np.random.RandomState(seed)
    a = torch.from_numpy(rs.standard_normal((B, T, feat_audio)).astype(np.float32))
    m = torch.from_numpy(rs.standard_normal((B, T, feat_motion)).astype(np.float32))
    t = torch.from_numpy(rs.standard_normal((B, 1, out)).astype(np.float32))
    return a.to(device), m.to(device), t.to(device)


def clone_batch(batch, device=None):
    """Deep copy (the reference's training_step mutates batch[2] in place, lstmformer.py:366)."""
    out = []
    for x, n in batch:
        x = x.clone() if device is None else x.to(device).clone()
        out.append((x, n.clone()))
    return out


def fill_params_randomstate(module: torch.nn.Module, seed: int = 0, scale: float = 0.08):
    """Deterministic weights from NumPy RandomState over the sorted state_dict.

    Both the reference (golden generation) and this build apply the same filler
    to identically named/shaped state_dicts, so full-width weights never need
    to be committed.  LayerNorm weights are drawn around 1.
    """
    rs = np.random.RandomState(seed)
    sd = module.state_dict()
    new = {}
    for k in sorted(sd.keys()):
        v = sd[k]
        arr = rs.standard_normal(tuple(v.shape)).astype(np.float32) * scale
        if "layer_norm.weight" in k or k.endswith("norm.weight"):
            arr = arr + 1.0
        new[k] = torch.from_numpy(arr).to(v.device)
    module.load_state_dict(new)
    return module
