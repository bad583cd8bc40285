"""Data-loader features on the MI355X: drop-in counterparts of the
reference's ``AudioPreprocessor`` (mr_gen/utils/preprocess/audio.py:6-67) and
``MotionPreprocessorNX`` (mr_gen/utils/preprocess/motion_nx.py:7-58).

Audio: the frames are never copied out of the waveform — one GEMM (``functional.gemm``, x6
arithmetic) multiplies them, read in place with row stride ``shift``, by the windowed DFT basis
[cos | sin] (a periodic Hann window folded in); ``mrg_fbank_finish`` forms |X_k|^2, applies
the HTK triangular mel filterbank of torchaudio's MelSpectrogram, takes log(max(., 1e-6)) and
appends the frame's log energy log(max(sum x^2, 1e-10)) (the reference computes that one in a
per-frame Python loop, audio.py:43-56); ``mrg_feature_delta`` stacks the deltas
(audio.py:58-67).  Results are float32 device tensors [frames - d, (nmels + 1)(d + 1)].

Motion: the npz slicing and the de-standardisation stay host-side numpy ops identical to the
reference's (they are the file read); the delta stacking runs on the device.

Files: WAV is read with the standard library (PCM 8/16/24/32-bit, what soundfile returns as
float32 in [-1, 1)); the reference reads through torchaudio's soundfile backend.
"""
from __future__ import annotations

import math
import wave as _wave
from typing import Optional

import numpy as np
import torch

from . import _lib
from . import functional as Fn


def dft_basis(nfft: int) -> torch.Tensor:
    """[2 * (nfft // 2 + 1), nfft] float32: rows k = w[n] cos(2 pi k n / N), then -w[n] sin(...)
    with w the periodic Hann window (torch.hann_window default, as MelSpectrogram uses)."""
    nf = nfft // 2 + 1
    n = np.arange(nfft, dtype=np.float64)
    w = 0.5 - 0.5 * np.cos(2.0 * math.pi * n / nfft)
    k = np.arange(nf, dtype=np.float64)[:, None]
    ang = 2.0 * math.pi * ((k * n[None, :]) % nfft) / nfft
    return torch.from_numpy(np.concatenate([w * np.cos(ang), -w * np.sin(ang)], 0).astype(np.float32))


def melscale_fbanks(n_freqs: int, f_min: float, f_max: float, n_mels: int, sample_rate: int) -> torch.Tensor:
    """HTK-scale triangular filterbank [n_freqs, n_mels], no area normalisation: the bank
    torchaudio.transforms.MelSpectrogram(sample_rate, n_fft, n_mels) builds (audio.py:16-22),
    computed in float32 like torchaudio does."""
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


def load_wav(path: str, start: int = 0, length: int = -1):
    """(waveform [channels, frames] float32 in [-1, 1), sample_rate), frames start..start+length
    (length -1: to the end), like the soundfile backend's load(path, frame_offset, num_frames)."""
    with _wave.open(path, "rb") as f:
        ch, width, sr, total = f.getnchannels(), f.getsampwidth(), f.getframerate(), f.getnframes()
        start = max(0, start)
        f.setpos(min(start, total))
        n = total - start if length < 0 else min(length, total - start)
        raw = f.readframes(max(0, n))
    if width == 1:
        x = (np.frombuffer(raw, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif width == 2:
        x = np.frombuffer(raw, "<i2").astype(np.float32) / 32768.0
    elif width == 3:
        b = np.frombuffer(raw, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        v = np.where(v >= 1 << 23, v - (1 << 24), v)
        x = v.astype(np.float32) / float(1 << 23)
    elif width == 4:
        x = (np.frombuffer(raw, "<i4").astype(np.float64) / 2147483648.0).astype(np.float32)
    else:
        raise ValueError(f"unsupported WAV sample width {width}")
    return torch.from_numpy(x.reshape(-1, ch).T.copy()), sr


def compute_delta(x: torch.Tensor, delta_order: int) -> torch.Tensor:
    """[x[d:], delta1[d-1:], delta2] (audio.py:58-67, motion_nx.py:49-58) on the device; x is
    [T, C] or a batch [N, T, C] of equal-length sequences."""
    if delta_order not in (0, 1, 2):
        raise ValueError("delta_order must be 0, 1 or 2")
    _lib.require_device(x)
    x = x.contiguous().float()
    T, C = x.shape[-2], x.shape[-1]
    N = x.shape[0] if x.dim() == 3 else 1
    out = torch.empty(*x.shape[:-2], max(T - delta_order, 0), C * (delta_order + 1), device=x.device,
                      dtype=torch.float32)
    if T <= delta_order or N == 0:
        return out  # empty, as the reference's slicing gives
    _lib.check(_lib.load().mrg_feature_delta(N, T, C, Fn._ptr(x), C, delta_order, Fn._ptr(out), Fn._stream()),
               "feature delta")
    return out


class AudioPreprocessor:
    """GPU ``AudioPreprocessor`` (audio.py:6-67): same config fields and call signature."""

    def __init__(self, cfg, device: Optional[torch.device] = None):
        self.cfg = cfg
        self.nfft = cfg.nfft
        self.shift = cfg.shift
        self.nmels = cfg.nmels
        self.sample_rate = cfg.sample_rate
        self.delta_order = cfg.delta_order
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.nfreq = self.nfft // 2 + 1
        if self.nfreq > 1025:
            raise ValueError("n_fft > 2048 is not supported")
        self.basis = dft_basis(self.nfft).to(self.device)
        self.melfb = melscale_fbanks(self.nfreq, 0.0, float(self.sample_rate // 2), self.nmels,
                                     self.sample_rate).contiguous().to(self.device)

    def __call__(self, wavepath: str, start: int, end: int) -> torch.Tensor:
        length = end if end == -1 else end - start
        waveform, sample_rate = load_wav(wavepath, start, length)
        if sample_rate != self.sample_rate:
            raise ValueError("sample_rate must be same as --sample-rate")
        out = self.features(waveform[0].to(self.device))
        assert len(out) != 0, f"start: {start}, end: {end}, stride: {1}"
        return out

    def fbank(self, waveform: torch.Tensor) -> torch.Tensor:
        """[frames, nmels + 1] (or [N, frames, nmels + 1] for a batch [N, samples] of equal-length
        clips, one launch each step): log mel energies and the log frame power (audio.py:33-36)."""
        _lib.require_device(waveform)
        x = waveform.contiguous().float()
        L = x.shape[-1]
        N = x.shape[0] if x.dim() == 2 else 1
        F = (L - self.nfft) // self.shift + 1
        if F <= 0:
            raise ValueError(f"waveform of {L} samples is shorter than n_fft={self.nfft}")
        nf, dev = self.nfreq, x.device
        rows = N * F
        spec = torch.empty(rows, 2 * nf, device=dev, dtype=torch.float32)
        # frame r of the batch: clip r // F, start (r % F) * shift (RowMap: ld_lo = shift, ld_hi = L)
        Fn.gemm(rows, 2 * nf, self.nfft, Fn._ptr(x), 0, self.shift, Fn._ptr(self.basis), 1, self.nfft,
                Fn._ptr(spec), 2 * nf, a_hi=L if N > 1 else 0, a_div=F if N > 1 else 0, device=dev)
        out = torch.empty(*x.shape[:-1], F, self.nmels + 1, device=dev, dtype=torch.float32)
        _lib.check(_lib.load().mrg_fbank_finish(rows, nf, self.nmels, Fn._ptr(spec), 2 * nf, Fn._ptr(self.melfb),
                                                Fn._ptr(x), self.shift, self.nfft, F, L, Fn._ptr(out),
                                                self.nmels + 1, Fn._stream()), "fbank finish")
        return out

    def features(self, waveform: torch.Tensor) -> torch.Tensor:
        """The __call__ result for a resident waveform [samples] (or a batch [N, samples])."""
        return self.compute_delta(self.fbank(waveform))

    def compute_log_power(self, waveform: torch.Tensor) -> torch.Tensor:
        return self.fbank(waveform)[:, -1].contiguous()

    def compute_delta(self, fbank: torch.Tensor) -> torch.Tensor:
        return compute_delta(fbank, self.delta_order)


class MotionPreprocessorNX:
    """``MotionPreprocessorNX`` (motion_nx.py:7-58); the delta stacking runs on the device."""

    def __init__(self, cfg, device: Optional[torch.device] = None):
        self.cfg = cfg
        self.delta_order: int = cfg.delta_order
        self.use_centroid: bool = cfg.use_centroid
        self.use_angle: bool = cfg.use_angle
        self.train_by_std: bool = cfg.train_by_std
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())

    def __call__(self, npz_path: str, start: int, end: int, stride: int) -> torch.Tensor:
        start += stride - 1
        end += stride - 1
        ac = np.load(npz_path)
        angle = ac["angle"][start:end:stride]
        centroid = ac["centroid"][start:end:stride]
        if not self.train_by_std:
            angle *= ac["angle_std"]
            angle += ac["angle_mean"]
            centroid *= ac["centroid_std"]
            centroid += ac["centroid_mean"]
        head_seq = torch.cat([torch.tensor(angle), torch.tensor(centroid)], dim=-1).to(torch.float32)
        out = self.compute_delta(head_seq.to(self.device))
        assert len(out) != 0, f"start: {start}, end: {end}, stride: {stride}, len: {len(ac['angle'])}\n{npz_path}"
        return out

    def compute_delta(self, head_seq: torch.Tensor) -> torch.Tensor:
        return compute_delta(head_seq, self.delta_order)
