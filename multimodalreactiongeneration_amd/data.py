"""Segment dataset and collate of the lstmformer / lstm_with_sampling loaders,
with the features computed on the MI355X.

``HeadMotionDatasetNX`` mirrors mr_gen/model/lstmformer/dataloader.py:20-110: a directory of
one-line JSON segment files written by DataBuilderNX (databuild_nx.py:296-342: per modality
``path``, ``seq`` / ``lead`` {start, end, stride}, motion ``offset``; ``target.shift_input_seq``),
each item the 7 tensors (partner fbank, partner motion, self motion, their lead windows, target)
— here device tensors from ``features.AudioPreprocessor`` / ``MotionPreprocessorNX``.
``collate_fn`` mirrors dataloader.py:114-121 (pack_sequence + pad_packed_sequence, batch_first,
padding -100): [(padded [B, Tmax, F], lengths int64)] * 7, padded by ``mrg_pad_sequences``.
"""
from __future__ import annotations

import json
import os
from typing import Any, Dict, List, Sequence

import torch

from . import _lib
from . import functional as Fn
from .features import AudioPreprocessor, MotionPreprocessorNX

PADDING_VALUE = -100.0


class HeadMotionDatasetNX(torch.utils.data.Dataset):
    def __init__(self, dataset_path: str, motion, audio, device=None) -> None:
        super().__init__()
        self.dataset_path = dataset_path
        self.data_list = self.load_segment_list()
        self.motion = motion
        self.audio = audio
        self.audio_preprocessor = AudioPreprocessor(audio, device)
        self.motion_preprocessor = MotionPreprocessorNX(motion, device)

    def __getitem__(self, index: int):
        with open(self.data_list[index], "r", encoding="utf-8") as f:
            lines = f.read().splitlines()
        if len(lines) > 1:
            raise ValueError("json file must have only one line.")
        jdic = json.loads(lines[0])
        pm, pa, sm, target = jdic["partner_motion"], jdic["partner_audio"], jdic["self_motion"], jdic["target"]
        op, os_ = pm["offset"], sm["offset"]
        ap, mp = self.audio_preprocessor, self.motion_preprocessor

        def motion(m, part, off):
            return mp(m["path"], m[part]["start"] - off, m[part]["end"] - off, m[part]["stride"])
        fbank_partner = ap(pa["path"], pa["seq"]["start"], pa["seq"]["end"])
        motion_partner = motion(pm, "seq", op)
        motion_self = motion(sm, "seq", os_)
        lead_fbank = ap(pa["path"], pa["lead"]["start"], pa["lead"]["end"])
        lead_partner = motion(pm, "lead", op)
        lead_self = motion(sm, "lead", os_)
        shift = target["shift_input_seq"]
        tgt = motion_self[shift:]
        motion_self = motion_self[: len(motion_self) - shift]
        return fbank_partner, motion_partner, motion_self, lead_fbank, lead_partner, lead_self, tgt

    def __len__(self) -> int:
        return len(self.data_list)

    def load_segment_list(self) -> List[str]:
        return [os.path.join(self.dataset_path, p) for p in os.listdir(self.dataset_path) if p.endswith(".json")]


def pad_sequences(seqs: Sequence[torch.Tensor], padding_value: float = PADDING_VALUE):
    """(padded [B, Tmax, F] on the sequences' device, lengths int64 on the host) like
    pad_packed_sequence(pack_sequence(seqs, enforce_sorted=False), batch_first=True)."""
    if not seqs:
        raise ValueError("empty batch")
    dev = seqs[0].device
    _lib.require_device(seqs[0])
    xs = [s.contiguous().float() for s in seqs]
    F = xs[0].shape[1] if xs[0].dim() == 2 else 1
    xs = [x.view(x.shape[0], F) for x in xs]
    lens = [x.shape[0] for x in xs]
    B, Tmax = len(xs), max(lens)
    out = torch.empty(B, Tmax, F, device=dev, dtype=torch.float32)
    table = torch.tensor([x.data_ptr() for x in xs], dtype=torch.int64).to(dev)
    dlens = torch.tensor(lens, dtype=torch.int32).to(dev)
    # the table and the sources are released to torch's stream-ordered caching allocator: any reuse
    # of their memory is queued behind this launch on the same stream
    _lib.check(_lib.load().mrg_pad_sequences(B, Tmax, F, Fn._ptr(table), Fn._ptr(dlens), padding_value,
                                             Fn._ptr(out), Fn._stream()), "pad sequences")
    if seqs[0].dim() == 1:
        out = out.view(B, Tmax)
    return out, torch.tensor(lens, dtype=torch.int64)


def collate_fn(batch):
    """lstmformer/dataloader.py:114-121 on device tensors: one (padded, lengths) pair per modal."""
    return [pad_sequences(list(modal)) for modal in zip(*batch)]
