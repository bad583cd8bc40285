"""Segment dataset + collate on the MI355X vs the reference's own
HeadMotionDatasetNX.__getitem__ / collate_fn outputs (tests/golden/dataset.npz; the reference
ran its orchestration with its MotionPreprocessorNX and, torchaudio being absent, the oracle's
audio restatement).  Motion tensors and collate: bit-exact; audio: 1e-4 relative."""
import json
import os
import wave

import numpy as np
import pytest
import torch

from tests.golden_util import load, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class _Cfg(dict):
    __getattr__ = dict.__getitem__


def _write_dataset(d, root):
    with wave.open(os.path.join(root, "partner.wav"), "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(16000)
        f.writeframes(d["files/partner_wav"].tobytes())
    for who in ("partner", "self"):
        pre = f"files/{who}_npz/"
        np.savez(os.path.join(root, f"{who}.npz"), **{k[len(pre):]: d[k] for k in d.files if k.startswith(pre)})
    seg = json.loads(str(d["segment_json"]))
    for k in ("partner_motion", "partner_audio", "self_motion"):
        seg[k]["path"] = os.path.join(root, seg[k]["path"])
    with open(os.path.join(root, "seg_0001.json"), "w", encoding="utf-8") as f:
        f.write(json.dumps(seg) + "\n")


def test_segment_dataset_item_vs_reference(tmp_path):
    from multimodalreactiongeneration_amd.data import HeadMotionDatasetNX
    d = load("dataset")
    _write_dataset(d, str(tmp_path))
    ds = HeadMotionDatasetNX(str(tmp_path), _Cfg(delta_order=2, use_centroid=True, use_angle=True, train_by_std=False),
                             _Cfg(nfft=400, shift=160, nmels=26, sample_rate=16000, delta_order=2), DEV)
    assert len(ds) == 1
    item = ds[0]
    for i, t in enumerate(item):
        ref = torch.from_numpy(d[f"item/{i}"])
        assert t.shape == ref.shape, i
        if i in (0, 3):  # audio
            assert rel_err(t, ref) < 1e-4, i
        else:            # motion / target: bit-exact
            assert torch.equal(t.cpu(), ref), i


def test_collate_vs_reference_bit_exact():
    from multimodalreactiongeneration_amd.data import collate_fn
    d = load("dataset")
    batch = [tuple(torch.from_numpy(d[f"collate_in/{b}/{m}"]).to(DEV) for m in range(2)) for b in range(4)]
    out = collate_fn(batch)
    for m, (padded, lens) in enumerate(out):
        assert torch.equal(padded.cpu(), torch.from_numpy(d[f"collate_out/{m}"])), m
        assert torch.equal(lens, torch.from_numpy(d[f"collate_len/{m}"])), m
        assert lens.dtype == torch.int64 and padded.device.type == "cuda"
