"""Data-loader features on the MI355X vs the reference's own outputs
(tests/golden/features.npz, produced by importing mr_gen's preprocessors) and, for the
MelSpectrogram part whose torchaudio dependency is absent here, vs the oracle restatement
(parity of that part unpinned).  Tolerance for the float pipeline 1e-4 relative; the delta
stacking and the motion path are bit-exact.
"""
import os
import wave

import numpy as np
import pytest
import torch

from tests.golden_util import load, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = 1e-4


class _Cfg(dict):
    __getattr__ = dict.__getitem__


def _audio_cfg(nmels=26, d=2):
    return _Cfg(nfft=400, shift=160, nmels=nmels, sample_rate=16000, delta_order=d)


@pytest.mark.parametrize("nmels,d", [(26, 2), (39, 0), (40, 1)])
def test_audio_features_vs_oracle(nmels, d):
    from multimodalreactiongeneration_amd.features import AudioPreprocessor
    from oracle import mrg_oracle as O
    wv = torch.from_numpy(load("features")["wave"])
    got = AudioPreprocessor(_audio_cfg(nmels, d), DEV).features(wv.to(DEV))
    torch.cuda.synchronize()
    ref = O.audio_features(wv, 16000, 400, 160, nmels, d)
    assert got.shape == ref.shape
    assert rel_err(got, ref) < TOL


def test_log_power_vs_reference_golden():
    from multimodalreactiongeneration_amd.features import AudioPreprocessor
    d = load("features")
    got = AudioPreprocessor(_audio_cfg(), DEV).compute_log_power(torch.from_numpy(d["wave"]).to(DEV))
    assert rel_err(got, d["log_power"]) < 1e-5


def test_delta_kernel_bit_exact_vs_reference_golden():
    from multimodalreactiongeneration_amd.features import compute_delta
    d = load("features")
    x = torch.from_numpy(d["delta_in"]).to(DEV)
    for k in range(3):
        assert torch.equal(compute_delta(x, k).cpu(), torch.from_numpy(d[f"delta{k}"])), k
    assert compute_delta(x[:2], 2).shape == (0, 81)  # the reference's empty slice (its caller asserts)


@pytest.mark.parametrize("by_std,d", [(0, 0), (0, 2), (1, 0), (1, 2)])
def test_motion_preprocessor_vs_reference_golden(tmp_path, by_std, d):
    from multimodalreactiongeneration_amd.features import MotionPreprocessorNX
    g = load("features")
    path = os.path.join(tmp_path, "m.npz")
    np.savez(path, **{k[4:]: g[k] for k in g.files if k.startswith("npz/")})
    mp = MotionPreprocessorNX(_Cfg(delta_order=d, use_centroid=True, use_angle=True, train_by_std=bool(by_std)), DEV)
    got = mp(path, 3, 33, 2)
    assert torch.equal(got.cpu(), torch.from_numpy(g[f"motion/std{by_std}/d{d}"]))


def test_audio_preprocessor_reads_wav_segment(tmp_path):
    """__call__(wavepath, start, end) on a 16-bit PCM file: the segment decoded as the
    soundfile backend does (x / 32768) and featurised, vs the oracle on the same samples."""
    from multimodalreactiongeneration_amd.features import AudioPreprocessor
    from oracle import mrg_oracle as O
    rs = np.random.RandomState(5)
    pcm = (rs.randn(16000) * 3000).astype(np.int16)
    path = os.path.join(tmp_path, "a.wav")
    with wave.open(path, "wb") as f:
        f.setnchannels(1)
        f.setsampwidth(2)
        f.setframerate(16000)
        f.writeframes(pcm.tobytes())
    ap = AudioPreprocessor(_audio_cfg(), DEV)
    got = ap(path, 1000, 9000)
    ref = O.audio_features(torch.from_numpy(pcm[1000:9000].astype(np.float32) / 32768.0), 16000, 400, 160, 26, 2)
    assert rel_err(got, ref) < TOL
    with pytest.raises(ValueError):
        AudioPreprocessor(_Cfg(nfft=400, shift=160, nmels=26, sample_rate=8000, delta_order=2), DEV)(path, 0, 4000)
    with pytest.raises(ValueError):
        ap.features(torch.zeros(300, device=DEV))


def test_audio_features_batched_clips_equal_per_clip():
    """A batch [N, samples] runs as one GEMM + one finish + one delta launch; every clip's
    rows equal its own single-clip result (same arithmetic, same order)."""
    from multimodalreactiongeneration_amd.features import AudioPreprocessor
    g = torch.Generator().manual_seed(9)
    waves = (torch.randn(5, 16000 * 2 + 77, generator=g) * 0.2).to(DEV)
    ap = AudioPreprocessor(_audio_cfg(40, 2), DEV)
    batch = ap.features(waves)
    for i in range(5):
        assert torch.equal(batch[i], ap.features(waves[i]))
