"""Data-loader features: one training batch's partner audio, 64 clips of
312 + 2 prediction frames (lead 12, delta order 2) at 16 kHz, nfft 400, hop 160, 26 mels.

    python tools/tools_bench_features.py        (on a GPU box)

GPU: AudioPreprocessor.features on the resident batch [64, samples] (one GEMM + one finish +
one delta launch) and clip by clip; CPU: the reference's algorithm (oracle.audio_features:
torch.stft MelSpectrogram + the per-frame log-power loop of audio.py:43-56), one thread as a
DataLoader worker runs it, on a sample of clips.
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd.features import AudioPreprocessor  # noqa: E402
from oracle import mrg_oracle as O  # noqa: E402


class _Cfg(dict):
    __getattr__ = dict.__getitem__


def main():
    N, F = 64, 314
    L = (F - 1) * 160 + 400
    g = torch.Generator().manual_seed(0)
    waves = torch.randn(N, L, generator=g) * 0.2
    ap = AudioPreprocessor(_Cfg(nfft=400, shift=160, nmels=26, sample_rate=16000, delta_order=2), "cuda:0")
    wd = waves.cuda()
    for _ in range(3):
        ap.features(wd)
    torch.cuda.synchronize()
    it = 50
    t0 = time.perf_counter()
    for _ in range(it):
        ap.features(wd)
    torch.cuda.synchronize()
    batch_ms = (time.perf_counter() - t0) / it * 1e3
    t0 = time.perf_counter()
    for _ in range(5):
        for i in range(N):
            ap.features(wd[i])
    torch.cuda.synchronize()
    per_clip_ms = (time.perf_counter() - t0) / 5 * 1e3
    torch.set_num_threads(1)
    S = 8
    O.audio_features(waves[0], 16000, 400, 160, 26, 2)
    t0 = time.perf_counter()
    for i in range(S):
        O.audio_features(waves[i], 16000, 400, 160, 26, 2)
    cpu_ms = (time.perf_counter() - t0) / S * N * 1e3
    print(json.dumps({"workload": "64 clips x 314 frames (50,640 samples) audio features, nfft 400 hop 160 26 mels, delta 2",
                      "gpu_batched_ms": round(batch_ms, 3), "gpu_clip_by_clip_ms": round(per_clip_ms, 2),
                      "cpu_reference_algorithm_ms": round(cpu_ms, 1), "cpu_sample": f"{S} clips, 1 thread, scaled to 64",
                      "speedup_batched_vs_cpu": round(cpu_ms / batch_ms, 1)}), flush=True)


if __name__ == "__main__":
    main()
