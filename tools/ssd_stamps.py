"""Diagnostics: per-frame phase times of the persistent scheduled-sampling decode forward
(decode_persist.hip, block 0's wall-clock stamps) on the C3 workload (B=64, T=300): median microseconds
per phase and per frame.

    python tools/ssd_stamps.py            (GPU box)
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib, configs as C  # noqa: E402
from multimodalreactiongeneration_amd.model import LSTMwithSample  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch  # noqa: E402

NAMES = ["z gather", "layer-1 input", "layer-1 gate/cell + layer-2 h gather", "layer-2 gate/cell + last h gather",
         "LayerNorm + FFN z + publish", "to next frame"]


def main():
    dev = torch.device("cuda", 0)
    mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=True)
    torch.manual_seed(0)
    m = LSTMwithSample(mc, oc, me).to(dev)
    T = 300
    batch = make_batch(B=64, T=T, lead=12, seed=1234, device=dev)
    mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5).to(dev)
    buf = torch.zeros(T * 8, dtype=torch.int64, device=dev)
    lib = _lib.load()
    for rep in range(2):
        lib.mrg_ssd_persist_debug_stamps(ctypes.c_void_p(buf.data_ptr()) if rep else None)
        with torch.no_grad():
            m.prediction(clone_batch(batch, dev), use_scheduled_sampling=True, sampling_mask=mask)
        torch.cuda.synchronize()
    lib.mrg_ssd_persist_debug_stamps(None)
    st = buf.view(T, 8).cpu().numpy().astype(np.float64) / 100.0   # 100 MHz -> us
    # phases: 0 start, 1 z gathered, 2 layer-1 input in LDS, 3 layer-2 h gathered, 4 last h gathered, 5 z done
    d = np.stack([st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2], st[:, 4] - st[:, 3],
                  st[:, 5] - st[:, 4], np.r_[st[1:, 0] - st[:-1, 5], np.nan]], 1)[1:-1]
    for k, nm in enumerate(NAMES):
        print(f"{np.nanmedian(d[:, k]):8.2f} us  {nm}")
    print(f"{np.median(st[2:, 0] - st[1:-1, 0]):8.2f} us per frame (median); forward {(st[-1, 5] - st[0, 0]) / 1e3:.3f} ms")


if __name__ == "__main__":
    main()
