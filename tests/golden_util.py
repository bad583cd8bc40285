"""Load committed golden fixtures (produced by tests/golden/make_golden.py from the reference)."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def config(d):
    return json.loads(str(d["meta/config"]))


def batch_from(d, device="cpu"):
    out = []
    for i in range(7):
        out.append((torch.from_numpy(d[f"in/{i}/x"]).to(device),
                    torch.from_numpy(d[f"in/{i}/len"])))
    return out


def prefixed(d, prefix, device="cpu"):
    return {k[len(prefix):]: torch.from_numpy(d[k]).to(device) for k in d.files if k.startswith(prefix)}


def rel_err(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()
