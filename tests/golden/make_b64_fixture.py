"""Fixtures for the benchmarked workloads at their full size (B=64, T=300), float64 oracle answers.

The oracle (oracle/mrg_oracle.py, the CPU restatement pinned to the reference's goldens by
tests/test_oracle_golden.py) is run ONCE here in float64 on exactly the bench's inputs, and a sample
of the result is stored, because the full gradients (up to 13 M values) are too large to commit and
a CPU run at this size is too slow for a GPU-box test.  Per training workload:

  loss; the model output when it is small; per parameter: max|g|, sum g, sum g^2, the gradient and
  the post-AdamW parameter at 256 seeded random indices plus the argmax |g| index; the float64 sum
  of every initial parameter (the GPU test first checks it rebuilt the same weights).

Workloads (``python tests/golden/make_b64_fixture.py [name ...]``, default all):

  metaformer_b64_f64       bench.py main: lstmformer r=1, torch.manual_seed(0) weights,
                           make_batch(B=64, T=300, seed=1234)                       (BASELINE configs[3])
  lstm_with_sample_ss_b64_f64
                           bench.py step_c3: LSTMwithSample scheduled sampling, torch.manual_seed(0)
                           weights, epoch 30, make_batch(B=64, T=300, lead=12, seed=1234), the first
                           mask draw RandomState(7).rand(300) < 0.5                 (BASELINE configs[2])
  simple_lstm_b64_f64      bench.py step_c2: SimpleLSTM fp32, torch.manual_seed(0) weights,
                           make_simple_batch(B=64, T=300)                           (BASELINE configs[1] shape)
  metaformer_gen_b64_f64   bench.py gen: Metaformer.prediction at B=64 on 40 frames (lead 12,
                           seed 1234), full generation and the RandomState(7) < 0.5 mask: the whole
                           prediction [64, 40, 6] is stored                          

float64 so each fixture is the exact answer the fp32 GPU path is measured against (the fp32 CPU
oracle itself is up to 3.8e-4 from it on the lstmformer's ReLU FeedForward input layer: see
tests/test_gpu_models.py::test_benchmark_schedule_b64_vs_oracle).  Reference call sites restated:
lstmformer.py:313-385,426-547; lstm_with_sample.py:278-301,339-433; simple_lstm.py:181-255.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer, LSTMwithSample, SimpleLSTM  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch, make_simple_batch  # noqa: E402
from oracle import mrg_oracle as O  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
NSAMPLE = 256


def _sampled(loss, grads, after, sd, y=None, seed=2024):
    rs = np.random.RandomState(seed)
    out = {"loss": np.float64(loss.item()),
           "param_sum": np.float64(sum(v.double().sum().item() for v in sd.values()))}
    if y is not None:
        out["y"] = y.double().numpy()
    for k in sorted(grads):
        g = grads[k].reshape(-1)
        a = after[k].reshape(-1)
        n = g.numel()
        idx = np.unique(np.concatenate([rs.randint(0, n, size=min(NSAMPLE, n)),
                                        [int(g.abs().argmax())]])).astype(np.int64)
        out[f"idx/{k}"] = idx
        out[f"g/{k}"] = g[idx].numpy()
        out[f"after/{k}"] = a[idx].numpy()
        out[f"stat/{k}"] = np.array([g.abs().max().item(), g.sum().item(), (g * g).sum().item()])
    return out


def _f64(sd):
    return {k: v.detach().double() for k, v in sd.items()}


def _b64(batch):
    return [(x.double(), n) for x, n in batch]


def metaformer_b64_f64():
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in Metaformer(mc, oc, me).state_dict().items()}
    batch = make_batch(B=64, T=300, ratio=1, seed=1234)
    loss, _, grads, after = O.run_train_step(O.metaformer_training_loss, _f64(sd), oc, mc, _b64(batch))
    return _sampled(loss, grads, after, sd)


def lstm_with_sample_ss_b64_f64():
    mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=True)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in LSTMwithSample(mc, oc, me).state_dict().items()}
    T = 300
    batch = make_batch(B=64, T=T, lead=12, seed=1234)
    mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5)
    loss, y, grads, after = O.run_train_step(O.lstm_with_sample_training_loss, _f64(sd), oc, mc, _b64(batch),
                                             sampling_mask=mask)
    out = _sampled(loss, grads, after, sd, y=y)
    out["sampling_mask"] = mask.numpy()
    return out


def simple_lstm_b64_f64():
    cfg, oc, me = C.simple_lstm_config()
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in SimpleLSTM(cfg, oc, me).state_dict().items()}
    a, mo, t = make_simple_batch(B=64, T=300)
    loss, y, grads, after = O.run_train_step(O.simple_lstm_training_loss, _f64(sd), oc, cfg,
                                             a.double(), mo.double(), t.double())
    return _sampled(loss, grads, after, sd, y=y)


def metaformer_gen_b64_f64():
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    sd = {k: v.detach().clone() for k, v in Metaformer(mc, oc, me).state_dict().items()}
    T = 40
    batch = make_batch(B=64, T=T, lead=12, seed=1234)
    masks = {"full": torch.ones(T, dtype=torch.bool),
             "ss": torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5)}
    out = {"param_sum": np.float64(sum(v.double().sum().item() for v in sd.values()))}
    with torch.no_grad():
        for name, mask in masks.items():
            out[f"pred/{name}"] = O.metaformer_prediction(_f64(sd), mc, _b64(batch), mask).numpy()
            out[f"mask/{name}"] = mask.numpy()
    return out


WORKLOADS = {f.__name__: f for f in (metaformer_b64_f64, lstm_with_sample_ss_b64_f64, simple_lstm_b64_f64,
                                     metaformer_gen_b64_f64)}


def main(names):
    torch.set_num_threads(os.cpu_count() or 8)
    for name in names or list(WORKLOADS):
        t0 = time.time()
        out = WORKLOADS[name]()
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **out)
        loss = f"loss {float(out['loss']):.9f}, " if "loss" in out else ""
        print(f"wrote {path}: {loss}{len(out)} arrays, {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
