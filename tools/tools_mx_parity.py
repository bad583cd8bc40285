"""Worst per-parameter gradient error vs the CPU oracle of the benchmark-width lstmformer step under
each recurrence / schedule mode (diagnostic for the MFMA recurrence and the encoder wavefront).

    python tools/tools_mx_parity.py            (on a GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib, configs as C  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch  # noqa: E402
from oracle import mrg_oracle as O  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / b.abs().max().clamp_min(1e-6)).item()


def main():
    B, T = int(os.environ.get("B", "4")), int(os.environ.get("T", "300"))
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to("cuda:0")
    batch = make_batch(B=B, T=T, seed=11)
    ref_loss, _, grads, _ = O.run_train_step(O.metaformer_training_loss, sd, oc, mc, clone_batch(batch))
    lib = _lib.load()
    for name, stack, mx in (("per-layer VALU", False, 0), ("per-layer MX", False, 2), ("stack default", True, 1),
                            ("stack VALU", True, 0)):
        lib.mrg_lstm_set_mx(mx, 0)
        m.metaformer.use_encoder_stack = stack
        for p in m.parameters():
            p.grad = None
        loss = m.training_step(clone_batch(batch, "cuda:0"))["loss"]
        loss.backward()
        torch.cuda.synchronize()
        errs = sorted(((rel(p.grad, grads[k]), k) for k, p in m.named_parameters()), reverse=True)
        print(f"{name:16s} loss rel {abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()):.2e}  worst grads: "
              + ", ".join(f"{e:.2e} {k.replace('metaformer.', '')[-60:]}" for e, k in errs[:3]), flush=True)


if __name__ == "__main__":
    main()
