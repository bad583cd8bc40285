"""Narrow down the split-fork wrong-gradient replay: deferral off, one side-stream fork
per weight-gradient product in the encoder stack, replayed gradients vs the same backward on one
stream, for variants of the fork pattern.

    python tools/tools_fork_variants.py          (GPU box)
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd import encoder_stack as ES  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402
from multimodalreactiongeneration_amd.graphs import capture  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402

_orig_wg = ES._EncoderStackFn._weight_grads
_orig_exit = Fn._side.__exit__
ERR = []
MODE = {"split": lambda l: True, "serialize": False}


def _wg(lib, ch, st, gr, l, *a):
    ES.SPLIT_FORKS = MODE["split"](l)
    return _orig_wg(lib, ch, st, gr, l, *a)


def _exit(self, *exc):
    on_side = self.ctx is not None
    r = _orig_exit(self, *exc)
    if on_side and MODE["serialize"]:
        torch.cuda.current_stream().wait_stream(Fn._SIDE[torch.device(self.dev).index or 0])
    return r


ES._EncoderStackFn._weight_grads = staticmethod(_wg)
Fn._side.__exit__ = _exit


def run(m, opt, batch, replay_it):
    def step():
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward()
    step()
    torch.cuda.synchronize()
    if replay_it:
        r = capture(step, 1)
        opt.flat_grad.fill_(-1.0)
        r()
        torch.cuda.synchronize()
        err = Fn._err_flag(torch.device("cuda:0"))
        ERR.append(int(err.item()))
        err.zero_()
    return {k: p.grad.clone() for k, p in m.named_parameters()}


def main():
    Fn.set_wgrad_defer(False)
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to("cuda:0")
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=64, T=300, ratio=1, seed=5, device="cuda:0")
    Fn.set_wgrad_stream(False)
    ref = run(m, opt, batch, False)
    Fn.set_wgrad_stream(True)
    variants = [("split all", lambda l: True, False), ("split all + main waits after each fork", lambda l: True, True),
                ("split layer 0 only", lambda l: l == 0, False), ("split layers >= 1", lambda l: l >= 1, False),
                ("split layer 4 only", lambda l: l == 4, False), ("no split", lambda l: False, False)]
    for name, pred, ser in variants:
        MODE["split"], MODE["serialize"] = pred, ser
        g = run(m, opt, batch, True)
        bad = [k for k in ref if not torch.equal(g[k], ref[k])]
        print(f"{name:42s}: {len(bad)} params differ; recurrence hand-off timeout flag after replay: {ERR[-1]}",
              flush=True)
        for k in bad[:60]:
            a, b = g[k].flatten(), ref[k].flatten()
            zero = (a == 0).float().mean().item()
            ratio = (a.double() @ b.double() / max(1e-30, (b.double() @ b.double()).item())).item()
            print(f"    {k.replace('metaformer.', '').replace('metaformer_blocks.', 'b').replace('embedding.modal_embeddings.', 'me')}"
                  f": zeros {zero:.2f} proj-ratio {ratio:+.3f} max|d| {(a - b).abs().max().item():.2e} "
                  f"max|ref| {b.abs().max().item():.2e}", flush=True)


if __name__ == "__main__":
    main()
