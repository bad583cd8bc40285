"""Diagnostics (timing only): what each kernel family costs the replayed headline step's wall time.

Each variant makes the named libmrg entry points return without launching (ctypes attributes of the
loaded library replaced by a no-op), captures the bench's step (B=64, T=300, r=1, weight gradients on
the side stream, deferred beside the backward recurrences) and times 20 replays.  The difference to
the base step is that family's share of the critical path (its kernel time minus what ran hidden
beside other work).  Results are meaningless numerically; never used by bench.py.

    python tools/critical_path.py [variant ...]        (on a GPU box)
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import _lib, configs as C, functional as Fn  # noqa: E402
from multimodalreactiongeneration_amd.graphs import capture  # noqa: E402
from multimodalreactiongeneration_amd.model import Metaformer  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch  # noqa: E402

VARIANTS = {
    "base": [],
    "side": ["SIDE"],                                    # every weight-gradient / param-reduce fork
    "ln_param": ["mrg_residual_layernorm_param_reduce"],
    "lstm_fwd": ["mrg_lstm_fwd"],
    "lstm_bwd": ["mrg_lstm_bwd"],
    "attn_fwd": ["mrg_attention_fwd"],
    "attn_bwd": ["mrg_attention_bwd"],
    "ln_fwd": ["mrg_residual_layernorm_fwd"],
    "ln_bwd": ["mrg_residual_layernorm_bwd"],
    "ln_fwd_tiny": ["TINY:mrg_residual_layernorm_fwd"],      # a 1-workgroup kernel in place of each launch
    "ln_fwd_batched": ["=mrg_residual_layernorm_fwd_batched"],
    "ln_fwd_plain": ["=mrg_residual_layernorm_fwd", "=mrg_residual_layernorm_fwd_map"],
    "gemm_batched": ["=mrg_gemm_x6g_batched"],
    "gemm_all": ["=mrg_gemm_x6g_batched", "=mrg_gemm_f32_ex", "=mrg_gemm_f32"],
}


def _noop(*a, **k):
    return 0


def run(names):
    lib = _lib.load()
    saved = {}
    for n in names:
        if n == "SIDE":
            continue
        tiny = n.startswith("TINY:")
        exact = n.startswith("=")
        n = n.split(":")[-1].lstrip("=")
        for sym in list(_lib.SIGNATURES):
            hit = sym == n if exact else (sym.startswith(n) and "workspace" not in sym and "bytes" not in sym)
            if hit:
                saved[sym] = getattr(lib, sym)
                busy = saved.get("mrg_debug_busy", lib.mrg_debug_busy)
                setattr(lib, sym, (lambda *a, busy=busy: busy(1, 64, 256, 0.5, a[-1])) if tiny else _noop)
    side_saved = None
    if "SIDE" in names:
        import multimodalreactiongeneration_amd.encoder_stack as ES
        import multimodalreactiongeneration_amd.integrate as IG
        side_saved = (Fn._on_side, ES._on_side, IG._on_side)
        Fn._on_side = ES._on_side = IG._on_side = lambda device, rows, keep, fn, writes=None: None
    try:
        dev = torch.device("cuda", 0)
        mc, oc, me = C.lstmformer_config(ratio=1)
        torch.manual_seed(0)
        m = Metaformer(mc, oc, me).to(dev)
        opt = m.configure_optimizers()["optimizer"]
        batch = make_batch(B=64, T=300, seed=1234, device=dev)
        one = torch.ones((), device=dev)

        def step():
            opt.zero_grad()
            m.training_step(list(batch))["loss"].backward(one)
            opt.step()
        replay = capture(step, 2, preserve=opt.state_tensors())
        for _ in range(5):
            replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / 20 * 1e3
    finally:
        for sym, f in saved.items():
            setattr(lib, sym, f)
        if side_saved is not None:
            import multimodalreactiongeneration_amd.encoder_stack as ES
            import multimodalreactiongeneration_amd.integrate as IG
            Fn._on_side, ES._on_side, IG._on_side = side_saved
        Fn._ERR.clear()


def main(argv):
    names = argv or list(VARIANTS)
    base = None
    for rep in range(2):
        for v in names:
            ms = run(VARIANTS[v])
            if v == "base":
                base = ms
            d = "" if base is None or v == "base" else f"  (saves {base - ms:+.3f} ms)"
            print(f"rep {rep} {v:10s} {ms:8.3f} ms/step{d}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
