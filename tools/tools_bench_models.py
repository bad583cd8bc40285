"""Step times of the other BASELINE configs (not the headline bench line): eager fwd+bwd+AdamW.

    python tools/tools_bench_models.py [steps] [C2|C3|C3tf|gen|gru|all] [graph]     (on a GPU box)

  graph=1 replays each step as one HIP graph (graphs.capture); C3's sampling mask then lives in a
  static device buffer refreshed from the host RNG draw before every replay.

  C2  simple_lstm, B=64, T=300 (fp32 arithmetic here; the BASELINE names bf16)
  C3  lstm_with_sampling, scheduled-sampling autoregressive training, B=64, T=300, lead 12,
      epoch 30/60 (sampling probability 0.5, mask from RandomState(7) as SURVEY §8d)
  C3' lstm_with_sampling teacher-forced, B=64, T=300
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # repo root
from multimodalreactiongeneration_amd import configs as C  # noqa: E402
from multimodalreactiongeneration_amd import functional as Fn  # noqa: E402
from multimodalreactiongeneration_amd.model import LSTMwithSample, SimpleLSTM  # noqa: E402
from multimodalreactiongeneration_amd.synthetic import make_batch, make_simple_batch, clone_batch  # noqa: E402

DEV = "cuda:0"


GRAPH = False


def timed(fn, steps, warm=2, pre=None):
    if GRAPH:
        from multimodalreactiongeneration_amd.graphs import capture
        replay = capture(fn, warm)

        def fn():
            if pre is not None:
                pre()
            replay()
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    only = sys.argv[2] if len(sys.argv) > 2 and sys.argv[2] != "all" else ""
    global GRAPH
    GRAPH = len(sys.argv) > 3 and sys.argv[3] == "1"
    out = {}
    torch.manual_seed(0)
    if only == "gen":
        return main_gen(steps, out)
    if only == "gru":
        return main_gru(steps, out)
    if only and only != "C2":
        return main_lws(steps, only, out)
    mc, oc, me = C.simple_lstm_config()
    m = SimpleLSTM(mc, oc, me).to(DEV)
    prec = os.environ.get("C2_PRECISION", "32")   # "bf16": the BASELINE configs[1] precision
    m.set_precision(prec)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_simple_batch(B=64, T=300, device=DEV)

    def step_simple():
        opt.zero_grad()
        m.training_step(batch)["loss"].backward()
        opt.step()
    ms = timed(step_simple, steps)
    out[f"C2_simple_lstm_{'fp32' if prec == '32' else prec}_B64_T300" + ("_graph" if GRAPH else "")] = {"ms_per_step": round(ms, 2), "frames_per_s": round(64 * 300 / ms * 1e3)}
    print(json.dumps(out), flush=True)
    if not only:
        main_lws(steps, only, out)
        main_gen(steps, out)


def main_gru(steps, out):
    """lstmformer with config_gru.yaml's embedding mixers (["gru"] * 3), B=64 T=300 r=1 train step."""
    from multimodalreactiongeneration_amd.model import Metaformer
    mc, oc, me = C.lstmformer_config(ratio=1, emb_mixers=("gru", "gru", "gru"))
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to(DEV)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=64, T=300, seed=1234, device=DEV)

    def step():
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward()
        opt.step()
    ms = timed(step, steps)
    key = "lstmformer_gru_B64_T300" + ("_graph" if GRAPH else "")
    out[key] = {"ms_per_step": round(ms, 2), "frames_per_s": round(64 * 300 / ms * 1e3)}
    print(json.dumps(out), flush=True)


def main_gen(steps, out):
    """lstmformer autoregressive generation (Metaformer.prediction, full_generation, no grad):
    SURVEY 8f rank 1; the reference logs this per clip in speed.log (visualize_metaformer.py)."""
    from multimodalreactiongeneration_amd.model import Metaformer
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to(DEV).eval()
    T = 300
    batch = make_batch(B=64, T=T, lead=12, seed=1234, device=DEV)
    mask = torch.ones(T, dtype=torch.bool, device=DEV) if GRAPH else None

    def gen():
        with torch.no_grad():
            m.prediction(batch, full_generation=True, sampling_mask=mask)
    ms = timed(gen, steps)
    key = "lstmformer_generation_B64_T300" + ("_graph" if GRAPH else "")
    out[key] = {"ms_per_clip_batch": round(ms, 2), "ms_per_frame": round(ms / T, 4),
                "frames_per_s": round(64 * T / ms * 1e3)}
    print(json.dumps(out), flush=True)


def main_lws(steps, only, out):
    for ss in (False, True):
        if only and only != ("C3" if ss else "C3tf"):
            continue
        mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=ss)
        torch.manual_seed(0)
        m = LSTMwithSample(mc, oc, me).to(DEV)
        m.current_epoch = 30
        opt = m.configure_optimizers()["optimizer"]
        batch = make_batch(B=64, T=300, lead=12 if ss else 0, seed=1234, device=DEV)
        mask = torch.from_numpy(np.random.RandomState(7).rand(300) < 0.5)
        if GRAPH:
            mask = mask.to(DEV)
        rng = np.random.RandomState(7)

        def refresh():  # the host draw of lstm_with_sample.py:389 into the static device mask
            mask.copy_(torch.from_numpy(rng.rand(300) < 0.5))

        def step_lws():
            opt.zero_grad()
            kw = {"sampling_mask": mask} if ss else {}
            m.training_step(batch if GRAPH else clone_batch(batch), **kw)["loss"].backward()
            opt.step()
        ms = timed(step_lws, steps, pre=refresh if ss else None)
        key = "C3_lstm_with_sampling_scheduled_sampling" if ss else "C3tf_lstm_with_sampling_teacher_forced"
        key += "_graph" if GRAPH else ""
        out[key] = {"ms_per_step": round(ms, 2), "frames_per_s": round(64 * 300 / ms * 1e3)}
        print(json.dumps(out), flush=True)
    Fn.check_errors()


if __name__ == "__main__":
    main()
