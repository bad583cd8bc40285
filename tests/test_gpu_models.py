"""Model-level parity on the MI355X: full training steps of the three models vs the reference goldens.

Each case loads the reference's weights (or regenerates them with the same
RandomState filler), runs ``training_step`` + backward + the fused AdamW on
the GPU, and compares loss, forward output, every parameter gradient and the
post-step parameters with what the reference itself produced
(tests/golden/*.npz).  Tolerance 1e-4 relative (fp32).
"""
import numpy as np
import pytest
import torch

from tests.golden_util import load, config, batch_from, prefixed, rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-4
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _done():
    yield
    from multimodalreactiongeneration_amd import functional as Fn
    torch.cuda.synchronize()
    Fn.check_errors()


def _build(cls, d, full_width_seed=None):
    cfg = config(d)
    m = cls(cfg["model"], cfg["optim"], cfg["metrics"])
    if full_width_seed is None:
        m.load_state_dict(prefixed(d, "param/"))
    else:
        from multimodalreactiongeneration_amd.synthetic import fill_params_randomstate
        fill_params_randomstate(m, full_width_seed)
    return m.to(DEV), cfg


def _check(d, m, loss, full=True):
    assert abs(loss.item() - float(d["loss"])) / abs(float(d["loss"])) < TOL
    for k, p in m.named_parameters():
        g = p.grad
        if f"grad/{k}" in d.files:
            assert rel_err(g, d[f"grad/{k}"]) < TOL, k
        elif f"gradsum/{k}" in d.files:
            ref = d[f"gradsum/{k}"]
            gg = g.double().cpu()
            assert abs(gg.sum().item() - ref[0]) <= TOL * max(abs(ref[0]), np.sqrt(ref[1]), 1e-6), k
            assert abs((gg ** 2).sum().item() - ref[1]) <= 1e-3 * max(ref[1], 1e-12), k


def _check_after(d, m):
    for k, p in m.named_parameters():
        if f"after/{k}" not in d.files:
            continue
        gref = torch.from_numpy(d[f"grad/{k}"])
        # AdamW's first step moves p by lr * g / (|g| + eps): entries with |g| within a few orders
        # of eps = 1e-8 turn a 1e-7 relative gradient difference into a visible update difference
        sel = gref.abs() > torch.clamp(1e-5 * gref.abs().max(), min=1e-6)
        if sel.any():
            assert rel_err(p.detach().cpu()[sel], torch.from_numpy(d[f"after/{k}"])[sel]) < TOL, k


def _train_step(m, batch, **kw):
    opt = m.configure_optimizers()["optimizer"]
    loss = m.training_step(batch, **kw)["loss"]
    loss.backward()
    torch.cuda.synchronize()
    return loss, opt


@pytest.mark.parametrize("name", ["metaformer_small_r1", "metaformer_small_r2_pad", "metaformer_gru_r2_pad"])
def test_metaformer_small_train_step(name):
    from multimodalreactiongeneration_amd.model import Metaformer
    d = load(name)
    m, cfg = _build(Metaformer, d)
    batch = batch_from(d, DEV)
    with torch.no_grad():
        m.eval()
        y_eval, _ = m.forward(*[(x.clone(), n) for x, n in batch[:-1]])
        assert rel_err(y_eval, d["y_eval"]) < TOL
        m.train()
        b2 = [(x.clone(), n) for x, n in batch]
        ms = b2[2][0]
        b2[2] = (ms * (ms != -100).float(), b2[2][1])
        y, _ = m.forward(*b2[:-1])
        assert rel_err(y, d["y"]) < TOL
    loss, opt = _train_step(m, batch)
    _check(d, m, loss)
    opt.step()
    torch.cuda.synchronize()
    _check_after(d, m)


def test_metaformer_full_width_train_step():
    from multimodalreactiongeneration_amd.model import Metaformer
    d = load("metaformer_full_r1")
    m, cfg = _build(Metaformer, d, full_width_seed=2)
    batch = batch_from(d, DEV)
    loss, _ = _train_step(m, batch)
    _check(d, m, loss)


def test_lstm_with_sample_teacher_forced():
    from multimodalreactiongeneration_amd.model import LSTMwithSample
    d = load("lstm_with_sample_tf")
    m, cfg = _build(LSTMwithSample, d)
    batch = batch_from(d, DEV)
    with torch.no_grad():
        y, _, _ = m.forward(*batch[:-1])
        assert rel_err(y, d["y"]) < TOL
    loss, opt = _train_step(m, batch)
    _check(d, m, loss)
    opt.step()
    torch.cuda.synchronize()
    _check_after(d, m)


def test_lstm_with_sample_scheduled_sampling():
    from multimodalreactiongeneration_amd.model import LSTMwithSample
    d = load("lstm_with_sample_ss")
    m, cfg = _build(LSTMwithSample, d)
    m.current_epoch = int(d["meta/epoch"])
    batch = batch_from(d, DEV)
    loss, opt = _train_step(m, batch, sampling_mask=torch.from_numpy(d["sampling_mask"]))
    _check(d, m, loss)
    opt.step()
    torch.cuda.synchronize()
    _check_after(d, m)


def test_lstm_with_sample_scheduled_sampling_graph_replay():
    """The same golden step with the mask in a device buffer, captured once as a HIP graph and
    replayed (graphs.capture): every gradient matches the reference's eager step."""
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import LSTMwithSample
    d = load("lstm_with_sample_ss")
    m, cfg = _build(LSTMwithSample, d)
    m.current_epoch = int(d["meta/epoch"])
    batch = batch_from(d, DEV)
    opt = m.configure_optimizers()["optimizer"]
    mask = torch.zeros(len(d["sampling_mask"]), dtype=torch.bool, device=DEV)
    loss_buf = torch.zeros((), device=DEV)

    def step():
        opt.zero_grad()
        loss = m.training_step(batch, sampling_mask=mask)["loss"]
        loss.backward()
        loss_buf.copy_(loss.detach())
    replay = capture(step, 1)
    mask.copy_(torch.from_numpy(d["sampling_mask"]))
    replay()
    torch.cuda.synchronize()
    _check(d, m, loss_buf)


def test_simple_lstm_train_step():
    from multimodalreactiongeneration_amd.model import SimpleLSTM
    d = load("simple_lstm_small")
    m, cfg = _build(SimpleLSTM, d)
    a, mo, t = (torch.from_numpy(d[k]).to(DEV) for k in ("in/audio", "in/motion", "in/target"))
    with torch.no_grad():
        assert rel_err(m.forward(a, mo), d["y"]) < TOL
    loss, opt = _train_step(m, (a, mo, t))
    _check(d, m, loss)
    opt.step()
    torch.cuda.synchronize()
    _check_after(d, m)


@pytest.mark.parametrize("ratio,B,T", [(1, 4, 300), (8, 2, 60)])
def test_metaformer_benchmark_width_vs_oracle(ratio, B, T):
    """Full benchmark architecture (H=256, 5 blocks, 5 encoder layers) at T=300 vs the CPU oracle."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    from oracle import mrg_oracle as O
    mc, oc, me = C.lstmformer_config(ratio=ratio)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    batch = make_batch(B=B, T=T, ratio=ratio, seed=11)
    loss = m.training_step(clone_batch(batch, DEV))["loss"]
    loss.backward()
    torch.cuda.synchronize()
    ref_loss, ref_y, grads, _ = O.run_train_step(O.metaformer_training_loss, sd, oc, mc, clone_batch(batch))
    assert abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()) < TOL
    errs = sorted(((rel_err(p.grad, grads[k]), k) for k, p in m.named_parameters()), reverse=True)
    assert errs[0][0] < TOL, errs[:6]


@pytest.mark.parametrize("mode", ["full", "tf", "ss"])
def test_metaformer_generation_golden(mode):
    """Metaformer.prediction (lstmformer.py:426-547) vs the reference's own output: T = 1 steps
    through the LSTM cell kernels, ratio 2, ragged padding; all three sampling modes."""
    from multimodalreactiongeneration_amd.model import Metaformer
    d = load("metaformer_gen_r2_pad")
    m, cfg = _build(Metaformer, d)
    m.eval()
    batch = batch_from(d, DEV)
    T = batch[1][0].shape[1]
    mask = {"full": torch.ones(T, dtype=torch.bool), "tf": torch.zeros(T, dtype=torch.bool),
            "ss": torch.from_numpy(d["sampling_mask"])}[mode]
    with torch.no_grad():
        pred, _ = m.prediction(batch, sampling_mask=mask)
    torch.cuda.synchronize()
    assert rel_err(pred, d[f"pred/{mode}"]) < TOL


def test_metaformer_generation_graph_replay():
    """The same generation captured once as a HIP graph with the mask in a device buffer and
    replayed for two different masks (graphs.capture)."""
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import Metaformer
    d = load("metaformer_gen_r2_pad")
    m, cfg = _build(Metaformer, d)
    m.eval()
    batch = batch_from(d, DEV)
    T = batch[1][0].shape[1]
    mask = torch.zeros(T, dtype=torch.bool, device=DEV)
    out = torch.zeros(batch[1][0].shape[0], T, 6, device=DEV)

    def gen():
        with torch.no_grad():
            out.copy_(m.prediction(batch, sampling_mask=mask)[0])
    replay = capture(gen, 1)
    for mode in ("ss", "full"):
        mask.copy_(torch.from_numpy(d["sampling_mask"]) if mode == "ss" else torch.ones(T, dtype=torch.bool))
        replay()
        torch.cuda.synchronize()
        assert rel_err(out, d[f"pred/{mode}"]) < TOL, mode


def test_metaformer_generation_benchmark_width_vs_oracle():
    """Benchmark architecture (H=256, 5 blocks, 5 encoder layers, r=1) generating 40 frames,
    scheduled-sampling mask RandomState(7) < 0.5, vs the CPU oracle restatement."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    from oracle import mrg_oracle as O
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).eval()
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    T = 40
    batch = make_batch(B=3, T=T, lead=4, seed=5)
    mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5)
    with torch.no_grad():
        pred, _ = m.prediction(clone_batch(batch, DEV), sampling_mask=mask)
        ref = O.metaformer_prediction(sd, mc, clone_batch(batch), mask)
    torch.cuda.synchronize()
    assert rel_err(pred, ref) < TOL


@pytest.mark.parametrize("defer,B", [(False, 8), (True, 64)])
def test_wgrad_side_stream_bitwise(defer, B):
    """Weight gradients on the side stream (functional._side), eager and graph-replayed, give the
    bit-identical gradients of the single-stream schedule (every kernel is deterministic).  With
    deferral the products run beside the next backward recurrence, which then takes one workgroup
    per CU (batch tile 4 instead of 2 at B = 64): the gradients are still bitwise the same."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to(DEV)
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=B, T=300, ratio=1, seed=5, device=DEV)

    def step():
        opt.zero_grad()
        m.training_step(list(batch))["loss"].backward()

    prev = Fn.set_wgrad_stream(False)
    prev_defer = Fn.set_wgrad_defer(defer)
    try:
        step()
        torch.cuda.synchronize()
        ref = opt.flat_grad.clone()
        Fn.set_wgrad_stream(True)
        step()
        torch.cuda.synchronize()
        assert torch.equal(opt.flat_grad, ref)
        replay = capture(step, 1)
        opt.flat_grad.zero_()
        replay()
        torch.cuda.synchronize()
        assert torch.equal(opt.flat_grad, ref)
        Fn.check_errors()
    finally:
        Fn.set_wgrad_stream(prev)
        Fn.set_wgrad_defer(prev_defer)


def test_metaformer_q9_broadcast_losses_golden():
    """the reference's genrt_loss (generation_step, lstmformer.py:410-424) and its
    scheduled-sampling training_step (:357-385) take the loss over target * motion_s_mask, a
    [T, B, T, F] broadcast (:434-435); ragged padding, delta_order 1, delta_loss_scale 2.  Loss,
    every gradient and the AdamW step vs the reference's own numbers."""
    from multimodalreactiongeneration_amd.model import Metaformer
    d = load("metaformer_q9_r2_pad")
    m, cfg = _build(Metaformer, d)
    m.current_epoch = int(d["meta/epoch"])
    batch = batch_from(d, DEV)
    m.eval()
    with torch.no_grad():
        pred, target4 = m.prediction([(x.clone(), n) for x, n in batch])
        assert rel_err(pred, d["gen/pred"]) < TOL
        assert tuple(target4.shape) == d["gen/target4"].shape
        assert torch.equal(target4.cpu(), torch.from_numpy(d["gen/target4"]))
        g = m.generation_step([(x.clone(), n) for x, n in batch])["loss"]
        assert abs(g.item() - float(d["genrt_loss"])) / float(d["genrt_loss"]) < TOL
    m.train()
    loss, opt = _train_step(m, batch, sampling_mask=torch.from_numpy(d["sampling_mask"]))
    _check(d, m, loss)
    opt.step()
    torch.cuda.synchronize()
    _check_after(d, m)


def test_lstm_with_sample_benchmark_width_vs_oracle():
    """BASELINE configs[2] architecture (H=256, sampler 2 x 128, r=1) at T=300: scheduled-sampling
    training step (mask RandomState(7) < 0.5, lead 12, ragged lengths) and the teacher-forced
    step, loss + every gradient vs the CPU oracle."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import LSTMwithSample
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    from oracle import mrg_oracle as O
    T = 300
    mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5)
    for scheduled in (True, False):
        mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=scheduled)
        torch.manual_seed(1)
        m = LSTMwithSample(mc, oc, me)
        m.current_epoch = 30
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        m = m.to(DEV)
        batch = make_batch(B=3, T=T, lead=12, seed=17, lengths=[300, 251, 177])
        kw = {"sampling_mask": mask} if scheduled else {}
        loss, _ = _train_step(m, clone_batch(batch, DEV), **kw)
        ref_loss, _, grads, _ = O.run_train_step(O.lstm_with_sample_training_loss, sd, oc, mc, clone_batch(batch),
                                                 **kw)
        assert abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()) < TOL, scheduled
        worst = max((rel_err(p.grad, grads[k]), k) for k, p in m.named_parameters())
        assert worst[0] < TOL, (scheduled, worst)


def test_simple_lstm_benchmark_width_vs_oracle():
    """BASELINE configs[1] architecture (bi-LSTM H=128 encoders x 2, 3 x 8-head cross attention,
    5-layer bi-LSTM decoder) at T=300, B=2, fp32: loss + every gradient vs the CPU oracle."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import SimpleLSTM
    from multimodalreactiongeneration_amd.synthetic import make_simple_batch
    from oracle import mrg_oracle as O
    cfg, oc, me = C.simple_lstm_config()
    torch.manual_seed(2)
    m = SimpleLSTM(cfg, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    a, mo, t = make_simple_batch(B=2, T=300, seed=19)
    loss, _ = _train_step(m, (a.to(DEV), mo.to(DEV), t.to(DEV)))
    ref_loss, _, grads, _ = O.run_train_step(O.simple_lstm_training_loss, sd, oc, cfg, a, mo, t)
    assert abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()) < TOL
    worst = max((rel_err(p.grad, grads[k]), k) for k, p in m.named_parameters())
    assert worst[0] < TOL, worst


@pytest.mark.parametrize("precision", ["32", "bf16"])
def test_simple_lstm_paired_encoders_match_sequential(precision):
    """configs[1] (B=64, T=300): the acoustic and motion encoders' recurrences sharing one launch per
    block (layers.paired_lstm_layerd, the default) give bitwise the loss and gradients of the two
    encoders run one after the other; the pairing did run (both LSTMs' paired results consumed)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import SimpleLSTM
    from multimodalreactiongeneration_amd.model import layers as LY
    from multimodalreactiongeneration_amd.synthetic import make_simple_batch
    cfg, oc, me = C.simple_lstm_config()
    torch.manual_seed(4)
    m = SimpleLSTM(cfg, oc, me).to(DEV)
    m.set_precision(precision)
    a, mo, t = (x.to(DEV) for x in make_simple_batch(B=64, T=300, seed=23))
    calls = []
    orig = LY.paired_lstm_layerd

    def spy(stacks, xs):
        out = orig(stacks, xs)
        calls.append(out is not None)
        return out
    res = {}
    try:
        LY_models = __import__("multimodalreactiongeneration_amd.model.models", fromlist=["x"])
        LY_models.paired_lstm_layerd = spy
        for pair in (True, False):
            m.pair_encoders = pair
            for p in m.parameters():
                p.grad = None
            loss, _ = _train_step(m, (a, mo, t))
            res[pair] = (loss.detach().clone(), [p.grad.clone() for p in m.parameters()])
    finally:
        LY_models.paired_lstm_layerd = orig
        m.pair_encoders = type(m).pair_encoders
    assert calls == [True]
    assert torch.equal(res[True][0], res[False][0])
    for g1, g0 in zip(res[True][1], res[False][1]):
        assert torch.equal(g1, g0)


def test_metaformer_q9_benchmark_width_vs_oracle():
    """Benchmark architecture (H=256, 5 blocks, 5 encoder layers, r=1), 24 frames, ragged: the
    scheduled-sampling training loss over the Q9 broadcast target + every gradient, and the
    genrt_loss, vs the CPU oracle."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    from oracle import mrg_oracle as O
    mc, oc, me = C.lstmformer_config(ratio=1, use_scheduled_sampling=True)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    T = 24
    batch = make_batch(B=3, T=T, lead=4, seed=23, lengths=[24, 19, 11])
    mask = torch.from_numpy(np.random.RandomState(7).rand(T) < 0.5)
    loss, _ = _train_step(m, clone_batch(batch, DEV), sampling_mask=mask)
    ref_loss, _, grads, _ = O.run_train_step(O.metaformer_ss_training_loss, sd, oc, mc, clone_batch(batch),
                                             sampling_mask=mask)
    assert abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()) < TOL
    worst = max((rel_err(p.grad, grads[k]), k) for k, p in m.named_parameters())
    assert worst[0] < TOL, worst
    with torch.no_grad():
        g = m.generation_step(clone_batch(batch, DEV))["loss"]
        ref_g = O.metaformer_genrt_loss(sd, mc, clone_batch(batch))
    assert abs(g.item() - ref_g.item()) / abs(ref_g.item()) < TOL


def test_simple_lstm_bf16_gate_vs_fp32_oracle():
    """BASELINE configs[1] is simple_lstm in bf16.  model.set_precision('bf16') runs every GEMM on
    bf16 operands (fp32 accumulation; recurrence state, LayerNorm, softmax, loss fp32).  Gate of
    SURVEY §8c: output <= 2e-2 and loss <= 1e-2 relative to the fp32 oracle, at benchmark width
    (T = 300, B = 2); gradients must still point the same way (cosine >= 0.99 per tensor)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import SimpleLSTM
    from multimodalreactiongeneration_amd.synthetic import make_simple_batch
    from oracle import mrg_oracle as O
    cfg, oc, me = C.simple_lstm_config()
    torch.manual_seed(2)
    m = SimpleLSTM(cfg, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV).set_precision("bf16")
    a, mo, t = make_simple_batch(B=2, T=300, seed=19)
    with torch.no_grad():
        y = m.forward(a.to(DEV), mo.to(DEV))
        y_ref = O.simple_lstm_forward(sd, cfg, a, mo)
    assert 0 < rel_err(y, y_ref) <= 2e-2, rel_err(y, y_ref)   # > 0: really bf16 arithmetic
    loss, _ = _train_step(m, (a.to(DEV), mo.to(DEV), t.to(DEV)))
    ref_loss, _, grads, _ = O.run_train_step(O.simple_lstm_training_loss, sd, oc, cfg, a, mo, t)
    assert abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()) <= 1e-2
    for k, p in m.named_parameters():
        g, r = p.grad.detach().double().cpu().flatten(), grads[k].double().flatten()
        if r.norm() > 1e-12:
            assert torch.nn.functional.cosine_similarity(g, r, dim=0) >= 0.99, k


@pytest.mark.parametrize("chunk,ratio,B,T", [(100, 1, 64, 300), (60, 1, 16, 300), (100, 1, 16, 250), (7, 2, 6, 40),
                                             (300, 1, 8, 50)])
def test_encoder_stack_matches_per_layer_schedule(chunk, ratio, B, T):
    """Block 0's embedding stacks as a (layer, time chunk) wavefront (encoder_stack.py) vs the
    per-layer schedule: same loss, output and every parameter gradient (fp32 reorderings only:
    weight-gradient sums run over time-major rows).  Ragged chunks (T % chunk != 0), audio at
    twice the frame rate (more chunks than the pose chains) and padded frames included."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import encoder_stack as ES
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    mc, oc, me = C.lstmformer_config(ratio=ratio)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to(DEV)
    lengths = [T] * B
    lengths[-1] = T - 5
    batch = make_batch(B=B, T=T, lead=3, ratio=ratio, seed=11, lengths=lengths, device=DEV)
    from multimodalreactiongeneration_amd import _lib
    lib = _lib.load()
    prev = ES.CHUNK
    out = []
    prev_mx = lib.mrg_lstm_set_mx(0, 0)   # one recurrence form on both sides: only the schedule differs
    try:
        ES.CHUNK = chunk
        for use in (False, True):
            m.metaformer.use_encoder_stack = use
            for p in m.parameters():
                p.grad = None
            y = m(*clone_batch(batch, DEV)[:-1])[0]
            loss = m.training_step(clone_batch(batch, DEV))["loss"]
            loss.backward()
            torch.cuda.synchronize()
            out.append((y.detach().clone(), loss.detach().clone(),
                        {k: p.grad.detach().clone() for k, p in m.named_parameters()}))
    finally:
        ES.CHUNK = prev
        lib.mrg_lstm_set_mx(prev_mx, 0)
        m.metaformer.use_encoder_stack = type(m.metaformer).use_encoder_stack
    (y0, l0, g0), (y1, l1, g1) = out
    assert rel_err(y1, y0) < 1e-5
    assert abs(l1.item() - l0.item()) <= 1e-6 * abs(l0.item())
    for k in g0:
        assert rel_err(g1[k], g0[k]) < 1e-5, k


@pytest.mark.parametrize("stack", [True, False])
def test_metaformer_benchmark_width_mfma_recurrence_vs_oracle(stack):
    """Benchmark architecture at T = 300 vs the CPU oracle with every H = 256 recurrence on the MFMA
    form (lstm_mx.hip, forced), through the encoder wavefront (encoder_stack.py) or per layer."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    from oracle import mrg_oracle as O
    lib = _lib.load()
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    m.metaformer.use_encoder_stack = stack
    batch = make_batch(B=4, T=300, seed=11)
    prev = lib.mrg_lstm_set_mx(2, 0)
    try:
        loss = m.training_step(clone_batch(batch, DEV))["loss"]
        loss.backward()
        torch.cuda.synchronize()
    finally:
        lib.mrg_lstm_set_mx(prev, 0)
    ref_loss, ref_y, grads, _ = O.run_train_step(O.metaformer_training_loss, sd, oc, mc, clone_batch(batch))
    assert abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()) < TOL
    worst = max(rel_err(p.grad, grads[k]) for k, p in m.named_parameters())
    assert worst < TOL, worst


@pytest.mark.parametrize("ratio,B,T", [(1, 64, 300), (2, 6, 40)])
def test_fused_integrator_matches_module_path(ratio, B, T):
    """Every block's integrator as one fused op (integrate.py: batched projections / LayerNorms, the
    concat written in place, the query gradient accumulated in GEMM epilogues) vs the per-module path:
    same output and loss (1e-5), ragged padding and audio at twice the frame rate included.  Gradients:
    at the small shape the two paths within 1e-5 of each other; at B = 64, T = 300 the two fp32
    summation orders may put a ReLU pre-activation near 0 on different sides, so EACH path is held to
    1e-4 on every gradient against the float64 oracle evaluated at its own ReLU sides (_tapped)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.model.metaformer import IntegrateModalBlock
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    from oracle import mrg_oracle as O
    mc, oc, me = C.lstmformer_config(ratio=ratio)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    lengths = [T] * B
    lengths[-1] = T - 5
    batch = make_batch(B=B, T=T, lead=3, ratio=ratio, seed=13, lengths=lengths)
    big = B * T >= 4096
    out = []
    try:
        for use in (False, True):
            IntegrateModalBlock.use_fused = use
            for p in m.parameters():
                p.grad = None
            y = m(*clone_batch(batch, DEV)[:-1])[0]
            loss, tap = _tapped(lambda: m.training_step(clone_batch(batch, DEV))["loss"])
            loss.backward()
            torch.cuda.synchronize()
            grads = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
            if big:
                ref = _oracle_f64_at(_relu_masks(m, tap), O.metaformer_training_loss, sd, oc, mc, clone_batch(batch))
                _check_vs_f64(m, loss.detach(), ref, after=False)
            out.append((y.detach().clone(), loss.detach().clone(), grads))
    finally:
        IntegrateModalBlock.use_fused = True
    (y0, l0, g0), (y1, l1, g1) = out
    assert rel_err(y1, y0) < 1e-5
    assert abs(l1.item() - l0.item()) <= 1e-5 * abs(l0.item())
    if not big:
        for k in g0:
            assert rel_err(g1[k], g0[k]) < 1e-5, (k, rel_err(g1[k], g0[k]))


# Whole-model B = 64 checks at the north_star's 1e-4 on EVERY gradient.  A ReLU pre-activation within
# fp32 rounding of 0 can take either side of the kink under a different summation order
# (tools/kink_census.py: 3 of 7.4 M between two GEMM settings of this forward), and one flipped row moves
# the cancellation-heavy LayerNorm-weight / embedding gradient sums by ~1e-4 of their max.  So the
# float64 oracle is evaluated AT the GPU forward's kinks: the fused FFN ops record each ReLU's side
# (functional.RELU_TAP) and the oracle multiplies by those masks instead of re-deciding them
# (oracle.RELU_MASKS).  The answer is then the exact function the GPU computed, and everything else
# (fp32 vs float64 rounding of the rest of the step) is held to 1e-4.


def _tapped(fn):
    """Run fn() with the FFN ReLU tap on: (fn's result, {Linear prefix: bool mask on the CPU})."""
    from multimodalreactiongeneration_amd import functional as Fn
    Fn.RELU_TAP = {}
    try:
        r = fn()
        torch.cuda.synchronize()
        tap = Fn.RELU_TAP
    finally:
        Fn.RELU_TAP = None
    return r, tap


def _relu_masks(m, tap):
    names = {p.data_ptr(): k for k, p in m.named_parameters()}
    out = {names[ptr][:-len("weight")]: v.cpu() for ptr, v in tap.items()}
    assert out and all(k.endswith("input.") for k in out), sorted(out)
    return out


def _oracle_f64_at(masks, loss_fn, sd, oc, mc, batch, **kw):
    """The oracle's fwd + loss + bwd + AdamW in float64 on the box's host cores, at the GPU's ReLU sides
    (LSTMs on the fused ATen op, equal to the per-step restatement: tests/test_oracle_golden.py)."""
    from oracle import mrg_oracle as O
    prev = O.RELU_MASKS, O.ATEN_LSTM
    O.RELU_MASKS, O.ATEN_LSTM = masks, True
    try:
        return O.run_train_step(loss_fn, {k: v.detach().cpu().double() for k, v in sd.items()}, oc, mc,
                                [(x.detach().cpu().double(), n.cpu()) for x, n in batch], **kw)
    finally:
        O.RELU_MASKS, O.ATEN_LSTM = prev


def _check_vs_f64(m, loss, ref, after=True, tol=TOL):
    """Loss, every full gradient and (after=True) the post-AdamW parameters vs the float64 answer."""
    ref_loss, _, grads, after_p = ref
    assert abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()) < tol, (loss.item(), ref_loss.item())
    worst = sorted((rel_err(p.grad, grads[k]), k) for k, p in m.named_parameters())
    print("worst gradient errors vs float64 at the GPU's kinks:", [(f"{e:.2e}", k) for e, k in worst[-4:]])
    assert worst[-1][0] < tol, worst[-1]
    if after:
        for k, p in m.named_parameters():
            g = grads[k].reshape(-1)
            sel = g.abs() > max(1e-5 * g.abs().max().item(), 1e-6)
            if sel.any():
                assert rel_err(p.detach().reshape(-1).cpu()[sel], after_p[k].reshape(-1)[sel]) < tol, k


def test_benchmark_schedule_b64_vs_oracle():
    """The benchmarked step exactly as bench.py runs it (B=64, T=300, r=1, bench weights and batch):
    encoder wavefront with the MFMA recurrences, deferred weight gradients beside the backward
    recurrences on the side stream, fused integrators, fwd + loss + bwd + AdamW captured as ONE HIP
    graph and replayed once, vs the oracle's float64 answer for the same inputs
    (tests/golden/metaformer_b64_f64.npz): loss, every parameter gradient (max|g|, L2 norm and 257
    sampled entries incl. the argmax) and the post-AdamW parameters at the sampled entries; then, at
    1e-4 on EVERY full gradient and the post-AdamW parameters, vs the float64 oracle run on the host
    at this forward's ReLU sides (see _tapped).
    Reference: lstmformer.py:313-333 (training_step, lossfun, configure_optimizers)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch
    d = load("metaformer_b64_f64")
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    assert abs(sum(v.double().sum().item() for v in m.state_dict().values()) - float(d["param_sum"])) < 1e-6, \
        "torch.manual_seed(0) init differs from the fixture's"
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    assert Fn.set_wgrad_stream(True) and Fn.set_wgrad_defer(True)   # the defaults bench.py runs with
    opt = m.configure_optimizers()["optimizer"]
    batch = make_batch(B=64, T=300, ratio=1, seed=1234, device=DEV)
    one = torch.ones((), device=DEV)
    loss_buf = torch.zeros((), device=DEV)

    def step():
        opt.zero_grad()
        loss = m.training_step(list(batch))["loss"]
        loss.backward(one)
        opt.step()
        loss_buf.copy_(loss.detach())
    # the forward the replay will run, eagerly, to record its ReLU sides (deterministic kernels: the
    # replay computes bitwise the same pre-activations)
    _, tap = _tapped(lambda: m.training_step(list(batch))["loss"])
    replay = capture(step, 2, preserve=opt.state_tensors())
    replay()
    torch.cuda.synchronize()
    Fn.check_errors()
    _check_sampled_fixture(d, m, loss_buf, loss_only=True)
    from oracle import mrg_oracle as O
    ref = _oracle_f64_at(_relu_masks(m, tap), O.metaformer_training_loss, sd, oc, mc,
                         make_batch(B=64, T=300, ratio=1, seed=1234))
    _check_vs_f64(m, loss_buf, ref)


def _check_sampled_fixture(d, m, loss, tol_of=lambda k: TOL, loss_only=False):
    """Loss, every parameter gradient (max|g|, L2 norm and the sampled entries incl. the argmax) and
    the post-AdamW parameters at the sampled entries vs a make_b64_fixture.py float64 fixture."""
    assert abs(loss.item() - float(d["loss"])) / abs(float(d["loss"])) < TOL, (loss.item(), float(d["loss"]))
    if loss_only:
        return
    worst = []
    for k, p in m.named_parameters():
        g = p.grad.detach().reshape(-1).double().cpu()
        idx = torch.from_numpy(d[f"idx/{k}"])
        gmax, _, g2 = d[f"stat/{k}"]
        tol = tol_of(k)
        scale = max(gmax, 1e-30)
        e_pt = (g[idx] - torch.from_numpy(d[f"g/{k}"])).abs().max().item() / scale
        e_max = abs(g.abs().max().item() - gmax) / scale
        e_l2 = abs(g.norm().item() - np.sqrt(g2)) / max(np.sqrt(g2), 1e-30)
        worst.append((max(e_pt, e_max, e_l2), k))
        assert e_pt < tol and e_max < tol and e_l2 < tol, (k, e_pt, e_max, e_l2)
        gref = torch.from_numpy(d[f"g/{k}"])
        sel = gref.abs() > max(1e-5 * gmax, 1e-6)
        if sel.any():
            a = p.detach().reshape(-1).double().cpu()[idx][sel]
            assert rel_err(a, torch.from_numpy(d[f"after/{k}"])[sel]) < tol, k
    worst.sort()
    print("worst gradient errors vs float64:", [(f"{e:.2e}", k) for e, k in worst[-5:]])


def _param_sum_matches(m, d):
    assert abs(sum(v.double().sum().item() for v in m.state_dict().values()) - float(d["param_sum"])) < 1e-6, \
        "torch.manual_seed(0) init differs from the fixture's"


def test_c3_scheduled_sampling_b64_vs_oracle():
    """BASELINE configs[2] exactly as bench.py's step_c3 times it: LSTMwithSample scheduled sampling,
    B=64, T=300, lead 12, torch.manual_seed(0) weights, epoch 30, the device mask holding the first
    RandomState(7) < 0.5 draw, fwd + loss + bwd + AdamW captured as ONE HIP graph (the fused per-frame
    decode, 16-row x 4-unit tiles over 256 workgroups) and replayed, vs the oracle's float64 answer
    (tests/golden/lstm_with_sample_ss_b64_f64.npz): loss, every gradient (max, L2, 257 samples),
    the post-AdamW parameters, and the eager prediction.  Reference: lstm_with_sample.py:278-301,379-433."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import LSTMwithSample
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    d = load("lstm_with_sample_ss_b64_f64")
    mc, oc, me = C.lstm_with_sampling_config(use_scheduled_sampling=True)
    torch.manual_seed(0)
    m = LSTMwithSample(mc, oc, me)
    _param_sum_matches(m, d)
    m.current_epoch = 30
    m = m.to(DEV)
    T = 300
    batch = make_batch(B=64, T=T, lead=12, seed=1234, device=DEV)
    mask = torch.from_numpy(d["sampling_mask"]).to(DEV)
    with torch.no_grad():
        y, _ = m.prediction(clone_batch(batch, DEV), use_scheduled_sampling=True, sampling_mask=mask)
    assert rel_err(y, d["y"]) < TOL
    opt = m.configure_optimizers()["optimizer"]
    loss_buf = torch.zeros((), device=DEV)

    def step_c3():
        opt.zero_grad()
        loss = m.training_step(batch, sampling_mask=mask)["loss"]
        loss.backward()
        opt.step()
        loss_buf.copy_(loss.detach())
    replay = capture(step_c3, 2, preserve=opt.state_tensors())
    replay()
    torch.cuda.synchronize()
    Fn.check_errors()
    _check_sampled_fixture(d, m, loss_buf)


def test_c2_simple_lstm_b64_vs_oracle():
    """BASELINE configs[1]'s shape in fp32 exactly as bench.py's step_c2 times it: SimpleLSTM B=64,
    T=300, torch.manual_seed(0) weights, paired encoder recurrences, HIP-graph replay of fwd + MSE +
    bwd + AdamW, vs the oracle's float64 answer (tests/golden/simple_lstm_b64_f64.npz): output,
    loss, every gradient (max, L2, 257 samples) and the post-AdamW parameters.
    Reference: simple_lstm.py:146-269 (with the Q3 unwrap)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import SimpleLSTM
    from multimodalreactiongeneration_amd.synthetic import make_simple_batch
    d = load("simple_lstm_b64_f64")
    cfg, oc, me = C.simple_lstm_config()
    torch.manual_seed(0)
    m = SimpleLSTM(cfg, oc, me).set_precision("32")
    _param_sum_matches(m, d)
    m = m.to(DEV)
    batch = make_simple_batch(B=64, T=300, device=DEV)
    with torch.no_grad():
        assert rel_err(m.forward(batch[0], batch[1]), d["y"]) < TOL
    opt = m.configure_optimizers()["optimizer"]
    loss_buf = torch.zeros((), device=DEV)

    def step_c2():
        opt.zero_grad()
        loss = m.training_step(batch)["loss"]
        loss.backward()
        opt.step()
        loss_buf.copy_(loss.detach())
    replay = capture(step_c2, 2, preserve=opt.state_tensors())
    replay()
    torch.cuda.synchronize()
    Fn.check_errors()
    _check_sampled_fixture(d, m, loss_buf)


def test_generation_b64_vs_oracle():
    """lstmformer generation (Metaformer.prediction) at the benchmarked batch B=64 with
    bench.py's weights and inputs, 40 frames, captured as one HIP graph with the mask in a device buffer
    and replayed for full generation and for the RandomState(7) < 0.5 scheduled-sampling mask, vs the
    oracle's float64 predictions (tests/golden/metaformer_gen_b64_f64.npz).  Reference: lstmformer.py:426-547."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.graphs import capture
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch
    d = load("metaformer_gen_b64_f64")
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    _param_sum_matches(m, d)
    m = m.to(DEV).eval()
    T = 40
    batch = make_batch(B=64, T=T, lead=12, seed=1234, device=DEV)
    mask = torch.ones(T, dtype=torch.bool, device=DEV)
    out = torch.zeros(64, T, 6, device=DEV)

    def gen():
        with torch.no_grad():
            out.copy_(m._generate(batch, sampling_mask=mask))
    replay = capture(gen, 1)
    for mode in ("ss", "full"):
        mask.copy_(torch.from_numpy(d[f"mask/{mode}"]))
        replay()
        torch.cuda.synchronize()
        assert rel_err(out, d[f"pred/{mode}"]) < TOL, mode


def test_encoder_stack_mfma_matches_per_layer_valu():
    """The encoder wavefront with its MFMA recurrences (the benchmarked form: 8 problems x 4 batch
    tiles x 3 chunks at B = 64) vs the per-layer schedule on the VALU recurrence: same loss within fp32
    reordering, and each schedule's every gradient within 1e-4 of the float64 oracle evaluated at that
    schedule's ReLU sides (the two fp32 orders may put a pre-activation near 0 on different sides)."""
    from multimodalreactiongeneration_amd import _lib
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    from oracle import mrg_oracle as O
    lib = _lib.load()
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    B, T = 64, 300
    lengths = [T] * B
    lengths[-1] = T - 5
    batch = make_batch(B=B, T=T, lead=3, seed=11, lengths=lengths)
    out = []
    prev = lib.mrg_lstm_set_mx(0, 0)
    try:
        for use, mx in ((False, 0), (True, 2)):
            lib.mrg_lstm_set_mx(mx, 0)
            m.metaformer.use_encoder_stack = use
            for p in m.parameters():
                p.grad = None
            loss, tap = _tapped(lambda: m.training_step(clone_batch(batch, DEV))["loss"])
            loss.backward()
            torch.cuda.synchronize()
            ref = _oracle_f64_at(_relu_masks(m, tap), O.metaformer_training_loss, sd, oc, mc, clone_batch(batch))
            _check_vs_f64(m, loss.detach(), ref, after=False)
            out.append(loss.detach().clone())
    finally:
        lib.mrg_lstm_set_mx(prev, 0)
        m.metaformer.use_encoder_stack = type(m.metaformer).use_encoder_stack
    assert abs(out[1].item() - out[0].item()) <= 1e-5 * abs(out[0].item())


def test_simple_lstm_configs0_shape_vs_oracle():
    """BASELINE configs[0]'s shape (simple_lstm, T=100, B=4) on the GPU vs the CPU oracle: loss, every
    gradient and the AdamW step at 1e-4 (simple_lstm.py:146-269)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import SimpleLSTM
    from multimodalreactiongeneration_amd.synthetic import make_simple_batch
    from oracle import mrg_oracle as O
    cfg, oc, me = C.simple_lstm_config()
    torch.manual_seed(0)
    m = SimpleLSTM(cfg, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    a, mo, t = make_simple_batch(B=4, T=100, seed=1234)
    opt = m.configure_optimizers()["optimizer"]
    loss = m.training_step((a.to(DEV), mo.to(DEV), t.to(DEV)))["loss"]
    loss.backward()
    opt.step()
    torch.cuda.synchronize()
    ref_loss, _, grads, after = O.run_train_step(O.simple_lstm_training_loss, sd, oc, cfg, a, mo, t)
    assert abs(loss.item() - ref_loss.item()) / abs(ref_loss.item()) < TOL
    for k, p in m.named_parameters():
        assert rel_err(p.grad, grads[k]) < TOL, k
        gref = grads[k]
        sel = gref.abs() > torch.clamp(1e-5 * gref.abs().max(), min=1e-6)
        if sel.any():
            assert rel_err(p.detach().cpu()[sel], after[k][sel]) < TOL, k


def test_kv_sink_two_forwards_one_backward():
    """The encoder outputs' shared key / value gradient (integrate.KVSink, drained by the encoder stack's
    backward) with TWO forwards over one batch before one backward: the gradients are twice the
    one-forward gradients (the sink must not depend on consumer order or forward count)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me).to(DEV)
    batch = make_batch(B=16, T=120, lead=3, seed=3, device=DEV)
    out = []
    for reps in (1, 2):
        for p in m.parameters():
            p.grad = None
        loss = sum(m.training_step(clone_batch(batch, DEV))["loss"] for _ in range(reps))
        loss.backward()
        torch.cuda.synchronize()
        out.append({k: p.grad.detach().clone() for k, p in m.named_parameters()})
    for k in out[0]:
        assert rel_err(out[1][k], 2.0 * out[0][k]) < 1e-5, k


def test_feature_input_gradient_vs_oracle():
    """Features that require a gradient (an upstream learnable module): the encoder wavefront returns
    none, so the model takes the per-layer schedule and the audio / pose gradients match the oracle's
    (ADVICE r03)."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch, clone_batch
    from oracle import mrg_oracle as O
    mc, oc, me = C.lstmformer_config(hidden=64, num_block=2, encoder_num_layer=2, bottleneck=16)
    torch.manual_seed(0)
    m = Metaformer(mc, oc, me)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    m = m.to(DEV)
    batch = make_batch(B=4, T=24, lead=3, seed=7)
    gb = clone_batch(batch, DEV)
    cb = clone_batch(batch)
    for i in (0, 1):   # partner audio and partner motion
        gb[i] = (gb[i][0].requires_grad_(True), gb[i][1])
        cb[i] = (cb[i][0].requires_grad_(True), cb[i][1])
    loss = m.training_step(gb)["loss"]
    loss.backward()
    torch.cuda.synchronize()
    params = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ref, _ = O.metaformer_training_loss(params, mc, cb)
    ref.backward()
    assert abs(loss.item() - ref.item()) / abs(ref.item()) < TOL
    for i in (0, 1):
        assert gb[i][0].grad is not None
        assert rel_err(gb[i][0].grad, cb[i][0].grad) < TOL, i


@pytest.mark.parametrize("loop", [True, False])
@pytest.mark.parametrize("B,T", [(37, 25), (64, 12), (3, 9)])
def test_generation_fused_frame_loop_matches_module_path(B, T, loop):
    """The fused frame loop (generate.py / gen.hip: other modalities' encoders and the one-key attention
    outputs hoisted over all frames; loop=True: the whole loop as one persistent launch with granule
    hand-offs between 16 workgroups per 8 rows, False: 26 launches per frame) vs the per-frame module
    forward the grad-enabled path runs, on ragged padded inputs (B not a multiple of the kernels' row
    tiles) under a scheduled-sampling mask: the predictions agree within fp32 reordering.
    Reference: lstmformer.py:426-547."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd import generate as G
    from multimodalreactiongeneration_amd.generate import plan_for
    from multimodalreactiongeneration_amd.model import Metaformer
    from multimodalreactiongeneration_amd.synthetic import make_batch
    mc, oc, me = C.lstmformer_config(ratio=1)
    torch.manual_seed(3)
    m = Metaformer(mc, oc, me).to(DEV).eval()
    assert plan_for(m) is not None
    lengths = [T] * B
    lengths[1] = T - 4
    batch = make_batch(B=B, T=T, lead=12, seed=5, lengths=lengths, device=DEV)
    mask = torch.from_numpy(np.random.RandomState(9).rand(T) < 0.5).to(DEV)
    prev = G._LOOP[0]
    G._LOOP[0] = loop
    try:
        with torch.no_grad():
            fast = m._generate(batch, sampling_mask=mask)
    finally:
        G._LOOP[0] = prev
    with torch.enable_grad():
        slow = m._generate(batch, sampling_mask=mask).detach()
    torch.cuda.synchronize()
    Fn.check_errors()
    assert fast.shape == slow.shape == (B, T, 6)
    assert rel_err(fast, slow) < 1e-5, rel_err(fast, slow)


@pytest.mark.parametrize("B,T,nl,FO", [(64, 40, 2, 6), (37, 25, 1, 6), (3, 9, 3, 8), (20, 30, 4, 1)])
def test_ssd_persistent_loop_matches_per_frame_launches(B, T, nl, FO):
    """The scheduled-sampling decode's forward frame loop as ONE persistent launch (ssd_loop.hip: 16
    workgroups per 8 rows, each layer's h handed over as granules, buffers alternating by frame
    parity) and its backward frame loop (ssd_loop_bwd_kernel, L >= 2), each on and off, vs the L + 1
    forward and 2L backward launches per frame of decode.hip, on the same inputs under a random sampling
    mask, ragged B, 1..4 layers and 1..8 output features (the per-frame kernels take FO <= 8): the prediction and, through the backward
    that reads every saved tensor (X_f's ms columns, X, gates, c, h, LayerNorm statistics, U, Z), the
    sampler-output and every parameter gradient agree within fp32 reordering.
    Reference: lstm_with_sample.py:379-433."""
    from multimodalreactiongeneration_amd import decode as D
    from multimodalreactiongeneration_amd import functional as Fn
    H, HB, SA, FMp = 256, 64, 128, 6
    F = SA + FMp + FO
    g = torch.Generator().manual_seed(B * 100 + nl)

    def u(*shape, k):
        return ((torch.rand(*shape, generator=g) * 2 - 1) * k).to(DEV)
    base = dict(w_f=u(H, F, k=F ** -0.5), b_f=u(H, k=F ** -0.5))
    layers = []
    for _ in range(nl):
        layers.append([u(4 * H, H, k=H ** -0.5), u(4 * H, H, k=H ** -0.5), u(4 * H, k=H ** -0.5),
                       u(4 * H, k=H ** -0.5), 1 + u(H, k=0.2), u(H, k=0.2)])
    ffn = [u(HB, H, k=H ** -0.5), u(HB, k=H ** -0.5), u(FO, HB, k=HB ** -0.5), u(FO, k=HB ** -0.5)]
    a_s = torch.randn(B, T, SA, generator=g).to(DEV)
    mp = torch.randn(B, T, FMp, generator=g).to(DEV)
    ms = torch.randn(B, T, FO, generator=g).to(DEV)
    mask = torch.from_numpy(np.random.RandomState(B + T).rand(T) < 0.5).to(DEV)
    dy = torch.randn(B, T, FO, generator=g).to(DEV)
    outs = []
    prev = D._LOOP[0], D._LOOP_BWD[0]
    try:
        for fwd, bwd in ((True, True), (False, True), (True, False), (False, False)):
            D._LOOP[0], D._LOOP_BWD[0] = fwd, bwd
            ps = [t.clone().requires_grad_(True) for t in [base["w_f"], base["b_f"]] + sum(layers, []) + ffn]
            a = a_s.clone().requires_grad_(True)
            lay = [ps[2 + 6 * i:8 + 6 * i] for i in range(nl)]
            y = D.scheduled_sampling_decode(a, mp, ms, mask, ps[0], ps[1], lay, ps[2 + 6 * nl:])
            (y * dy).sum().backward()
            torch.cuda.synchronize()
            Fn.check_errors()
            outs.append((y.detach(), a.grad, [p.grad for p in ps]))
    finally:
        D._LOOP[0], D._LOOP_BWD[0] = prev
    y1, a1, g1 = outs[-1]
    for v, (y0, a0, g0) in enumerate(outs[:-1]):
        assert y0.shape == (B, T, FO)
        assert rel_err(y0, y1) < 1e-5, (v, rel_err(y0, y1))
        assert rel_err(a0, a1) < 1e-5, (v, rel_err(a0, a1))
        for i, (p, q) in enumerate(zip(g0, g1)):
            if q is None or q.abs().max() == 0:   # W_hh (zero state): exactly zero on both paths
                assert p is None or p.abs().max() == 0, (v, i)
                continue
            assert rel_err(p, q) < 1e-5, (v, i, rel_err(p, q))
