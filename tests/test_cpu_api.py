"""CPU-only checks: the C-ABI library loads and exports what include/mrg.h declares; the
drop-in API matches the reference's module tree; the product path refuses CPU tensors."""
import os
import re

import pytest
import torch

from tests.model_shapes import keys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


HEADERS = ("mrg.h", "mrg_tuning.h")   # the drop-in boundary; tuning / measurement / test hooks


def _header_text(name="mrg.h"):
    return open(os.path.join(ROOT, "include", name)).read()


def _header_functions(names=HEADERS):
    out = set()
    for name in names:
        src = re.sub(r"/\*.*?\*/", "", _header_text(name), flags=re.S)
        out.update(re.findall(r"\b(mrg_[a-z0-9_]+)\s*\(", src))
    return sorted(out)


def test_boundary_header_holds_no_tuning_hooks():
    """include/mrg.h is the drop-in boundary only: the tuning knobs, probes, fault injection and the
    structural GEMM variants live in include/mrg_tuning.h; the pre-split weight
    planes and their products are the step's path since round 5 (gemm_wide.hip), so they are boundary."""
    boundary = set(_header_functions(("mrg.h",)))
    tuning = set(_header_functions(("mrg_tuning.h",)))
    assert not boundary & tuning
    for name in ("mrg_gemm_x6_variant", "mrg_gemm_force_tile", "mrg_ssd_gate_cell_fwd_dbg", "mrg_gemm_set_wide",
                 "mrg_lstm_debug_inject", "mrg_lstm_debug_stamps", "mrg_probe_start"):
        assert name in tuning and name not in boundary, name
    for name in ("mrg_split_planes_batched", "mrg_gemm_x6_planes", "mrg_gemm_x6_planes_batched"):
        assert name in boundary, name


def test_library_exports_every_header_symbol():
    import ctypes
    from multimodalreactiongeneration_amd import _lib
    lib = _lib.load()
    declared = _header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature"
    assert lib.mrg_version() >= 100
    assert lib.mrg_lstm_supported_hidden(256) and not lib.mrg_lstm_supported_hidden(12)


def test_workspace_size_helpers():
    from multimodalreactiongeneration_amd import _lib
    lib = _lib.load()
    # split-K slabs, then room for the row sums of A (fused bias gradients) or the column-sum partials
    assert lib.mrg_gemm_workspace_bytes(256, 256, 8) == (8 * 256 * 256 + 512 * 256) * 4
    assert lib.mrg_gemm_workspace_bytes(256, 256, 1) == 512 * 256 * 4
    assert lib.mrg_gemm_workspace_bytes(1024, 256, 1024) == (1024 * 1024 * 256 + 1024 * 1024) * 4
    assert lib.mrg_lstm_fwd_xbuf_bytes(64, 256) == 2 * 64 * 256 * 8
    assert lib.mrg_lstm_bwd_xbuf_bytes(64, 256) == 2 * 64 * 16 * 256 * 8
    assert lib.mrg_attention_bwd_workspace_bytes(2, 4, 300) == 2 * 4 * 300 * 4


@pytest.mark.parametrize("name,builder", [("Metaformer", "lstmformer_config"),
                                          ("LSTMwithSample", "lstm_with_sampling_config"),
                                          ("SimpleLSTM", "simple_lstm_config")])
def test_state_dict_matches_reference(name, builder):
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd import model as M
    m = getattr(M, name)(*getattr(C, builder)())
    got = {k: list(v.shape) for k, v in m.state_dict().items()}
    ref = keys(name)
    assert list(got) == list(ref)          # same keys, same order
    assert got == ref


def test_metaformer_r8_state_dict_and_param_count():
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    m = Metaformer(*C.lstmformer_config(ratio=8))
    assert {k: list(v.shape) for k, v in m.state_dict().items()} == keys("Metaformer_r8")
    assert sum(p.numel() for p in m.parameters()) == 13_052_678
    assert m.ratio == 8


def test_reference_constructor_errors():
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    mc, oc, me = C.lstmformer_config()
    mc["pred_fps"] = 30.0
    with pytest.raises(ValueError):
        Metaformer(mc, oc, me)
    mc, oc, me = C.lstmformer_config()
    mc["loss_type"] = "bogus"
    with pytest.raises(ValueError):
        Metaformer(mc, oc, me)


def test_mask_descriptor_dense_matches_reference_golden():
    import numpy as np
    from multimodalreactiongeneration_amd.model.masks import gen_attention_mask
    from tests.golden_util import load
    d = load("attention_masks")
    for i in range(5):
        m = gen_attention_mask(torch.from_numpy(d[f"case{i}/main"]), torch.from_numpy(d[f"case{i}/other"]),
                               int(d[f"case{i}/heads"]))
        assert torch.equal(m.dense(), torch.from_numpy(d[f"case{i}/mask"]))
        assert m.view(-1, 3, 3) is m


def test_product_path_has_no_cpu_fallback():
    from multimodalreactiongeneration_amd import functional as Fn
    x = torch.randn(4, 8)
    w = torch.nn.Parameter(torch.randn(3, 8))
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        Fn.linear(x, w, None)


def test_split_state_quirks():
    from multimodalreactiongeneration_amd.model.mixers import split_state
    assert split_state(None, None) == (None, None, [])
    first, rest, prev = split_state([1, 2, 3], [9])
    assert first == 1 and rest == [2, 3] and prev == [9]
    with pytest.raises(IndexError):  # reference quirk: an empty list is not treated as "no state"
        split_state([], None)


def test_mixer_argument_selection():
    from multimodalreactiongeneration_amd.model.mixers import mixer_layerd_argments_select
    cfg = mixer_layerd_argments_select("lstm", hidden_size=32, num_heads=4, num_layerd=3, bogus=1)
    assert cfg["hidden_size"] == 32 and cfg["num_layerd"] == 3 and "num_heads" not in cfg and "bogus" not in cfg
    cfg = mixer_layerd_argments_select("mha", hidden_size=32, num_heads=4, self_attention=False)
    assert cfg["num_heads"] == 4 and cfg["self_attention"] is False and cfg["max_context_len"] == 125
    with pytest.raises(ValueError):
        mixer_layerd_argments_select("rnn", hidden_size=8)


def test_gen_target_dict():
    from multimodalreactiongeneration_amd.configs import AttrDict
    from multimodalreactiongeneration_amd.model import gen_target_dict
    assert gen_target_dict(AttrDict(use_centroid=True, use_angle=True, delta_order=0)) == \
        {"centroid": (0, 3), "angle": (3, 6)}
    d2 = gen_target_dict(AttrDict(use_centroid=True, use_angle=True, delta_order=2))
    assert d2["delta2-angle"] == (15, 18)


def test_synthetic_batch_format():
    from multimodalreactiongeneration_amd.synthetic import make_batch
    b = make_batch(B=3, T=5, lead=2, ratio=2, lengths=[5, 3, 1])
    assert isinstance(b, list) and len(b) == 7
    assert b[0][0].shape == (3, 10, 40) and b[3][0].shape == (3, 4, 40)
    assert (b[1][0][1, 3:] == -100).all() and (b[0][0][1, 6:] == -100).all()
    assert b[1][1].tolist() == [5, 3, 1]


@pytest.mark.parametrize("model_type", ["lstmformer", "lstm_with_sampling", "simple_lstm"])
def test_checkpoint_round_trip_through_load_model(tmp_path, model_type):
    """model_loader.load_model (model_loader.py:13-26): a Lightning-shaped checkpoint
    {"state_dict", "epoch", "global_step", optimizer / scheduler states} written with torch.save
    loads through the pickle-free weights_only path into a fresh model, bit-exact."""
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import models as M
    build = {"lstmformer": (C.lstmformer_config, dict(hidden=32, num_block=2, encoder_num_layer=2, bottleneck=16)),
             "lstm_with_sampling": (C.lstm_with_sampling_config, dict(hidden=32, sampler_hidden=16, bottleneck=8)),
             "simple_lstm": (C.simple_lstm_config, dict(hidden=32, lstm=16, bottleneck=8, att_heads=4))}
    fn, kw = build[model_type]
    mc, oc, me = fn(**kw)
    cls = {"lstmformer": M.Metaformer, "lstm_with_sampling": M.LSTMwithSample, "simple_lstm": M.SimpleLSTM}
    torch.manual_seed(11)
    src = cls[model_type](mc, oc, me)
    sd = src.state_dict()
    ckpt = {"state_dict": sd, "epoch": 7, "global_step": 1234, "pytorch-lightning_version": "2.0.2",
            "optimizer_states": [{"state": {0: {"step": torch.tensor(3.0), "exp_avg": torch.zeros(3)}},
                                  "param_groups": [{"lr": 5e-6, "weight_decay": 1e-2, "params": [0]}]}],
            "lr_schedulers": [{"T_max": 100, "last_epoch": 7, "base_lrs": [5e-6]}]}
    path = tmp_path / "last.ckpt"
    torch.save(ckpt, path)
    cfg = {"model": mc, "optim": oc, "metrics": me}
    got = M.load_model(model_type, str(path), cfg)
    out = got.state_dict()
    assert list(out.keys()) == list(sd.keys())
    for k in sd:
        assert torch.equal(out[k], sd[k]), k
    # a bare state_dict file (no Lightning wrapper) loads too
    torch.save(sd, tmp_path / "bare.pt")
    got2 = M.load_model(model_type, str(tmp_path / "bare.pt"), cfg)
    assert all(torch.equal(got2.state_dict()[k], sd[k]) for k in sd)
    with pytest.raises(ValueError):
        M.load_model("gru_former", str(path), cfg)


def test_ctypes_signatures_match_header_arity():
    """Every binding in _lib.SIGNATURES declares as many arguments as include/mrg.h gives the entry."""
    from multimodalreactiongeneration_amd import _lib
    h = "\n".join(_header_text(n) for n in HEADERS)
    for name, (_res, args) in _lib.SIGNATURES.items():
        m = re.search(r"^(?:const\s+)?\w+\s*\**\s*" + name + r"\s*\(([^;]*?)\);", h, re.S | re.M)
        assert m, name
        params = [x for x in m.group(1).split(",") if x.strip() and x.strip() != "void"]
        assert len(params) == len(args), (name, len(params), len(args))


def test_comm_entry_points_load_without_a_gpu():
    """The RCCL C-ABI resolves librccl at run time: the library loads and reports the 128-byte id
    size with no GPU and no communicator."""
    from multimodalreactiongeneration_amd import _lib
    lib = _lib.load()
    assert lib.mrg_comm_id_bytes() == 128
    assert lib.mrg_comm_available() in (0, 1)
    assert lib.mrg_comm_destroy(None) == 0


def test_kv_sink_refuses_stale_sum_from_an_earlier_backward():
    """integrate.KVSink: a sum left by a backward pass whose producer never drained it is
    detected by the next pass's first write (the autograd graph task is recorded) instead of being added
    onto; a drained sink starts over."""
    import torch
    from multimodalreactiongeneration_amd.integrate import KVSink
    sink = KVSink()
    firsts = []

    class Consumer(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.clone()

        @staticmethod
        def backward(ctx, g):
            firsts.append(sink.begin_write())
            sink.written += 1
            return g

    x = torch.ones(3, requires_grad=True)
    (Consumer.apply(x) + Consumer.apply(x)).sum().backward()   # two consumers, one pass
    assert firsts == [True, False]
    with pytest.raises(RuntimeError, match="never drained"):
        Consumer.apply(x).sum().backward()                     # the first pass never drained
    sink.drain()
    firsts.clear()
    Consumer.apply(x).sum().backward()
    assert firsts == [True]


def test_side_stream_flush_conflicts():
    """functional._conflicts: a flush on the side stream waits for the recurrence stream when one of its
    items writes a gradient buffer the recurrence stream wrote in this backward, or names none."""
    from multimodalreactiongeneration_amd import functional as Fn
    a, b = torch.zeros(64), torch.zeros(64)
    va = a[16:32]
    rec = Fn._writes((a,))
    assert Fn._conflicts([(None, (), None, Fn._writes((va,)))], rec)          # a view of the same buffer
    assert not Fn._conflicts([(None, (), None, Fn._writes((b, None)))], rec)   # a different buffer
    assert Fn._conflicts([(None, (), None, None)], rec)                       # unknown writes
    assert Fn._conflicts([(None, (), None, Fn._writes((b,)))], None)          # recurrence stream unknown
