"""Run the Python orchestration of a fused op on the CPU against a stand-in libmrg (every entry point
returns 0, size helpers return sizes): catches Python-level errors (wrong argument counts, bad
indexing, shape mistakes) in the launch plumbing before a GPU run.  Nothing is computed.

    python tools/tools_mock_lib.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from multimodalreactiongeneration_amd import _lib  # noqa: E402


class MockLib:
    def __init__(self, real):
        self.real = real
        self.calls = []

    def __getattr__(self, name):
        sig = _lib.SIGNATURES.get(name)
        if sig is None:
            raise AttributeError(name)
        res, args = sig

        def fn(*a):
            if len(a) != len(args):
                raise TypeError(f"{name}: {len(a)} arguments, signature has {len(args)}")
            self.calls.append(name)
            if name.endswith("_bytes"):
                return getattr(self.real, name)(*a)
            if name in ("mrg_lstm_supported_hidden",):
                return 1
            if name == "mrg_gemm_get_mode":
                return 1
            return 0
        return fn


def main():
    real = _lib.load()
    mock = MockLib(real)
    _lib.load = lambda: mock
    _lib.require_device = lambda *a, **k: None
    _lib.cu_count = lambda *a, **k: 256
    from multimodalreactiongeneration_amd import functional as Fn
    from multimodalreactiongeneration_amd import encoder_stack as ES
    from multimodalreactiongeneration_amd import block_stack as BS
    from multimodalreactiongeneration_amd import integrate as IG
    for mod in (Fn, ES, BS, IG):
        mod._stream = lambda: ctypes.c_void_p(0)
    Fn.set_wgrad_stream(False)
    Fn.zero_ = lambda t: t.zero_()
    from multimodalreactiongeneration_amd import configs as C
    from multimodalreactiongeneration_amd.model import Metaformer
    for ratio, T, B in ((1, 40, 4), (2, 30, 3)):
        mc, oc, me = C.lstmformer_config(hidden=64, num_block=3, encoder_num_layer=2, bottleneck=16, ratio=ratio)
        torch.manual_seed(0)
        m = Metaformer(mc, oc, me)
        E = 64
        blocks = []
        for b in list(m.metaformer.metaformer_blocks)[1:]:
            lay = b.embedding.modal_embeddings[0].mixer[0]
            lstm = lay.mixer.module.mixer
            ln1, ffl, ln2 = lay.mixer.layer_norm, list(lay.feed_forward.feed_forward.module.children())[0], \
                lay.feed_forward.feed_forward.layer_norm
            flat = [*lstm.direction_params(0), ln1.weight, ln1.bias, ffl.weight, ffl.bias, ln2.weight, ln2.bias]
            for integ in b.integrator.integrators:
                blk = integ.mixer[0]
                mha = blk.mixer.module.mixer[0].mha
                ffw = blk.feed_forward.feed_forward
                lin = list(ffw.module.children())[0]
                flat += [mha.in_proj_weight, mha.in_proj_bias, mha.out_proj.weight, mha.out_proj.bias,
                         blk.mixer.layer_norm.weight, blk.mixer.layer_norm.bias, lin.weight, lin.bias,
                         ffw.layer_norm.weight, ffw.layer_norm.bias]
            flat += [b.integrator.cat_linear.weight, b.integrator.cat_linear.bias]
            ff = b.feedforward.feed_forward
            mods = list(ff.module.children())
            flat += [mods[0].weight, mods[0].bias, mods[2].weight, mods[2].bias, ff.layer_norm.weight,
                     ff.layer_norm.bias]
            blocks.append(flat)
        x = torch.randn(B, T, E, requires_grad=True)
        kvs = [torch.randn(B, T * ratio, E, requires_grad=True), torch.randn(B, T, E, requires_grad=True)]
        sinks = [IG.KVSink(), None]
        qpad = torch.zeros(B, T, dtype=torch.uint8)
        kpads = [torch.zeros(B, T * ratio, dtype=torch.uint8), torch.zeros(B, T, dtype=torch.uint8)]
        for chunk in (7, 40):
            mock.calls.clear()
            y = BS.block_stack(x, kvs, [qpad, qpad], kpads, blocks, 4, True, 1e-5, sinks, chunk=chunk)
            nf = len(mock.calls)
            y.backward(torch.ones_like(y))
            print(f"ratio {ratio} T {T} chunk {chunk}: forward {nf} calls, backward {len(mock.calls) - nf}; "
                  f"sink written {sinks[0].written}, own kv grad {kvs[1].grad is not None}", flush=True)
            sinks[0].drain()


if __name__ == "__main__":
    main()
