"""Import the upstream reference (read-only, /root/reference) for golden-vector generation.

Used ONLY by ``make_golden.py`` in the build container.  The reference needs
pytorch_lightning / omegaconf / torchmetrics, none of which are installed, so we
register minimal stand-ins in ``sys.modules`` and
skip ``mr_gen/__init__.py`` (it imports cv2 / mediapipe).  Reference files are
never modified or copied; the GPU box never imports this module.
"""
import os
import sys
import types

import torch
from torch import nn

REF_ROOT = os.environ.get("MRG_REFERENCE_ROOT", "/root/reference")


def _mod(name, **attrs):
    m = types.ModuleType(name)
    m.__dict__.update(attrs)
    sys.modules[name] = m
    return m


class _LightningModule(nn.Module):
    current_epoch = 0

    def log(self, *a, **k):
        pass

    def log_dict(self, *a, **k):
        pass

    @property
    def device(self):
        return next(self.parameters()).device


class AttrDict(dict):
    """Attribute access + .get, like an OmegaConf DictConfig."""

    def __getattr__(self, k):
        if k in self:
            return self[k]
        raise AttributeError(k)

    def __setattr__(self, k, v):
        self[k] = v


class _NoMetric(nn.Module):
    def __init__(self, *a, **k):
        super().__init__()

    def forward(self, *a, **k):
        return {}


_LOADED = {}


def load_reference():
    """Return a namespace with the reference classes (Metaformer, LSTMwithSample, SimpleLSTM, ...)."""
    if _LOADED:
        return _LOADED["ns"]
    if not os.path.isdir(os.path.join(REF_ROOT, "mr_gen")):
        raise RuntimeError(f"reference not found under {REF_ROOT}")
    sys.dont_write_bytecode = True
    _mod("pytorch_lightning", LightningModule=_LightningModule,
         LightningDataModule=object, Trainer=object)
    _mod("pytorch_lightning.utilities")
    _mod("pytorch_lightning.utilities.types", STEP_OUTPUT=object,
         EVAL_DATALOADERS=object, TRAIN_DATALOADERS=object)
    _mod("omegaconf", DictConfig=AttrDict)
    _mod("torchmetrics", Metric=_NoMetric, MeanSquaredError=_NoMetric,
         MetricCollection=_NoMetric)
    r = os.path.join(REF_ROOT, "mr_gen")
    _mod("mr_gen").__path__ = [r]
    _mod("mr_gen.utils").__path__ = [os.path.join(r, "utils")]
    _mod("mr_gen.databuild", DataBuilderNX=None, DataBuilder=None)
    _mod("mr_gen.utils.preprocess", AudioPreprocessor=None,
         MotionPreprocessorNX=None, MotionPreprocessor=None)
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)

    from mr_gen.model.lstmformer.lstmformer import Metaformer
    from mr_gen.model.lstm_with_sampling.lstm_with_sample import LSTMwithSample
    from mr_gen.model.simple_lstm import simple_lstm as S
    from mr_gen.model.utils.multi_modal_metaformer import gen_attention_mask

    # SimpleLSTM.forward feeds (tensor, hxs) tuples into nn.MultiheadAttention
    # (simple_lstm.py:69-71,95-97,140-143) and crashes as written.
    # The only runnable interpretation: take element [0] of LSTMLayerd's output.
    S.AcousticEncoder.forward = lambda self, a: self.acostic_lstm(self.embed_layer(a))[0]
    S.MotionEncoder.forward = lambda self, h: self.motion_lstm(self.embed_layer(h))[0]
    S.MotionDecoder.forward = lambda self, x: self.mapping(
        self.seq_reshape(self.decoder_lstm(x)[0]))

    ns = types.SimpleNamespace(Metaformer=Metaformer, LSTMwithSample=LSTMwithSample,
                               SimpleLSTM=S.SimpleLSTM, gen_attention_mask=gen_attention_mask)
    _LOADED["ns"] = ns
    return ns


def load_preprocessors():
    """The reference's AudioPreprocessor / MotionPreprocessorNX classes (mr_gen/utils/preprocess).

    torchaudio is not installed: ``torchaudio.transforms`` and the soundfile backend are
    registered as empty stand-ins so audio.py imports; only the pure-torch methods
    (compute_log_power, compute_delta) are exercised through them.  MotionPreprocessorNX needs
    only numpy / torch and runs unchanged.
    """
    import importlib.util
    sys.dont_write_bytecode = True
    _mod("torchaudio")
    _mod("torchaudio.transforms", MelSpectrogram=None)
    _mod("torchaudio._backend")
    _mod("torchaudio._backend.soundfile_backend", load=None)
    base = os.path.join(REF_ROOT, "mr_gen", "utils", "preprocess")
    out = {}
    for name in ("audio", "motion_nx"):
        spec = importlib.util.spec_from_file_location(f"_ref_preprocess_{name}", os.path.join(base, name + ".py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        out[name] = mod
    return types.SimpleNamespace(AudioPreprocessor=out["audio"].AudioPreprocessor,
                                 MotionPreprocessorNX=out["motion_nx"].MotionPreprocessorNX)
