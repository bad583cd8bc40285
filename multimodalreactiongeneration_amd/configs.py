"""Config builders mirroring the reference's Hydra YAML (resolved) for the three models.

The reference reads ``cfg.model`` / ``cfg.optim`` / ``cfg.metrics`` (OmegaConf
``DictConfig``) with attribute access and ``.get``.  ``AttrDict`` gives the
same surface with no OmegaConf dependency.

Sources:
  lstmformer          mr_gen/model/lstmformer/config.yaml:5-104,143-150
  lstm_with_sampling  mr_gen/model/lstm_with_sampling/config.yaml:28-69
  simple_lstm         mr_gen/model/simple_lstm/config.yaml:30-110
Benchmark overrides (SURVEY §8 / BASELINE.md §3): nmels=39, delta_order=0
(40-d audio, 6-d pose), pred_fps=100 (r=1) or 12.5 (r=8).
"""
from __future__ import annotations


class AttrDict(dict):
    """dict with attribute access (OmegaConf-DictConfig-like surface)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v

    def copy(self):
        return AttrDict(self)


def as_attr(cfg):
    """Accept a dict / AttrDict / DictConfig-like object; return something with attr access + .get."""
    if isinstance(cfg, AttrDict):
        return cfg
    if isinstance(cfg, dict):
        return AttrDict(cfg)
    return cfg


def _optim(lr=5e-6):
    return AttrDict(use_optimizer="adam", momentum=0.9, weight_decay=1e-2, lr=lr,
                    use_lr_sched=True, batch_size=128, max_epochs=100)


def _metrics(delta_order=0):
    return AttrDict(use_centroid=True, use_angle=True, delta_order=delta_order)


def lstmformer_config(hidden=256, num_block=5, encoder_num_layer=5, num_heads=4,
                      bottleneck=64, nmels=39, delta_order=0, ratio=1, lr=5e-6,
                      loss_type="huber", emb_mixers=("lstm", "lstm", "lstm"), delta_loss_scale=1,
                      use_scheduled_sampling=False, max_epochs=60):
    """Resolved mr_gen/model/lstmformer/config.yaml model section (+ bench overrides)."""
    model = AttrDict(
        main_modal_idx=2, hidden_size=hidden, num_block=num_block, dropout=0.0,
        num_layerd=1, encoder_num_layer=encoder_num_layer, num_internal_layer=1,
        residual=True, residual_layer_norm=True, bias=True,
        emb_mixers=list(emb_mixers),  # config_gru.yaml:50-52: ["gru"] * 3
        bottleneck_size=bottleneck, nonlinearity="none", ffn_nonlinearity="relu",
        proj_size=0, num_heads=num_heads, add_bias_kv=False, add_zero_attn=False,
        max_context_len=10, repeat_with_encoder=False, interlayer_residual=False,
        interlayer_residual_norm=True, sampling_rate=16000, shift=160,
        pred_fps=100.0 / ratio, modalities=["audio", "motion", "motion"],
        use_centroid=True, use_angle=True, nmels=nmels, delta_order=delta_order,
        loss_type=loss_type, loss_reduction="mean", huber_delta=1.0, smoothl1_beta=1.0,
        delta_loss_scale=delta_loss_scale, use_scheduled_sampling=use_scheduled_sampling,
        max_epochs=max_epochs)
    return model, _optim(lr), _metrics(delta_order)


def lstm_with_sampling_config(hidden=256, sampler_hidden=128, sampler_layers=2,
                              num_layers=2, bottleneck=64, nmels=39, delta_order=0,
                              ratio=1, lr=5e-6, use_scheduled_sampling=False,
                              max_epochs=60):
    """Resolved mr_gen/model/lstm_with_sampling/config.yaml model section."""
    model = AttrDict(
        nmels=nmels, delta_order=delta_order, use_centroid=True, use_angle=True,
        sampler_hidden_size=sampler_hidden, sampler_num_layers=sampler_layers,
        sampler_dropout_rate=0, sampling_rate=16000, shift=160, fps=25,
        pred_fps=100.0 / ratio, hidden_size=hidden, bottleneck_size=bottleneck,
        num_layers=num_layers, num_lstm=1, dropout_rate=0.0, use_layer_norm=True,
        use_relu=True, use_mixing=False, use_residual=True, delta_loss_scale=1,
        loss_type="huber", loss_reduction="mean", huber_delta=1.0, smoothl1_beta=1.0,
        use_scheduled_sampling=use_scheduled_sampling, max_epochs=max_epochs)
    return model, _optim(lr), _metrics(delta_order)


def simple_lstm_config(hidden=256, lstm=128, bottleneck=64, att_heads=8,
                       att_layers=3, enc_layers=2, dec_layers=5, feat_audio=40,
                       feat_motion=6, output_size=6, mapping=64, lr=5e-6):
    """Resolved mr_gen/model/simple_lstm/config.yaml model section (40-d / 6-d bench shapes)."""
    cfg = AttrDict(
        acostic_feat_size=feat_audio, motion_feat_size=feat_motion,
        motion_num_lstm=1, acostic_num_lstm=1,
        acostic_num_layers=enc_layers, motion_num_layers=enc_layers,
        acostic_lstm_size=lstm, motion_lstm_size=lstm,
        acostic_lstm_out_size=hidden, motion_lstm_out_size=hidden,
        acostic_affine_size=hidden, motion_affine_size=hidden,
        acostic_bottleneck_size=bottleneck, motion_bottleneck_size=bottleneck,
        acostic_output_size=hidden, motion_output_size=hidden,
        att_heads=att_heads, att_num_layers=att_layers, att_use_residual=True,
        att_use_layer_norm=True, dropout_rate=0, output_size=output_size,
        bidirectional=True, use_layer_norm=True, use_relu=True, use_mixing=True,
        use_residual=True, decoder_num_layers=dec_layers, decoder_num_lstm=1,
        decoder_lstm_size=lstm, decoder_affine_size=hidden,
        decoder_bottleneck_size=bottleneck, decoder_output_size=hidden,
        decoder_mapping_size=mapping, decoder_bidirectional=True,
        decoder_use_layer_norm=True, decoder_use_relu=True, decoder_use_mixing=True,
        decoder_use_residual=True, delta_loss_scale=1, all_static=True)
    return cfg, _optim(lr), _metrics(0)
