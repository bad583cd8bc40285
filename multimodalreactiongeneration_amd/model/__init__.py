"""Drop-in counterparts of ``mr_gen.model`` (Metaformer, LSTMwithSample, SimpleLSTM) and ``mr_gen.model.utils``."""
from .layers import (LSTM, Linear, LayerNorm, MultiheadAttention, MHAforSequentail, ResidualConnection,
                     FeedForward, LSTMSampler, LSTMModule, LSTMBlock, LSTMLayerd,
                     MultiModalAttentionBlockSequential, MultimodalAttentionBlock, MultimodalAttention)
from .masks import gen_attention_mask, BlockCausalMask
from .mixers import (LSTMMixer, MHAMixer, LSTMMixerBlock, MHAMixerBlock, LSTMMixerLayerd, MHAMixerLayerd,
                     MixerBlockFactory, MixerLayerdFactory, split_state, mixer_layerd_argments_select,
                     feedforward_block_argments)
from .metaformer import (MultiModalEmbedding, IntegrateModalBlock, MultiModalMetaformerBlock,
                         MultiModalMetaformer, check_form_modal_num)
from .models import Metaformer, LSTMwithSample, SimpleLSTM, load_model, gen_target_dict, MODEL_TYPE

PADDING_VALUE = -100
