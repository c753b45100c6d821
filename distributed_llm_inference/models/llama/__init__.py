from .cache import KVPool, PartialLlamaSinkCache  # noqa: F401
from .model import LlamaBlock  # noqa: F401
from .modules import (LlamaAttention, LlamaDecoderLayer, LlamaMLP, RMSNorm,  # noqa: F401
                      apply_rotary_pos_emb, rotate_half)

# reference-compatible aliases (models/llama/modules.py:23, 117 in the reference)
OptimizedLlamaDecoderLayer = LlamaDecoderLayer
OptimizedLlamaInferenceAttention = LlamaAttention
