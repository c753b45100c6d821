"""Model families: Llama (primary) and GPT-2 (CPU plumbing config)."""
from .common import AttnMetadata, Linear  # noqa: F401
from .embed_head import Embedding, LMHead  # noqa: F401
from .gpt2.model import GPT2Block  # noqa: F401
from .llama.cache import KVPool, PartialLlamaSinkCache  # noqa: F401
from .llama.model import LlamaBlock  # noqa: F401
from .stage import CausalLMStage, make_block  # noqa: F401
