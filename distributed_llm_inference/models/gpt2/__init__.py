from .model import GPT2Block, GPT2Layer  # noqa: F401
