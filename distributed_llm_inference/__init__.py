"""distributed_llm_inference — MI355X-native distributed LLM inference.

Same capabilities, Python API and ``distribute`` CLI as Dylan102938/distributed-llm-inference,
re-designed for AMD Instinct MI355X (gfx950): hand-written CDNA4 HIP kernels (MFMA paged attention,
fused RMSNorm, RoPE + paged KV write, sampling, fp8), RCCL point-to-point pipeline over xGMI, a
native C++ host runtime (KV block manager, shared-memory control channels) and hipGraph decode.
"""
__version__ = "0.1.0"

from .config import PRESETS, CacheConfig, ModelSpec, ServeConfig, plan_stages, resolve_model  # noqa: F401
