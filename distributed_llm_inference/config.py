"""Model / stage / serving configuration.

The reference takes its model description straight from ``transformers.AutoConfig``
(``/root/reference/distributed_llm_inference/utils/model.py:83``) and reads a handful of
``LlamaConfig`` fields (``models/llama/model.py:19-23``, ``modules.py:44-45``).  This framework
owns its model code, so it parses the HF ``config.json`` itself into a small, frozen
:class:`ModelSpec` that every layer (kernels, KV pool sizing, pipeline planner) shares.  No
network access and no HF import are needed at runtime.

Unlike the reference (bug B9 in SURVEY.md) ``rms_norm_eps`` is honoured.
"""
from __future__ import annotations

import dataclasses
import json
import math
import os
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple


@dataclass(frozen=True)
class ModelSpec:
    """Architecture description shared by every stage of a pipeline."""

    arch: str = "llama"  # "llama" | "gpt2"
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[Tuple[Tuple[str, Any], ...]] = None  # frozen dict items
    max_position_embeddings: int = 8192
    tie_word_embeddings: bool = False
    pad_token_id: Optional[int] = None
    bos_token_id: Optional[int] = 128000
    eos_token_id: Optional[int] = 128001
    hidden_act: str = "silu"
    pretraining_tp: int = 1
    attention_bias: bool = False
    mlp_bias: bool = False
    name: str = "custom"
    # Llama-family variants: "llama" | "mistral" | "qwen2" (the HF model_type)
    model_type: str = "llama"
    # bias on o_proj; None = same as attention_bias (Llama).  Qwen2 has q/k/v bias only.
    o_proj_bias: Optional[bool] = None
    # Mistral-style sliding-window attention length (None = full causal attention)
    sliding_window: Optional[int] = None
    # HF config.output_hidden_states: what LlamaBlock.forward does when its argument is None
    # (reference models/llama/model.py:35-37)
    output_hidden_states: bool = False

    @property
    def rope_type(self) -> Optional[str]:
        rs = self.rope_scaling_dict
        return None if not rs else rs.get("rope_type", rs.get("type"))

    @property
    def has_o_proj_bias(self) -> bool:
        return self.attention_bias if self.o_proj_bias is None else self.o_proj_bias

    # ------------------------------------------------------------------ derived
    @property
    def group_size(self) -> int:
        return self.num_heads // self.num_kv_heads

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def rope_scaling_dict(self) -> Optional[Dict[str, Any]]:
        return dict(self.rope_scaling) if self.rope_scaling is not None else None

    def layer_param_count(self) -> int:
        h, i = self.hidden_size, self.intermediate_size
        if self.arch == "gpt2":
            return 4 * h * h + 4 * h + 2 * h * i + i + h + 4 * h
        return h * self.qkv_size + self.q_size * h + 3 * h * i + 2 * h

    def param_count(self) -> int:
        emb = self.vocab_size * self.hidden_size
        head = 0 if self.tie_word_embeddings else emb
        return self.num_layers * self.layer_param_count() + emb + head + self.hidden_size

    def kv_bytes_per_token_per_layer(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_kv_heads * self.head_dim * dtype_bytes

    def replace(self, **kw) -> "ModelSpec":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        d["rope_scaling"] = self.rope_scaling_dict
        return d

    # ------------------------------------------------------------------ parsing
    @classmethod
    def from_hf_config(cls, cfg: Any) -> "ModelSpec":
        """Build from a HF ``config.json`` path / directory / dict / ``PretrainedConfig``."""
        if isinstance(cfg, (str, os.PathLike)):
            p = str(cfg)
            if os.path.isdir(p):
                p = os.path.join(p, "config.json")
            with open(p) as f:
                cfg = json.load(f)
        elif not isinstance(cfg, dict):
            cfg = cfg.to_dict()
        mt = cfg.get("model_type", "llama")
        if mt == "gpt2":
            h = cfg.get("n_embd", 768)
            nh = cfg.get("n_head", 12)
            return cls(
                arch="gpt2",
                vocab_size=cfg.get("vocab_size", 50257),
                hidden_size=h,
                intermediate_size=cfg.get("n_inner") or 4 * h,
                num_layers=cfg.get("n_layer", 12),
                num_heads=nh,
                num_kv_heads=nh,
                head_dim=h // nh,
                rms_norm_eps=cfg.get("layer_norm_epsilon", 1e-5),
                rope_theta=0.0,
                max_position_embeddings=cfg.get("n_positions", 1024),
                tie_word_embeddings=True,
                pad_token_id=cfg.get("pad_token_id"),
                bos_token_id=cfg.get("bos_token_id", 50256),
                eos_token_id=cfg.get("eos_token_id", 50256),
                hidden_act=cfg.get("activation_function", "gelu_new"),
                attention_bias=True,
                mlp_bias=True,
                name=cfg.get("_name_or_path", "gpt2") or "gpt2",
            )
        if mt not in ("llama", "mistral", "qwen2"):
            raise ValueError(f"unsupported model_type {mt!r} (supported: llama, mistral, qwen2, gpt2)")
        # Qwen2: q/k/v projections always carry a bias, o_proj never does (no config key)
        qwen2 = mt == "qwen2"
        sw = cfg.get("sliding_window")
        if qwen2 and not cfg.get("use_sliding_window", False):
            sw = None
        nh = cfg["num_attention_heads"]
        h = cfg["hidden_size"]
        # transformers 4.x: rope_theta + rope_scaling; transformers 5.x: rope_parameters
        rp = cfg.get("rope_parameters") or {}
        rope_theta = cfg.get("rope_theta", rp.get("rope_theta", 10000.0))
        rs = cfg.get("rope_scaling") or ({k: v for k, v in rp.items() if k != "rope_theta"}
                                         if rp else None)
        if rs is not None and rs.get("rope_type", rs.get("type")) in (None, "default"):
            rs = None
        eos = cfg.get("eos_token_id")
        if isinstance(eos, list):
            eos = eos[0]
        return cls(
            arch="llama",
            vocab_size=cfg["vocab_size"],
            hidden_size=h,
            intermediate_size=cfg["intermediate_size"],
            num_layers=cfg["num_hidden_layers"],
            num_heads=nh,
            num_kv_heads=cfg.get("num_key_value_heads") or nh,
            head_dim=cfg.get("head_dim") or h // nh,
            rms_norm_eps=cfg.get("rms_norm_eps", 1e-6),
            rope_theta=float(rope_theta),
            rope_scaling=tuple(sorted(rs.items())) if rs else None,
            max_position_embeddings=cfg.get("max_position_embeddings", 4096),
            tie_word_embeddings=bool(cfg.get("tie_word_embeddings", False)),
            pad_token_id=cfg.get("pad_token_id"),
            bos_token_id=cfg.get("bos_token_id"),
            eos_token_id=eos,
            hidden_act=cfg.get("hidden_act", "silu"),
            pretraining_tp=cfg.get("pretraining_tp", 1) or 1,
            attention_bias=True if qwen2 else bool(cfg.get("attention_bias", False)),
            mlp_bias=bool(cfg.get("mlp_bias", False)),
            name=cfg.get("_name_or_path", mt) or mt,
            model_type=mt,
            o_proj_bias=False if qwen2 else None,
            sliding_window=int(sw) if sw else None,
            output_hidden_states=bool(cfg.get("output_hidden_states", False)),
        )

    def to_hf_dict(self) -> Dict[str, Any]:
        """Inverse of :meth:`from_hf_config` (used to write ``config.json`` for random-init dirs)."""
        if self.arch == "gpt2":
            return dict(
                model_type="gpt2", vocab_size=self.vocab_size, n_embd=self.hidden_size,
                n_inner=self.intermediate_size, n_layer=self.num_layers, n_head=self.num_heads,
                layer_norm_epsilon=self.rms_norm_eps, n_positions=self.max_position_embeddings,
                activation_function=self.hidden_act, bos_token_id=self.bos_token_id,
                eos_token_id=self.eos_token_id,
            )
        arch_name = {"llama": "LlamaForCausalLM", "mistral": "MistralForCausalLM",
                     "qwen2": "Qwen2ForCausalLM"}[self.model_type]
        extra: Dict[str, Any] = {}
        if self.model_type == "mistral":
            extra["sliding_window"] = self.sliding_window
        if self.model_type == "qwen2":
            extra.update(use_sliding_window=self.sliding_window is not None,
                         sliding_window=self.sliding_window)
        return dict(
            extra, model_type=self.model_type, architectures=[arch_name],
            vocab_size=self.vocab_size,
            hidden_size=self.hidden_size, intermediate_size=self.intermediate_size,
            num_hidden_layers=self.num_layers, num_attention_heads=self.num_heads,
            num_key_value_heads=self.num_kv_heads, head_dim=self.head_dim,
            rms_norm_eps=self.rms_norm_eps, rope_theta=self.rope_theta,
            rope_scaling=self.rope_scaling_dict,
            max_position_embeddings=self.max_position_embeddings,
            tie_word_embeddings=self.tie_word_embeddings, pad_token_id=self.pad_token_id,
            bos_token_id=self.bos_token_id, eos_token_id=self.eos_token_id,
            hidden_act=self.hidden_act, pretraining_tp=self.pretraining_tp,
            attention_bias=self.attention_bias, mlp_bias=self.mlp_bias,
            output_hidden_states=self.output_hidden_states,
        )


_LLAMA3_ROPE = (("factor", 8.0), ("high_freq_factor", 4.0), ("low_freq_factor", 1.0),
                ("original_max_position_embeddings", 8192), ("rope_type", "llama3"))

PRESETS: Dict[str, ModelSpec] = {
    "llama-3-8b": ModelSpec(name="llama-3-8b"),
    "llama-3-70b": ModelSpec(
        name="llama-3-70b", hidden_size=8192, intermediate_size=28672, num_layers=80,
        num_heads=64, num_kv_heads=8),
    "llama-3.1-8b": ModelSpec(name="llama-3.1-8b", rope_scaling=_LLAMA3_ROPE,
                              max_position_embeddings=131072),
    "llama-3.1-70b": ModelSpec(
        name="llama-3.1-70b", hidden_size=8192, intermediate_size=28672, num_layers=80,
        num_heads=64, num_kv_heads=8, rope_scaling=_LLAMA3_ROPE, max_position_embeddings=131072),
    "llama-2-7b": ModelSpec(
        name="llama-2-7b", vocab_size=32000, hidden_size=4096, intermediate_size=11008,
        num_layers=32, num_heads=32, num_kv_heads=32, rope_theta=10000.0, rms_norm_eps=1e-5,
        max_position_embeddings=4096, bos_token_id=1, eos_token_id=2),
    "gpt2": ModelSpec(
        name="gpt2", arch="gpt2", vocab_size=50257, hidden_size=768, intermediate_size=3072,
        num_layers=12, num_heads=12, num_kv_heads=12, head_dim=64, rms_norm_eps=1e-5,
        rope_theta=0.0, max_position_embeddings=1024, tie_word_embeddings=True,
        bos_token_id=50256, eos_token_id=50256, hidden_act="gelu_new", attention_bias=True,
        mlp_bias=True),
    "mistral-7b": ModelSpec(
        name="mistral-7b", model_type="mistral", vocab_size=32000, hidden_size=4096,
        intermediate_size=14336, num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128,
        rms_norm_eps=1e-5, rope_theta=10000.0, max_position_embeddings=32768, bos_token_id=1,
        eos_token_id=2, sliding_window=4096),
    "qwen2-7b": ModelSpec(
        name="qwen2-7b", model_type="qwen2", vocab_size=152064, hidden_size=3584,
        intermediate_size=18944, num_layers=28, num_heads=28, num_kv_heads=4, head_dim=128,
        rms_norm_eps=1e-6, rope_theta=1000000.0, max_position_embeddings=32768,
        bos_token_id=151643, eos_token_id=151645, attention_bias=True, o_proj_bias=False),
    # tiny configs for CPU tests / smoke
    "tiny-llama": ModelSpec(
        name="tiny-llama", vocab_size=512, hidden_size=128, intermediate_size=256, num_layers=4,
        num_heads=4, num_kv_heads=2, head_dim=32, max_position_embeddings=2048,
        rope_theta=10000.0, bos_token_id=1, eos_token_id=2),
    # 8 layers: one per rank in the 8-rank CPU rehearsals of the PP=8 paths
    "tiny-llama-8l": ModelSpec(
        name="tiny-llama-8l", vocab_size=512, hidden_size=128, intermediate_size=256, num_layers=8,
        num_heads=4, num_kv_heads=2, head_dim=32, max_position_embeddings=2048,
        rope_theta=10000.0, bos_token_id=1, eos_token_id=2),
    "tiny-gpt2": ModelSpec(
        name="tiny-gpt2", arch="gpt2", vocab_size=512, hidden_size=128, intermediate_size=512,
        num_layers=4, num_heads=4, num_kv_heads=4, head_dim=32, max_position_embeddings=512,
        rope_theta=0.0, tie_word_embeddings=True, bos_token_id=1, eos_token_id=2,
        hidden_act="gelu_new", attention_bias=True, mlp_bias=True),
}


def resolve_model(model: Any) -> ModelSpec:
    """Accept a preset name, a ``config.json`` path/dir, a dict, a HF config or a ModelSpec."""
    if isinstance(model, ModelSpec):
        return model
    if isinstance(model, str):
        key = model.lower().replace("meta-llama/", "").replace("_", "-")
        key = key.replace("meta-llama-3", "llama-3")
        if key in PRESETS:
            return PRESETS[key]
        if os.path.exists(model):
            return ModelSpec.from_hf_config(model)
        raise ValueError(f"unknown model {model!r}: not a preset ({sorted(PRESETS)}) nor a path")
    return ModelSpec.from_hf_config(model)


# ---------------------------------------------------------------------------------------------
# Stage placement (pipeline planner).  The reference's server stub wants to "choose optimal block
# ids" (server/server.py:7-8) and the worker owns [block_index_start, block_index_end)
# (server/worker.py:13-14).  On one MI355X node every GPU is identical and fully connected, so the
# optimal placement is the contiguous, cost-balanced split below.  The first stage also pays the
# embedding gather and the last stage the LM head, so their layer counts are trimmed by the
# equivalent layer cost.
# ---------------------------------------------------------------------------------------------
def plan_stages(spec: ModelSpec, num_stages: int,
                weights: Optional[Sequence[float]] = None,
                head_rotation: bool = False) -> List[Tuple[int, int]]:
    """Split ``spec.num_layers`` into ``num_stages`` contiguous ``[start, end)`` ranges.

    ``weights`` (optional, one per stage) expresses relative stage speed (e.g. for a degraded GPU
    during rebalancing); the default is uniform hardware.  ``head_rotation``: the decode steps'
    LM head runs on every rank in turn (runtime/head.py), so its cost is shared evenly instead of
    trimming the last stage.
    """
    L = spec.num_layers
    if num_stages < 1:
        raise ValueError("num_stages must be >= 1")
    if num_stages > L:
        raise ValueError(f"cannot split {L} layers into {num_stages} stages")
    w = list(weights) if weights is not None else [1.0] * num_stages
    if len(w) != num_stages or min(w) <= 0:
        raise ValueError("weights must be positive, one per stage")
    # LM head (+ final norm + sampling) in layer-equivalents of decode time.  By bytes/FLOPs the
    # head is vocab*hidden / layer_params (1.22 layers for Llama-3-70B), but its single wide GEMM
    # runs far more efficiently than a layer (which also carries attention, norms, activation):
    # measured on MI355X at 512 rows, head + sampling 0.78 ms vs 1.06 ms per layer
    # (profiles/pp1_bf16_b512_decode_breakdown.txt) -> factor 0.6.
    head_cost = 0.6 * spec.vocab_size * spec.hidden_size / max(1, spec.layer_param_count())
    extra = [0.0] * num_stages
    if num_stages > 1:
        if head_rotation:
            extra = [head_cost / num_stages] * num_stages
        else:
            extra[-1] += head_cost
    total = (L + sum(extra))
    tw = sum(w)
    # start below the proportional target, then hand out the remaining layers one at a time to
    # the stage whose time after taking it is smallest: this minimises the slowest stage, which
    # sets the pipeline's throughput
    targets = [total * wi / tw - ei for wi, ei in zip(w, extra)]
    counts = [max(1, int(math.floor(t))) for t in targets]
    while sum(counts) > L:
        i = max((k for k in range(num_stages) if counts[k] > 1),
                key=lambda k: (counts[k] + extra[k]) / w[k])
        counts[i] -= 1
    while sum(counts) < L:
        i = min(range(num_stages), key=lambda k: ((counts[k] + 1 + extra[k]) / w[k], k))
        counts[i] += 1
    out, s = [], 0
    for c in counts:
        out.append((s, s + c))
        s += c
    return out


@dataclass
class CacheConfig:
    """KV-cache policy for one stage.

    ``window_length``/``num_sink_tokens`` mirror ``PartialLlamaSinkCache(window_length,
    num_sink_tokens)`` (reference ``models/llama/cache.py:11``).  ``window_length=0`` means a full
    (non-evicting) cache sized from HBM.
    """

    block_size: int = 64
    num_blocks: Optional[int] = None  # None -> sized from free HBM
    gpu_memory_utilization: float = 0.90
    window_length: int = 0
    num_sink_tokens: int = 0
    max_chunk: int = 512  # extra ring headroom so a prefill chunk never evicts keys it needs
    dtype: str = "bf16"   # "bf16" | "fp8" (e4m3fn: half the decode-attention bytes, 2x tokens)
    k_scale: float = 1.0  # fp8 cache stores k / k_scale and v / v_scale
    v_scale: float = 1.0

    def __post_init__(self):
        if self.dtype not in ("bf16", "fp8"):
            raise ValueError(f"KV cache dtype must be 'bf16' or 'fp8', got {self.dtype!r}")

    @property
    def windowed(self) -> bool:
        return self.window_length > 0

    @property
    def torch_dtype(self):
        import torch
        return torch.float8_e4m3fn if self.dtype == "fp8" else torch.bfloat16

    @property
    def dtype_bytes(self) -> int:
        return 1 if self.dtype == "fp8" else 2


@dataclass
class KernelPolicy:
    """Which hand-written kernel takes each hot-path product (read by ``ops`` at every call, so a
    captured hipGraph keeps the choice it was captured with).  The defaults are the measured
    winners; the fields exist for the trade-offs that are real and for A/B runs.  Set from
    ``EngineConfig.kernels`` / ``distribute --kernels k=v,...`` / ``bench.py --kernels``; the
    ``DLI_KERNELS`` environment variable (same syntax) overrides them."""

    # bf16 decode projections on the one-wave-per-SIMD gemm4 kernel (else the 8-wave gemm_tile):
    # 70B decode step 75.0 vs 77.7 ms (profiles/r4/gemm4_step_ab.txt)
    gemm4: bool = True
    # fp8 decode projections on gemm4 (16x16x128 block-scaled MFMA, G4S8 k-loop; bit-identical
    # to gemm_tile) instead of gemm_tile: "all", "none", or a "+"-separated subset of qkv / o /
    # gate_up / down.  gate|up: 202 vs 219 us alone, +1.9 % tok/s in-step; the others win 2-7 %
    # alone but stay within noise in-step (profiles/r5/fp8_gemm4_16x16.md)
    fp8_gemm4: str = "gate_up"
    # bf16 gemm4 k-loop schedule at decode M (<= 2 row tiles of 256): 8 / 9 = 4 / 6 with the
    # weight stream non-temporal, or 4, 6 (csrc/kernels/gemm4.hip G4Sched; 8: +1.4 % tok/s over
    # 6 in-step, profiles/r5/gemm4_sched_nt.md)
    gemm4_decode_sched: int = 8
    # split-K partials of the deferred projections (QKV, O, down) stored as bf16 (else fp32);
    # consumers always sum in fp32 (profiles/bf16_partials_ab.txt, docs/parity.md C6)
    bf16_partials: bool = True
    # split-K partials summed by their consumer kernel (RMSNorm / RoPE / quantiser) instead of a
    # reduce pass; with fp32 partials both are bit-identical (the tests' reference path)
    defer_splitk: bool = True
    # fp8: SwiGLU / attention outputs handed to the next projection as MX (e8m0 per 128-column
    # block, quantised in the producer's epilogue) instead of bf16 + a per-row quantiser pass
    fp8_mx: bool = True
    # hand-written tile GEMMs for the decode projections at all (False: hipBLASLt everywhere)
    tile_gemms: bool = True
    # hipBLASLt for the products the tile kernels do not take well (M < 128, the LM head).  None = automatic: off when pipeline ranks share a GPU (DLI_SHARE_GPU), because its
    # stream-K kernels wait on each other's workgroups (README "What else couples streams")
    library_gemms: Optional[bool] = None
    # largest M that stays on the tile kernels when library GEMMs are on (0: no bound - large-M
    # prefill products run on gemm4 / gemm_tile too).  Above 2048 hipBLASLt stays: at the
    # headline's 16384-row prefill chunks it runs the 70B projections at 1.63 PF against gemm4's
    # 1.36 (rocprof, profiles/r6/pgemm/top_*.txt; prefill 25.5 vs 29.2 s).  A single-prompt TTFT
    # reads the other way (32k: 4.89 vs 5.55 s) only because the first request pays hipBLASLt's
    # lazy code-object loads for its new shapes - a one-time cost, not a per-request one.
    tile_gemm_max_m: int = 2048
    # ... and the executor runs each such projection once at start-up (StageExecutor.
    # warm_prefill_gemms), so the first long prompt does not pay hipBLASLt's code-object loads
    warm_library_gemms: bool = True
    # run the partial last wave of whole-K bf16 gemm_tile products stream-K (neutral in-step)
    stream_k_tail: bool = False
    # 1-2 decode rows on the weight-streaming GEMVs, with the input RMSNorm, RoPE/KV write and
    # SwiGLU fused into them (else the batch path)
    gemv: bool = True
    # ... with the RMSNorms fused into the QKV / gate|up GEMVs (bit-identical norm arithmetic)
    gemv_norm: bool = True
    # LLM.int8: a resident transposed int8 copy of every weight for the outlier-column gather
    # (1.6 vs 2.9 ms per 70B step, but one more byte per weight: a third less KV capacity)
    int8_transposed: bool = False
    # prefill attention on the 32x32x16-MFMA kernel (csrc/kernels/attn_prefill32.hip: 32 query
    # rows per wave, 64-key steps) wherever it applies (bf16 full cache, head_dim 128, any GQA
    # group incl. MHA, no custom mask); else attention.hip's 16x16x32 kernel
    prefill_m32: bool = True

    _FP8_SHAPES = ("qkv", "o", "gate_up", "down")

    def __post_init__(self):
        if self.gemm4_decode_sched not in (4, 6, 8, 9):
            raise ValueError(f"gemm4_decode_sched={self.gemm4_decode_sched}: 4, 6, 8 or 9")
        sel = self.fp8_gemm4
        if sel not in ("all", "none") and any(
                x not in self._FP8_SHAPES for x in sel.split("+")):
            raise ValueError(f"fp8_gemm4={sel!r}: 'all', 'none' or a '+' list of "
                             f"{'/'.join(self._FP8_SHAPES)}")

    def fp8_on_gemm4(self, shape: str) -> bool:
        return self.gemm4 and (self.fp8_gemm4 == "all" or shape in self.fp8_gemm4.split("+"))

    def with_overrides(self, spec: str) -> "KernelPolicy":
        """``"gemm4=0,library_gemms=auto"`` applied on top of this policy."""
        if not spec or not spec.strip():
            return self
        kw: Dict[str, Any] = {}
        names = {f.name: f for f in dataclasses.fields(self)}
        for item in spec.split(","):
            if not item.strip():
                continue
            k, _, v = item.partition("=")
            k, v = k.strip(), v.strip()
            if k not in names:
                raise ValueError(f"unknown kernel policy field {k!r} (known: {sorted(names)})")
            if k == "fp8_gemm4":
                kw[k] = v
            elif names[k].type in (int, "int"):
                kw[k] = int(v)
            elif k == "library_gemms" and v.lower() in ("auto", "none", ""):
                kw[k] = None
            elif v.lower() in ("1", "true", "on", "yes"):
                kw[k] = True
            elif v.lower() in ("0", "false", "off", "no"):
                kw[k] = False
            else:
                raise ValueError(f"kernel policy {k}={v!r}: expected 0/1")
        return dataclasses.replace(self, **kw)


@dataclass
class ServeConfig:
    max_batch_size: int = 256
    max_num_batched_tokens: int = 8192
    num_micro_batches: int = 0  # 0 -> num_stages (+0) for a full pipeline
    max_seq_len: int = 8192
    use_graphs: bool = True
    # decode steps' LM head + sampling on every pipeline rank in turn (runtime/head.py) instead of
    # the last stage only; env DLI_HEAD_ROTATION=0/1 overrides
    head_rotation: bool = True
    graph_batch_sizes: List[int] = field(default_factory=lambda: [1, 2, 4, 8, 16, 32, 64, 96, 128,
                                                                  160, 192, 224, 256])
