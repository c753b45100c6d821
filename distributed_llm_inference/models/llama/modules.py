"""Llama decoder layer on the CDNA4 kernels.

Reference: ``OptimizedLlamaDecoderLayer`` / ``OptimizedLlamaInferenceAttention``
(/root/reference/distributed_llm_inference/models/llama/modules.py:23-184).  Same computation,
intended semantics (SURVEY B1/B2/B6/B7/B8/B9 fixed), MI355X-first data flow per layer:

    normed, residual = add_rmsnorm(h, residual)            # csrc/kernels/norm.hip
    qkv  = normed @ W_qkv^T                                 # ONE fused GEMM (hipBLASLt / fp8)
    q    = rope_cache(qkv) ; k,v -> paged KV cache          # csrc/kernels/rope_cache.hip
    o    = paged attention (decode split-K | prefill)       # csrc/kernels/attention.hip (MFMA)
    a    = o @ W_o^T
    normed, residual = add_rmsnorm(a, residual)
    h    = silu_mul(normed @ W_gate_up^T) @ W_down^T        # fused gate|up GEMM + activation.hip
                                                            # (decode: SwiGLU in the tile GEMM epilogue)

The residual stream is carried *separately* from the layer output, so each residual add is fused
into the following RMSNorm kernel (one HBM pass) instead of being a standalone elementwise op.
``pretraining_tp`` (reference modules.py:44-59, 107-110) is single-device weight slicing that is
mathematically identical to the unsliced projection; it is accepted and ignored.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn

from ... import ops
from ...config import ModelSpec
from ..common import AttnMetadata, Linear


def rotate_half(x: torch.Tensor) -> torch.Tensor:
    """``cat(-x2, x1)`` over the last dim (HF / reference ``rotate_half``)."""
    x1, x2 = x.chunk(2, dim=-1)
    return torch.cat((-x2, x1), dim=-1)


def apply_rotary_pos_emb(q: torch.Tensor, k: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                         unsqueeze_dim: int = 1) -> Tuple[torch.Tensor, torch.Tensor]:
    """Reference ``apply_rotary_pos_emb`` (modules.py:17-20) with the intended broadcasting (B2):
    ``cos``/``sin`` [B, T, D] are unsqueezed over the head axis of q [B, H, T, D] / k [B, KVH, T, D],
    and the rotation is computed in fp32.  The runtime path fuses RoPE into the KV-cache write
    kernel (csrc/kernels/rope_cache.hip); this helper serves library users and tests."""
    c = cos.unsqueeze(unsqueeze_dim).float()
    s = sin.unsqueeze(unsqueeze_dim).float()
    qf, kf = q.float(), k.float()
    return ((qf * c + rotate_half(qf) * s).to(q.dtype), (kf * c + rotate_half(kf) * s).to(k.dtype))


class RMSNorm(nn.Module):
    def __init__(self, hidden: int, eps: float, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden, dtype=dtype, device=device), requires_grad=False)
        self.eps = eps

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                residual_out: Optional[torch.Tensor] = None):
        return ops.rms_norm(x, self.weight, self.eps, residual=residual, residual_out=residual_out)


class LlamaAttention(nn.Module):
    def __init__(self, spec: ModelSpec, layer_idx: int, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.layer_idx = layer_idx
        self.num_heads = spec.num_heads
        self.num_kv_heads = spec.num_kv_heads
        self.head_dim = spec.head_dim
        self.scale = spec.head_dim ** -0.5
        self.qkv_proj = Linear(spec.hidden_size, spec.qkv_size, bias=spec.attention_bias,
                               dtype=dtype, device=device)
        self.o_proj = Linear(spec.q_size, spec.hidden_size, bias=spec.has_o_proj_bias, dtype=dtype,
                             device=device)
        self.qkv_proj.role, self.o_proj.role = "qkv", "o"

    def forward(self, normed: Optional[torch.Tensor], meta: AttnMetadata, k_cache: torch.Tensor,
                v_cache: torch.Tensor, cos_sin: torch.Tensor, x_q=None, defer_reduce: bool = False,
                norm: Optional[ops.RowNorm] = None):
        """``norm``: ``normed`` is the UN-normalised row and the QKV GEMV applies the input
        RMSNorm itself (1-2 decode rows, LlamaDecoderLayer._forward_gemv)."""
        q = None
        if norm is not None:
            # 1-2 rows: RMSNorm -> QKV -> RoPE / KV write in one GEMV launch when it applies
            q = self.qkv_proj.gemv_qkv_rope(normed, meta, k_cache, v_cache, cos_sin,
                                            self.num_heads, self.num_kv_heads, self.head_dim,
                                            norm=norm)
            q_sink = None
            if q is None:
                qkv = self.qkv_proj.gemv(normed, norm=norm)
                if qkv is None:
                    raise RuntimeError("fused-norm QKV: the GEMV does not take this product")
        else:
            # split-K partials of the QKV GEMM are summed inside the RoPE / KV-write kernel
            qkv = self.qkv_proj(normed, x_q, defer_reduce=True)
        if q is None:
            q, q_sink = ops.rope_cache(qkv, meta.positions, meta.slot_mapping, cos_sin,
                                       self.num_heads, self.num_kv_heads, self.head_dim, k_cache,
                                       v_cache, window=meta.window, want_sink=meta.want_sink,
                                       k_scale=meta.k_scale, v_scale=meta.v_scale)
        T = q.shape[0]
        if meta.custom_mask is not None:
            # reference-API custom 4-D additive mask (reference model.py:115-119, modules.py:92-94):
            # the prefill kernel's masked variant (any T, full cache) adds it before the online
            # softmax in place of the causal mask
            o = ops.attn_prefill(q, None, k_cache, v_cache, meta.block_tables, meta.seq_lens,
                                 meta.q_start, meta.max_q, self.scale, k_scale=meta.k_scale,
                                 v_scale=meta.v_scale, mask=meta.custom_mask)
        elif meta.is_decode:
            op = self.o_proj
            mx = (op.is_fp8 and op.bias is None and ops.policy().fp8_mx
                  and ops.attn_decode_mx_ok(self.head_dim, meta.num_splits))
            if mx and q.is_cuda:
                sp = ops.tile_gemm_splits_fp8(T, op.out_features, op.in_features)
                mx = bool(sp) and ops.mx_tileable(op.in_features, sp)
            if mx:
                # fp8 O projection: the attention epilogue quantises its output itself (one e8m0
                # scale per head row), consumed by the block-scaled MFMA -- no bf16 [T, nh*D]
                # store and no per-row quantisation pass
                o = ops.attn_decode(q, q_sink, k_cache, v_cache, meta.block_tables, meta.seq_lens,
                                    self.scale, meta.n_sink, meta.sink_pad, meta.ring, meta.window,
                                    num_splits=meta.num_splits, workspace=meta.workspace,
                                    k_scale=meta.k_scale, v_scale=meta.v_scale, mx_out=True)
                return op(None, x_q=o, defer_reduce=defer_reduce)
            o = ops.attn_decode(q, q_sink, k_cache, v_cache, meta.block_tables, meta.seq_lens,
                                self.scale, meta.n_sink, meta.sink_pad, meta.ring, meta.window,
                                num_splits=meta.num_splits, workspace=meta.workspace,
                                k_scale=meta.k_scale, v_scale=meta.v_scale)
        else:
            o = ops.attn_prefill(q, q_sink, k_cache, v_cache, meta.block_tables, meta.seq_lens,
                                 meta.q_start, meta.max_q, self.scale, meta.n_sink, meta.sink_pad,
                                 meta.ring, meta.window, k_scale=meta.k_scale,
                                 v_scale=meta.v_scale, tile_map=meta.tile_map)
        o = o.view(T, self.num_heads * self.head_dim)
        return self.o_proj(o, defer_reduce=defer_reduce)


class LlamaMLP(nn.Module):
    def __init__(self, spec: ModelSpec, device=None, dtype=torch.bfloat16):
        super().__init__()
        if spec.hidden_act != "silu":
            raise ValueError(f"unsupported Llama activation {spec.hidden_act!r}")
        self.intermediate_size = spec.intermediate_size
        self.gate_up_proj = Linear(spec.hidden_size, 2 * spec.intermediate_size, bias=spec.mlp_bias,
                                   dtype=dtype, device=device)
        self.down_proj = Linear(spec.intermediate_size, spec.hidden_size, bias=spec.mlp_bias,
                                dtype=dtype, device=device)
        self.gate_up_proj.role, self.down_proj.role = "gate_up", "down"
        # True once gate_up_proj.weight's rows are in ops.swiglu_interleave order, so the tile
        # GEMM's epilogue can apply SwiGLU itself (no [M, 2I] intermediate, no silu_mul launch)
        self.fused_swiglu = False

    def set_fused_swiglu(self, on: bool) -> None:
        """Permute gate_up_proj's rows in place to / from the fused-SwiGLU tile order (bf16
        weights, or fp8 weights + their per-channel scales when the fp8 tile path is on)."""
        w = self.gate_up_proj
        if on == self.fused_swiglu:
            return
        if w.bias is not None or w.out_features % 256:
            return
        perm = ops.swiglu_interleave if on else ops.swiglu_deinterleave
        with torch.no_grad():
            if w.is_int8:
                # LLM.int8: rows of the int8 weight and its per-channel scale, columns of the
                # transposed copy; the outlier columns are gathered from these per product
                w.weight_int8.copy_(perm(w.weight_int8))
                w.weight_scale.copy_(perm(w.weight_scale.reshape(-1, 1)).reshape(w.weight_scale.shape))
                if w.weight_int8_t is not None:
                    w.weight_int8_t.copy_(perm(w.weight_int8_t.t()).t())
            elif w.is_fp8:
                # per-output-channel quantisation commutes with the row permutation
                w.weight_fp8.copy_(perm(w.weight_fp8.view(torch.uint8)).view(w.weight_fp8.dtype))
                w.weight_scale.copy_(perm(w.weight_scale.reshape(-1, 1)).reshape(w.weight_scale.shape))
            else:
                w.weight.data.copy_(perm(w.weight.data))
        self.fused_swiglu = on

    def forward(self, normed: Optional[torch.Tensor], x_q=None, defer_reduce: bool = False,
                norm: Optional[ops.RowNorm] = None):
        gp = self.gate_up_proj
        if norm is not None:   # un-normalised rows: the gate|up GEMV applies the RMSNorm itself
            h = gp.gemv(normed, swiglu=True, norm=norm)
            if h is None:
                raise RuntimeError("fused-norm gate|up: the GEMV does not take this product")
            return self.down_proj(h, defer_reduce=defer_reduce)
        if self.fused_swiglu and ops.policy().gemv:
            # 1-2 decode rows: SwiGLU in the weight-streaming GEMV's epilogue (any weight dtype)
            h = gp.gemv_swiglu(normed, x_q)
            if h is not None:
                return self.down_proj(h, defer_reduce=defer_reduce)
        if self.fused_swiglu and gp.is_int8:
            # SwiGLU in the int8 tile GEMM's epilogue, after the fused bf16 outlier product
            h = ops.llm_int8_linear(normed, gp.weight_int8, gp.weight_scale, gp.int8_threshold,
                                    wq_t=gp.weight_int8_t, swiglu=True)
            return self.down_proj(h, defer_reduce=defer_reduce)
        if self.fused_swiglu and gp.is_fp8:
            xq, xs = x_q if x_q is not None else ops.quant_rowwise(normed)
            if xq.is_cuda and ops.tile_gemm_splits_fp8(xq.shape[0], gp.out_features,
                                                        gp.in_features):
                dp = self.down_proj
                dsp = ops.tile_gemm_splits_fp8(xq.shape[0], dp.out_features, dp.in_features)
                g4 = ops.policy().fp8_on_gemm4("gate_up")
                if (ops.policy().fp8_mx and dsp and dp.bias is None
                        and ops.mx_tileable(dp.in_features, dsp)):
                    # SwiGLU output quantised in the epilogue with per-(row, 128-column) e8m0
                    # scales, consumed by the down projection's block-scaled MFMA: no bf16 h,
                    # no per-row quantisation pass
                    h = ops.gemm_tile_fp8(xq, xs, gp.weight_fp8, gp.weight_scale, swiglu=True,
                                          mx_out=True, gemm4=g4)
                    return dp(None, x_q=h, defer_reduce=defer_reduce)
                # fp8 gate|up on the block-scaled tile kernel, SwiGLU in its epilogue (bf16 out;
                # down_proj quantises it: one [M, I] pass instead of silu_mul_quant's [M, 2I])
                h = ops.gemm_tile_fp8(xq, xs, gp.weight_fp8, gp.weight_scale, swiglu=True,
                                      gemm4=g4)
            else:
                h = ops.swiglu_interleaved(gp(None, (xq, xs)))
            return self.down_proj(h, defer_reduce=defer_reduce)
        if self.fused_swiglu:
            if gp.tile_splits(normed):
                h = ops.gemm_tile(normed, gp.weight, swiglu=True)
            else:
                h = ops.swiglu_interleaved(gp(normed))
            return self.down_proj(h, defer_reduce=defer_reduce)
        gu = gp(normed, x_q)
        if self.down_proj.is_fp8:  # SwiGLU fused with the fp8 quantisation of down_proj's input
            if not gu.is_cuda and ops.policy().fp8_mx and self.down_proj.bias is None:
                # CPU reference of the GPU tile path: h handed over in MX form (per-(row,
                # 128-column) e8m0 scales), as the fused SwiGLU epilogue quantises it
                return self.down_proj(None, x_q=ops.mx_quantize(ops.silu_mul(gu)),
                                      defer_reduce=defer_reduce)
            return self.down_proj(None, ops.silu_mul_quant(gu), defer_reduce=defer_reduce)
        return self.down_proj(ops.silu_mul(gu), defer_reduce=defer_reduce)


class LlamaDecoderLayer(nn.Module):
    """One decoder layer; ``layer_idx`` is the GLOBAL layer index (as in the reference)."""

    def __init__(self, spec: ModelSpec, layer_idx: int, device=None, dtype=torch.bfloat16):
        super().__init__()
        self.layer_idx = layer_idx
        self.hidden_size = spec.hidden_size
        self.self_attn = LlamaAttention(spec, layer_idx, device, dtype)
        self.mlp = LlamaMLP(spec, device, dtype)
        self.input_layernorm = RMSNorm(spec.hidden_size, spec.rms_norm_eps, device, dtype)
        self.post_attention_layernorm = RMSNorm(spec.hidden_size, spec.rms_norm_eps, device, dtype)

    def forward(self, hidden, residual: Optional[torch.Tensor], meta: AttnMetadata,
                k_cache: torch.Tensor, v_cache: torch.Tensor, cos_sin: torch.Tensor,
                defer_out: bool = False):
        """``defer_out``: the returned hidden state may be ``ops.SplitKPartials`` (the next
        layer's input RMSNorm reduces them); the O projection's partials always go straight
        into the post-attention RMSNorm."""
        if self._gemv_norms(hidden):
            return self._forward_gemv(hidden, residual, meta, k_cache, v_cache, cos_sin, defer_out)
        if self.self_attn.qkv_proj.is_fp8:
            return self._forward_fp8(hidden, residual, meta, k_cache, v_cache, cos_sin, defer_out)
        first = residual is None
        if first:
            # first layer of the stage: the input IS the residual; never modify it in place (it
            # may be a hipGraph's static input buffer that warmup / capture replays re-read)
            residual = hidden
            normed, _ = self.input_layernorm(hidden)
        else:
            normed, residual = self.input_layernorm(hidden, residual)
        attn = self.self_attn(normed, meta, k_cache, v_cache, cos_sin, defer_reduce=True)
        normed, residual = self.post_attention_layernorm(
            attn, residual, residual_out=torch.empty_like(residual) if first else None)
        return self.mlp(normed, defer_reduce=defer_out), residual

    def _gemv_norms(self, hidden) -> bool:
        """1-2 decode rows whose four projections all run on the weight-streaming GEMV: the two
        RMSNorms then run inside the QKV and gate|up GEMVs (``_forward_gemv``)."""
        if (not isinstance(hidden, torch.Tensor) or not hidden.is_cuda or hidden.dim() != 2
                or hidden.dtype != torch.bfloat16 or not hidden.is_contiguous()
                or not (ops.policy().gemv and ops.policy().gemv_norm)):
            return False
        M = hidden.shape[0]
        a, m = self.self_attn, self.mlp
        return (M * self.hidden_size * 2 <= 65536 and m.fused_swiglu
                and a.qkv_proj.gemv_ok(M) and a.o_proj.gemv_ok(M)
                and m.gate_up_proj.gemv_ok(M, swiglu=True) and m.down_proj.gemv_ok(M))

    def _forward_gemv(self, hidden, residual, meta, k_cache, v_cache, cos_sin, defer_out=False):
        """1-2 decode rows: input RMSNorm fused into the QKV GEMV, post-attention RMSNorm into the
        gate|up GEMV (which also applies SwiGLU): per layer QKV, RoPE/KV, attention, O, gate|up,
        down -- two launches fewer than the unfused order, same normalised rows (bit-identical
        norm arithmetic, gemv.hip).  The residual stream moves to fresh buffers (the GEMV writes
        it once while every workgroup still reads the old one)."""
        ln1, ln2 = self.input_layernorm, self.post_attention_layernorm
        if residual is None:   # first layer of the stage: the input IS the residual
            n1, res = ops.RowNorm(ln1.weight, ln1.eps), hidden
        else:
            res = torch.empty_like(residual)
            n1 = ops.RowNorm(ln1.weight, ln1.eps, residual, res)
        attn = self.self_attn(hidden, meta, k_cache, v_cache, cos_sin, norm=n1)
        res2 = torch.empty_like(res)
        n2 = ops.RowNorm(ln2.weight, ln2.eps, res, res2)
        return self.mlp(attn, norm=n2, defer_reduce=defer_out), res2

    def _forward_fp8(self, hidden, residual, meta, k_cache, v_cache, cos_sin, defer_out=False):
        """fp8 weights: every RMSNorm is fused with the fp8 quantisation of the GEMM input that
        follows it (quant.hip), so the bf16 normalised activation never touches HBM."""
        ln1, ln2 = self.input_layernorm, self.post_attention_layernorm
        first = residual is None
        if first:  # input is the residual; never modify it in place (graph static input)
            residual = hidden
            xq = ops.quant_rowwise(hidden, norm_w=ln1.weight, eps=ln1.eps)
        else:
            xq = ops.quant_rowwise(hidden, residual, ln1.weight, ln1.eps)
        # the O projection's split-K partials (tile path) are summed inside the quantiser
        attn = self.self_attn(None, meta, k_cache, v_cache, cos_sin, x_q=xq, defer_reduce=True)
        res_out = torch.empty_like(residual) if first else residual
        xq = ops.quant_rowwise(attn, residual, ln2.weight, ln2.eps, residual_out=res_out)
        # defer_out: the down projection's split-K partials go into the next layer's quantiser
        return self.mlp(None, x_q=xq, defer_reduce=defer_out), res_out

    # ------------------------------------------------------------------ weights
    def load_hf_state_dict(self, sd: dict) -> None:
        """Load a HF ``LlamaDecoderLayer`` state dict (keys relative to ``model.layers.{i}.``),
        fusing q|k|v and gate|up into the single GEMM weights."""
        def g(k):
            if k not in sd:
                raise KeyError(f"parameter {k} not found in state dict for layer {self.layer_idx}")
            return sd[k]
        dt = self.input_layernorm.weight.dtype
        with torch.no_grad():
            qkv = torch.cat([g("self_attn.q_proj.weight"), g("self_attn.k_proj.weight"),
                             g("self_attn.v_proj.weight")], 0)
            self.self_attn.qkv_proj.weight.copy_(qkv.to(dt))
            self.self_attn.o_proj.weight.copy_(g("self_attn.o_proj.weight").to(dt))
            if self.self_attn.qkv_proj.bias is not None:   # Llama attention_bias, Qwen2
                self.self_attn.qkv_proj.bias.copy_(torch.cat(
                    [g("self_attn.q_proj.bias"), g("self_attn.k_proj.bias"),
                     g("self_attn.v_proj.bias")], 0).to(dt))
            if self.self_attn.o_proj.bias is not None:     # Llama attention_bias (not Qwen2)
                self.self_attn.o_proj.bias.copy_(g("self_attn.o_proj.bias").to(dt))
            gu = torch.cat([g("mlp.gate_proj.weight"), g("mlp.up_proj.weight")], 0)
            if self.mlp.fused_swiglu:
                gu = ops.swiglu_interleave(gu)
            self.mlp.gate_up_proj.weight.copy_(gu.to(dt))
            self.mlp.down_proj.weight.copy_(g("mlp.down_proj.weight").to(dt))
            if self.mlp.gate_up_proj.bias is not None:     # Llama mlp_bias
                self.mlp.gate_up_proj.bias.copy_(torch.cat(
                    [g("mlp.gate_proj.bias"), g("mlp.up_proj.bias")], 0).to(dt))
                self.mlp.down_proj.bias.copy_(g("mlp.down_proj.bias").to(dt))
            self.input_layernorm.weight.copy_(g("input_layernorm.weight").to(dt))
            self.post_attention_layernorm.weight.copy_(g("post_attention_layernorm.weight").to(dt))

    def hf_state_dict(self) -> dict:
        """Inverse of :meth:`load_hf_state_dict` (used to write checkpoints / test parity)."""
        a, m = self.self_attn, self.mlp
        q, k, v = a.qkv_proj.weight.split([a.num_heads * a.head_dim,
                                           a.num_kv_heads * a.head_dim,
                                           a.num_kv_heads * a.head_dim], 0)
        gu = m.gate_up_proj.weight
        if m.fused_swiglu:
            gu = ops.swiglu_deinterleave(gu)
        gate, up = gu.split([m.intermediate_size, m.intermediate_size], 0)
        sd = {
            "self_attn.q_proj.weight": q, "self_attn.k_proj.weight": k,
            "self_attn.v_proj.weight": v, "self_attn.o_proj.weight": a.o_proj.weight,
            "mlp.gate_proj.weight": gate, "mlp.up_proj.weight": up,
            "mlp.down_proj.weight": m.down_proj.weight,
            "input_layernorm.weight": self.input_layernorm.weight,
            "post_attention_layernorm.weight": self.post_attention_layernorm.weight,
        }
        if a.qkv_proj.bias is not None:
            qb, kb, vb = a.qkv_proj.bias.split([a.num_heads * a.head_dim,
                                                a.num_kv_heads * a.head_dim,
                                                a.num_kv_heads * a.head_dim], 0)
            sd.update({"self_attn.q_proj.bias": qb, "self_attn.k_proj.bias": kb,
                       "self_attn.v_proj.bias": vb})
        if a.o_proj.bias is not None:
            sd["self_attn.o_proj.bias"] = a.o_proj.bias
        if m.gate_up_proj.bias is not None:
            gb, ub = m.gate_up_proj.bias.split([m.intermediate_size, m.intermediate_size], 0)
            sd.update({"mlp.gate_proj.bias": gb, "mlp.up_proj.bias": ub,
                       "mlp.down_proj.bias": m.down_proj.bias})
        return sd
