"""Plain-PyTorch reference implementations of every kernel in ``csrc/kernels``.

They serve two purposes only:
  1. the fp32 numerics oracle for the GPU kernel tests (``tests/test_kernels_gpu.py``);
  2. the CPU execution path (GPT-2 / tiny-Llama CPU plumbing config, CPU unit tests).
On a GPU tensor the HIP kernels are ALWAYS used (``ops/__init__.py`` never falls back silently).

Cache layouts are identical to the kernels':
  k_cache [num_blocks, nkv, block_size, D] (bf16, or fp8 e4m3fn storing k / k_scale),
  v_cache [num_blocks, nkv, block_size/8, D, 8] (V^T in 8-key groups: element (key, d) at
  [key // 8, d, key % 8]).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------- normalisation
def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float,
             residual: Optional[torch.Tensor] = None, residual_out: Optional[torch.Tensor] = None
             ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    if residual is not None:
        dst = residual if residual_out is None else residual_out
        dst.copy_((x.float() + residual.float()).to(residual.dtype))
        x = residual = dst
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype), residual


def layer_norm(x, w, b, eps, residual=None, residual_out=None):
    if residual is not None:
        dst = residual if residual_out is None else residual_out
        dst.copy_((x.float() + residual.float()).to(residual.dtype))
        x = residual = dst
    y = F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)
    return y.to(x.dtype), residual


# ----------------------------------------------------------------------------- activations
def silu_mul(x: torch.Tensor) -> torch.Tensor:
    i = x.shape[-1] // 2
    return (F.silu(x[..., :i].float()) * x[..., i:].float()).to(x.dtype)


def gelu_bias(x: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    xf = x.float() + (bias.float() if bias is not None else 0.0)
    return F.gelu(xf, approximate="tanh").to(x.dtype)


# ----------------------------------------------------------------------------- rope + cache
def _rotate(x: torch.Tensor, cs: torch.Tensor) -> torch.Tensor:
    """x [T, H, D] (any float), cs [T, D] fp32 (cos | sin halves) -> rotated fp32."""
    D = x.shape[-1]
    half = D // 2
    c = cs[:, None, :half]
    s = cs[:, None, half:]
    x1, x2 = x[..., :half].float(), x[..., half:].float()
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def rope_cache(qkv: torch.Tensor, positions: Optional[torch.Tensor],
               slot_mapping: Optional[torch.Tensor], cos_sin: Optional[torch.Tensor],
               nh: int, nkv: int, D: int, k_cache: torch.Tensor, v_cache: torch.Tensor,
               window: int = 0, want_sink: bool = False, k_scale: float = 1.0,
               v_scale: float = 1.0) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    T = qkv.shape[0]
    q = qkv[:, : nh * D].reshape(T, nh, D)
    k = qkv[:, nh * D: (nh + nkv) * D].reshape(T, nkv, D)
    v = qkv[:, (nh + nkv) * D: (nh + 2 * nkv) * D].reshape(T, nkv, D)
    q_sink = None
    if cos_sin is not None:
        maxp = cos_sin.shape[0]
        pos = positions.long().clamp(0, maxp - 1)
        cs = cos_sin[pos]
        qr = _rotate(q, cs).to(qkv.dtype)
        kr = _rotate(k, cs).to(qkv.dtype)
        if want_sink:
            ps = torch.minimum(positions.long(), torch.full_like(positions.long(), window - 1))
            q_sink = _rotate(q, cos_sin[ps.clamp(0, maxp - 1)]).to(qkv.dtype)
    else:
        qr, kr = q.clone(), k.clone()
        if want_sink:
            q_sink = q.clone()
    if slot_mapping is not None:
        bs = k_cache.shape[2]
        sm = slot_mapping.long()
        ok = sm >= 0
        if ok.any():
            blk, off = sm[ok] // bs, sm[ok] % bs
            if k_cache.dtype == torch.bfloat16:
                k_cache[blk, :, off, :] = kr[ok]
                v_cache[blk, :, off // 8, :, off % 8] = v[ok]
            else:  # fp8 cache: stored = x / scale (from the bf16-rounded value, as the kernel)
                k_cache[blk, :, off, :] = (kr[ok].float() / k_scale).to(k_cache.dtype)
                v_cache[blk, :, off // 8, :, off % 8] = (v[ok].float() / v_scale).to(v_cache.dtype)
    return qr.contiguous(), (q_sink.contiguous() if q_sink is not None else None)


# ----------------------------------------------------------------------------- attention
def _gather_seq(k_cache, v_cache, block_table, nslots, k_scale=1.0, v_scale=1.0):
    """Return K [nslots, nkv, D], V [nslots, nkv, D] in slot order (fp8 caches dequantised)."""
    bs = k_cache.shape[2]
    nb = (nslots + bs - 1) // bs
    blocks = block_table[:nb].long()
    K = k_cache[blocks].permute(0, 2, 1, 3).reshape(nb * bs, k_cache.shape[1], -1)[:nslots]
    V = v_cache[blocks].permute(0, 2, 4, 1, 3).reshape(nb * bs, v_cache.shape[1], -1)[:nslots]
    if K.dtype != torch.bfloat16 and K.dtype != torch.float32:
        K, V = K.float() * k_scale, V.float() * v_scale
    return K, V


def _ring_abs(u: torch.Tensor, L: int, n_sink: int, sink_pad: int, ring: int) -> torch.Tensor:
    o = u - sink_pad
    newest = (L - 1 - n_sink) % ring
    back = (newest - o) % ring
    return (L - 1) - back


def _attend_one(q_cols: torch.Tensor, q_sink_cols: Optional[torch.Tensor], qpos: torch.Tensor,
                K: torch.Tensor, V: torch.Tensor, L: int, scale: float, n_sink: int,
                sink_pad: int, ring: int, window: int) -> torch.Tensor:
    """q_cols [n, nh, D] with absolute positions qpos [n]; K/V [slots, nkv, D] -> [n, nh, D] fp32."""
    n, nh, D = q_cols.shape
    nkv = K.shape[1]
    G = nh // nkv
    Kf = K.float().repeat_interleave(G, dim=1)  # [S, nh, D]
    Vf = V.float().repeat_interleave(G, dim=1)
    S = K.shape[0]
    u = torch.arange(S, device=K.device)
    if ring <= 0:
        # full cache: slot == absolute position
        vis = u[None, :] <= qpos[:, None]  # [n, S]
        vis &= (u < L)[None, :]
        scores = torch.einsum("nhd,shd->nhs", q_cols.float(), Kf) * scale
        scores = scores.masked_fill(~vis[:, None, :], float("-inf"))
    else:
        is_sink = u < n_sink
        a = torch.where(is_sink, u, _ring_abs(u, L, n_sink, sink_pad, ring))
        roll_valid = (u >= sink_pad) & ((u - sink_pad) < max(0, min(ring, L - n_sink)))
        vis_roll = roll_valid[None, :] & (a[None, :] >= n_sink) & (a[None, :] <= qpos[:, None]) \
            & ((qpos[:, None] - a[None, :]) < (window - n_sink))
        vis_sink = (is_sink & (u < min(n_sink, L)))[None, :] & (u[None, :] <= qpos[:, None])
        s_roll = torch.einsum("nhd,shd->nhs", q_cols.float(), Kf) * scale
        qs = q_sink_cols if q_sink_cols is not None else q_cols
        s_sink = torch.einsum("nhd,shd->nhs", qs.float(), Kf) * scale
        scores = torch.where(is_sink[None, None, :], s_sink, s_roll)
        vis = torch.where(is_sink[None, :], vis_sink, vis_roll)
        scores = scores.masked_fill(~vis[:, None, :], float("-inf"))
    p = torch.softmax(scores, dim=-1)
    p = torch.nan_to_num(p, nan=0.0)
    return torch.einsum("nhs,shd->nhd", p, Vf)


def attn_decode(q, q_sink, k_cache, v_cache, block_tables, seq_lens, scale,
                n_sink=0, sink_pad=0, ring=0, window=0, k_scale=1.0, v_scale=1.0) -> torch.Tensor:
    B, nh, D = q.shape
    out = torch.zeros_like(q)
    for b in range(B):
        L = int(seq_lens[b])
        if L <= 0:
            continue
        nslots = L if ring <= 0 else (L if L <= n_sink else sink_pad + min(ring, L - n_sink))
        K, V = _gather_seq(k_cache, v_cache, block_tables[b], nslots, k_scale, v_scale)
        qpos = torch.tensor([L - 1], device=q.device)
        o = _attend_one(q[b:b + 1], q_sink[b:b + 1] if q_sink is not None else None, qpos, K, V,
                        L, scale, n_sink, sink_pad, ring, window)
        out[b] = o[0].to(q.dtype)
    return out


def attn_prefill(q, q_sink, k_cache, v_cache, block_tables, seq_lens, q_start, scale,
                 n_sink=0, sink_pad=0, ring=0, window=0, k_scale=1.0, v_scale=1.0) -> torch.Tensor:
    out = torch.zeros_like(q)
    B = seq_lens.numel()
    for b in range(B):
        s0, s1 = int(q_start[b]), int(q_start[b + 1])
        ql = s1 - s0
        if ql == 0:
            continue
        L = int(seq_lens[b])
        nslots = L if ring <= 0 else (L if L <= n_sink else sink_pad + min(ring, L - n_sink))
        K, V = _gather_seq(k_cache, v_cache, block_tables[b], nslots, k_scale, v_scale)
        qpos = torch.arange(L - ql, L, device=q.device)
        o = _attend_one(q[s0:s1], q_sink[s0:s1] if q_sink is not None else None, qpos, K, V, L,
                        scale, n_sink, sink_pad, ring, window)
        out[s0:s1] = o.to(q.dtype)
    return out


def attn_custom_mask(q, k_cache, v_cache, block_tables, seq_lens, q_start, scale, mask,
                     k_scale=1.0, v_scale=1.0) -> torch.Tensor:
    """Attention under a caller-supplied pre-inverted additive mask (reference model.py:115-119,
    modules.py:92-94): ``scores = q k^T * scale + mask[b, :, :, :L]``, fp32 softmax.  ``mask`` is
    [B, 1 | nh, T_b, >= L] with 0 = attend, large negative = masked; row b's queries are the last
    T_b positions of its L cached keys (full, non-windowed cache).  No causal mask is added: the
    custom mask IS the mask, exactly as in the reference."""
    out = torch.zeros_like(q)
    nh = q.shape[1]
    for b in range(seq_lens.numel()):
        s0, s1 = int(q_start[b]), int(q_start[b + 1])
        ql = s1 - s0
        if ql == 0:
            continue
        L = int(seq_lens[b])
        K, V = _gather_seq(k_cache, v_cache, block_tables[b], L, k_scale, v_scale)
        G = nh // K.shape[1]
        Kf = K.float().repeat_interleave(G, dim=1)
        Vf = V.float().repeat_interleave(G, dim=1)
        scores = torch.einsum("nhd,shd->hns", q[s0:s1].float(), Kf) * scale    # [nh, ql, L]
        mb = mask[b, :, -ql:, :L].to(device=q.device, dtype=torch.float32)    # [1|nh, ql, L]
        # entries <= -1e4 mask the key outright (exactly what exp gives next to any live score);
        # a query row with no live key outputs zeros (padding rows: the reference's eager
        # softmax over finfo.min would average V there, HF's SDPA path unmasks such rows)
        live = mb > -1e4
        p = torch.softmax((scores + mb).masked_fill(~live, float("-inf")), dim=-1)
        p = torch.nan_to_num(p, nan=0.0) * live.any(-1, keepdim=True)
        out[s0:s1] = torch.einsum("hns,shd->nhd", p, Vf).to(q.dtype)
    return out


# ----------------------------------------------------------------------------- sampling
def sample(logits: torch.Tensor, temperature: Optional[torch.Tensor] = None,
           top_k: Optional[torch.Tensor] = None, top_p: Optional[torch.Tensor] = None,
           generator: Optional[torch.Generator] = None, seeds: Optional[torch.Tensor] = None,
           step: Optional[torch.Tensor] = None,
           counters: Optional[torch.Tensor] = None) -> torch.Tensor:
    """With ``seeds`` (one per row) each row draws from its own generator seeded by
    (seed, counter) — ``counters[b]`` (the token's position in its sequence) or else ``step`` —
    like the HIP kernel's counter-based hash: a sequence's samples do not depend on which other
    rows share the batch.  (The random streams differ from the kernel's.)"""
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    st = int(step.reshape(-1)[0]) if step is not None else 0
    for b in range(B):
        g = generator
        if seeds is not None:
            c = int(counters[b]) if counters is not None else st
            g = torch.Generator(device=logits.device)
            g.manual_seed((int(seeds[b]) * 0x9E3779B97F4A7C15 + c * 0xBF58476D1CE4E5B9)
                          & 0x7FFFFFFFFFFFFFFF)
        x = logits[b].float()
        t = float(temperature[b]) if temperature is not None else 0.0
        if not t > 0:
            out[b] = int(torch.argmax(x))
            continue
        x = x / t
        k = int(top_k[b]) if top_k is not None else 0
        if 0 < k < V:
            thr = torch.topk(x, k).values[-1]
            x = x.masked_fill(x < thr, float("-inf"))
        p = float(top_p[b]) if top_p is not None else 1.0
        if p < 1.0:
            probs = torch.softmax(x, -1)
            sp, si = torch.sort(probs, descending=True)
            cum = torch.cumsum(sp, 0)
            keep_n = int(torch.searchsorted(cum, torch.tensor(p * float(cum[-1])))) + 1
            thr = sp[min(keep_n, V) - 1]
            x = x.masked_fill(probs < thr, float("-inf"))
        probs = torch.softmax(x, -1)
        out[b] = int(torch.multinomial(probs, 1, generator=g))
    return out


# ----------------------------------------------------------------------------- rope table
def build_cos_sin(head_dim: int, max_pos: int, theta: float, rope_scaling=None,
                  device=None, max_position_embeddings: Optional[int] = None,
                  seq_len: Optional[int] = None) -> torch.Tensor:
    """fp32 table [max_pos, head_dim] = (cos | sin) of the rotate-half convention, with the
    configured frequency scaling: llama3 (HF ``_compute_llama3_parameters``), linear, and
    dynamic NTK (HF ``_compute_dynamic_ntk_parameters``: for a forward whose longest position is
    ``seq_len`` > ``max_position_embeddings`` the base grows to theta * ((factor * seq_len /
    max_pe) - (factor - 1)) ** (d / (d - 2)); the caller builds such a table per forward,
    models/llama/model.py)."""
    if rope_scaling and rope_scaling.get("rope_type", rope_scaling.get("type")) == "dynamic":
        if max_position_embeddings is None:
            raise ValueError("dynamic rope scaling needs max_position_embeddings")
        if seq_len is not None and seq_len > max_position_embeddings:
            f = float(rope_scaling["factor"])
            theta = theta * ((f * seq_len / max_position_embeddings) - (f - 1)) ** (
                head_dim / (head_dim - 2))
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    attn_factor = 1.0
    if rope_scaling:
        rt = rope_scaling.get("rope_type", rope_scaling.get("type"))
        if rt == "llama3":
            factor = rope_scaling["factor"]
            lo = rope_scaling.get("low_freq_factor", 1.0)
            hi = rope_scaling.get("high_freq_factor", 4.0)
            old = rope_scaling.get("original_max_position_embeddings", 8192)
            lo_wl, hi_wl = old / lo, old / hi
            wl = 2 * math.pi / inv_freq
            scaled = torch.where(wl > lo_wl, inv_freq / factor, inv_freq)
            smooth = (old / wl - lo) / (hi - lo)
            smoothed = (1 - smooth) * scaled / factor + smooth * scaled
            is_med = (wl >= hi_wl) & (wl <= lo_wl)
            inv_freq = torch.where(is_med, smoothed, scaled)
        elif rt == "linear":
            inv_freq = inv_freq / rope_scaling["factor"]
        elif rt == "dynamic":
            pass  # the base itself was rescaled above (seq_len past max_position_embeddings)
        else:
            raise ValueError(f"unsupported rope_scaling type {rt!r}")
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv_freq)
    cs = torch.cat([freqs.cos() * attn_factor, freqs.sin() * attn_factor], dim=-1)
    return cs.to(torch.float32).to(device) if device is not None else cs.to(torch.float32)


# ----------------------------------------------------------------------------- payload digest
_M64 = (1 << 64) - 1


def digest_parts(t: torch.Tensor) -> torch.Tensor:
    """[1, 2] int64: the two order-sensitive sums of csrc/kernels/digest.hip over ``t``'s 32-bit
    words (the bytes, zero-padded to whole words), wrapped mod 2^64 in int64."""
    b = t.detach().contiguous().reshape(-1).view(torch.uint8).cpu()
    if b.numel() % 4:
        b = torch.cat([b, torch.zeros(4 - b.numel() % 4, dtype=torch.uint8)])
    w = b.view(torch.int32).to(torch.int64) & 0xFFFFFFFF
    i = torch.arange(w.numel(), dtype=torch.int64)
    s1 = (w * (2 * i + 1)).sum()
    s2 = ((w ^ 0x9E3779B9) * (((i * 0x85EBCA6B) & 0xFFFFFFFF) + 1)).sum()
    return torch.stack([s1, s2]).view(1, 2)


def digest_fold(parts: torch.Tensor) -> Tuple[int, int]:
    """The digest (s1, s2) as unsigned 64-bit ints from per-workgroup partials [n, 2]."""
    p = parts.detach().cpu().tolist()
    return (sum(r[0] & _M64 for r in p) & _M64, sum(r[1] & _M64 for r in p) & _M64)
