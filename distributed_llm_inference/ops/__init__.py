"""Operator front-end: GPU tensors -> hand-written CDNA4 HIP kernels, CPU tensors -> torch reference.

There is deliberately no silent fallback: a GPU tensor with the native extension missing raises
(``NativeKernelsMissing``), so a GPU run can never "pass" on an eager PyTorch path.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Optional, Tuple

import torch

from ..config import KernelPolicy
from . import reference as ref

_C = None
_POLICY: Optional[KernelPolicy] = None


def policy() -> KernelPolicy:
    """The process's :class:`~config.KernelPolicy` (``DLI_KERNELS`` applied on top)."""
    global _POLICY
    if _POLICY is None:
        _POLICY = KernelPolicy().with_overrides(os.environ.get("DLI_KERNELS", ""))
    return _POLICY


def set_policy(p: KernelPolicy) -> KernelPolicy:
    """Install ``p`` (``DLI_KERNELS`` still overrides it); returns the previous policy."""
    global _POLICY
    prev = policy()
    _POLICY = p.with_overrides(os.environ.get("DLI_KERNELS", ""))
    return prev


@contextlib.contextmanager
def kernel_policy(**fields):
    """Temporarily change policy fields (tests, A/B probes): ``with kernel_policy(gemm4=False):``."""
    import dataclasses
    prev = policy()
    global _POLICY
    _POLICY = dataclasses.replace(prev, **fields)
    try:
        yield _POLICY
    finally:
        _POLICY = prev


class NativeKernelsMissing(RuntimeError):
    pass


def native():
    """The compiled ``_C`` extension (kernels + RCCL).  Raises if it was not built."""
    global _C
    if _C is None:
        try:
            from .. import _C as mod  # type: ignore[attr-defined]
        except ImportError as e:  # pragma: no cover - depends on build state
            raise NativeKernelsMissing(
                "distributed_llm_inference native kernels are not built; run "
                "`python -m distributed_llm_inference._build` (hipcc, gfx950)") from e
        _C = mod
    return _C


def native_available() -> bool:
    try:
        native()
        return True
    except NativeKernelsMissing:
        return False


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# ----------------------------------------------------------------------------- normalisation
class SplitKPartials:
    """The un-reduced output of a split-K tile GEMM: partial products ``parts [S, M, N]``, bf16
    by default (:func:`bf16_partials`), fp32 with ``KernelPolicy.bf16_partials=False``;
    consumers always sum them in fp32.

    ``gemm_tile(..., defer_reduce=True)`` returns this instead of running the reduction pass;
    ``rms_norm`` sums the partials while it reads them (norm.hip ``x_parts``), so the reduce
    kernel and the bf16 [M, N] round trip through HBM disappear.  Any other consumer calls
    :meth:`materialize`."""

    __slots__ = ("parts",)

    def __init__(self, parts: torch.Tensor):
        self.parts = parts

    @property
    def shape(self):
        return torch.Size(self.parts.shape[1:])

    @property
    def device(self):
        return self.parts.device

    dtype = torch.bfloat16
    is_cuda = True

    def materialize(self) -> torch.Tensor:
        if self.parts.dtype != torch.float32:   # bf16 partials (fp8 path): summed in fp32
            return self.parts.float().sum(0).to(torch.bfloat16)
        out = torch.empty(self.parts.shape[1:], dtype=torch.bfloat16, device=self.parts.device)
        native().splitk_reduce(out, self.parts)
        return out


def bf16_partials() -> bool:
    """Split-K partials of the deferred projections (QKV, O, down) stored as bf16
    (``KernelPolicy.bf16_partials``, default) for every operand precision: half the partial
    traffic of the GEMM epilogue and of the consumer that sums them (RMSNorm / RoPE); each
    partial carries one extra bf16 rounding (~2^-9 relative) before the fp32 sum.  Measured on the
    default bench (same box, interleaved): 6468-6482 -> 6556-6574 tok/s
    (profiles/bf16_partials_ab.txt).  End-to-end bound vs the fp32 CPU reference:
    tests/test_engine_gpu.py::test_bf16_splitk_partials_end_to_end_vs_cpu_reference; listed in
    docs/parity.md (C6)."""
    return policy().bf16_partials


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None, residual_out: Optional[torch.Tensor] = None
             ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """``r = x + residual`` written to ``residual_out`` (default: in place into ``residual``);
    ``out = RMSNorm(r or x) * w``.  Returns ``(out, r)``.  ``x`` may be :class:`SplitKPartials`."""
    if isinstance(x, SplitKPartials):
        out = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device) if out is None else out
        native().rms_norm_splitk(out, x.parts, residual, w, float(eps), residual_out)
        return out, (residual_out if residual_out is not None else residual)
    if not _gpu(x):
        y, r = ref.rms_norm(x, w, eps, residual, residual_out)
        if out is not None:
            out.copy_(y)
            y = out
        return y, r
    out = torch.empty_like(x) if out is None else out
    native().rms_norm(out, x, residual, w, float(eps), residual_out)
    return out, (residual_out if residual_out is not None else residual)


def layer_norm(x, w, b, eps, residual=None, out=None, residual_out=None):
    if not _gpu(x):
        y, r = ref.layer_norm(x, w, b, eps, residual, residual_out)
        if out is not None:
            out.copy_(y)
            y = out
        return y, r
    out = torch.empty_like(x) if out is None else out
    native().layer_norm(out, x, residual, w, b, float(eps), residual_out)
    return out, (residual_out if residual_out is not None else residual)


# ----------------------------------------------------------------------------- activations
def silu_mul(x: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not _gpu(x):
        y = ref.silu_mul(x)
        return out.copy_(y) if out is not None else y
    if out is None:
        out = torch.empty(*x.shape[:-1], x.shape[-1] // 2, dtype=x.dtype, device=x.device)
    native().silu_mul(out, x)
    return out


def gelu_bias(x: torch.Tensor, bias: Optional[torch.Tensor] = None,
              out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not _gpu(x):
        y = ref.gelu_bias(x, bias)
        return out.copy_(y) if out is not None else y
    out = torch.empty_like(x) if out is None else out
    native().gelu_bias(out, x, bias)
    return out


def add(a: torch.Tensor, b: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    if not _gpu(a):
        y = (a.float() + b.float()).to(a.dtype)
        return out.copy_(y) if out is not None else y
    out = torch.empty_like(a) if out is None else out
    native().add(out, a, b)
    return out


# ----------------------------------------------------------------------------- rope + cache
def rope_cache(qkv: torch.Tensor, positions: Optional[torch.Tensor],
               slot_mapping: Optional[torch.Tensor], cos_sin: Optional[torch.Tensor], nh: int,
               nkv: int, head_dim: int, k_cache: torch.Tensor, v_cache: torch.Tensor,
               window: int = 0, want_sink: bool = False, q_out: Optional[torch.Tensor] = None,
               q_sink_out: Optional[torch.Tensor] = None, k_scale: float = 1.0,
               v_scale: float = 1.0):
    """Rotate q/k, write k/v to the paged cache; returns ``(q [T, nh, D], q_sink or None)``.
    fp8 (e4m3fn) caches store ``k / k_scale`` and ``v / v_scale``.  ``qkv`` may be
    :class:`SplitKPartials` (summed while loaded, bit-identical to the reduce pass)."""
    if isinstance(qkv, SplitKPartials):
        T = qkv.shape[0]
        if q_out is None:
            q_out = torch.empty(T, nh, head_dim, dtype=torch.bfloat16, device=qkv.device)
        if want_sink and q_sink_out is None:
            q_sink_out = torch.empty_like(q_out)
        native().rope_cache(qkv.parts, positions, slot_mapping, cos_sin, q_out,
                            q_sink_out if want_sink else None, int(window), k_cache, v_cache,
                            int(nh), int(nkv), float(k_scale), float(v_scale))
        return q_out, (q_sink_out if want_sink else None)
    if not _gpu(qkv):
        q, qs = ref.rope_cache(qkv, positions, slot_mapping, cos_sin, nh, nkv, head_dim, k_cache,
                               v_cache, window, want_sink, k_scale, v_scale)
        if q_out is not None:
            q_out.copy_(q)
            q = q_out
        if qs is not None and q_sink_out is not None:
            q_sink_out.copy_(qs)
            qs = q_sink_out
        return q, qs
    T = qkv.shape[0]
    if q_out is None:
        q_out = torch.empty(T, nh, head_dim, dtype=qkv.dtype, device=qkv.device)
    if want_sink and q_sink_out is None:
        q_sink_out = torch.empty_like(q_out)
    native().rope_cache(qkv, positions, slot_mapping, cos_sin, q_out,
                        q_sink_out if want_sink else None, int(window), k_cache, v_cache,
                        int(nh), int(nkv), float(k_scale), float(v_scale))
    return q_out, (q_sink_out if want_sink else None)


# ----------------------------------------------------------------------------- attention
def decode_splits(batch: int, nkv: int, group: int, max_len: int, cu: int = 256,
                  kv_fp8: bool = False) -> int:
    """Split-K factor for decode.  The kernel runs one wave per (sequence, kv head, 16-head group,
    split); aim for ~4 waves per CU (measured best on the 70B head config from B = 1 to 16, 8k-32k
    contexts: profiles/attn_decode_microbench.json) while keeping >= 1 key step per split.  Splits come
    in multiples of 4 from 4 up (a workgroup's 4 waves merge theirs in LDS, csrc/kernels/
    attention.hip), so B = 1 at 8k context runs 256 splits (2048 waves) instead of the 64 the
    unmerged partial traffic used to allow.  An fp8 cache streams half the bytes per key step, so
    where the bf16 rule already splits (2-16) it takes twice the splits (B = 64 at 4k: 104 -> 98 us,
    B = 16 at 8k: 58 -> 56 us; one split stays best at large batch and 128 at B = 1:
    profiles/attn_fp8kv_split_sweep.json)."""
    waves = batch * nkv * ((group + 15) // 16)
    if waves >= 8 * cu:
        return 1
    target = 4 * cu
    want = (target + waves - 1) // waves
    max_useful = max(1, (max_len + 31) // 32)
    s = int(max(1, min(want, max_useful, 512)))
    if kv_fp8 and 2 <= s <= 16:
        s = min(2 * s, max_useful)
    if s >= 4:
        return s // 4 * 4
    return 2 if s == 3 else s


def attn_decode_mx_ok(head_dim: int, num_splits: int) -> bool:
    """Whether :func:`attn_decode` can hand its output over as :class:`MxFp8` (one e8m0 scale
    per head row = one 128-column block of the O projection's input; single-split decode)."""
    return head_dim == 128 and num_splits == 1


def attn_decode(q, q_sink, k_cache, v_cache, block_tables, seq_lens, scale, n_sink=0, sink_pad=0,
                ring=0, window=0, num_splits=1, workspace=None, out=None, k_scale=1.0, v_scale=1.0,
                mx_out: bool = False):
    """Paged GQA decode attention -> bf16 ``[T, nh, D]``; ``mx_out`` (needs
    :func:`attn_decode_mx_ok`): the same values (rounded to bf16) quantised in the kernel's
    epilogue to :class:`MxFp8` ``[T, nh * D]`` for the fp8 O projection, replacing a separate
    per-row quantisation pass."""
    if mx_out and not attn_decode_mx_ok(q.shape[-1], num_splits):
        raise ValueError("attn_decode(mx_out=True) needs head_dim 128 and one split")
    if not _gpu(q):
        y = ref.attn_decode(q, q_sink, k_cache, v_cache, block_tables, seq_lens, scale, n_sink,
                            sink_pad, ring, window, k_scale, v_scale)
        if mx_out:
            return mx_quantize(y.to(torch.bfloat16).reshape(q.shape[0], -1))
        return out.copy_(y) if out is not None else y
    if mx_out:
        T, nh, D = q.shape
        nb = (T + 63) // 64
        q8 = torch.empty(T, nh * D, dtype=torch.float8_e4m3fn, device=q.device)
        sc = torch.empty(nh * nb * 64, dtype=torch.uint8, device=q.device)
        # the kernel writes only q8 / sc: no bf16 output (nothing held in a graph's pool)
        dummy = q.new_empty((0, nh, D))
        native().attn_decode(dummy, q, q_sink, k_cache, v_cache, block_tables, seq_lens,
                             float(scale), int(n_sink), int(sink_pad), int(ring), int(window), 1,
                             None, None, float(k_scale), float(v_scale), q8, sc)
        return MxFp8(q8, sc)
    out = torch.empty_like(q) if out is None else out
    part_o = part_ml = None
    if num_splits > 1:
        if workspace is None:
            workspace = decode_workspace(q.shape[0], q.shape[1], q.shape[2], num_splits, q.device)
        part_o, part_ml = workspace[0], workspace[1]
    native().attn_decode(out, q, q_sink, k_cache, v_cache, block_tables, seq_lens, float(scale),
                         int(n_sink), int(sink_pad), int(ring), int(window), int(num_splits),
                         part_o, part_ml, float(k_scale), float(v_scale))
    return out


def decode_workspace(rows: int, nh: int, head_dim: int, splits: int, device):
    """Split-K decode workspace: fp32 partial O and (max, sum) per split (sized for the unmerged
    worst case; the kernel uses splits / 4 of it when its workgroups merge their splits)."""
    return (torch.empty(splits * rows * nh * head_dim, dtype=torch.float32, device=device),
            torch.empty(splits * rows * nh * 2, dtype=torch.float32, device=device))


PREFILL_QB = 1   # 16-token query blocks per prefill wave (attention.hip QB; 2 was +2 % on 2k-4k
                 # chunks but -25 % on 16-token ones: profiles/attn_prefill_qb_ab.json)
PREFILL_QB_LONG = 1024   # from this longest chunk on, 32-token tiles (attn_prefill32.hip: 8 waves
                         # per workgroup, staggered halves) beat 16-token ones (4 waves, two
                         # workgroups per CU): 2k-on-6k 962-980 vs 935-954 TFLOP/s; below it
                         # the 16-token tiles win (512-token prompts 414-432 vs 397)
                         # (profiles/r6/prefill/)


def prefill_qb_for(max_q: int) -> int:
    """The prefill tile choice for a batch whose longest chunk is ``max_q`` tokens: one
    function, so the tile map and the kernel launch always agree."""
    return 2 if max_q >= PREFILL_QB_LONG else PREFILL_QB


def prefill_tile_tokens(nh: int, nkv: int, qb: int = PREFILL_QB) -> int:
    """Query tokens per prefill workgroup tile (attention.hip: 16 * TPW * QB, TPW = 4 / HPW)."""
    G = nh // nkv
    hpw = 4 if G % 4 == 0 else (2 if G % 2 == 0 else 1)
    return 16 * (4 // hpw) * qb


def prefill_tiles(q_lens, nh: int, nkv: int, out=None, qb: Optional[int] = None) -> torch.Tensor:
    """Compact (sequence, token-tile) work list of the prefill kernel: one row per tile that
    holds query tokens.  A 1-token decode row mixed into a prefill batch gets a single tile
    instead of ``max_q / tile`` empty workgroups.  Returns int32 [n_tiles, 2] (or fills ``out``)."""
    import numpy as np
    if qb is None:
        qb = prefill_qb_for(max(q_lens) if len(q_lens) else 0)
    tt = prefill_tile_tokens(nh, nkv, qb)
    ql = np.asarray(q_lens, dtype=np.int64)
    nt = (ql + tt - 1) // tt
    b = np.repeat(np.arange(len(ql), dtype=np.int32), nt)
    starts = np.repeat(np.cumsum(nt) - nt, nt)
    tile = (np.arange(int(nt.sum())) - starts).astype(np.int32)
    m = np.stack([b, tile], axis=1)
    if out is not None:
        out.numpy()[: len(m)] = m
        return out[: len(m)]
    return torch.from_numpy(np.ascontiguousarray(m))


def attn_prefill(q, q_sink, k_cache, v_cache, block_tables, seq_lens, q_start, max_q, scale,
                 n_sink=0, sink_pad=0, ring=0, window=0, out=None, k_scale=1.0, v_scale=1.0,
                 tile_map=None, mask=None, qb: Optional[int] = None):
    """Paged varlen prefill attention.  ``mask``: the reference API's pre-inverted 4-D additive
    mask ``[B, 1 | nh, T, >= L]`` (0 = attend, large negative = masked; the last ``q_len_b`` rows
    of sequence b) - it replaces the causal mask (full cache, any T incl. 1).  ``qb``: 16-token
    query blocks per wave (1 or 2; ``tile_map`` must be built with the same value)."""
    if not _gpu(q):
        if mask is not None:
            y = ref.attn_custom_mask(q, k_cache, v_cache, block_tables, seq_lens, q_start, scale,
                                     mask, k_scale, v_scale)
        else:
            y = ref.attn_prefill(q, q_sink, k_cache, v_cache, block_tables, seq_lens, q_start,
                                 scale, n_sink, sink_pad, ring, window, k_scale, v_scale)
        return out.copy_(y) if out is not None else y
    out = torch.empty_like(q) if out is None else out
    if qb is None:
        qb = prefill_qb_for(int(max_q))
    if mask is not None:
        if ring:
            raise ValueError("custom 4-D masks need a full (non-windowed) cache")
        mask = mask.to(device=q.device, dtype=torch.float32).contiguous()
        tile_map = None   # dense grid: the masked kernel runs one query block per wave
    native().attn_prefill(out, q, q_sink, k_cache, v_cache, block_tables, seq_lens, q_start,
                          int(max_q), float(scale), int(n_sink), int(sink_pad), int(ring),
                          int(window), float(k_scale), float(v_scale), tile_map, int(qb), mask,
                          bool(policy().prefill_m32))
    return out


# ----------------------------------------------------------------------------- payload digest
def digest(t: torch.Tensor, nblocks: int = 256) -> torch.Tensor:
    """Hop-integrity digest partials of ``t`` (csrc/kernels/digest.hip on the current stream;
    torch on the CPU); fold them with :func:`digest_fold`.  Returns [nblocks, 2] int64."""
    if not _gpu(t) or (t.numel() * t.element_size()) % 4:
        return ref.digest_parts(t)
    t = t.contiguous()
    part = torch.empty(nblocks, 2, dtype=torch.int64, device=t.device)
    native().digest(part, t)
    return part


digest_fold = ref.digest_fold


# ----------------------------------------------------------------------------- sampling
def sample(logits: torch.Tensor, temperature: Optional[torch.Tensor] = None,
           top_k: Optional[torch.Tensor] = None, top_p: Optional[torch.Tensor] = None,
           seeds: Optional[torch.Tensor] = None, step: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, logprobs: Optional[torch.Tensor] = None,
           generator: Optional[torch.Generator] = None,
           counters: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``seeds`` + ``counters`` (int64 per row: the sampled token's position in its sequence) key
    each row's randomness, so a seeded request samples the same tokens in any batch / pipeline;
    without ``counters`` the device ``step`` and the row index do."""
    if not _gpu(logits):
        y = ref.sample(logits, temperature, top_k, top_p, generator, seeds=seeds, step=step,
                       counters=counters)
        return out.copy_(y) if out is not None else y
    if out is None:
        out = torch.empty(logits.shape[0], dtype=torch.int32, device=logits.device)
    native().sample(out, logprobs, logits, temperature, top_k, top_p, seeds, step, counters)
    return out


# ----------------------------------------------------------------------------- fp8
FP8 = torch.float8_e4m3fn
FP8_MAX = 448.0


def quant_rowwise(x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                  norm_w: Optional[torch.Tensor] = None, eps: float = 0.0,
                  residual_out: Optional[torch.Tensor] = None):
    """Per-row dynamic fp8-e4m3 quantisation, optionally of ``RMSNorm(x + residual)``.

    With ``residual`` the sum ``x + residual`` is written back to ``residual_out`` (default: in
    place into ``residual``) exactly like :func:`rms_norm`.  Returns ``(q, scale[rows, 1])``.
    ``x`` may be :class:`SplitKPartials` (summed on load)."""
    if isinstance(x, SplitKPartials):
        q = torch.empty(x.shape, dtype=FP8, device=x.device)
        s = torch.empty(x.shape[0], 1, dtype=torch.float32, device=x.device)
        native().quant_rowwise(q, s, x.parts, residual, norm_w, float(eps), residual_out)
        return q, s
    K = x.shape[-1]
    rows = x.numel() // K
    if not _gpu(x):
        if residual is not None:
            s = (x.float() + residual.float()).to(x.dtype)
            (residual if residual_out is None else residual_out).copy_(s)
            x = s
        if norm_w is not None:
            x, _ = ref.rms_norm(x, norm_w, eps)
        return _quant_ref(x.reshape(rows, K), x.shape)
    q = torch.empty(x.shape, dtype=FP8, device=x.device)
    s = torch.empty(rows, 1, dtype=torch.float32, device=x.device)
    native().quant_rowwise(q, s, x, residual, norm_w, float(eps), residual_out)
    return q, s


def silu_mul_quant(x: torch.Tensor):
    """``silu(x[:, :I]) * x[:, I:]`` quantised per row to fp8: returns ``(q [T, I], scale [T, 1])``."""
    T, I = x.shape[0], x.shape[1] // 2
    if not _gpu(x):
        return _quant_ref(silu_mul(x), (T, I))
    q = torch.empty(T, I, dtype=FP8, device=x.device)
    s = torch.empty(T, 1, dtype=torch.float32, device=x.device)
    native().silu_mul_quant(q, s, x)
    return q, s


def _quant_ref(x2: torch.Tensor, shape):
    xf = x2.float()
    s = xf.abs().amax(-1).clamp_min(1e-12) / FP8_MAX
    s = torch.where(xf.abs().amax(-1) > 0, s, torch.ones_like(s))
    q = (xf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return q.reshape(shape), s.reshape(-1, 1)


def quantize_weight_fp8(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Offline per-output-channel fp8 quantisation of a [N, K] weight: returns (w_fp8, scale[1, N])."""
    wf = w.float()
    s = wf.abs().amax(-1).clamp_min(1e-12) / FP8_MAX
    q = (wf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return q, s.reshape(1, -1).contiguous()


def softmax_scale(head_dim: int) -> float:
    return 1.0 / math.sqrt(head_dim)


# ----------------------------------------------------------------------------- tile GEMM
def _swiglu_src(n2: int, device) -> torch.Tensor:
    """Row ``c`` of the interleaved weight is row ``src[c]`` of the fused [gate; up] weight."""
    if n2 % 256:
        raise ValueError("swiglu_interleave needs 2I % 256 == 0")
    c = torch.arange(n2, device=device)
    tile, cl = c // 256, c % 256
    wave, f, lc = cl // 64, (cl % 64) // 16, cl % 16
    out_col = tile * 128 + wave * 32 + (f // 2) * 16 + lc
    return torch.where(f % 2 == 0, out_col, n2 // 2 + out_col)


def swiglu_interleave(w_gate_up: torch.Tensor) -> torch.Tensor:
    """Reorder the rows of a fused ``[gate; up]`` weight ([2I, K]) for ``gemm_tile(swiglu=True)``.

    Tile-local column c (256 per tile) = wave ``c // 64``, n-fragment ``f = (c % 64) // 16``,
    lane column ``c % 16``; fragments 2p / 2p+1 carry gate / up of output column
    ``tile * 128 + wave * 32 + p * 16 + c % 16`` (csrc/kernels/gemm_tile.hip epilogue)."""
    return w_gate_up.index_select(0, _swiglu_src(w_gate_up.shape[0], w_gate_up.device)).contiguous()


def swiglu_deinterleave(w: torch.Tensor) -> torch.Tensor:
    """Inverse of ``swiglu_interleave``."""
    out = torch.empty_like(w)
    out[_swiglu_src(w.shape[0], w.device)] = w
    return out


def gemm_tile(x: torch.Tensor, w: torch.Tensor, splits: int = 1, swiglu: bool = False,
              out: Optional[torch.Tensor] = None, workspace: Optional[torch.Tensor] = None,
              defer_reduce: bool = False):
    """``x [M, K] @ w[N, K]^T`` with the 256x256 LDS-DMA MFMA kernel (N % 256 == 0, K % 64 == 0).
    ``swiglu=True``: ``w`` is a ``swiglu_interleave``d [gate; up] weight and the result is
    ``silu(x @ gate^T) * (x @ up^T)`` ([M, N/2]).  ``defer_reduce`` (split-K only): return the
    partials as :class:`SplitKPartials` for a consumer that reduces them (``rms_norm``): bf16
    under :func:`bf16_partials` (the default), else fp32."""
    M, N = x.shape[0], w.shape[0]
    if _gpu(x) and policy().gemm4:
        return _gemm4(x, w, splits, swiglu, out, defer_reduce)
    if defer_reduce and splits > 1 and _gpu(x) and not swiglu and policy().defer_splitk:
        if bf16_partials():
            parts = torch.empty(splits, M, N, dtype=torch.bfloat16, device=x.device)
            native().gemm_tile(parts, x, w, int(splits), 4)
            return SplitKPartials(parts)
        parts = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
        dummy = torch.empty(M, 0, dtype=torch.bfloat16, device=x.device)   # C is unused
        native().gemm_tile(dummy, x, w, int(splits), 1, parts.view(-1))
        return SplitKPartials(parts)
    if not _gpu(x):
        if swiglu:
            h = (x.float() @ swiglu_deinterleave(w).float().t()).to(x.dtype).float()
            r = (torch.nn.functional.silu(h[:, :N // 2]) * h[:, N // 2:]).to(x.dtype)
        else:
            r = (x.float() @ w.float().t()).to(x.dtype)
        return out.copy_(r) if out is not None else r
    if out is None:
        out = torch.empty(M, N // 2 if swiglu else N, dtype=x.dtype, device=x.device)
    if splits == 1 and tile_gemm_stream_k(M, N, x.device):
        splits = 0   # data-parallel waves + stream-K tail (csrc/kernels/gemm_tile.hip SkArgs)
        if workspace is None or workspace.numel() < native().gemm_tile_sk_workspace_floats():
            workspace = torch.empty(native().gemm_tile_sk_workspace_floats(), dtype=torch.float32,
                                    device=x.device)
    if splits > 1 and workspace is None:
        workspace = torch.empty(splits * M * N, dtype=torch.float32, device=x.device)
    native().gemm_tile(out, x, w, int(splits), 2 if swiglu else 0, workspace)
    return out


def _gemm4(x: torch.Tensor, w: torch.Tensor, splits: int, swiglu: bool,
           out: Optional[torch.Tensor], defer_reduce: bool,
           xs: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
           x_mx: Optional[torch.Tensor] = None):
    """:func:`gemm_tile`'s contract on gemm4: same epilogues (bf16 store, fused SwiGLU, split-K
    partials handed to the consumer or reduced here), bit-identical results for bf16.  fp8 e4m3
    operands (``xs`` [M] / ``ws`` [N] scales, or ``x_mx``: MX activation scales) run the
    block-scaled 16x16x128 MFMA with gemm_tile's fragment pairing (:func:`gemm_tile_fp8` /
    :func:`gemm_tile_fp8_mx`'s contracts, bit-identical results)."""
    M, N = x.shape[0], w.shape[0]
    splits = max(1, int(splits))
    fp8 = xs is not None or x_mx is not None
    # bf16 decode-size schedule from the policy; fp8 and larger M: the kernel's default
    var = policy().gemm4_decode_sched if (not fp8 and M <= 512) else -1
    if splits > 1 and defer_reduce and not swiglu and policy().defer_splitk:
        bf = bf16_partials()
        parts = torch.empty(splits, M, N, dtype=torch.bfloat16 if bf else torch.float32,
                            device=x.device)
        native().gemm4(parts, x, w, splits, 4 if bf else 1, 0, xs, ws, var, a_mx=x_mx)
        return SplitKPartials(parts)
    if out is None:
        out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=x.device)
    if splits == 1:
        native().gemm4(out, x, w, 1, 2 if swiglu else 0, 0, xs, ws, var, a_mx=x_mx)
        return out
    if swiglu:
        raise ValueError("gemm4: fused SwiGLU takes whole-K tiles (splits = 1)")
    parts = torch.empty(splits, M, N, dtype=torch.float32, device=x.device)
    native().gemm4(parts, x, w, splits, 1, 0, xs, ws, var, a_mx=x_mx)
    native().splitk_reduce(out, parts)
    return out


def gemm4_mx_ok(K: int, splits: int) -> bool:
    """Whether gemm4 takes MX activations over K with this split count (its LDS scale slab holds
    64 k-tiles; csrc/kernels/gemm4.hip kG4MxKt)."""
    return mx_tileable(K, splits)


_CU_COUNT = {}


def device_cus(device) -> int:
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    if idx not in _CU_COUNT:
        _CU_COUNT[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _CU_COUNT[idx]


def tile_gemm_stream_k(M: int, N: int, device) -> bool:
    """Whether a whole-K (splits = 1) bf16 ``gemm_tile`` should run its last, partial wave of tiles
    as a stream-K tail: more tiles than CUs and a remainder of at least half the CUs (Llama-3-70B
    gate|up at M = 512: 448 tiles = 256 whole + 192 shared k-wise by 256 workgroups, instead of a
    second wave with 64 idle CUs).  Opt-in: in isolation (back-to-back
    launches) it is 6-12 % faster (profiles/gemm_sk_bench.json), but inside the decode step the
    gate|up GEMM runs at the same ~386 us either way (rocprofv3, profiles/stream_k_decode_ab.txt),
    and bench.py is unchanged within noise.  In the decode step the whole-tile kernel already runs
    25 % faster than in the isolated loop (386 vs 480 us), so the idle-CU tail is not what bounds
    it there; a GRBM_GUI_ACTIVE pass shows the stream-K variant at a ~1 % lower clock.
    (``KernelPolicy.stream_k_tail``.)"""
    if not policy().stream_k_tail:
        return False
    cus = device_cus(device)
    tiles = ((M + 255) // 256) * (N // 256)
    return tiles > cus and tiles % cus >= cus // 2


TILE_GEMM_MIN_M = 128    # below: too few rows to fill a 256-row tile (hipBLASLt / skinny path)
TILE_GEMM_WIDE_N = 65536  # vocabulary-wide LM heads: hipBLASLt's wide-N solutions
TILE_MAX_SPLITS = 8      # norm / quant / rope consumers sum up to 8 partials (SPLITS_SWITCH)
_CUS = 256


def library_gemms() -> bool:
    """Whether products the tile kernel does not take well (M < 128, the vocabulary-wide LM head)
    may go to hipBLASLt (default).  Off, every tileable product stays on the tile
    kernel: hipBLASLt picks stream-K solutions for some of these shapes - persistent kernels
    sized to the CU count whose workgroups wait for each other's partial tiles - and two of
    them in flight at once (the head stream next to the compute stream, or ranks sharing one
    GPU) can each hold CUs the other needs.  Measured: every hipBLASLt kernel torch picks for the
    70B decode shapes at M = 1..4096 is stream-K (``SK3``, profiles/streams/blaslt_streamk.txt);
    8 pipeline ranks sharing one GPU at 32 rows per micro-batch stalled in 4 of 4 runs with them
    and completed with this off.  ``KernelPolicy.library_gemms``; automatic (None): off when
    ranks share a GPU (``DLI_SHARE_GPU=1``)."""
    lib = policy().library_gemms
    if lib is None:
        return os.environ.get("DLI_SHARE_GPU", "0") != "1"
    return bool(lib)


def tile_gemm_splits(M: int, N: int, K: int, elem_bytes: int = 2) -> int:
    """Split-K factor for ``gemm_tile`` on an [M, K] x [N, K]^T product, or 0 = not eligible.

    Picks the split that best fills the 256 CUs with whole waves of 256x256 tiles (ties -> fewer
    splits), e.g. 70B at M = 512: QKV 80 tiles x 3, O / down 64 x 4, gate|up 448 x 1 (measured
    best per shape, profiles/gemm_tile_bench.json).  ``KernelPolicy.tile_gemms=False`` disables
    the tile kernels (hipBLASLt everywhere)."""
    if not policy().tile_gemms:
        return 0
    lib = library_gemms()
    if N % 256 or (K * elem_bytes) % 128 or M < 1:
        return 0
    max_m = policy().tile_gemm_max_m
    k_tiles = K * elem_bytes // 128
    tiles = ((M + 255) // 256) * (N // 256)
    if lib:
        if M < TILE_GEMM_MIN_M:
            return 0
        if N >= TILE_GEMM_WIDE_N:
            return 0  # the 128256-wide LM head: hipBLASLt's wide-N solutions (690 vs 824 us)
        if max_m > 0 and (M > max_m or tiles > 2 * _CUS):
            return 0  # the round-5 rule (large-M products to hipBLASLt), for A/B runs
    best, best_util = 1, 0.0
    for s in range(1, TILE_MAX_SPLITS + 1):
        if s > k_tiles or (s > 1 and tiles * s > 2 * _CUS):
            break
        if (s - 1) * (-(-k_tiles // s)) >= k_tiles:
            continue   # the kernels give every split >= 1 k-tile (16 k-tiles can't go 7 ways)
        work = tiles * s
        util = work / (_CUS * ((work + _CUS - 1) // _CUS))
        if util > best_util + 1e-9:
            best, best_util = s, util
    return best


# ----------------------------------------------------------------------------- LLM.int8
def quantize_weight_int8(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-wise (per output channel) absmax int8 weights, as bitsandbytes' ``Linear8bitLt``
    stores them (reference utils/model.py:93-113): returns (w_int8 [N, K], scale [N])."""
    wf = w.float()
    s = wf.abs().amax(-1).clamp_min(1e-12) / 127.0
    q = torch.round(wf / s[:, None]).clamp(-127, 127).to(torch.int8)
    return q, s.contiguous()


def quant_rowwise_int8(x: torch.Tensor, outlier: Optional[torch.Tensor] = None
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-row absmax int8 quantisation of ``x [rows, K]``; columns with ``outlier[c] != 0`` are
    zeroed (LLM.int8 computes them in bf16).  Returns (q int8, scale [rows])."""
    rows, K = x.shape
    if not _gpu(x):
        xf = x.float()
        if outlier is not None:
            xf = xf * (outlier == 0).to(xf.dtype)
        s = xf.abs().amax(-1).clamp_min(0)
        s = torch.where(s > 0, s / 127.0, torch.ones_like(s))
        return torch.round(xf / s[:, None]).clamp(-127, 127).to(torch.int8), s
    q = torch.empty(rows, K, dtype=torch.int8, device=x.device)
    s = torch.empty(rows, dtype=torch.float32, device=x.device)
    native().quant_rowwise_int8(q, s, x.contiguous(), outlier)
    return q, s


LLM_INT8_MAX_OUTLIERS = 64   # static outlier-column capacity (graph-capturable shapes)
LLM_INT8_SELECT_MAX_K = 32768   # int8_outlier.hip select kernel: 1024 threads x 32 columns


def llm_int8_linear(x: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor, threshold: float = 6.0,
                    max_outliers: int = LLM_INT8_MAX_OUTLIERS,
                    wq_t: Optional[torch.Tensor] = None, swiglu: bool = False,
                    defer_reduce: bool = False):
    """LLM.int8 matmul ``x [M, K] @ W^T`` with ``W ~= wq * ws[:, None]`` (int8, per-channel).

    Mixed-precision decomposition as in bitsandbytes ``Linear8bitLt(threshold=...)``: feature
    columns whose magnitude exceeds ``threshold`` anywhere in the batch are multiplied in bf16
    (with the dequantised weight columns); every other column goes through per-row int8
    quantisation and the int8 MFMA tile GEMM (``gemm_tile.hip``, v_mfma_i32_16x16x64_i8), whose
    epilogue adds the bf16 outlier product (one bf16 MFMA k-step per 32 outlier columns).  To keep
    shapes static (hipGraph decode) the outlier set is the ``max_outliers`` largest columns that
    pass the threshold; ``threshold <= 0`` disables the decomposition.  ``wq_t``: optional
    transposed copy ``[K, N]`` of ``wq`` (GPU) that makes the outlier weight-column gather
    coalesced.  ``swiglu``: ``wq`` / ``ws`` rows in ``swiglu_interleave`` order, returns
    ``silu(gate) * up`` ([M, N/2]).  ``defer_reduce``: a split-K product returns its partials
    (:class:`SplitKPartials`, the outlier product inside split 0's) for a consumer to reduce."""
    M, K = x.shape
    N = wq.shape[0]
    outl = None   # (x_out [M, J], w_out [N, J]) bf16: the outlier product
    flags = None
    ol_cnt = None   # device int32 [1]: outlier columns kept (dynamic gathers, fused epilogue)
    tile_ok = _gpu(x) and N % 256 == 0 and K % 128 == 0 and M > 0
    if threshold > 0 and M > 0:
        J = min(max_outliers, K)
        # int8_outlier.hip: colmax / radix select / two gathers (select: K <= 1024 x 32 columns;
        # the coalesced gather from the transposed copy needs N % 4 == 0)
        if _gpu(x) and K % 8 == 0 and K <= LLM_INT8_SELECT_MAX_K:
            if wq_t is not None and N % 4 != 0:
                wq_t = None
            # fused epilogue: it reads only the ceil(cnt / 32) live 32-column chunks, so the
            # gathers skip the rest (no outliers -> no gather traffic, no outlier MFMA steps)
            dynamic = tile_ok
            flags, xo, wo, cnt = native().llm_int8_outliers(
                x.contiguous(), wq, ws.float().contiguous(), float(threshold), int(J), wq_t,
                dynamic)
            ol_cnt = cnt if dynamic else None
        else:
            # same rule as the kernel: |x| >= threshold; above J such columns, strictly above
            # the (J+1)-th largest column maximum (ties at that cut dropped)
            colmax = x.abs().amax(0).float()
            n_pass = int((colmax >= threshold).sum())
            if n_pass > J:
                cut = colmax.topk(J + 1).values[-1]
                on = colmax > cut
            else:
                on = colmax >= threshold
            cols = on.nonzero().flatten()
            idx = torch.zeros(J, dtype=torch.long, device=x.device)
            idx[:cols.numel()] = cols
            sel = torch.zeros(J, dtype=torch.bool, device=x.device)
            sel[:cols.numel()] = True
            flags = on.to(torch.uint8)
            xo = x.index_select(1, idx) * sel.to(x.dtype)
            wo = (wq.index_select(1, idx).float() * ws[:, None] * sel).to(x.dtype)
        outl = (xo, wo)
    xq, xs = quant_rowwise_int8(x, flags)
    if tile_ok:
        sp = tile_gemm_splits(max(M, TILE_GEMM_MIN_M), N, K, elem_bytes=1) or 1
        if swiglu:
            sp = 1
        xo = wo = None
        if outl is not None:
            xo, wo = outl
            J = xo.shape[1]
            if J % 32:   # the epilogue's bf16 MFMA k-step: zero-pad to a multiple of 32
                pad = 32 - J % 32
                xo = torch.nn.functional.pad(xo, (0, pad))
                wo = torch.nn.functional.pad(wo, (0, pad))
            xo, wo = xo.contiguous(), wo.contiguous()
        if defer_reduce and sp > 1 and not swiglu and policy().defer_splitk:
            if bf16_partials():   # bf16 partials (epilogue 4), as on the fp8 path
                parts = torch.empty(sp, M, N, dtype=torch.bfloat16, device=x.device)
                native().gemm_tile(parts, xq, wq, int(sp), 4, None, xs, ws, xo, wo,
                                   ol_cnt=ol_cnt)
                return SplitKPartials(parts)
            parts = torch.empty(sp, M, N, dtype=torch.float32, device=x.device)
            dummy = torch.empty(M, 0, dtype=torch.bfloat16, device=x.device)   # C is unused
            native().gemm_tile(dummy, xq, wq, int(sp), 1, parts.view(-1), xs, ws, xo, wo,
                               ol_cnt=ol_cnt)
            return SplitKPartials(parts)
        y = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=x.device)
        ws_ = torch.empty(sp * M * N, dtype=torch.float32, device=x.device) if sp > 1 else None
        native().gemm_tile(y, xq, wq, int(sp), 2 if swiglu else 0, ws_, xs, ws, xo, wo,
                           ol_cnt=ol_cnt)
        return y
    # CPU / untileable shapes: dequantised reference
    y = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).t()
    if outl is not None:
        y = y + outl[0].float() @ outl[1].float().t()
    y = y.to(torch.bfloat16)
    return swiglu_interleaved(y) if swiglu else y


def gemm_tile_fp8(xq: torch.Tensor, xs: torch.Tensor, wq: torch.Tensor, ws: torch.Tensor,
                  splits: int = 1, swiglu: bool = False, out: Optional[torch.Tensor] = None,
                  workspace: Optional[torch.Tensor] = None, defer_reduce: bool = False,
                  mx_out: bool = False, gemm4: bool = False):
    """fp8 e4m3 tile GEMM: ``(xq [M, K] @ wq[N, K]^T) * xs[M] * ws[N]`` -> bf16, on the
    block-scaled K=128 MFMA (2x the bf16 MFMA rate; unit block scales, per-row / per-channel
    scales applied in the epilogue).  ``swiglu``: ``wq`` / ``ws`` rows in swiglu_interleave order.
    ``defer_reduce`` (split-K): return :class:`SplitKPartials` (scaled partials, bf16 under
    :func:`bf16_partials`).
    ``mx_out`` (with ``swiglu``): return the SwiGLU output as :class:`MxFp8`, quantised in the
    epilogue (needs N % 256 == 0).  ``gemm4``: run on the one-wave-per-SIMD kernel (the caller
    decides per shape: ``KernelPolicy.fp8_on_gemm4``)."""
    M, N = xq.shape[0], wq.shape[0]
    if mx_out:
        if not swiglu:
            raise ValueError("gemm_tile_fp8: mx_out is an output of the SwiGLU epilogue")
        if not _gpu(xq):
            return mx_quantize(gemm_tile_fp8(xq, xs, wq, ws, swiglu=True))
        I = N // 2
        q = torch.empty(M, I, dtype=torch.float8_e4m3fn, device=xq.device)
        sc = torch.empty(I // 128 * ((M + 63) // 64) * 64, dtype=torch.uint8, device=xq.device)
        if gemm4:
            native().gemm4(q, xq, wq, 1, 3, 0, xs.reshape(-1).contiguous(),
                           ws.reshape(-1).contiguous(), out_mx=sc)
        else:
            native().gemm_tile(q, xq, wq, 1, 3, None, xs.reshape(-1).contiguous(),
                               ws.reshape(-1).contiguous(), out_mx=sc)
        return MxFp8(q, sc)
    if _gpu(xq) and gemm4 and xq.shape[1] % 128 == 0:
        return _gemm4(xq, wq, splits, swiglu, out, defer_reduce,
                      xs.reshape(-1).contiguous(), ws.reshape(-1).contiguous())
    if defer_reduce and splits > 1 and _gpu(xq) and not swiglu and policy().defer_splitk:
        if bf16_partials():
            parts = torch.empty(splits, M, N, dtype=torch.bfloat16, device=xq.device)
            native().gemm_tile(parts, xq, wq, int(splits), 4, None,
                               xs.reshape(-1).contiguous(), ws.reshape(-1).contiguous())
            return SplitKPartials(parts)
        parts = torch.empty(splits, M, N, dtype=torch.float32, device=xq.device)
        dummy = torch.empty(M, 0, dtype=torch.bfloat16, device=xq.device)   # C is unused
        native().gemm_tile(dummy, xq, wq, int(splits), 1, parts.view(-1),
                           xs.reshape(-1).contiguous(), ws.reshape(-1).contiguous())
        return SplitKPartials(parts)
    if not _gpu(xq):
        h = (xq.float() * xs.reshape(-1, 1).float()) @ (wq.float() * ws.reshape(-1, 1).float()).t()
        if swiglu:
            return swiglu_interleaved(h.to(torch.bfloat16), out)
        r = h.to(torch.bfloat16)
        return out.copy_(r) if out is not None else r
    if out is None:
        out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=xq.device)
    if splits > 1 and workspace is None:
        workspace = torch.empty(splits * M * N, dtype=torch.float32, device=xq.device)
    native().gemm_tile(out, xq, wq, int(splits), 2 if swiglu else 0, workspace,
                       xs.reshape(-1).contiguous(), ws.reshape(-1).contiguous())
    return out


class MxFp8:
    """fp8 e4m3 activations with one power-of-two (e8m0) scale per (row, 128-column block), as
    the fp8 gate|up tile GEMM's SwiGLU epilogue writes them (gemm_tile.hip kSwiGLUMx) and the down
    projection consumes them on the block-scaled MFMA's per-lane scale operand (kFp8Mx).
    ``sc`` is uint8 in gemm_tile.hip's ``mx_off`` layout: byte of (row r, block kt) at
    ``(kt * nb + r // 64) * 64 + (r % 16) * 4 + (r % 64) // 16``, ``nb = ceil(M / 64)``."""

    __slots__ = ("q", "sc")

    def __init__(self, q: torch.Tensor, sc: torch.Tensor):
        self.q, self.sc = q, sc

    @property
    def shape(self):
        return self.q.shape

    def exponents(self) -> torch.Tensor:
        """int32 [M, K / 128]: the scale exponents (value = q * 2 ** e)."""
        M, K = self.q.shape
        nb = (M + 63) // 64
        r = torch.arange(M, device=self.sc.device)
        idx = (r // 64) * 64 + (r % 16) * 4 + (r % 64) // 16
        return self.sc.view(K // 128, nb * 64)[:, idx].t().to(torch.int32) - 127

    def dequantize(self) -> torch.Tensor:
        e = self.exponents().float()
        return self.q.float() * torch.exp2(e).repeat_interleave(128, dim=1)


def mx_quantize(h: torch.Tensor) -> MxFp8:
    """Reference MX quantiser (same rule as the kSwiGLUMx epilogue): per (row, 128-column block)
    the smallest 2^k with amax / 2^k <= 448, q = e4m3(h / 2^k)."""
    M, K = h.shape
    nb = (M + 63) // 64
    hf = h.float().view(M, K // 128, 128)
    am = hf.abs().amax(-1)
    ratio = am / 448.0
    m, e = torch.frexp(ratio)                       # ratio = m * 2^e, m in [0.5, 1)
    k = torch.where(m == 0.5, e - 1, e)             # exact powers of two: 2^(e-1) == ratio
    k = torch.where(am > 0, k, torch.zeros_like(k)).clamp(-126, 126)
    q = (hf * torch.exp2(-k.float())[..., None]).clamp(-448, 448).view(M, K).to(torch.float8_e4m3fn)
    sc = torch.full((K // 128, nb * 64), 127, dtype=torch.uint8, device=h.device)
    r = torch.arange(M, device=h.device)
    idx = (r // 64) * 64 + (r % 16) * 4 + (r % 64) // 16
    sc[:, idx] = (k + 127).to(torch.uint8).t()
    return MxFp8(q, sc.view(-1))


MX_MAX_KTILES = 64   # k-tiles of scales one kFp8Mx workgroup keeps in LDS (gemm_tile.hip kMxMaxKt)


def mx_tileable(K: int, splits: int) -> bool:
    """Whether a kFp8Mx tile GEMM over K with this split count fits its LDS scale slot."""
    kt = K // 128
    return splits >= 1 and K % 128 == 0 and -(-kt // splits) <= MX_MAX_KTILES


def gemm_tile_fp8_mx(a: MxFp8, wq: torch.Tensor, ws: torch.Tensor, splits: int = 1,
                     defer_reduce: bool = False, gemm4: bool = False):
    """fp8 tile GEMM on MX activations: ``(q * 2^e) @ (wq * ws)^T`` with the e8m0 scales applied
    by the MFMA itself (kFp8Mx); bf16 out, or :class:`SplitKPartials` when deferring."""
    xq = a.q
    M, N = xq.shape[0], wq.shape[0]
    if not _gpu(xq):
        y = a.dequantize() @ (wq.float() * ws.reshape(-1, 1).float()).t()
        return y.to(torch.bfloat16)
    if not mx_tileable(xq.shape[1], splits):
        raise ValueError(f"gemm_tile_fp8_mx: K={xq.shape[1]} with {splits} splits exceeds the "
                         f"{MX_MAX_KTILES}-k-tile scale slot")
    ws = ws.reshape(-1).contiguous()
    if gemm4:
        return _gemm4(xq, wq, splits, False, None, defer_reduce, None, ws, x_mx=a.sc)
    if defer_reduce and splits > 1 and policy().defer_splitk:
        if bf16_partials():
            parts = torch.empty(splits, M, N, dtype=torch.bfloat16, device=xq.device)
            native().gemm_tile(parts, xq, wq, int(splits), 4, None, None, ws, a_mx=a.sc)
            return SplitKPartials(parts)
        parts = torch.empty(splits, M, N, dtype=torch.float32, device=xq.device)
        dummy = torch.empty(M, 0, dtype=torch.bfloat16, device=xq.device)   # C is unused
        native().gemm_tile(dummy, xq, wq, int(splits), 1, parts.view(-1), None, ws, a_mx=a.sc)
        return SplitKPartials(parts)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=xq.device)
    workspace = (torch.empty(splits * M * N, dtype=torch.float32, device=xq.device)
                 if splits > 1 else None)
    native().gemm_tile(out, xq, wq, int(splits), 0, workspace, None, ws, a_mx=a.sc)
    return out


def tile_gemm_splits_fp8(M: int, N: int, K: int) -> int:
    """``tile_gemm_splits`` for the fp8 kernels (every fp8 decode projection runs on the
    hand-written block-scaled MFMA tile kernels: QKV / O / down split-K with their partials
    reduced by the consumer kernels, gate|up with the fused SwiGLU epilogue;
    profiles/fp8_tile_all_vs_long.json)."""
    return tile_gemm_splits(M, N, K, elem_bytes=1)


def swiglu_interleaved(gu: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """silu(gate) * up from a GEMM output whose columns follow ``swiglu_interleave``'s order
    (shapes the fused tile epilogue does not take: prefill chunks, 1-2 row batches)."""
    M, n2 = gu.shape
    if not _gpu(gu):
        v = gu.float().reshape(M, n2 // 256, 4, 2, 2, 16)
        y = (torch.nn.functional.silu(v[..., 0, :]) * v[..., 1, :]).reshape(M, n2 // 2).to(gu.dtype)
        return out.copy_(y) if out is not None else y
    if out is None:
        out = torch.empty(M, n2 // 2, dtype=gu.dtype, device=gu.device)
    native().silu_mul(out, gu, True)
    return out


# ----------------------------------------------------------------------------- skinny GEMM
SKINNY_MAX_M = 4        # kernel limit
SKINNY_DISPATCH_M = 2   # Linear uses it up to here: measured faster than hipBLASLt at M <= 2 on
                        # every Llama-3-70B decode shape (5.3-6.9 vs 4.3-6.0 TB/s), slower at M = 4


class RowNorm:
    """The input RMSNorm a skinny GEMM applies to its rows itself (1-2 decode rows, GPU): the
    GEMV multiplies ``rmsnorm(x + res_in) * w`` (bit-identical to :func:`rms_norm`'s output) and
    writes ``res_out = x + res_in`` once -- one launch instead of two.  ``res_out`` must be a
    different buffer than ``res_in``; ``res_in=None``: no residual add (x itself is normalised)."""

    __slots__ = ("w", "eps", "res_in", "res_out")

    def __init__(self, w: torch.Tensor, eps: float, res_in: Optional[torch.Tensor] = None,
                 res_out: Optional[torch.Tensor] = None):
        if res_out is not None and (res_in is None or res_out.data_ptr() == res_in.data_ptr()):
            raise ValueError("RowNorm: res_out needs res_in and must not alias it")
        self.w, self.eps, self.res_in, self.res_out = w, float(eps), res_in, res_out

    def apply(self, x: torch.Tensor) -> torch.Tensor:
        """The normalised rows (CPU reference path; also writes res_out)."""
        y, _ = rms_norm(x, self.w, self.eps, residual=self.res_in,
                        residual_out=self.res_out if self.res_in is not None else None)
        return y

    def kwargs(self) -> dict:
        return dict(norm_w=self.w, res_in=self.res_in, res_out=self.res_out, eps=self.eps)


def _swiglu_ref(y: torch.Tensor) -> torch.Tensor:
    """CPU reference of the fused-SwiGLU GEMV epilogue: bf16 gate / up, interleaved columns."""
    return swiglu_interleaved(y.to(torch.bfloat16))


def skinny_gemm_int8(x: torch.Tensor, wq: torch.Tensor, w_scale: torch.Tensor,
                     bias: Optional[torch.Tensor] = None, swiglu: bool = False,
                     norm: Optional[RowNorm] = None) -> torch.Tensor:
    """``y = (x . wq^T) * w_scale`` for 1-2 bf16 decode rows with LLM.int8 weights (int8 [N, K],
    per-row scale): the weight stream at 1 byte per weight, activations kept in bf16 (no
    activation quantisation, so no outlier split is needed: every column is exact bf16 x int8).
    ``swiglu``: ``wq`` is a swiglu_interleave'd gate|up weight; returns silu(gate) * up."""
    M, N = x.shape[0], wq.shape[0]
    if not _gpu(x):
        if norm is not None:
            x = norm.apply(x)
        y = x.float() @ (wq.float() * w_scale.reshape(-1, 1)).t()
        if bias is not None:
            y = y + bias.float()
        return _swiglu_ref(y) if swiglu else y.to(torch.bfloat16)
    out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=x.device)
    native().skinny_gemm_int8(out, x.contiguous(), wq, w_scale.reshape(-1).contiguous(), bias,
                              swiglu, **(norm.kwargs() if norm is not None else {}))
    return out


def skinny_gemm_fp8(x: torch.Tensor, w8: torch.Tensor, w_scale: torch.Tensor,
                    x_scale: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
                    swiglu: bool = False, norm: Optional[RowNorm] = None) -> torch.Tensor:
    """``y = (x . w8^T) * w_scale (* x_scale)`` for 1-2 decode rows: fp8 e4m3 weights [N, K]
    with one scale per output row, activations bf16 or fp8 with one scale per row (the fused
    RMSNorm quantiser's output), weight-streaming GEMV (csrc/kernels/gemv.hip)."""
    M, N = x.shape[0], w8.shape[0]
    if norm is not None and x_scale is not None:
        raise ValueError("skinny_gemm_fp8: the fused norm takes bf16 rows")
    if not _gpu(x):
        if norm is not None:
            x = norm.apply(x)
        xf = x.float() * x_scale.reshape(-1, 1) if x_scale is not None else x.float()
        y = (xf @ (w8.float() * w_scale.reshape(-1, 1)).t())
        if bias is not None:
            y = y + bias.float()
        return _swiglu_ref(y) if swiglu else y.to(torch.bfloat16)
    out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=x.device)
    native().skinny_gemm_fp8(out, x.contiguous(),
                             None if x_scale is None else x_scale.reshape(-1).contiguous(), w8,
                             w_scale.reshape(-1).contiguous(), bias, swiglu,
                             **(norm.kwargs() if norm is not None else {}))
    return out


def skinny_gemm_qkv_rope(x: torch.Tensor, w: torch.Tensor, w_scale: Optional[torch.Tensor],
                         bias: Optional[torch.Tensor], positions: Optional[torch.Tensor],
                         slot_mapping: Optional[torch.Tensor], cos_sin: Optional[torch.Tensor],
                         nh: int, nkv: int, head_dim: int, k_cache: torch.Tensor,
                         v_cache: torch.Tensor, k_scale: float = 1.0, v_scale: float = 1.0,
                         norm: Optional[RowNorm] = None) -> torch.Tensor:
    """1-2 decode rows: the fused QKV projection (bf16, fp8 or int8 weights ``w`` [(nh + 2 nkv) D,
    K], per-row ``w_scale`` for 8-bit) with :func:`rope_cache`'s work in the GEMV epilogue --
    returns q [M, nh, D] rotated, k (rotated) and v written to the paged caches -- and the
    input RMSNorm in its prologue when ``norm`` is given.  One launch instead of three."""
    M = x.shape[0]
    if not _gpu(x):
        if norm is not None:
            x = norm.apply(x)
        wf = w.float() if w_scale is None else w.float() * w_scale.reshape(-1, 1)
        qkv = x.float() @ wf.t()
        if bias is not None:
            qkv = qkv + bias.float()
        q, _ = rope_cache(qkv.to(torch.bfloat16), positions, slot_mapping, cos_sin, nh, nkv,
                          head_dim, k_cache, v_cache, k_scale=k_scale, v_scale=v_scale)
        return q
    q = torch.empty(M, nh, head_dim, dtype=torch.bfloat16, device=x.device)
    native().skinny_gemm_qkv_rope(q, x.contiguous(), w,
                                  None if w_scale is None else w_scale.reshape(-1).contiguous(),
                                  bias, positions, slot_mapping, cos_sin, k_cache, v_cache,
                                  int(nh), int(nkv), float(k_scale), float(v_scale),
                                  **(norm.kwargs() if norm is not None else {}))
    return q


def skinny_gemm(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, swiglu: bool = False,
                norm: Optional[RowNorm] = None) -> torch.Tensor:
    """``x [M, K] @ w[N, K]^T (+ bias)`` for M <= 4 with the weight-streaming HIP kernel;
    ``swiglu`` (M <= 2): ``w`` is a swiglu_interleave'd gate|up weight, returns silu(gate) * up."""
    if not _gpu(x):
        if norm is not None:
            x = norm.apply(x)
        y = x.float() @ w.float().t() + (bias.float() if bias is not None else 0.0)
        y = _swiglu_ref(y) if swiglu else y.to(x.dtype)
        return out.copy_(y) if out is not None else y
    if out is None:
        out = torch.empty(x.shape[0], w.shape[0] // 2 if swiglu else w.shape[0], dtype=x.dtype,
                          device=x.device)
    native().skinny_gemm(out, x, w, bias, swiglu, **(norm.kwargs() if norm is not None else {}))
    return out

