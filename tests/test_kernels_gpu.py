"""Numerics of every CDNA4 HIP kernel against the plain-PyTorch fp32 reference (ops/reference.py).

Run on an MI355X: ``python -m pytest tests -m gpu``.
"""
import math

import pytest
import torch

from distributed_llm_inference import ops
from distributed_llm_inference.ops import reference as ref

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _close(a, b, atol, rtol=0.0, msg=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs()
    tol = atol + rtol * b.abs()
    bad = (err > tol)
    assert not bad.any(), f"{msg} max err {err.max().item():.4g} at {bad.nonzero()[:5].tolist()}"


@pytest.mark.parametrize("rows,hidden", [(1, 128), (5, 4096), (7, 8192), (3, 1000 * 8)])
@pytest.mark.parametrize("with_res", [False, True])
def test_rms_norm(gpu, rows, hidden, with_res):
    torch.manual_seed(0)
    x = torch.randn(rows, hidden, device=gpu, dtype=BF)
    w = (1 + 0.1 * torch.randn(hidden, device=gpu)).to(BF)
    r = torch.randn(rows, hidden, device=gpu, dtype=BF) if with_res else None
    r_ref = r.clone().cpu() if with_res else None
    y, r2 = ops.rms_norm(x, w, 1e-5, residual=r)
    y_ref, r_ref2 = ref.rms_norm(x.cpu(), w.cpu(), 1e-5, residual=r_ref)
    _close(y, y_ref, 2e-2, 1e-2, "rms_norm")
    if with_res:
        _close(r2, r_ref2, 1e-2, 1e-2, "residual")


def test_layer_norm(gpu):
    x = torch.randn(9, 768, device=gpu, dtype=BF)
    w = torch.randn(768, device=gpu, dtype=BF)
    b = torch.randn(768, device=gpu, dtype=BF)
    y, _ = ops.layer_norm(x, w, b, 1e-5)
    y_ref, _ = ref.layer_norm(x.cpu(), w.cpu(), b.cpu(), 1e-5)
    _close(y, y_ref, 5e-2, 2e-2, "layer_norm")


def test_silu_mul_gelu_add(gpu):
    x = torch.randn(13, 2 * 1024, device=gpu, dtype=BF)
    _close(ops.silu_mul(x), ref.silu_mul(x.cpu()), 1e-2, 1e-2, "silu_mul")
    b = torch.randn(2048, device=gpu, dtype=BF)
    _close(ops.gelu_bias(x, b), ref.gelu_bias(x.cpu(), b.cpu()), 2e-2, 1e-2, "gelu")
    y = torch.randn_like(x)
    _close(ops.add(x, y), (x.float() + y.float()), 1e-2, 1e-2, "add")


def _make_cache(nblocks, nkv, bs, D, dev):
    k = torch.randn(nblocks, nkv, bs, D, device=dev, dtype=BF)
    v = torch.randn(nblocks, nkv, bs // 8, D, 8, device=dev, dtype=BF)
    return k, v


@pytest.mark.parametrize("nh,nkv,D", [(32, 8, 128), (8, 8, 64), (4, 2, 32)])
@pytest.mark.parametrize("window", [0, 64])
def test_rope_cache(gpu, nh, nkv, D, window):
    torch.manual_seed(1)
    T, bs, nblocks = 37, 64, 16
    qkv = torch.randn(T, (nh + 2 * nkv) * D, device=gpu, dtype=BF)
    pos = torch.randint(0, 300, (T,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(nblocks * bs, device=gpu)[:T].to(torch.int64)
    slots[3] = -1  # a token that is not written
    cs = ref.build_cos_sin(D, 512, 500000.0, device=gpu)
    k1, v1 = _make_cache(nblocks, nkv, bs, D, gpu)
    k2, v2 = k1.clone().cpu(), v1.clone().cpu()
    q, qs = ops.rope_cache(qkv, pos, slots, cs, nh, nkv, D, k1, v1, window=window,
                           want_sink=window > 0)
    q_r, qs_r = ref.rope_cache(qkv.cpu(), pos.cpu(), slots.cpu(), cs.cpu(), nh, nkv, D, k2, v2,
                               window, window > 0)
    _close(q, q_r, 2e-2, 1e-2, "q")
    if window:
        _close(qs, qs_r, 2e-2, 1e-2, "q_sink")
    _close(k1, k2, 2e-2, 1e-2, "k_cache")
    _close(v1, v2, 0.0, 0.0, "v_cache")


@pytest.mark.parametrize("nh,nkv,D,S", [(64, 8, 128, 3), (4, 2, 32, 2)])
@pytest.mark.parametrize("fp8", [False, True])
def test_rope_cache_from_splitk_partials_bit_identical(gpu, nh, nkv, D, S, fp8):
    """qkv given as un-reduced fp32 split-K partials == reduce pass, then rope_cache."""
    torch.manual_seed(4)
    T, bs, nblocks = 29, 64, 8
    parts = torch.randn(S, T, (nh + 2 * nkv) * D, device=gpu)
    pos = torch.randint(0, 300, (T,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(nblocks * bs, device=gpu)[:T].to(torch.int64)
    slots[5] = -1
    cs = ref.build_cos_sin(D, 512, 500000.0, device=gpu)
    k1, v1 = _make_cache(nblocks, nkv, bs, D, gpu)
    if fp8:
        k1, v1 = k1.to(torch.float8_e4m3fn), v1.to(torch.float8_e4m3fn)
    k2, v2 = k1.clone(), v1.clone()
    qkv = ops.SplitKPartials(parts).materialize()
    q1, qs1 = ops.rope_cache(qkv, pos, slots, cs, nh, nkv, D, k1, v1, window=100, want_sink=True,
                             k_scale=0.5, v_scale=0.25)
    q2, qs2 = ops.rope_cache(ops.SplitKPartials(parts), pos, slots, cs, nh, nkv, D, k2, v2,
                             window=100, want_sink=True, k_scale=0.5, v_scale=0.25)
    assert torch.equal(q1, q2) and torch.equal(qs1, qs2)
    assert torch.equal(k1.view(torch.uint8), k2.view(torch.uint8))
    assert torch.equal(v1.view(torch.uint8), v2.view(torch.uint8))


@pytest.mark.parametrize("nh,nkv,D,S", [(64, 8, 128, 3), (8, 8, 64, 0), (4, 2, 32, 2)])
@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("parts_bf16", [False, True])
def test_rope_cache_v8_bit_identical_to_v4(gpu, nh, nkv, D, S, fp8, parts_bf16):
    """The 16-byte kernel (default for D % 16 == 0) computes every element exactly as the
    4-element kernel - which runs when a bf16 qkv row stride is not a multiple of 8 - fed the
    reduced input (split-K partials summed in fp32 in split order, rounded to bf16 once): q,
    q_sink, K and V^T caches, bf16 / fp32 / bf16 partials."""
    if S == 0 and parts_bf16:
        pytest.skip("no partials")
    torch.manual_seed(21)
    T, bs, nblocks = 41, 64, 8
    width = (nh + 2 * nkv) * D
    if S:
        parts = torch.randn(S, T, width, device=gpu)
        parts = parts.to(torch.bfloat16) if parts_bf16 else parts
        src = ops.SplitKPartials(parts)
        acc = parts[0].float()
        for i in range(1, S):
            acc = acc + parts[i].float()
        red = acc.to(BF)
    else:
        src = red = torch.randn(T, width, device=gpu, dtype=BF)
    # the same values at a row stride of width + 4 (not a multiple of 8): the 4-element kernel
    odd = torch.zeros(T, width + 4, device=gpu, dtype=BF)
    odd[:, :width] = red
    src_v4 = odd[:, :width]
    pos = torch.randint(0, 300, (T,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(nblocks * bs, device=gpu)[:T].to(torch.int64)
    slots[7] = -1
    cs = ref.build_cos_sin(D, 512, 500000.0, device=gpu)
    k1, v1 = _make_cache(nblocks, nkv, bs, D, gpu)
    if fp8:
        k1, v1 = k1.to(torch.float8_e4m3fn), v1.to(torch.float8_e4m3fn)
    k2, v2 = k1.clone(), v1.clone()
    outs = []
    for x, (k, v) in ((src, (k1, v1)), (src_v4, (k2, v2))):
        outs.append(ops.rope_cache(x, pos, slots, cs, nh, nkv, D, k, v, window=100,
                                   want_sink=True, k_scale=0.5, v_scale=0.25))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(k1.view(torch.uint8), k2.view(torch.uint8))
    assert torch.equal(v1.view(torch.uint8), v2.view(torch.uint8))


@pytest.mark.parametrize("fp8", [False, True])
def test_rope_cache_bf16_partials_match_fp32_partials(gpu, fp8):
    """bf16 split-K partials (fp8 path, gemm_tile epilogue 4) are summed in fp32 in split order:
    bit-identical to the same values given as fp32 partials."""
    torch.manual_seed(14)
    nh, nkv, D, S, T, bs, nblocks = 64, 8, 128, 3, 29, 64, 8
    pb = torch.randn(S, T, (nh + 2 * nkv) * D, device=gpu).to(torch.bfloat16)
    pos = torch.randint(0, 300, (T,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(nblocks * bs, device=gpu)[:T].to(torch.int64)
    cs = ref.build_cos_sin(D, 512, 500000.0, device=gpu)
    k1, v1 = _make_cache(nblocks, nkv, bs, D, gpu)
    if fp8:
        k1, v1 = k1.to(torch.float8_e4m3fn), v1.to(torch.float8_e4m3fn)
    k2, v2 = k1.clone(), v1.clone()
    q1, _ = ops.rope_cache(ops.SplitKPartials(pb.float()), pos, slots, cs, nh, nkv, D, k1, v1)
    q2, _ = ops.rope_cache(ops.SplitKPartials(pb), pos, slots, cs, nh, nkv, D, k2, v2)
    assert torch.equal(q1, q2)
    assert torch.equal(k1.view(torch.uint8), k2.view(torch.uint8))
    assert torch.equal(v1.view(torch.uint8), v2.view(torch.uint8))


@pytest.mark.parametrize("S,rows,K", [(4, 512, 8192), (3, 33, 1024)])
def test_quant_rowwise_bf16_partials_match_fp32_partials(gpu, S, rows, K):
    torch.manual_seed(S + rows + 1)
    pb = torch.randn(S, rows, K, device=gpu).to(torch.bfloat16)
    res = torch.randn(rows, K, device=gpu, dtype=BF)
    w = torch.randn(K, device=gpu, dtype=BF)
    r1, r2 = res.clone(), res.clone()
    q1, s1 = ops.quant_rowwise(ops.SplitKPartials(pb.float()), r1, w, 1e-5)
    q2, s2 = ops.quant_rowwise(ops.SplitKPartials(pb), r2, w, 1e-5)
    assert torch.equal(q1.view(torch.uint8), q2.view(torch.uint8))
    assert torch.equal(s1, s2) and torch.equal(r1, r2)


@pytest.mark.parametrize("M,N,K,splits", [(512, 1024, 8192, 4), (300, 768, 2048, 3)])
def test_gemm_tile_fp8_bf16_partials(gpu, M, N, K, splits):
    """gemm_tile epilogue 4 (fp8, split-K partials rounded to bf16) against the fp32 partials."""
    torch.manual_seed(M + K)
    xq, xs = ops.quant_rowwise(torch.randn(M, K, device=gpu).to(BF))
    wq, ws = ops.quantize_weight_fp8((torch.randn(N, K, device=gpu) / K ** 0.5).to(BF))
    with ops.kernel_policy(bf16_partials=False):
        pf = ops.gemm_tile_fp8(xq, xs, wq, ws, splits, defer_reduce=True).parts
    pb = ops.gemm_tile_fp8(xq, xs, wq, ws, splits, defer_reduce=True).parts
    assert pb.dtype == BF and pf.dtype == torch.float32
    assert torch.equal(pb, pf.to(BF))


@pytest.mark.parametrize("M,N,K,splits", [(512, 1024, 8192, 4), (300, 768, 2048, 3)])
def test_gemm_tile_bf16_operand_bf16_partials(gpu, M, N, K, splits):
    """bf16 operands, bf16 partials (default): epilogue 4 writes each split's fp32 partial rounded to
    bf16 - exactly the fp32 partials' rounding - and RMSNorm over them stays within one bf16
    ulp-scale of the fp32-partials result."""
    torch.manual_seed(M + K + 1)
    x = torch.randn(M, K, device=gpu).to(BF)
    w = (torch.randn(N, K, device=gpu) / K ** 0.5).to(BF)
    with ops.kernel_policy(bf16_partials=False):
        pf = ops.gemm_tile(x, w, splits, defer_reduce=True).parts
    pb = ops.gemm_tile(x, w, splits, defer_reduce=True).parts
    assert pb.dtype == BF and pf.dtype == torch.float32
    assert torch.equal(pb, pf.to(BF))
    nw = torch.rand(N, device=gpu).to(BF) + 0.5
    r1 = torch.randn(M, N, device=gpu).to(BF)
    r2 = r1.clone()
    y1, _ = ops.rms_norm(ops.SplitKPartials(pf), nw, 1e-5, r1)
    y2, _ = ops.rms_norm(ops.SplitKPartials(pb), nw, 1e-5, r2)
    _close(y2, y1, 2e-2, 2e-2, "rms over bf16 partials")
    _close(r2, r1, 2e-2, 2e-2, "residual over bf16 partials")


def _tables(B, max_blocks, nblocks, dev, seed=0):
    g = torch.Generator().manual_seed(seed)
    perm = torch.randperm(nblocks, generator=g)[: B * max_blocks]
    return perm.reshape(B, max_blocks).to(torch.int32).to(dev)


@pytest.mark.parametrize("nh,nkv,D", [(64, 8, 128), (32, 8, 128), (12, 12, 64), (4, 2, 32)])
@pytest.mark.parametrize("splits", [1, 3])
def test_attn_decode(gpu, nh, nkv, D, splits):
    torch.manual_seed(2)
    bs, B = 64, 6
    lens = torch.tensor([1, 0, 33, 64, 257, 1000], dtype=torch.int32)
    max_blocks = (int(lens.max()) + bs - 1) // bs
    nblocks = B * max_blocks + 3
    kc, vc = _make_cache(nblocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, nblocks, gpu)
    q = torch.randn(B, nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    out = ops.attn_decode(q, None, kc, vc, bt, lens.to(gpu), scale, num_splits=splits)
    out_r = ref.attn_decode(q.cpu(), None, kc.cpu(), vc.cpu(), bt.cpu(), lens, scale)
    _close(out, out_r, 2e-2, 2e-2, "decode")


@pytest.mark.parametrize("splits", [1, 2])
def test_attn_decode_window(gpu, splits):
    torch.manual_seed(3)
    nh, nkv, D, bs = 32, 8, 128, 64
    n_sink, sink_pad, window, ring = 4, 32, 100, 160
    lens = torch.tensor([3, 50, 104, 200, 517], dtype=torch.int32)
    B = lens.numel()
    max_blocks = (sink_pad + ring + bs - 1) // bs
    nblocks = B * max_blocks
    kc, vc = _make_cache(nblocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, nblocks, gpu, seed=1)
    q = torch.randn(B, nh, D, device=gpu, dtype=BF)
    qs = torch.randn(B, nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    out = ops.attn_decode(q, qs, kc, vc, bt, lens.to(gpu), scale, n_sink, sink_pad, ring, window,
                          num_splits=splits)
    out_r = ref.attn_decode(q.cpu(), qs.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), lens, scale, n_sink,
                            sink_pad, ring, window)
    _close(out, out_r, 2e-2, 2e-2, "decode-window")


@pytest.mark.parametrize("splits", [1, 2, 4, 12, 64, 256, 6, 3])
def test_attn_decode_long_context(gpu, splits):
    """16k-32k contexts (70B head config) through every split path: one split, workgroup-merged
    splits with nothing left to merge (2, 4), groups of 4 merged in LDS whose partials the combine
    kernel finishes (12, 64, 256), pairs merged in LDS then combined (6), unmerged splits (3)."""
    torch.manual_seed(21)
    nh, nkv, D, bs = 64, 8, 128, 64
    lens = torch.tensor([16384, 32768 - 5, 20001], dtype=torch.int32)
    B = lens.numel()
    max_blocks = (int(lens.max()) + bs - 1) // bs
    nblocks = B * max_blocks
    kc, vc = _make_cache(nblocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, nblocks, gpu, seed=7)
    q = torch.randn(B, nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    out = ops.attn_decode(q, None, kc, vc, bt, lens.to(gpu), scale, num_splits=splits)
    out_r = ref.attn_decode(q.cpu(), None, kc.cpu(), vc.cpu(), bt.cpu(), lens, scale)
    _close(out, out_r, 1e-2, 2e-2, f"decode-long-s{splits}")


@pytest.mark.parametrize("splits", [1, 8, 64])
def test_attn_decode_window_multi_wrap(gpu, splits):
    """StreamingLLM ring at a realistic window (W = 4096, 4 sinks) after several wraps of the
    ring, scored in slot space against the re-rotation-free reference."""
    torch.manual_seed(22)
    nh, nkv, D, bs = 64, 8, 128, 64
    n_sink, sink_pad, window = 4, 64, 4096
    ring = window - n_sink + 60   # ring rounded up to whole 32-slot steps (>= window - sinks)
    ring = (ring + 31) // 32 * 32
    lens = torch.tensor([3, 4000, 4097, 9000, 13001], dtype=torch.int32)
    B = lens.numel()
    max_blocks = (sink_pad + ring + bs - 1) // bs
    nblocks = B * max_blocks
    kc, vc = _make_cache(nblocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, nblocks, gpu, seed=8)
    q = torch.randn(B, nh, D, device=gpu, dtype=BF)
    qs = torch.randn(B, nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    out = ops.attn_decode(q, qs, kc, vc, bt, lens.to(gpu), scale, n_sink, sink_pad, ring, window,
                          num_splits=splits)
    out_r = ref.attn_decode(q.cpu(), qs.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), lens, scale, n_sink,
                            sink_pad, ring, window)
    _close(out, out_r, 1e-2, 2e-2, f"decode-window-wrap-s{splits}")


@pytest.mark.parametrize("nh,nkv,D", [(32, 8, 128), (8, 8, 64), (4, 2, 32)])
@pytest.mark.parametrize("tiles", [False, True])
@pytest.mark.parametrize("qb", ["1", "2"])
def test_attn_prefill(gpu, nh, nkv, D, tiles, qb):
    qb = int(qb)   # 16-token query blocks per wave
    torch.manual_seed(4)
    bs = 64
    q_lens = [5, 64, 130, 1, 1, 1]  # mixed batch: prefill chunks and decode rows
    ctx = [0, 10, 70, 300, 3, 129]  # tokens already in the cache before this chunk
    lens = torch.tensor([a + b for a, b in zip(q_lens, ctx)], dtype=torch.int32)
    B = len(q_lens)
    q_start = torch.tensor([0] + list(torch.cumsum(torch.tensor(q_lens), 0)), dtype=torch.int32)
    T = int(q_start[-1])
    max_blocks = (int(lens.max()) + bs - 1) // bs
    nblocks = B * max_blocks
    kc, vc = _make_cache(nblocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, nblocks, gpu, seed=2)
    q = torch.randn(T, nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    tm = ops.prefill_tiles(q_lens, nh, nkv, qb=qb).to(gpu) if tiles else None
    out = ops.attn_prefill(q, None, kc, vc, bt, lens.to(gpu), q_start.to(gpu), max(q_lens), scale,
                           tile_map=tm, qb=qb)
    out_r = ref.attn_prefill(q.cpu(), None, kc.cpu(), vc.cpu(), bt.cpu(), lens, q_start, scale)
    _close(out, out_r, 2e-2, 2e-2, "prefill")


@pytest.mark.parametrize("heads", ["one", "per_head"])
@pytest.mark.parametrize("D", [64, 128])
def test_attn_prefill_custom_mask(gpu, heads, D):
    """The reference API's pre-inverted 4-D additive mask in the HIP prefill kernel (masked
    variant) against the fp32 oracle ref.attn_custom_mask: ragged lengths, mixed chunk / decode
    rows, a mask that opens future keys (no causal mask is added), finfo.min and -inf entries,
    a row open to a single key and a row masked with finfo.min everywhere (zeros)."""
    torch.manual_seed(11)
    nh, nkv, bs = 8, 2, 64
    q_lens = [9, 1, 40, 3]
    ctx = [0, 77, 30, 129]
    lens = [a + b for a, b in zip(q_lens, ctx)]
    B, Tm, Km = len(q_lens), max(q_lens), max(lens) + 5
    q_start = torch.tensor([0] + list(torch.cumsum(torch.tensor(q_lens), 0)), dtype=torch.int32)
    T = int(q_start[-1])
    max_blocks = (max(lens) + bs - 1) // bs
    kc, vc = _make_cache(B * max_blocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, B * max_blocks, gpu, seed=7)
    q = torch.randn(T, nh, D, device=gpu, dtype=BF)
    Hm = 1 if heads == "one" else nh
    neg = torch.finfo(torch.float32).min
    mask = torch.where(torch.rand(B, Hm, Tm, Km) < 0.3, torch.tensor(neg), torch.tensor(0.0))
    mask += torch.randn(B, Hm, Tm, Km) * 0.5 * (mask == 0)   # graded biases, max stays ~0
    mask[0, :, -1, :] = float("-inf")    # -inf everywhere ...
    mask[0, :, -1, 0] = 0.0              # ... except one key
    mask[2, :, -5, :] = neg              # a row masked with finfo.min everywhere (-> zeros)
    mask = mask.clamp(max=0.0)
    scale = 1 / math.sqrt(D)
    lens_t = torch.tensor(lens, dtype=torch.int32)
    out = ops.attn_prefill(q, None, kc, vc, bt, lens_t.to(gpu), q_start.to(gpu), max(q_lens),
                           scale, mask=mask.to(gpu))
    out_r = ref.attn_custom_mask(q.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), lens_t, q_start, scale,
                                 mask)
    _close(out, out_r, 2e-2, 2e-2, "prefill-custom-mask")
    # a mask that only re-states causality equals the causal kernel
    causal = torch.full((B, 1, Tm, Km), neg)
    for b in range(B):
        for t in range(q_lens[b]):
            causal[b, 0, Tm - q_lens[b] + t, : lens[b] - q_lens[b] + t + 1] = 0.0
    out_c = ops.attn_prefill(q, None, kc, vc, bt, lens_t.to(gpu), q_start.to(gpu), max(q_lens),
                             scale, mask=causal.to(gpu))
    out_p = ops.attn_prefill(q, None, kc, vc, bt, lens_t.to(gpu), q_start.to(gpu), max(q_lens),
                             scale)
    _close(out_c, out_p.cpu().float(), 1e-2, 1e-2, "custom-causal-vs-causal")


@pytest.mark.parametrize("qb", ["1", "2"])
def test_attn_prefill_window(gpu, qb):
    qb = int(qb)
    torch.manual_seed(5)
    nh, nkv, D, bs = 8, 2, 64, 64
    n_sink, sink_pad, window, ring = 4, 32, 96, 192
    q_lens = [40, 7]
    lens = torch.tensor([40, 300], dtype=torch.int32)
    B = 2
    q_start = torch.tensor([0, 40, 47], dtype=torch.int32)
    max_blocks = (sink_pad + ring + bs - 1) // bs
    kc, vc = _make_cache(B * max_blocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, B * max_blocks, gpu, seed=3)
    q = torch.randn(47, nh, D, device=gpu, dtype=BF)
    qs = torch.randn(47, nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    out = ops.attn_prefill(q, qs, kc, vc, bt, lens.to(gpu), q_start.to(gpu), 40, scale, n_sink,
                           sink_pad, ring, window, qb=qb)
    out_r = ref.attn_prefill(q.cpu(), qs.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), lens, q_start, scale,
                             n_sink, sink_pad, ring, window)
    _close(out, out_r, 2e-2, 2e-2, "prefill-window")


@pytest.mark.parametrize("qb", ["1", "2"])
@pytest.mark.parametrize("nh,nkv", [(32, 8), (16, 16)])
@pytest.mark.parametrize("n_sink", [0, 4, 40])
def test_attn_prefill_m32_sliding_window(gpu, qb, nh, nkv, n_sink):
    """attn_prefill32.hip on windowed ring caches: Mistral's sliding window (no sinks) and
    StreamingLLM sink windows (4 sinks; 40, which spill into the step's second half): rolling keys
    by ring offset, slot sink_pad + (a - n_sink) % ring, window mask q - (W - n_sink) < a <= q,
    the sinks as one extra step scored against q_sink; chunks on top of a wrapped ring, against
    the fp32 oracle (ring semantics of cache.py / ring_abs) and attention.hip's kernel."""
    qb = int(qb)
    torch.manual_seed(17 + n_sink)
    D, bs, window = 128, 64, 200
    q_lens = [300, 1, 64, 130, 17, 3]
    ctx = [0, 899, 636, 400, 1000, 0]
    lens = torch.tensor([a + b for a, b in zip(q_lens, ctx)], dtype=torch.int32)
    sink_pad = ((n_sink + 31) // 32) * 32
    ring = ((window - n_sink + max(q_lens) - 1 + 31) // 32) * 32   # the block manager's sizing
    B = len(q_lens)
    q_start = torch.tensor([0] + list(torch.cumsum(torch.tensor(q_lens), 0)), dtype=torch.int32)
    max_blocks = (sink_pad + ring + bs - 1) // bs
    kc, vc = _make_cache(B * max_blocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, B * max_blocks, gpu, seed=4)
    q = torch.randn(int(q_start[-1]), nh, D, device=gpu, dtype=BF)
    qs = torch.randn(int(q_start[-1]), nh, D, device=gpu, dtype=BF) if n_sink else None
    scale = 1 / math.sqrt(D)
    tm = ops.prefill_tiles(q_lens, nh, nkv, qb=qb).to(gpu)
    args = (kc, vc, bt, lens.to(gpu), q_start.to(gpu), max(q_lens), scale, n_sink, sink_pad, ring,
            window)
    out = ops.attn_prefill(q, qs, *args, tile_map=tm, qb=qb)
    out_r = ref.attn_prefill(q.cpu(), qs.cpu() if n_sink else None, kc.cpu(), vc.cpu(), bt.cpu(),
                             lens, q_start, scale, n_sink, sink_pad, ring, window)
    _close(out, out_r, 2e-2, 2e-2, f"prefill-m32-window-{nh}/{nkv}-s{n_sink}-qb{qb}")
    with ops.kernel_policy(prefill_m32=False):
        out_l = ops.attn_prefill(q, qs, *args, tile_map=tm, qb=qb)
    _close(out, out_l, 2e-2, 2e-2, "prefill-m32-window-vs-legacy")


@pytest.mark.parametrize("qb", ["1", "2"])
@pytest.mark.parametrize("nh,nkv,window", [(64, 8, 0), (32, 8, 0), (16, 16, 0), (64, 8, 200)])
def test_attn_prefill_m32_fp8_kv(gpu, qb, nh, nkv, window):
    """attn_prefill32.hip on fp8 e4m3 caches (runs widened to bf16 on their way into LDS, K's
    scale in the softmax scale, V's in the normalisation) against the fp32 oracle and
    attention.hip's fp8 kernel: 8-wave and 4-wave workgroups (groups of 8 at both tile sizes, 4
    and MHA at the long-chunk tiles; the others fall back), full cache and a sliding window."""
    qb = int(qb)
    torch.manual_seed(23)
    D, bs, ks, vs = 128, 64, 2.0, 0.5
    q_lens = [300, 1, 64, 130, 17]
    ctx = [0, 899, 36, 400, 10]
    lens = torch.tensor([a + b for a, b in zip(q_lens, ctx)], dtype=torch.int32)
    ring = ((window + max(q_lens) - 1 + 31) // 32) * 32 if window else 0
    B = len(q_lens)
    q_start = torch.tensor([0] + list(torch.cumsum(torch.tensor(q_lens), 0)), dtype=torch.int32)
    max_blocks = ((ring or int(lens.max())) + bs - 1) // bs
    kc, vc = _make_cache_fp8(B * max_blocks, nkv, bs, D, gpu, ks, vs)
    bt = _tables(B, max_blocks, B * max_blocks, gpu, seed=6)
    q = torch.randn(int(q_start[-1]), nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    tm = ops.prefill_tiles(q_lens, nh, nkv, qb=qb).to(gpu)
    args = (kc, vc, bt, lens.to(gpu), q_start.to(gpu), max(q_lens), scale, 0, 0, ring, window)
    out = ops.attn_prefill(q, None, *args, tile_map=tm, qb=qb, k_scale=ks, v_scale=vs)
    out_r = ref.attn_prefill(q.cpu(), None, kc.cpu(), vc.cpu(), bt.cpu(), lens, q_start, scale,
                             0, 0, ring, window, k_scale=ks, v_scale=vs)
    _close(out, out_r, 2e-2, 2e-2, f"prefill-m32-fp8-{nh}/{nkv}-w{window}-qb{qb}")
    with ops.kernel_policy(prefill_m32=False):
        out_l = ops.attn_prefill(q, None, *args, tile_map=tm, qb=qb, k_scale=ks, v_scale=vs)
    _close(out, out_l, 2e-2, 2e-2, "prefill-m32-fp8-vs-legacy")


def test_sample_greedy_and_topk1(gpu):
    torch.manual_seed(6)
    B, V = 9, 128256
    logits = torch.randn(B, V, device=gpu, dtype=BF) * 3
    greedy = ops.sample(logits)
    assert torch.equal(greedy.cpu().long(), logits.float().argmax(-1).cpu())
    t = torch.full((B,), 0.7, device=gpu)
    k1 = torch.ones(B, dtype=torch.int32, device=gpu)
    # fp32 logits: bf16 rows of 128k values contain tied maxima, which top-k=1 keeps together
    lf = torch.randn(B, V, device=gpu) * 3
    s = ops.sample(lf, temperature=t, top_k=k1, seeds=torch.arange(B, device=gpu))
    assert torch.equal(s.cpu().long(), lf.argmax(-1).cpu())
    lp = torch.empty(B, device=gpu)
    ops.sample(logits.float(), out=torch.empty(B, dtype=torch.int32, device=gpu), logprobs=lp)
    lp_ref = torch.log_softmax(logits.float(), -1).max(-1).values
    _close(lp, lp_ref, 1e-3, 1e-3, "logprob")


@pytest.mark.parametrize("V", [128256, 1000, 1003])
def test_sample_greedy_ties_take_the_lowest_index(gpu, V):
    """16-byte greedy path (bf16, V % 8 == 0) and the element-wise one agree with torch's argmax,
    ties included (the lowest index wins)."""
    torch.manual_seed(V)
    B = 5
    logits = torch.randn(B, V, device=gpu).clamp(-4, 4).to(BF)
    logits[:, V // 3] = 9.0
    logits[:, V - 2] = 9.0
    logits[1, 0] = 9.0
    out = ops.sample(logits)
    assert torch.equal(out.cpu().long(), logits.float().argmax(-1).cpu())
    assert out[1].item() == 0 and out[0].item() == V // 3


def test_sample_distribution(gpu):
    # V small, many rows with the same logits -> empirical frequencies ~ softmax
    V, B = 16, 4096
    base = torch.linspace(-2, 2, V, device=gpu)
    logits = base.repeat(B, 1).contiguous()
    t = torch.ones(B, device=gpu)
    s = ops.sample(logits, temperature=t, seeds=torch.arange(B, device=gpu) * 7919)
    freq = torch.bincount(s.long().cpu(), minlength=V).float() / B
    p = torch.softmax(base.cpu(), -1)
    assert (freq - p).abs().max() < 0.03
    # top-k=4 keeps only the 4 largest
    s = ops.sample(logits, temperature=t, top_k=torch.full((B,), 4, dtype=torch.int32, device=gpu),
                   seeds=torch.arange(B, device=gpu))
    assert int(s.min()) >= V - 4
    # top-p=0.5 keeps the smallest top set with mass >= 0.5
    sp, _ = torch.sort(p, descending=True)
    need = int((torch.cumsum(sp, 0) < 0.5).sum()) + 1
    s = ops.sample(logits, temperature=t, top_p=torch.full((B,), 0.5, device=gpu),
                   seeds=torch.arange(B, device=gpu))
    assert int(s.min()) >= V - need


def test_quant_rowwise(gpu):
    x = torch.randn(17, 4096, device=gpu, dtype=BF) * 3
    q, s = ops.quant_rowwise(x)
    deq = q.float() * s
    rel = (deq - x.float()).abs().max() / x.float().abs().max()
    assert rel < 0.07
    w = (1 + 0.1 * torch.randn(4096, device=gpu)).to(BF)
    r = torch.randn_like(x)
    r2 = r.clone()
    q2, s2 = ops.quant_rowwise(x, residual=r, norm_w=w, eps=1e-5)
    y, _ = ref.rms_norm(x.cpu(), w.cpu(), 1e-5, residual=r2.cpu())
    deq2 = (q2.float() * s2).cpu()
    assert (deq2 - y.float()).abs().max() / y.float().abs().max() < 0.07


def test_quant_rowwise_residual_out_of_place(gpu):
    x = torch.randn(9, 8192, device=gpu, dtype=BF)
    r = torch.randn_like(x)
    w = (1 + 0.1 * torch.randn(8192, device=gpu)).to(BF)
    r0, ro = r.clone(), torch.empty_like(r)
    q, s = ops.quant_rowwise(x, r, w, 1e-5, residual_out=ro)
    assert torch.equal(r, r0)  # input residual untouched
    _close(ro, x.float() + r0.float(), 1e-2, 1e-2, "residual_out")
    # identical to the CPU reference path (same bf16 rounding before quantisation)
    rc = r0.cpu().clone()
    qc, sc = ops.quant_rowwise(x.cpu(), rc, w.cpu(), 1e-5)
    torch.testing.assert_close(s.cpu(), sc, rtol=1e-2, atol=0)
    deq, deqc = q.float().cpu() * s.cpu(), qc.float() * sc
    assert (deq - deqc).abs().max() / deqc.abs().max() < 0.07


@pytest.mark.parametrize("T,I", [(1, 512), (33, 3584), (256, 28672)])
def test_silu_mul_quant(gpu, T, I):
    x = torch.randn(T, 2 * I, device=gpu, dtype=BF) * 2
    q, s = ops.silu_mul_quant(x)
    assert q.shape == (T, I) and s.shape == (T, 1)
    y = ref.silu_mul(x.cpu()).float()
    sr = y.abs().amax(-1, keepdim=True) / 448.0
    torch.testing.assert_close(s.cpu(), sr, rtol=1e-2, atol=1e-6)
    deq = q.float().cpu() * s.cpu()
    assert (deq - y).abs().max() / y.abs().max() < 0.07


def test_rms_norm_residual_out_of_place(gpu):
    x = torch.randn(5, 4096, device=gpu, dtype=BF)
    r = torch.randn(5, 4096, device=gpu, dtype=BF)
    w = torch.ones(4096, device=gpu, dtype=BF)
    r0 = r.clone()
    ro = torch.empty_like(r)
    y, r2 = ops.rms_norm(x, w, 1e-5, residual=r, residual_out=ro)
    assert r2 is ro and torch.equal(r, r0)  # input residual untouched
    _close(ro, x.float() + r0.float(), 1e-2, 1e-2, "residual_out")
    y_ref, _ = ref.rms_norm(x.cpu(), w.cpu(), 1e-5, residual=r0.cpu().clone())
    _close(y, y_ref, 2e-2, 1e-2, "rms_norm")


# ------------------------------------------------------------------------------ fp8 KV cache
F8 = torch.float8_e4m3fn


def _make_cache_fp8(nblocks, nkv, bs, D, dev, ks, vs):
    k, v = _make_cache(nblocks, nkv, bs, D, dev)
    return (k.float() / ks).to(F8), (v.float() / vs).to(F8)


@pytest.mark.parametrize("window", [0, 64])
def test_rope_cache_fp8(gpu, window):
    torch.manual_seed(11)
    nh, nkv, D, T, bs, nblocks = 32, 8, 128, 29, 64, 8
    qkv = torch.randn(T, (nh + 2 * nkv) * D, device=gpu, dtype=BF) * 3
    pos = torch.randint(0, 300, (T,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(nblocks * bs, device=gpu)[:T].to(torch.int64)
    cs = ref.build_cos_sin(D, 512, 500000.0, device=gpu)
    ks, vs = 0.5, 2.0
    k1, v1 = _make_cache_fp8(nblocks, nkv, bs, D, gpu, ks, vs)
    k2, v2 = k1.clone().cpu(), v1.clone().cpu()
    q, _ = ops.rope_cache(qkv, pos, slots, cs, nh, nkv, D, k1, v1, window=window,
                          want_sink=window > 0, k_scale=ks, v_scale=vs)
    q_r, _ = ref.rope_cache(qkv.cpu(), pos.cpu(), slots.cpu(), cs.cpu(), nh, nkv, D, k2, v2,
                            window, window > 0, ks, vs)
    _close(q, q_r, 2e-2, 1e-2, "q")
    # the same fp8 encoding up to one rounding step of the bf16 intermediate
    kd = (k1.float().cpu() - k2.float()).abs()
    assert (kd <= 0.13 * k2.float().abs() + 1e-3).all(), kd.max()  # <= one e4m3 step
    assert (kd > 0).float().mean() < 0.01  # and almost always bit-identical
    assert torch.equal(v1.cpu().view(torch.uint8), v2.view(torch.uint8))


@pytest.mark.parametrize("splits,D", [(1, 128), (3, 128), (4, 128), (8, 128), (12, 128),
                                      (64, 128), (6, 128), (4, 64), (1, 64), (4, 32), (3, 32)])
def test_attn_decode_fp8_kv(gpu, splits, D):
    """fp8 KV decode through every split path (ungrouped 1 / 3, workgroup-merged 4 / 8, merged +
    combined 12 / 64, pairs 6) with the head-dim-permuted 16-byte loads (D % 64 == 0) and the
    8-byte path (D = 32)."""
    torch.manual_seed(12)
    nh, nkv, bs, B = 64, 8, 64, 5
    lens = torch.tensor([1, 33, 64, 257, 700], dtype=torch.int32)
    max_blocks = (int(lens.max()) + bs - 1) // bs
    nblocks = B * max_blocks
    ks, vs = 0.25, 1.5
    kc, vc = _make_cache_fp8(nblocks, nkv, bs, D, gpu, ks, vs)
    bt = _tables(B, max_blocks, nblocks, gpu, seed=4)
    q = torch.randn(B, nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    out = ops.attn_decode(q, None, kc, vc, bt, lens.to(gpu), scale, num_splits=splits,
                          k_scale=ks, v_scale=vs)
    out_r = ref.attn_decode(q.cpu(), None, kc.cpu(), vc.cpu(), bt.cpu(), lens, scale,
                            k_scale=ks, v_scale=vs)
    _close(out, out_r, 2e-2, 2e-2, "decode-fp8")


@pytest.mark.parametrize("kv_fp8", [False, True])
@pytest.mark.parametrize("B,nh,nkv,D", [(512, 64, 8, 128), (1024, 64, 8, 128), (512, 16, 8, 64),
                                        (512, 8, 8, 32)])
def test_attn_decode_one_step_loop_large_batch(gpu, kv_fp8, B, nh, nkv, D):
    """Large one-split batches (B x 8 kv heads >= 16 waves per CU: attention.hip decode_grid runs
    the one-step loop at 4 waves per SIMD) against the fp32 reference on sampled sequences, and
    bit for bit against the same sequences run as small batches (the two-step loop): both
    loops walk the keys in the same order through the same online-softmax arithmetic."""
    torch.manual_seed(B + kv_fp8 + D)
    bs = 64
    lens = torch.randint(1, 300, (B,), dtype=torch.int32)
    lens[:3] = torch.tensor([1, 32, 299], dtype=torch.int32)
    max_blocks = (int(lens.max()) + bs - 1) // bs
    nblocks = B * max_blocks
    ks = vs = 1.0
    if kv_fp8:
        ks, vs = 0.25, 1.5
        kc, vc = _make_cache_fp8(nblocks, nkv, bs, D, gpu, ks, vs)
    else:
        kc, vc = _make_cache(nblocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, nblocks, gpu, seed=7)
    q = torch.randn(B, nh, D, device=gpu, dtype=BF)
    lg = lens.to(gpu)
    scale = 1 / math.sqrt(D)
    out = ops.attn_decode(q, None, kc, vc, bt, lg, scale, num_splits=1, k_scale=ks, v_scale=vs)
    parts = [ops.attn_decode(q[i:i + 64], None, kc, vc, bt[i:i + 64], lg[i:i + 64], scale,
                             num_splits=1, k_scale=ks, v_scale=vs) for i in range(0, B, 64)]
    torch.cuda.synchronize()
    assert torch.equal(out, torch.cat(parts, 0))
    idx = torch.tensor([0, 1, 2] + list(range(5, B, B // 29)))
    out_r = ref.attn_decode(q[idx].cpu(), None, kc.cpu(), vc.cpu(), bt[idx].cpu(), lens[idx],
                            scale, k_scale=ks, v_scale=vs)
    _close(out[idx], out_r, 2e-2, 2e-2, "decode one-step")


@pytest.mark.parametrize("B", [5, 64, 130])
@pytest.mark.parametrize("kv_fp8", [False, True])
def test_attn_decode_mx_output_bit_exact(gpu, B, kv_fp8):
    """attn_decode(mx_out=True): the epilogue's MX fp8 hand-off (one e8m0 scale per head row)
    equals ops.mx_quantize of the bf16 output bit for bit, incl. the padding-row scales."""
    torch.manual_seed(B)
    nh, nkv, D, bs = 16, 4, 128, 64
    lens = torch.randint(1, 700, (B,), dtype=torch.int32)
    nblk = int(((lens + bs - 1) // bs).sum()) + 1
    q = (torch.randn(B, nh, D) * 2.0).to(torch.bfloat16).to(gpu)
    kc = (torch.randn(nblk, nkv, bs, D) * 0.5)
    vc = (torch.randn(nblk, nkv, bs // 8, D, 8) * 3.0)
    ks = vs = 1.0
    if kv_fp8:
        ks, vs = 0.25, 0.5
        kc = (kc / ks).to(torch.float8_e4m3fn)
        vc = (vc / vs).to(torch.float8_e4m3fn)
    else:
        kc, vc = kc.to(torch.bfloat16), vc.to(torch.bfloat16)
    kc, vc = kc.to(gpu), vc.to(gpu)
    maxb = int(((lens + bs - 1) // bs).max())
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    nxt = 1
    for b in range(B):
        n = int((lens[b] + bs - 1) // bs)
        bt[b, :n] = torch.arange(nxt, nxt + n)
        nxt += n
    bt, lens_g = bt.to(gpu), lens.to(gpu)
    scale = D ** -0.5
    ref_o = ops.attn_decode(q, None, kc, vc, bt, lens_g, scale, num_splits=1, k_scale=ks, v_scale=vs)
    ref = ops.mx_quantize(ref_o.reshape(B, nh * D))
    mx = ops.attn_decode(q, None, kc, vc, bt, lens_g, scale, num_splits=1, k_scale=ks, v_scale=vs,
                         mx_out=True)
    assert torch.equal(mx.sc.cpu(), ref.sc.cpu())
    assert torch.equal(mx.q.view(torch.uint8).cpu(), ref.q.view(torch.uint8).cpu())


@pytest.mark.parametrize("splits", [1, 4, 12])
def test_attn_decode_fp8_kv_window_sinks(gpu, splits):
    """fp8 KV in StreamingLLM window mode: the sink segment is scored with q_sink, which must
    follow the same permuted head-dim map as q."""
    torch.manual_seed(23)
    nh, nkv, D, bs = 64, 8, 128, 64
    n_sink, sink_pad, window = 4, 64, 512
    ring = (window - n_sink + 31) // 32 * 32
    lens = torch.tensor([3, 300, 513, 2000], dtype=torch.int32)
    B = lens.numel()
    max_blocks = (sink_pad + ring + bs - 1) // bs
    nblocks = B * max_blocks
    ks, vs = 0.5, 2.0
    kc, vc = _make_cache_fp8(nblocks, nkv, bs, D, gpu, ks, vs)
    bt = _tables(B, max_blocks, nblocks, gpu, seed=9)
    q = torch.randn(B, nh, D, device=gpu, dtype=BF)
    qs = torch.randn(B, nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    out = ops.attn_decode(q, qs, kc, vc, bt, lens.to(gpu), scale, n_sink, sink_pad, ring, window,
                          num_splits=splits, k_scale=ks, v_scale=vs)
    out_r = ref.attn_decode(q.cpu(), qs.cpu(), kc.cpu(), vc.cpu(), bt.cpu(), lens, scale, n_sink,
                            sink_pad, ring, window, k_scale=ks, v_scale=vs)
    _close(out, out_r, 2e-2, 2e-2, f"decode-fp8-window-s{splits}")


@pytest.mark.parametrize("qb", ["1", "2"])
def test_attn_prefill_long_chunks(gpu, qb):
    """70B head config, long causal chunks on top of cached context (multi-tile workgroups, the
    diagonal inside a two-block wave tile, a chunk length that is not a tile multiple)."""
    qb = int(qb)
    torch.manual_seed(24)
    nh, nkv, D, bs = 64, 8, 128, 64
    q_lens, ctx = [1000, 77, 2048], [0, 900, 64]
    lens = torch.tensor([a + b for a, b in zip(q_lens, ctx)], dtype=torch.int32)
    B = len(q_lens)
    q_start = torch.tensor([0] + list(torch.cumsum(torch.tensor(q_lens), 0)), dtype=torch.int32)
    max_blocks = (int(lens.max()) + bs - 1) // bs
    kc, vc = _make_cache(B * max_blocks, nkv, bs, D, gpu)
    bt = _tables(B, max_blocks, B * max_blocks, gpu, seed=6)
    q = torch.randn(int(q_start[-1]), nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    tm = ops.prefill_tiles(q_lens, nh, nkv, qb=qb).to(gpu)
    out = ops.attn_prefill(q, None, kc, vc, bt, lens.to(gpu), q_start.to(gpu), max(q_lens), scale,
                           tile_map=tm, qb=qb)
    out_r = ref.attn_prefill(q.cpu(), None, kc.cpu(), vc.cpu(), bt.cpu(), lens, q_start, scale)
    _close(out, out_r, 2e-2, 2e-2, f"prefill-long-qb{qb}")


@pytest.mark.parametrize("nh,nkv", [(64, 8), (32, 8), (64, 4), (16, 8), (16, 16), (28, 4)])
@pytest.mark.parametrize("qb", ["1", "2"])
@pytest.mark.parametrize("ramp", [False, True])
def test_attn_prefill_m32(gpu, nh, nkv, qb, ramp):
    """attn_prefill32.hip (32x32x16 MFMA, 64-key steps, deferred softmax max) against the fp32
    oracle and against attention.hip's kernel: GQA groups of 8 / 4 / 16 (two workgroups per kv
    head), pairs (two heads x 32- or 64-token tiles), MHA and Qwen2's odd group of 7 (one head x
    64- or 128-token tiles), 16- and 32-token tiles, chunks on top of cached context, a chunk
    ending mid-step, decode rows in the batch.  ``ramp``: keys scaled up along the sequence, so
    the running max keeps growing by more than the deferral threshold (every rescale branch
    fires, cdna T13 hazard)."""
    qb = int(qb)
    torch.manual_seed(31)
    D, bs = 128, 64
    q_lens = [300, 1, 33, 64, 96, 2]
    ctx = [0, 500, 31, 64, 200, 0]
    lens = torch.tensor([a + b for a, b in zip(q_lens, ctx)], dtype=torch.int32)
    B = len(q_lens)
    q_start = torch.tensor([0] + list(torch.cumsum(torch.tensor(q_lens), 0)), dtype=torch.int32)
    max_blocks = (int(lens.max()) + bs - 1) // bs
    kc, vc = _make_cache(B * max_blocks, nkv, bs, D, gpu)
    if ramp:   # slot s of every page scaled by 1 + 6 (page_pos * bs + s) / L: later keys louder
        bt_cpu = _tables(B, max_blocks, B * max_blocks, "cpu", seed=9)
        scale_k = torch.ones(B * max_blocks, 1, bs, 1)
        for b in range(B):
            for j in range(max_blocks):
                pos = j * bs + torch.arange(bs, dtype=torch.float32)
                scale_k[int(bt_cpu[b, j]), 0, :, 0] = 1 + 6 * pos / max(int(lens[b]), 1)
        kc = (kc.float() * scale_k.to(gpu)).to(BF)
    bt = _tables(B, max_blocks, B * max_blocks, gpu, seed=9)
    q = torch.randn(int(q_start[-1]), nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    tm = ops.prefill_tiles(q_lens, nh, nkv, qb=qb).to(gpu)
    out = ops.attn_prefill(q, None, kc, vc, bt, lens.to(gpu), q_start.to(gpu), max(q_lens), scale,
                           tile_map=tm, qb=qb)
    out_r = ref.attn_prefill(q.cpu(), None, kc.cpu(), vc.cpu(), bt.cpu(), lens, q_start, scale)
    _close(out, out_r, 2e-2, 2e-2, f"prefill-m32-{nh}/{nkv}-qb{qb}-ramp{ramp}")
    with ops.kernel_policy(prefill_m32=False):
        out_l = ops.attn_prefill(q, None, kc, vc, bt, lens.to(gpu), q_start.to(gpu), max(q_lens),
                                 scale, tile_map=tm, qb=qb)
    _close(out, out_l, 2e-2, 2e-2, "prefill-m32-vs-legacy")
    # dense grid (no tile map) gives the same result
    out_d = ops.attn_prefill(q, None, kc, vc, bt, lens.to(gpu), q_start.to(gpu), max(q_lens),
                             scale, qb=qb)
    assert torch.equal(out, out_d)


def test_attn_prefill_fp8_kv(gpu):
    torch.manual_seed(13)
    nh, nkv, D, bs = 32, 8, 128, 64
    q_lens, ctx = [5, 64, 130], [0, 10, 300]
    lens = torch.tensor([a + b for a, b in zip(q_lens, ctx)], dtype=torch.int32)
    B = len(q_lens)
    q_start = torch.tensor([0] + list(torch.cumsum(torch.tensor(q_lens), 0)), dtype=torch.int32)
    max_blocks = (int(lens.max()) + bs - 1) // bs
    ks, vs = 2.0, 0.5
    kc, vc = _make_cache_fp8(B * max_blocks, nkv, bs, D, gpu, ks, vs)
    bt = _tables(B, max_blocks, B * max_blocks, gpu, seed=5)
    q = torch.randn(int(q_start[-1]), nh, D, device=gpu, dtype=BF)
    scale = 1 / math.sqrt(D)
    out = ops.attn_prefill(q, None, kc, vc, bt, lens.to(gpu), q_start.to(gpu), max(q_lens), scale,
                           k_scale=ks, v_scale=vs)
    out_r = ref.attn_prefill(q.cpu(), None, kc.cpu(), vc.cpu(), bt.cpu(), lens, q_start, scale,
                             k_scale=ks, v_scale=vs)
    _close(out, out_r, 2e-2, 2e-2, "prefill-fp8")


@pytest.mark.parametrize("S,rows,K", [(4, 512, 8192), (3, 33, 1024)])
@pytest.mark.parametrize("with_norm", [False, True])
def test_quant_rowwise_from_splitk_partials_bit_identical(gpu, S, rows, K, with_norm):
    torch.manual_seed(S + rows)
    parts = torch.randn(S, rows, K, device=gpu)
    res = torch.randn(rows, K, device=gpu, dtype=BF)
    w = torch.randn(K, device=gpu, dtype=BF) if with_norm else None
    x = ops.SplitKPartials(parts).materialize()
    r1, r2 = res.clone(), res.clone()
    q1, s1 = ops.quant_rowwise(x, r1, w, 1e-5)
    q2, s2 = ops.quant_rowwise(ops.SplitKPartials(parts), r2, w, 1e-5)
    assert torch.equal(q1.view(torch.uint8), q2.view(torch.uint8))
    assert torch.equal(s1, s2) and torch.equal(r1, r2)


@pytest.mark.parametrize("V", [128256, 32000, 50304])
def test_sample_register_path_matches_radix_path(gpu, V):
    """The register-resident top-k / top-p search (sampling.hip sample_row_regs, bf16 logits with
    V % 8 == 0) keeps the same set as the radix-histogram path (the same values as fp32 logits)
    and draws the same Gumbel sample: identical tokens for seeded rows over temperatures, top-k
    and top-p values."""
    torch.manual_seed(V)
    B = 24
    logits = (torch.randn(B, V, device=gpu) * torch.linspace(0.5, 6, B, device=gpu)[:, None]).to(BF)
    t = torch.linspace(0.3, 1.5, B, device=gpu)
    ks = torch.tensor([0, 1, 2, 5, 40, 1000, V - 1, V] * 3, dtype=torch.int32, device=gpu)
    ps = torch.tensor([1.0, 0.9, 0.5, 0.99, 0.1, 0.7] * 4, device=gpu)
    seeds = torch.arange(B, device=gpu) * 7919 + 3
    ctr = torch.arange(B, device=gpu, dtype=torch.int64) + 100
    out = {}
    for path, lg in (("1", logits), ("0", logits.float())):
        lp = torch.empty(B, device=gpu)
        tok = ops.sample(lg, temperature=t, top_k=ks, top_p=ps, seeds=seeds, counters=ctr,
                         logprobs=lp)
        out[path] = (tok.cpu(), lp.cpu())
    assert torch.equal(out["1"][0], out["0"][0]), (out["1"][0], out["0"][0])
    _close(out["1"][1], out["0"][1], 1e-4, 1e-4, "logprobs")


@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("fp8_act", [False, True])
def test_skinny_gemm_fp8(gpu, M, fp8_act):
    """fp8-weight GEMV (gemv.hip skinny_gemm_fp8_kernel) against the fp32 product of the same
    dequantised operands: bf16 rows, or fp8 rows with per-row scales (quant_rowwise's output)."""
    torch.manual_seed(M + 2 * fp8_act)
    N, K = 2050, 8192
    w = torch.randn(N, K, device=gpu) * 0.02
    wq, ws = ops.quantize_weight_fp8(w.to(BF))
    x = torch.randn(M, K, device=gpu, dtype=BF)
    bias = torch.randn(N, device=gpu, dtype=BF)
    wd = wq.float() * ws.reshape(-1, 1)
    if fp8_act:
        xq, xs = ops.quant_rowwise(x)
        y = ops.skinny_gemm_fp8(xq, wq, ws, xs, bias)
        xd = xq.float() * xs.reshape(-1, 1)
    else:
        y = ops.skinny_gemm_fp8(x, wq, ws, None, bias)
        xd = x.float()
    ref = xd @ wd.t() + bias.float()
    _close(y.float(), ref, 2e-2, 2e-2, "skinny fp8")


@pytest.mark.parametrize("M", [1, 2])
def test_skinny_gemm_int8(gpu, M):
    """int8-weight GEMV (LLM.int8 weights, bf16 rows) against the fp32 product of the same
    dequantised weights."""
    torch.manual_seed(M)
    N, K = 2050, 8192
    w = torch.randn(N, K, device=gpu) * 0.02
    wq, ws = ops.quantize_weight_int8(w)
    x = torch.randn(M, K, device=gpu, dtype=BF)
    y = ops.skinny_gemm_int8(x, wq, ws)
    ref = x.float() @ (wq.float() * ws.reshape(-1, 1)).t()
    _close(y.float(), ref, 2e-2, 2e-2, "skinny int8")


@pytest.mark.parametrize("wdtype", ["bf16", "fp8", "fp8-act", "int8"])
@pytest.mark.parametrize("M", [1, 2])
def test_skinny_gemm_swiglu(gpu, M, wdtype):
    """Fused-SwiGLU GEMV epilogue (gemv.hip SW variants) on a swiglu_interleave'd gate|up
    weight against silu(gate) * up of the fp32 product of the same dequantised operands."""
    torch.manual_seed(7 * M + len(wdtype))
    I, K = 1024, 4096
    w = torch.randn(2 * I, K, device=gpu) * 0.02
    wi = ops.swiglu_interleave(w.to(BF))
    x = torch.randn(M, K, device=gpu, dtype=BF)
    if wdtype == "bf16":
        y = ops.skinny_gemm(x, wi, swiglu=True)
        gu = x.float() @ wi.float().t()
    elif wdtype == "int8":
        wq, ws = ops.quantize_weight_int8(wi.float())
        y = ops.skinny_gemm_int8(x, wq, ws, swiglu=True)
        gu = x.float() @ (wq.float() * ws.reshape(-1, 1)).t()
    else:
        wq, ws = ops.quantize_weight_fp8(wi)
        wd = wq.float() * ws.reshape(-1, 1)
        if wdtype == "fp8-act":
            xq, xs = ops.quant_rowwise(x)
            y = ops.skinny_gemm_fp8(xq, wq, ws, xs, swiglu=True)
            gu = (xq.float() * xs.reshape(-1, 1)) @ wd.t()
        else:
            y = ops.skinny_gemm_fp8(x, wq, ws, swiglu=True)
            gu = x.float() @ wd.t()
    ref = ops.swiglu_interleaved(gu.to(BF).cpu()).float()
    assert y.shape == (M, I)
    _close(y.float().cpu(), ref, 2e-2, 2e-2, f"skinny swiglu {wdtype}")


@pytest.mark.parametrize("wdtype", ["bf16", "fp8", "int8"])
@pytest.mark.parametrize("M", [1, 2])
@pytest.mark.parametrize("swiglu", [False, True])
@pytest.mark.parametrize("resid", [False, True])
def test_skinny_gemm_fused_norm_bit_identical(gpu, M, wdtype, swiglu, resid):
    """The GEMV's fused input RMSNorm (gemv.hip gemv_norm_prologue) reproduces rms_norm's
    normalised rows bit for bit, so fused == rms_norm -> GEMV exactly; res_out = x + res_in."""
    torch.manual_seed(M * 31 + swiglu * 7 + resid)
    N, K = (2048 if swiglu else 1536), 8192
    x = torch.randn(M, K, device=gpu, dtype=BF)
    res = torch.randn(M, K, device=gpu, dtype=BF) if resid else None
    res0 = res.clone() if resid else None
    nw = (1 + 0.1 * torch.randn(K, device=gpu)).to(BF)
    w = (torch.randn(N, K, device=gpu) * 0.02).to(BF)
    if wdtype == "fp8":
        wq, ws = ops.quantize_weight_fp8(w)
        f = lambda xx, **kw: ops.skinny_gemm_fp8(xx, wq, ws, None, swiglu=swiglu, **kw)  # noqa: E731
    elif wdtype == "int8":
        wq, ws = ops.quantize_weight_int8(w.float())
        f = lambda xx, **kw: ops.skinny_gemm_int8(xx, wq, ws, swiglu=swiglu, **kw)  # noqa: E731
    else:
        f = lambda xx, **kw: ops.skinny_gemm(xx, w, swiglu=swiglu, **kw)  # noqa: E731
    r_sep = res.clone() if resid else None
    normed, _ = ops.rms_norm(x, nw, 1e-5, residual=r_sep)      # r_sep <- x + res in place
    ref = f(normed)
    r_out = torch.empty_like(x) if resid else None
    got = f(x, norm=ops.RowNorm(nw, 1e-5, res, r_out))
    torch.cuda.synchronize()
    assert torch.equal(got, ref), (got.float() - ref.float()).abs().max().item()
    if resid:
        assert torch.equal(r_out, r_sep)
        assert torch.equal(res, res0)   # res_in untouched (not aliased)


@pytest.mark.parametrize("wdtype", ["bf16", "fp8", "int8"])
@pytest.mark.parametrize("kv_fp8", [False, True])
@pytest.mark.parametrize("M", [1, 2])
def test_skinny_gemm_qkv_rope_matches_gemv_then_rope_cache(gpu, wdtype, kv_fp8, M):
    """The fused QKV GEMV with RoPE + paged KV write in its epilogue (gemv.hip kEpRope) produces
    the same q and the same cache bytes as the GEMV followed by rope_cache (one slot skipped
    with -1 when M = 2), with and without the fused input RMSNorm."""
    torch.manual_seed(11 * M + kv_fp8 + len(wdtype))
    nh, nkv, D, bs, K, nblk = 8, 2, 128, 64, 2048, 4
    N = (nh + 2 * nkv) * D
    x = torch.randn(M, K, device=gpu, dtype=BF)
    w = (torch.randn(N, K, device=gpu) * 0.02).to(BF)
    if wdtype == "fp8":
        wq, ws = ops.quantize_weight_fp8(w)
    elif wdtype == "int8":
        wq, ws = ops.quantize_weight_int8(w.float())
    else:
        wq, ws = w, None
    cs = ops.reference.build_cos_sin(D, 4096, 500000.0, None, device=gpu)
    pos = torch.tensor([37, 4000][:M], device=gpu, dtype=torch.int32)
    slots = torch.tensor([5, -1][:M] if M == 2 else [70], device=gpu, dtype=torch.int64)
    kdt = torch.float8_e4m3fn if kv_fp8 else BF
    nw = (1 + 0.1 * torch.randn(K, device=gpu)).to(BF)
    for norm in (None, ops.RowNorm(nw, 1e-5)):
        caches = []
        for _ in range(2):
            kc = torch.zeros(nblk, nkv, bs, D, device=gpu).to(kdt)
            vc = torch.zeros(nblk, nkv, bs // 8, D, 8, device=gpu).to(kdt)
            caches.append((kc, vc))
        xin = x if norm is None else norm.apply(x)
        if wdtype == "bf16":
            qkv = ops.skinny_gemm(xin, wq)
        elif wdtype == "fp8":
            qkv = ops.skinny_gemm_fp8(xin, wq, ws)
        else:
            qkv = ops.skinny_gemm_int8(xin, wq, ws)
        q_ref, _ = ops.rope_cache(qkv, pos, slots, cs, nh, nkv, D, *caches[0], k_scale=0.5,
                                  v_scale=0.25)
        q = ops.skinny_gemm_qkv_rope(x, wq, ws, None, pos, slots, cs, nh, nkv, D, *caches[1],
                                     k_scale=0.5, v_scale=0.25, norm=norm)
        torch.cuda.synchronize()
        assert torch.equal(q, q_ref)
        for a, b in zip(caches[0], caches[1]):
            assert torch.equal(a.view(torch.uint8), b.view(torch.uint8))


@pytest.mark.parametrize("shape,dtype", [((512, 8192), BF), ((3, 5, 7), torch.float32),
                                         ((1 << 20,), torch.int32), ((2,), BF)])
def test_digest_matches_reference(gpu, shape, dtype):
    """csrc/kernels/digest.hip (hop integrity, parallel/integrity.py): the folded partial sums
    equal the torch reference bit for bit at any grid size, and one flipped bit changes them."""
    torch.manual_seed(40)
    t = (torch.randn(shape, device=gpu) * 100).to(dtype)
    want = ops.digest_fold(ref.digest_parts(t.cpu()))
    for nb in (1, 7, 256):
        assert ops.digest_fold(ops.digest(t, nblocks=nb)) == want, nb
    u = t.clone()
    u.view(torch.uint8).view(-1)[u.numel() * u.element_size() // 2] ^= 0x10
    assert ops.digest_fold(ops.digest(u)) != want
