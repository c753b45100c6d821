"""Hand-written GEMMs (csrc/kernels/gemm_tile.hip, gemv.hip) vs fp32 PyTorch references."""
import pytest
import torch

from distributed_llm_inference import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K", [(1, 8), (7, 1000), (8192, 8192), (10, 28672 + 8)])
@pytest.mark.parametrize("bias", [False, True])
def test_skinny_gemm_matches_fp32(gpu, M, N, K, bias):
    if K % 8:
        K += 8 - K % 8
    torch.manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=gpu, dtype=torch.bfloat16) if bias else None
    y = ops.skinny_gemm(x, w, b)
    ref = x.float() @ w.float().t() + (b.float() if bias else 0.0)
    err = (y.float() - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err


def test_linear_uses_skinny_path_for_small_batches(gpu):
    from distributed_llm_inference.models.common import Linear
    lin = Linear(4096, 6144, device=gpu)
    torch.nn.init.normal_(lin.weight, std=0.02)
    for M in (1, 2, 3, 64):
        x = torch.randn(M, 4096, device=gpu, dtype=torch.bfloat16)
        y = lin(x)
        ref = x.float() @ lin.weight.float().t()
        assert (y.float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())


# ------------------------------------------------------------------ 256x256 tile GEMM (gemm_tile.hip)
_TILE_CASES = [(256, 256, 64, 1), (256, 256, 128, 1), (512, 512, 1024, 1), (100, 768, 512, 1),
               (512, 1024, 4096, 4), (300, 512, 8192, 3), (1, 256, 256, 1), (512, 256, 192, 2),
               (777, 512, 320, 5)]


@pytest.mark.parametrize("M,N,K,splits", _TILE_CASES)
def test_gemm_tile_matches_fp32(gpu, M, N, K, splits):
    torch.manual_seed(M * 3 + N + K)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    y = ops.gemm_tile(x, w, splits=splits)
    ref = x.float() @ w.float().t()
    err = (y.float() - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err


def test_gemm_tile_asymmetric_identity(gpu):
    x = torch.eye(256, 128, device=gpu, dtype=torch.bfloat16)
    w = (torch.arange(256 * 128, device=gpu, dtype=torch.float32).reshape(256, 128) % 251).to(torch.bfloat16)
    assert torch.equal(ops.gemm_tile(x, w).float(), x.float() @ w.float().t())


@pytest.mark.parametrize("M,I,K", [(512, 512, 1024), (77, 256, 256), (256, 1024, 512)])
def test_gemm_tile_fused_swiglu(gpu, M, I, K):
    torch.manual_seed(M + I)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(2 * I, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    wi = ops.swiglu_interleave(w)
    y = ops.gemm_tile(x, wi, swiglu=True)
    h = (x.float() @ w.float().t()).to(torch.bfloat16)
    ref = ops.silu_mul(h).float()
    assert (y.float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())
    # the unfused fallback on interleaved columns computes the same thing
    y2 = ops.swiglu_interleaved(torch.nn.functional.linear(x, wi))
    assert (y2.float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())


def test_llama_mlp_fused_swiglu_matches_unfused(gpu):
    from distributed_llm_inference.config import PRESETS
    from distributed_llm_inference.models.llama.modules import LlamaMLP
    spec = PRESETS["llama-3-8b"].replace(hidden_size=512, intermediate_size=1024)
    mlp = LlamaMLP(spec, device=gpu)
    torch.manual_seed(1)
    for p in mlp.parameters():
        p.data.normal_(0, 0.02)
    for M in (1, 2, 64, 256, 512):
        x = torch.randn(M, 512, device=gpu, dtype=torch.bfloat16)
        mlp.set_fused_swiglu(False)
        a = mlp(x).float()
        sd_before = mlp.gate_up_proj.weight.clone()
        mlp.set_fused_swiglu(True)
        b = mlp(x).float()
        assert (a - b).abs().max().item() < 2e-2 * max(1e-3, a.abs().max().item()), M
        mlp.set_fused_swiglu(False)
        assert torch.equal(mlp.gate_up_proj.weight, sd_before)


def test_linear_dispatches_decode_batches_to_tile_gemm(gpu, monkeypatch):
    from distributed_llm_inference.models.common import Linear
    lin = Linear(1024, 2048, device=gpu)
    torch.nn.init.normal_(lin.weight, std=0.02)
    calls = []
    real = ops.gemm_tile
    monkeypatch.setattr(ops, "gemm_tile", lambda *a, **k: calls.append(k.get("splits")) or real(*a, **k))
    x = torch.randn(512, 1024, device=gpu, dtype=torch.bfloat16)
    y = lin(x)
    assert calls, "M=512 decode batch did not use the tile GEMM"
    ref = x.float() @ lin.weight.float().t()
    assert (y.float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())


def test_no_library_gemms_keeps_small_and_wide_products_on_the_tile_kernel(gpu, monkeypatch):
    """KernelPolicy.library_gemms=False (the default when ranks share a GPU): M < 128 and the wide
    LM head stay on the
    tile kernel (hipBLASLt's choices there are stream-K persistent kernels); the rotating head's
    projection always does (LMHead.project(tile=True))."""
    from distributed_llm_inference.config import PRESETS
    from distributed_llm_inference.models.common import Linear
    from distributed_llm_inference.models.embed_head import LMHead
    cm = ops.kernel_policy(library_gemms=False)
    cm.__enter__()
    calls = []
    real = ops.gemm_tile
    monkeypatch.setattr(ops, "gemm_tile", lambda *a, **k: calls.append(a[1].shape) or real(*a, **k))
    lin = Linear(1024, 2048, device=gpu)
    torch.nn.init.normal_(lin.weight, std=0.02)
    for M in (3, 32, 127):
        x = torch.randn(M, 1024, device=gpu, dtype=torch.bfloat16)
        ref = x.float() @ lin.weight.float().t()
        assert (lin(x).float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())
    assert len(calls) == 3, calls
    cm.__exit__(None, None, None)   # library GEMMs allowed again: the head's tile=True still holds
    spec = PRESETS["llama-3-8b"].replace(hidden_size=1024, vocab_size=256 * 300)
    head = LMHead(spec, device=gpu).init_random(3)
    x = torch.randn(32, 1024, device=gpu, dtype=torch.bfloat16)
    calls.clear()
    y = head.project(x, tile=True)
    assert calls, "the rotating head's projection did not use the tile GEMM"
    ref = x.float() @ head.proj.weight.float().t()
    assert (y.float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("M,N,K,splits", [(256, 256, 128, 1), (512, 512, 2048, 1), (100, 768, 1024, 3),
                                          (512, 1024, 8192, 4), (33, 256, 384, 1)])
def test_gemm_tile_fp8_matches_dequantised_fp32(gpu, M, N, K, splits):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=gpu)
    w = torch.randn(N, K, device=gpu) / K ** 0.5
    xq, xs = ops.quant_rowwise(x.to(torch.bfloat16))
    wq, ws = ops.quantize_weight_fp8(w.to(torch.bfloat16))
    ref = (xq.float() * xs.reshape(-1, 1)) @ (wq.float() * ws.reshape(-1, 1)).t()
    y = ops.gemm_tile_fp8(xq, xs, wq, ws, splits).float()
    assert (y - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


def test_gemm_tile_fp8_exact_integers_and_swiglu(gpu):
    # exact small integers: any k-pairing mistake between the operands shows up bit-exactly
    xi = torch.zeros(256, 128, device=gpu)
    xi[torch.arange(128), torch.arange(128)] = 1.0
    wi = (torch.arange(256 * 128, device=gpu, dtype=torch.float32).reshape(256, 128) % 13) - 6
    one = torch.ones(256, device=gpu)
    y = ops.gemm_tile_fp8(xi.to(torch.float8_e4m3fn), one, wi.to(torch.float8_e4m3fn), one).float()
    assert torch.equal(y, xi @ wi.t())
    x = torch.randn(512, 1024, device=gpu).to(torch.bfloat16)
    w = (torch.randn(1024, 1024, device=gpu) / 32).to(torch.bfloat16)
    xq, xs = ops.quant_rowwise(x)
    wq, ws = ops.quantize_weight_fp8(w)
    ref = ops.silu_mul(((xq.float() * xs) @ (wq.float() * ws.reshape(-1, 1)).t()).to(torch.bfloat16)).float()
    wqi = ops.swiglu_interleave(wq.view(torch.uint8)).view(wq.dtype)
    wsi = ops.swiglu_interleave(ws.reshape(-1, 1)).reshape(-1)
    y = ops.gemm_tile_fp8(xq, xs, wqi, wsi, swiglu=True).float()
    assert (y - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


# ------------------------------------------------------------------ fp8 MX activations (kSwiGLUMx -> kFp8Mx)
@pytest.mark.parametrize("M", [512, 300, 64, 1])
@pytest.mark.parametrize("gemm4", [False, True])
def test_gemm_tile_fp8_swiglu_mx_epilogue_matches_reference_quantiser(gpu, M, gemm4):
    # same main loop as the bf16-output SwiGLU epilogue: its h, quantised by the reference MX rule,
    # must give the kernel's fp8 bytes and e8m0 scales bit for bit (pad rows of the last 64-row
    # block carry scale 127); for gemm_tile (8 waves) and gemm4 (one wave per SIMD, kG4SwiGLUMx),
    # and the two kernels' outputs are the same bytes (same 16x16x128 MFMA, same k pairing)
    torch.manual_seed(M)
    K, I = 1024, 768
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    w = (torch.randn(2 * I, K, device=gpu) / 32 * torch.rand(2 * I, 1, device=gpu) * 4).to(torch.bfloat16)
    xq, xs = ops.quant_rowwise(x)
    wq, ws = ops.quantize_weight_fp8(w)
    wqi = ops.swiglu_interleave(wq.view(torch.uint8)).view(wq.dtype)
    wsi = ops.swiglu_interleave(ws.reshape(-1, 1)).reshape(-1)
    h = ops.gemm_tile_fp8(xq, xs, wqi, wsi, swiglu=True, gemm4=gemm4)
    a = ops.gemm_tile_fp8(xq, xs, wqi, wsi, swiglu=True, mx_out=True, gemm4=gemm4)
    ref = ops.mx_quantize(h)
    assert torch.equal(a.sc, ref.sc)
    assert torch.equal(a.q.view(torch.uint8), ref.q.view(torch.uint8))
    if gemm4:
        with ops.kernel_policy(gemm4=False):
            h0 = ops.gemm_tile_fp8(xq, xs, wqi, wsi, swiglu=True)
            a0 = ops.gemm_tile_fp8(xq, xs, wqi, wsi, swiglu=True, mx_out=True)
        assert torch.equal(h, h0)
        assert torch.equal(a.sc, a0.sc) and torch.equal(a.q.view(torch.uint8), a0.q.view(torch.uint8))
    # and the MX representation stays within fp8 resolution of h
    err = (a.dequantize() - h.float()).abs()
    bmax = h.float().abs().view(M, -1, 128).amax(-1).repeat_interleave(128, 1)
    assert (err <= h.float().abs() * 2 ** -4 + bmax * 2 ** -17).all()


@pytest.mark.parametrize("M,N,K,splits", [(512, 1024, 8192, 1), (512, 8192, 28672, 4),
                                          (300, 512, 4096, 2), (77, 256, 1024, 1)])
@pytest.mark.parametrize("gemm4", [False, True])
def test_gemm_tile_fp8_mx_matches_dequantised_fp32(gpu, M, N, K, splits, gemm4):
    torch.manual_seed(M + N + K)
    # rows and 128-column blocks of very different magnitudes: per-block scales matter
    h = (torch.randn(M, K, device=gpu) * torch.exp2(torch.randint(-6, 7, (M, K // 128), device=gpu)
                                                    ).repeat_interleave(128, 1).float()).to(torch.bfloat16)
    a = ops.mx_quantize(h)
    w = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    wq, ws = ops.quantize_weight_fp8(w)
    ref = a.dequantize() @ (wq.float() * ws.reshape(-1, 1)).t()
    y = ops.gemm_tile_fp8_mx(a, wq, ws, splits, gemm4=gemm4).float()
    assert (y - ref).abs().max().item() < 1e-2 * ref.abs().max().item()
    if gemm4:   # same MFMA, k pairing and split ranges as gemm_tile: the same bits
        with ops.kernel_policy(gemm4=False):
            y0 = ops.gemm_tile_fp8_mx(a, wq, ws, splits).float()
        assert torch.equal(y, y0)
    if splits > 1:
        parts = ops.gemm_tile_fp8_mx(a, wq, ws, splits, defer_reduce=True, gemm4=gemm4)
        assert isinstance(parts, ops.SplitKPartials)
        assert (parts.parts.sum(0) - ref).abs().max().item() < 1e-2 * ref.abs().max().item()
        if gemm4:
            with ops.kernel_policy(gemm4=False):
                p0 = ops.gemm_tile_fp8_mx(a, wq, ws, splits, defer_reduce=True)
            assert torch.equal(parts.parts, p0.parts)


def test_gemm_tile_fp8_mx_rejects_oversized_k_split(gpu):
    a = ops.mx_quantize(torch.randn(256, 128 * 65, device=gpu).to(torch.bfloat16))
    wq, ws = ops.quantize_weight_fp8(torch.randn(256, 128 * 65, device=gpu).to(torch.bfloat16))
    with pytest.raises(ValueError):
        ops.gemm_tile_fp8_mx(a, wq, ws, 1)


# ------------------------------------------------------------------ LLM.int8 (int8 MFMA tile GEMM)
def test_gemm_tile_int8_exact_and_random(gpu):
    xi = torch.zeros(256, 128, device=gpu)
    xi[torch.arange(128), torch.arange(128)] = 1.0
    wi = (torch.arange(256 * 128, device=gpu, dtype=torch.float32).reshape(256, 128) % 29) - 14
    one = torch.ones(256, device=gpu)
    y = torch.empty(256, 256, device=gpu, dtype=torch.bfloat16)
    ops.native().gemm_tile(y, xi.to(torch.int8), wi.to(torch.int8), 1, 0, None, one, one)
    assert torch.equal(y.float(), xi @ wi.t())
    for M, N, K, sp in ((512, 1024, 4096, 4), (77, 512, 384, 1), (300, 768, 2048, 3)):
        x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
        w = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
        xq, xs = ops.quant_rowwise_int8(x)
        wq, ws = ops.quantize_weight_int8(w)
        ref = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).t()
        out = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
        wsp = torch.empty(sp * M * N, device=gpu) if sp > 1 else None
        ops.native().gemm_tile(out, xq, wq, sp, 0, wsp, xs, ws)
        assert (out.float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()


def test_quant_rowwise_int8_kernel_matches_reference(gpu):
    x = torch.randn(37, 1024, device=gpu).to(torch.bfloat16)
    flags = torch.zeros(1024, dtype=torch.uint8, device=gpu)
    flags[[3, 500, 1023]] = 1
    q, s = ops.quant_rowwise_int8(x, flags)
    qr, sr = ops.quant_rowwise_int8(x.cpu(), flags.cpu())
    assert torch.allclose(s.cpu(), sr, rtol=1e-6)
    assert (q.cpu().int() - qr.int()).abs().max().item() <= 1   # rounding of exact halves


def test_llm_int8_linear_gpu_matches_cpu_and_bf16(gpu):
    torch.manual_seed(0)
    M, K, N = 64, 1024, 512
    x = torch.randn(M, K)
    x[:, [11, 600]] *= 50.0
    xb = x.to(torch.bfloat16)
    w = (torch.randn(N, K) / K ** 0.5).to(torch.bfloat16)
    wq, ws = ops.quantize_weight_int8(w)
    y_cpu = ops.llm_int8_linear(xb, wq, ws, 6.0).float()
    y_gpu = ops.llm_int8_linear(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0).float().cpu()
    ref = xb.float() @ w.float().t()
    assert ((y_gpu - y_cpu).norm() / y_cpu.norm()).item() < 5e-3
    assert ((y_gpu - ref).norm() / ref.norm()).item() < 0.02


@pytest.mark.parametrize("M,K,N,n_out", [(512, 1024, 1024, 5), (300, 2048, 512, 80), (7, 1024, 256, 3),
                                         (130, 4096, 768, 0)])
def test_llm_int8_fused_outlier_epilogue_swiglu_and_partials(gpu, M, K, N, n_out):
    """The bf16 outlier product runs inside the int8 tile GEMM's epilogue: plain store, fused
    SwiGLU (pairwise-interleaved int8 rows + scales) and deferred split-K partials (the outlier
    term in split 0 only) all match the dequantised CPU reference."""
    torch.manual_seed(M + K + n_out)
    x = torch.randn(M, K)
    if n_out:
        x[:, torch.randperm(K)[:n_out]] *= 40.0
    xb = x.to(torch.bfloat16)
    w = (torch.randn(N, K) / K ** 0.5).to(torch.bfloat16)
    wq, ws = ops.quantize_weight_int8(w)
    ref = ops.llm_int8_linear(xb, wq, ws, 6.0).float()                 # CPU reference path
    y = ops.llm_int8_linear(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0).float().cpu()
    assert ((y - ref).norm() / ref.norm()).item() < 5e-3
    p = ops.llm_int8_linear(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0, defer_reduce=True)
    if isinstance(p, ops.SplitKPartials):
        assert p.parts.shape[0] > 1
        yp = p.parts.float().sum(0).cpu()
        assert ((yp - ref).norm() / ref.norm()).item() < 5e-3
    wqi = ops.swiglu_interleave(wq.to(gpu))
    wsi = ops.swiglu_interleave(ws.to(gpu).reshape(-1, 1)).reshape(-1)
    h = ops.llm_int8_linear(xb.to(gpu), wqi, wsi, 6.0, swiglu=True).float().cpu()
    href = ops.silu_mul(ref.to(torch.bfloat16)).float()
    assert ((h - href).norm() / href.norm()).item() < 1e-2


def test_llm_int8_dynamic_outlier_chunks_ignore_stale_columns(gpu):
    """The fused path gathers only the live 32-column outlier chunks and the epilogue multiplies
    only those: a product with few outliers right after one with many (same shapes, so the
    caching allocator hands back buffers still holding the previous call's columns) and one with
    none must match the CPU reference, for the store, split-K partial and SwiGLU epilogues."""
    M, K, N = 256, 4096, 1024
    torch.manual_seed(7)
    w = (torch.randn(N, K) / K ** 0.5).to(torch.bfloat16)
    wq, ws = ops.quantize_weight_int8(w)
    wqg, wsg = wq.to(gpu), ws.to(gpu)
    wqi = ops.swiglu_interleave(wqg)
    wsi = ops.swiglu_interleave(wsg.reshape(-1, 1)).reshape(-1)
    for n_out in (70, 3, 40, 0, 64):
        x = torch.randn(M, K)
        if n_out:
            x[:, torch.randperm(K)[:n_out]] *= 40.0
        xb = x.to(torch.bfloat16)
        ref = ops.llm_int8_linear(xb, wq, ws, 6.0).float()
        y = ops.llm_int8_linear(xb.to(gpu), wqg, wsg, 6.0).float().cpu()
        assert ((y - ref).norm() / ref.norm()).item() < 5e-3, n_out
        p = ops.llm_int8_linear(xb.to(gpu), wqg, wsg, 6.0, defer_reduce=True)
        yp = p.parts.float().sum(0).cpu() if isinstance(p, ops.SplitKPartials) else p.float().cpu()
        assert ((yp - ref).norm() / ref.norm()).item() < 5e-3, n_out
        h = ops.llm_int8_linear(xb.to(gpu), wqi, wsi, 6.0, swiglu=True).float().cpu()
        href = ops.silu_mul(ref.to(torch.bfloat16)).float()
        assert ((h - href).norm() / href.norm()).item() < 1e-2, n_out


def _llm_int8_outliers_ref(x, wq, ws, threshold, J):
    """fp32 PyTorch reference of int8_outlier.hip: the <= J largest column maxima above
    `threshold` (distinct values), in column order, padded with (column 0, weight 0)."""
    colmax = x.float().abs().amax(0)
    vals, _ = colmax.sort(descending=True)
    if (colmax >= threshold).sum() <= J:
        on = colmax >= threshold     # bitsandbytes: |A| >= threshold
    else:
        on = colmax > vals[J].item()  # strictly above the (J+1)-th largest; ties dropped
    cols = on.nonzero().flatten()
    idx = torch.zeros(J, dtype=torch.long)
    idx[:cols.numel()] = cols
    sel = torch.zeros(J)
    sel[:cols.numel()] = 1.0
    xo = (x.float()[:, idx] * sel).to(torch.bfloat16)
    wo = ((wq.float()[:, idx] * ws[:, None]).to(torch.bfloat16).float() * sel).to(torch.bfloat16)
    return on.to(torch.uint8), xo, wo


# (K, outlier columns planted): below the 64-column cap (threshold cut) and above it (radix
# select of the 65th largest column maximum), K = 28672 is the 70B down projection (28 / thread)
# M = 1 / 96 / 300 / 512: column-max row loop tail only, and the 4-deep unrolled body + tail
@pytest.mark.parametrize("K,n_out,M", [(1024, 5, 96), (8192, 40, 512), (8192, 300, 1),
                                       (28672, 1000, 300), (4096, 0, 96), (8200, 30, 130)])
def test_llm_int8_outlier_kernels_match_reference(gpu, K, n_out, M):
    torch.manual_seed(K + n_out)
    N, J = 512, 64
    x = torch.randn(M, K) * 0.5
    cols = torch.randperm(K)[:n_out]
    xb = x.to(torch.bfloat16)
    # distinct bf16 magnitudes >= 8 (consecutive bit patterns: no ties at the cut), random rows
    planted = (torch.randperm(n_out).to(torch.int16) + 0x4100).view(torch.bfloat16)
    xb[torch.randint(0, M, (n_out,)), cols] = planted
    wq = torch.randint(-127, 128, (N, K), dtype=torch.int8)
    ws = torch.rand(N) * 0.01 + 1e-3
    flags, xo, wo, cnt = ops.native().llm_int8_outliers(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0, J)
    rf, rx, rw = _llm_int8_outliers_ref(xb, wq, ws, 6.0, J)
    assert int(flags.sum()) == min(n_out, J) == int(cnt.item())
    assert torch.equal(flags.cpu(), rf)
    assert torch.equal(xo.cpu(), rx)
    assert torch.equal(wo.cpu(), rw)
    # the coalesced gather from the transposed weight copy gives the same bits
    wq_t = wq.t().contiguous().to(gpu)
    _, _, wo_t, _ = ops.native().llm_int8_outliers(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0, J, wq_t)
    assert torch.equal(wo_t.cpu(), rw)
    # dynamic: only the live 32-column chunks are written, and those bit-exactly
    live = min(J, (min(n_out, J) + 31) // 32 * 32)
    for wt in (None, wq_t):
        _, xd, wd, c = ops.native().llm_int8_outliers(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0, J,
                                                      wt, True)
        assert int(c.item()) == min(n_out, J)
        assert torch.equal(xd[:, :live].cpu(), rx[:, :live])
        assert torch.equal(wd[:, :live].cpu(), rw[:, :live])


def test_llm_int8_select_ties_at_the_cut_and_early_exit(gpu):
    """More than J columns pass the threshold: distinct maxima end the radix select early (the
    located value alone in its bin), tied maxima at the cut run every pass and drop the whole tie;
    both must pick the reference's set exactly."""
    K, M, N, J = 4096, 64, 256, 64
    wq = torch.randint(-127, 128, (N, K), dtype=torch.int8)
    ws = torch.rand(N) * 0.01 + 1e-3
    for vals in ([9.0] * 40 + [8.0] * 60, [float(v) for v in torch.linspace(7.0, 500.0, 150)],
                 [7.5] * 100):
        torch.manual_seed(len(vals))
        xb = (torch.randn(M, K) * 0.5).to(torch.bfloat16)
        cols = torch.randperm(K)[:len(vals)]
        xb[torch.randint(0, M, (len(vals),)), cols] = torch.tensor(vals).to(torch.bfloat16)
        flags, xo, wo, cnt = ops.native().llm_int8_outliers(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0, J)
        rf, rx, rw = _llm_int8_outliers_ref(xb, wq, ws, 6.0, J)
        assert torch.equal(flags.cpu(), rf), vals[:3]
        assert int(cnt.item()) == int(rf.sum())
        assert torch.equal(xo.cpu(), rx) and torch.equal(wo.cpu(), rw)


# the transposed-copy gather's tails: partial 16-column blocks / max_out % 8 != 0 and partial
# 256-row n-tiles (N % 256 != 0), bit-exact against the reference
@pytest.mark.parametrize("N,J", [(260, 20), (1028, 40), (512, 64)])
def test_llm_int8_gather_wt_tails(gpu, N, J):
    torch.manual_seed(N + J)
    K, M = 2048, 64
    xb = (torch.randn(M, K) * 0.5).to(torch.bfloat16)
    cols = torch.randperm(K)[:J + 7]
    planted = (torch.randperm(J + 7).to(torch.int16) + 0x4100).view(torch.bfloat16)
    xb[torch.randint(0, M, (J + 7,)), cols] = planted
    wq = torch.randint(-127, 128, (N, K), dtype=torch.int8)
    ws = torch.rand(N) * 0.01 + 1e-3
    _, _, rw = _llm_int8_outliers_ref(xb, wq, ws, 6.0, J)
    wq_t = wq.t().contiguous().to(gpu)
    _, _, wo_t, _ = ops.native().llm_int8_outliers(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0, J, wq_t)
    assert torch.equal(wo_t.cpu(), rw)


def test_llm_int8_threshold_is_inclusive_and_cpu_gpu_agree(gpu):
    """|x| == threshold is an outlier (bitsandbytes' >=), on the GPU kernel and the CPU path."""
    K, N, M = 1024, 256, 8
    xb = (torch.randn(M, K) * 0.3).to(torch.bfloat16)
    xb[3, 17] = 6.0        # exactly at the threshold
    xb[5, 900] = -7.5
    wq = torch.randint(-127, 128, (N, K), dtype=torch.int8)
    ws = torch.rand(N) * 0.01 + 1e-3
    fg, _, _, _ = ops.native().llm_int8_outliers(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0, 64)
    assert fg.cpu()[17] == 1 and fg.cpu()[900] == 1 and int(fg.sum()) == 2
    y_cpu = ops.llm_int8_linear(xb, wq, ws, 6.0).float()
    y_gpu = ops.llm_int8_linear(xb.to(gpu), wq.to(gpu), ws.to(gpu), 6.0).float().cpu()
    assert ((y_gpu - y_cpu).norm() / y_cpu.norm()).item() < 5e-3


# ------------------------------------------------- stream-K tail (gemm_tile splits = 0, SkArgs)
def _sk_workspace(gpu):
    n = ops.native().gemm_tile_sk_workspace_floats()
    ws = torch.empty(n, dtype=torch.float32, device=gpu)
    ws.view(torch.int32)[1023] = 0   # the kernel's spin-timeout counter
    return ws


# tiles = ceil(M/256) * N/256 on 256 CUs: 448 (tail 192, 2 owners per tile, the 70B gate|up
# case), 384 with K = 256 (4 k-tiles, 2 per workgroup), 288 (tail 32: 8 workgroups per tile,
# a 7-deep predecessor chain), 260 with K = 4096 (tail 4: 64 workgroups per tile)
@pytest.mark.parametrize("M,N,K", [(512, 57344, 1024), (256, 98304, 256), (512, 36864, 2048),
                                   (300, 33280, 4096)])
@pytest.mark.parametrize("swiglu", [False, True])
def test_gemm_tile_stream_k_matches_fp32(gpu, M, N, K, swiglu):
    if ops.device_cus(gpu) != 256:
        pytest.skip("shapes sized for 256 CUs")
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    ws = _sk_workspace(gpu)
    out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=gpu)
    wi = ops.swiglu_interleave(w) if swiglu else w
    h = x.float() @ w.float().t()
    ref = ops.silu_mul(h.to(torch.bfloat16)).float() if swiglu else h
    tol = 2e-2 * max(1.0, ref.abs().max().item())
    for it in range(3):   # repeated launches: flags re-zeroed, L1/L2 hold the previous slabs
        out.zero_()
        ops.native().gemm_tile(out, x, wi, 0, 2 if swiglu else 0, ws)
        err = (out.float() - ref).abs().max().item()
        assert err < tol, (it, err)
    torch.cuda.synchronize()
    assert int(ws.view(torch.int32)[1023].item()) == 0, "stream-K hand-off spin timed out"


def test_gemm_tile_stream_k_dispatch_and_graph(gpu, monkeypatch):
    """With KernelPolicy.stream_k_tail ops.gemm_tile picks the stream-K tail for the 70B gate|up
    shape, also under graph replay."""
    cm = ops.kernel_policy(stream_k_tail=True, gemm4=False)
    cm.__enter__()
    if ops.device_cus(gpu) != 256:
        pytest.skip("shape sized for 256 CUs")
    M, I, K = 512, 28672, 512
    assert ops.tile_gemm_stream_k(M, 2 * I, gpu)
    assert not ops.tile_gemm_stream_k(M, 8192, gpu)       # 64 tiles: split-K instead
    torch.manual_seed(5)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(2 * I, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    wi = ops.swiglu_interleave(w)
    ref = ops.silu_mul((x.float() @ w.float().t()).to(torch.bfloat16)).float()
    out = torch.empty(M, I, dtype=torch.bfloat16, device=gpu)
    ops.gemm_tile(x, wi, swiglu=True, out=out)       # warm-up outside capture
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.gemm_tile(x, wi, swiglu=True, out=out)
    for _ in range(3):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert (out.float() - ref).abs().max().item() < 2e-2 * max(1.0, ref.abs().max().item())


# ------------------------------------- split-K partials reduced inside the consumer RMSNorm
@pytest.mark.parametrize("S,M,H", [(3, 512, 8192), (4, 300, 4096), (2, 7, 1024)])
@pytest.mark.parametrize("mode", ["none", "inplace", "out_of_place"])
def test_rms_norm_splitk_bit_identical_to_reduce_then_norm(gpu, S, M, H, mode):
    torch.manual_seed(S * M + H)
    parts = torch.randn(S, M, H, device=gpu)
    w = torch.randn(H, device=gpu, dtype=torch.bfloat16)
    res = torch.randn(M, H, device=gpu, dtype=torch.bfloat16) if mode != "none" else None
    x = ops.SplitKPartials(parts).materialize()
    assert torch.equal(x, parts.sum(0).to(torch.bfloat16)) or \
        (x.float() - parts.sum(0)).abs().max().item() < 1e-2
    r1 = res.clone() if res is not None else None
    r2 = res.clone() if res is not None else None
    ro1 = torch.empty_like(res) if mode == "out_of_place" else None
    ro2 = torch.empty_like(res) if mode == "out_of_place" else None
    y1, rr1 = ops.rms_norm(x, w, 1e-5, residual=r1, residual_out=ro1)
    y2, rr2 = ops.rms_norm(ops.SplitKPartials(parts), w, 1e-5, residual=r2, residual_out=ro2)
    assert torch.equal(y1, y2)
    if res is not None:
        assert torch.equal(rr1, rr2)
        if mode == "out_of_place":
            assert torch.equal(r2, res)   # residual_in untouched


@pytest.mark.parametrize("bf16_parts", ["0", "1"])
def test_gemm_tile_defer_reduce_feeds_rms_norm(gpu, monkeypatch, bf16_parts):
    """fp32 partials (KernelPolicy.bf16_partials=False): the consumer's sum is bit-identical to the
    reduce pass; bf16 partials (default): each partial carries one extra bf16 rounding - close,
    not equal."""
    cm = ops.kernel_policy(bf16_partials=bf16_parts == "1")
    cm.__enter__()
    torch.manual_seed(11)
    M, N, K = 512, 8192, 8192
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    nw = torch.randn(N, device=gpu, dtype=torch.bfloat16)
    res = torch.randn(M, N, device=gpu, dtype=torch.bfloat16)
    sp = ops.tile_gemm_splits(M, N, K)
    assert sp > 1
    p = ops.gemm_tile(x, w, splits=sp, defer_reduce=True)
    assert isinstance(p, ops.SplitKPartials) and p.parts.shape == (sp, M, N)
    y_ref = ops.gemm_tile(x, w, splits=sp)
    a, ra = ops.rms_norm(y_ref, nw, 1e-5, residual=res.clone())
    b, rb = ops.rms_norm(p, nw, 1e-5, residual=res.clone())
    if bf16_parts == "0":
        assert p.parts.dtype == torch.float32
        assert torch.equal(p.materialize(), y_ref)
        assert torch.equal(a, b) and torch.equal(ra, rb)
    else:
        assert p.parts.dtype == torch.bfloat16
        tol = 2e-2 * y_ref.float().abs().max().item()
        assert (p.materialize().float() - y_ref.float()).abs().max().item() < tol
        assert (rb.float() - ra.float()).abs().max().item() < tol
        assert (b.float() - a.float()).abs().max().item() < 2e-2 * a.float().abs().max().item()


@pytest.mark.parametrize("M", [512, 300, 40, 1100])   # <= 512: decode schedule v8 (NT weights); 1100: v4
@pytest.mark.parametrize("N,K,splits,epi", [(2048, 1024, 1, 0), (4096, 2048, 1, 2),
                                            (1024, 4096, 3, 1), (1024, 4096, 4, 4),
                                            (7680, 512, 1, 0),
                                            # 1-3 k-tiles per split: every tail of the k-loop
                                            (256, 64, 1, 0), (512, 128, 1, 2), (256, 192, 1, 0),
                                            (768, 320, 2, 1)])
def test_gemm4_bit_identical_to_gemm_tile(gpu, M, N, K, splits, epi):
    """gemm4.hip (one wave per SIMD, asm-ordered k-loop) runs the same MFMA over the same k order
    as gemm_tile: bf16 store, SwiGLU and fp32 / bf16 split-K partials must match it bit for bit,
    for full and partial M tiles and persistent grids (7680 / 256 x 2 = 60 tiles, few CUs)."""
    torch.manual_seed(M + N + splits)
    a = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    b = (torch.randn(N, K, device=gpu) * 0.05).to(torch.bfloat16)
    nat = ops.native()
    if epi in (1, 4):
        ref = torch.empty(splits, M, N, device=gpu, dtype=torch.float32)
        nat.gemm_tile(torch.empty(M, 0, device=gpu, dtype=torch.bfloat16), a, b, splits, 1,
                      ref.view(-1))
        if epi == 4:
            ref = ref.to(torch.bfloat16)
        out = torch.empty(splits, M, N, device=gpu, dtype=ref.dtype)
    else:
        cols = N // 2 if epi == 2 else N
        ref = torch.empty(M, cols, device=gpu, dtype=torch.bfloat16)
        nat.gemm_tile(ref, a, b, 1, epi)
        out = torch.empty_like(ref)
    # automatic persistent grid, and a small grid that loops over tiles; every decode-size
    # schedule (NT weight streams 8 / 9 included) gives the same bits
    for grid, var in ((0, -1), (7, -1), (0, 4), (0, 6), (0, 8), (0, 9)):
        out.fill_(7.0)
        nat.gemm4(out, a, b, splits, epi, grid, None, None, var)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (grid, var, (out.float() - ref.float()).abs().max().item())


def _q8(x):
    s = (x.float().abs().amax(1) / 448.0).clamp_min(1e-12)
    return (x.float() / s[:, None]).to(torch.float8_e4m3fn), s.contiguous()


@pytest.mark.parametrize("M", [512, 300, 40])
@pytest.mark.parametrize("N,K,splits,epi", [(2048, 1024, 1, 0), (4096, 2048, 1, 2),
                                            (1024, 4096, 3, 1), (1024, 4096, 4, 4),
                                            (7680, 512, 1, 0),
                                            # 1-3 k-tiles per split: every tail of the k-loop
                                            (256, 128, 1, 0), (512, 256, 1, 2), (256, 384, 1, 0),
                                            (768, 640, 2, 1)])
def test_gemm4_fp8_bit_identical_to_gemm_tile_fp8(gpu, M, N, K, splits, epi):
    """fp8 gemm4 (block-scaled 16x16x128 MFMA with gemm_tile's fragment pairing, unit block scales,
    per-row x per-channel scales in the epilogue) against gemm_tile's fp8 path on the same
    quantised operands -- bit for bit, bf16 / SwiGLU stores and fp32 / bf16 split-K partials --
    and against the fp32 product of the dequantised operands."""
    torch.manual_seed(M + N + splits + 1)
    a, sa = _q8(torch.randn(M, K, device=gpu))
    b, sb = _q8(torch.randn(N, K, device=gpu) * 0.05)
    nat = ops.native()
    full = (a.float() * sa[:, None]) @ (b.float() * sb[:, None]).t()
    if epi == 1:
        ref = torch.empty(splits, M, N, device=gpu, dtype=torch.float32)
        nat.gemm_tile(torch.empty(M, 0, device=gpu, dtype=torch.bfloat16), a, b, splits, 1,
                      ref.view(-1), sa, sb)
        out = torch.empty_like(ref)
        f32 = full
    elif epi == 4:
        ref = torch.empty(splits, M, N, device=gpu, dtype=torch.bfloat16)
        nat.gemm_tile(ref, a, b, splits, 4, None, sa, sb)
        out = torch.empty_like(ref)
        f32 = full
    else:
        cols = N // 2 if epi == 2 else N
        ref = torch.empty(M, cols, device=gpu, dtype=torch.bfloat16)
        nat.gemm_tile(ref, a, b, 1, epi, None, sa, sb)
        out = torch.empty_like(ref)
        f32 = ops.swiglu_interleaved(full.cpu()).to(gpu) if epi == 2 else full   # fp32 reference
    scale = f32.abs().max().item()
    for grid in (0, 7):
        out.fill_(7.0)
        nat.gemm4(out, a, b, splits, epi, grid, sa, sb)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (grid, (out.float() - ref.float()).abs().max().item())
        got = out.float().sum(0) if epi in (1, 4) else out.float()
        assert (got - f32).abs().max().item() < 2e-2 * scale, grid


@pytest.mark.parametrize("M,K,I", [(512, 8192, 28672), (300, 2048, 1536), (40, 1024, 768)])
def test_gemm4_fp8_mx_chain_gate_up_to_down(gpu, M, K, I):
    """The fp8 MLP hand-off on gemm4 end to end: gate|up + SwiGLU quantised to MX in gemm4's
    epilogue, consumed by the down projection on gemm4's MX operand - against the same chain on
    gemm_tile, and the down product against the fp32 product of the dequantised MX activations
    (a shared partial M tile, the 70B shape with its 4-way split-K)."""
    torch.manual_seed(M + I)
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    wgu = (torch.randn(2 * I, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    wd = (torch.randn(K, I, device=gpu) / I ** 0.5).to(torch.bfloat16)
    xq, xs = ops.quant_rowwise(x)
    gq, gs = ops.quantize_weight_fp8(wgu)
    gqi = ops.swiglu_interleave(gq.view(torch.uint8)).view(gq.dtype)
    gsi = ops.swiglu_interleave(gs.reshape(-1, 1)).reshape(-1)
    dq, ds = ops.quantize_weight_fp8(wd)
    sp = ops.tile_gemm_splits_fp8(M, K, I) or 1
    outs = {}
    for g4 in (False, True):
        h = ops.gemm_tile_fp8(xq, xs, gqi, gsi, swiglu=True, mx_out=True, gemm4=g4)
        y = ops.gemm_tile_fp8_mx(h, dq, ds, sp, gemm4=g4).float()
        ref = h.dequantize() @ (dq.float() * ds.reshape(-1, 1)).t()
        assert (y - ref).abs().max().item() < 1e-2 * ref.abs().max().item(), g4
        outs[g4] = (h.dequantize(), y)
    assert torch.equal(outs[True][0], outs[False][0])   # same MX bytes and scales
    assert torch.equal(outs[True][1], outs[False][1])
