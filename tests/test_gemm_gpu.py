"""Hand-written decode GEMM (csrc/kernels/gemm.hip) vs an fp32 PyTorch reference."""
import pytest
import torch

from distributed_llm_inference import ops

pytestmark = pytest.mark.gpu


_CASES = [(M, N, K, bn, splits)
          for M in (1, 37, 128, 256)
          for N, K in ((128, 128), (256, 1024), (384, 2048))
          for bn, splits in ((128, 1), (64, 1), (128, 2), (64, 4))
          if N % bn == 0 and (K // 64) % splits == 0]  # only tileable shapes


@pytest.mark.parametrize("M,N,K,bn,splits", _CASES)
def test_gemm_nt_matches_fp32(gpu, M, N, K, bn, splits):
    torch.manual_seed(M + N + K)
    x = torch.randn(M, K, device=gpu, dtype=torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    y = ops.gemm_nt(x, w, splits=splits, bn=bn)
    ref = x.float() @ w.float().t()
    err = (y.float() - ref).abs().max().item()
    assert err < 2e-2 * max(1.0, ref.abs().max().item()), err


def test_gemm_nt_asymmetric_identity(gpu):
    # A = I (rows 0..M-1 of identity) with an asymmetric B catches transposed C writes
    M, K, N = 64, 128, 128
    x = torch.eye(M, K, device=gpu, dtype=torch.bfloat16)
    w = torch.arange(N * K, device=gpu, dtype=torch.float32).reshape(N, K).remainder(251).to(torch.bfloat16)
    y = ops.gemm_nt(x, w, splits=1, bn=128)
    assert torch.equal(y.float(), w.float().t()[:M])


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
