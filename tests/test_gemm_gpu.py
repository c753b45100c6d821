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
