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
