"""Hand-written decode GEMM (csrc/kernels/gemm.hip) vs an fp32 PyTorch reference."""
import pytest
import torch

from distributed_llm_inference import ops

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M", [1, 37, 128, 256])
@pytest.mark.parametrize("N,K", [(128, 128), (256, 1024), (384, 2048)])
@pytest.mark.parametrize("bn,splits", [(128, 1), (64, 1), (128, 2), (64, 4)])
def test_gemm_nt_matches_fp32(gpu, M, N, K, bn, splits):
    if N % bn or (K // 64) % splits:
        pytest.skip("shape not tileable")
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
