"""Out-of-bounds canaries for the HIP kernels (race detection / sanitizers).

GPU AddressSanitizer is not available on the MI355X pool, so every kernel that writes memory is
run on a VIEW into a larger buffer whose guard regions (before and after the view, and the unused
blocks of the KV caches) are filled with a sentinel.  Any store outside the logical output — a
wrong grid bound, a tail-handling bug, an off-by-one in the slot arithmetic — flips a guard word.
Shapes are chosen with ragged tails (row counts / widths that are not multiples of the tile).
"""
import pytest
import torch

from distributed_llm_inference import ops
from distributed_llm_inference.ops import reference as ref

pytestmark = pytest.mark.gpu
BF = torch.bfloat16
G = 4096  # guard elements on each side
SENT = -12345.0


def _guarded(shape, dtype, dev, fill=SENT):
    n = 1
    for s in shape:
        n *= s
    buf = torch.full((G + n + G,), fill, dtype=dtype, device=dev)
    return buf, buf[G:G + n].view(*shape)


def _check(buf, n, what):
    head, tail = buf[:G], buf[G + n:]
    s = torch.tensor(SENT, dtype=buf.dtype)
    assert bool((head.cpu() == s).all()), f"{what}: write before the output"
    assert bool((tail.cpu() == s).all()), f"{what}: write after the output"


@pytest.mark.parametrize("rows,hidden", [(1, 128), (7, 8192), (33, 5120)])
def test_norm_canaries(gpu, rows, hidden):
    x = torch.randn(rows, hidden, device=gpu, dtype=BF)
    w = torch.ones(hidden, device=gpu, dtype=BF)
    buf, out = _guarded((rows, hidden), BF, gpu)
    rbuf, res = _guarded((rows, hidden), BF, gpu)
    res.copy_(torch.randn_like(x))
    rob, rout = _guarded((rows, hidden), BF, gpu)
    ops.rms_norm(x, w, 1e-5, residual=res, out=out, residual_out=rout)
    torch.cuda.synchronize()
    for b, what in ((buf, "rms_norm out"), (rbuf, "residual in"), (rob, "residual out")):
        _check(b, rows * hidden, what)
    b2 = torch.zeros(hidden, device=gpu, dtype=BF)
    buf2, out2 = _guarded((rows, hidden), BF, gpu)
    ops.layer_norm(x, w, b2, 1e-5, out=out2)
    torch.cuda.synchronize()
    _check(buf2, rows * hidden, "layer_norm out")


@pytest.mark.parametrize("T,I", [(1, 128), (13, 3584), (5, 1000 * 8)])
def test_activation_canaries(gpu, T, I):
    x = torch.randn(T, 2 * I, device=gpu, dtype=BF)
    buf, out = _guarded((T, I), BF, gpu)
    ops.silu_mul(x, out=out)
    y = torch.randn(T, 2 * I, device=gpu, dtype=BF)
    buf2, out2 = _guarded((T, 2 * I), BF, gpu)
    ops.add(x, y, out=out2)
    buf3, out3 = _guarded((T, 2 * I), BF, gpu)
    ops.gelu_bias(x, torch.zeros(2 * I, device=gpu, dtype=BF), out=out3)
    torch.cuda.synchronize()
    _check(buf, T * I, "silu_mul")
    _check(buf2, T * 2 * I, "add")
    _check(buf3, T * 2 * I, "gelu_bias")


def test_rope_cache_writes_only_its_slots(gpu):
    nh, nkv, D, bs, nblocks, T = 8, 2, 128, 64, 12, 50
    qkv = torch.randn(T, (nh + 2 * nkv) * D, device=gpu, dtype=BF)
    pos = torch.arange(T, device=gpu, dtype=torch.int32)
    # the tokens land in blocks 3 and 7 only; every other block must stay at the sentinel
    slots = torch.cat([torch.arange(3 * bs, 3 * bs + 32), torch.arange(7 * bs + 5, 7 * bs + 23)])
    slots = slots.to(torch.int64).to(gpu)
    kc = torch.full((nblocks, nkv, bs, D), SENT, device=gpu, dtype=BF)
    vc = torch.full((nblocks, nkv, bs // 8, D, 8), SENT, device=gpu, dtype=BF)
    cs = ref.build_cos_sin(D, 256, 500000.0, device=gpu)
    qbuf, q_out = _guarded((T, nh, D), BF, gpu)
    ops.rope_cache(qkv, pos, slots, cs, nh, nkv, D, kc, vc, q_out=q_out)
    torch.cuda.synchronize()
    _check(qbuf, T * nh * D, "rope q_out")
    s = torch.tensor(SENT, dtype=BF)
    written = torch.zeros(nblocks * bs, dtype=torch.bool)
    written[slots.cpu()] = True
    k_slot = kc.cpu().permute(0, 2, 1, 3).reshape(nblocks * bs, -1)
    v_slot = vc.cpu().permute(0, 2, 4, 1, 3).reshape(nblocks * bs, -1)
    for name, c in (("k_cache", k_slot), ("v_cache", v_slot)):
        untouched = (c == s).all(-1)
        assert bool(untouched[~written].all()), f"{name}: write outside the slot mapping"
        assert not bool(untouched[written].any()), f"{name}: a mapped slot was not written"


@pytest.mark.parametrize("splits", [1, 3])
def test_attn_decode_canaries(gpu, splits):
    nh, nkv, D, bs, B = 64, 8, 128, 64, 5
    lens = torch.tensor([1, 70, 129, 300, 7], dtype=torch.int32)
    nb = 5
    kc = torch.randn(B * nb, nkv, bs, D, device=gpu, dtype=BF)
    vc = torch.randn(B * nb, nkv, bs // 8, D, 8, device=gpu, dtype=BF)
    bt = torch.arange(B * nb, dtype=torch.int32, device=gpu).view(B, nb)
    q = torch.randn(B, nh, D, device=gpu, dtype=BF)
    buf, out = _guarded((B, nh, D), BF, gpu)
    ops.attn_decode(q, None, kc, vc, bt, lens.to(gpu), D ** -0.5, num_splits=splits, out=out)
    torch.cuda.synchronize()
    _check(buf, B * nh * D, "attn_decode")


def test_quant_canaries(gpu):
    T, K = 9, 8192
    x = torch.randn(T, K, device=gpu, dtype=BF)
    q, s = ops.quant_rowwise(x)
    assert q.shape == (T, K) and s.shape == (T, 1)
    # the fused SwiGLU quantiser at a width that is not a multiple of its 512-thread row tile
    x2 = torch.randn(T, 2 * 1000 * 8, device=gpu, dtype=BF)
    q2, s2 = ops.silu_mul_quant(x2)
    torch.cuda.synchronize()
    deq = q2.float() * s2
    y = ref.silu_mul(x2.cpu()).float()
    assert (deq.cpu() - y).abs().max() / y.abs().max() < 0.07
