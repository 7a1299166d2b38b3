"""GEMV fusions (gemv2.hip: RMSNorm prologue at M <= 4, bias, zero-fill side job) and the two-level
argmax, each against a plain PyTorch fp32 reference of the same op."""
import math

import numpy as np
import pytest
import torch

from mipipe.utils import quants as Q

pytestmark = pytest.mark.gpu


def nmse(a, b):
    a, b = a.double(), b.double()
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def _weights(qt, n, k, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(x, qt)
    return raw, torch.from_numpy(Q.dequantize(raw, qt).reshape(n, k))


def _xg_f16(xf, gamma):
    # the deferred norm's rounding point: f16(x * gamma); rsqrt(mean(x^2) + eps) scales the output
    return (xf * gamma).half().float()


def _rs(xf, eps):
    return torch.rsqrt((xf * xf).mean(-1, keepdim=True) + eps)


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q5_K, Q.Q6_K, Q.Q8_0, Q.Q4_0, Q.F16])
@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("nsplit", [1, 3, 7])
def test_gemv_fused_atomic_fused_norm_bias(cuda, native, qt, M, nsplit):
    from mipipe.ops.kernels import PackedWeight, gemv_fused, EPI_ATOMIC
    n, k = 96, 1792   # 7 super-blocks: uneven splits
    raw, deq = _weights(qt, n, k, 11 + qt)
    w = PackedWeight(raw, qt, n, k)
    xf = torch.randn(M, k) * 4
    gamma = torch.rand(k) + 0.5
    bias = torch.randn(n)
    base = torch.randn(M, n)
    ssq = torch.full((M,), 3.0).cuda()
    y = gemv_fused(w, EPI_ATOMIC, xf=xf.cuda(), gamma=gamma.cuda(), eps=1e-5, bias=bias.cuda(),
                   y=base.clone().cuda(), nsplit=nsplit, ssq=ssq)
    # ATOMIC: unscaled accumulation + bias; the sums of squares are published for the consumer
    ref = base + _xg_f16(xf, gamma) @ deq.T + bias
    assert nmse(y.cpu(), ref) < 1e-5
    torch.testing.assert_close(ssq.cpu(), 3.0 + (xf.double() ** 2).sum(-1).float(), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K])
@pytest.mark.parametrize("M", [1, 4])
def test_gemv_fused_store_norm_matches_unfused(cuda, native, qt, M):
    """Fused norm + GEMV == rmsnorm kernel + GEMV (same f16 rounding point), up to summation order."""
    from mipipe.ops.kernels import PackedWeight, gemv, gemv_fused, rmsnorm, EPI_STORE
    n, k = 200, 4096
    raw, deq = _weights(qt, n, k, 3)
    w = PackedWeight(raw, qt, n, k)
    xf = (torch.randn(M, k) * 2).cuda()
    gamma = (torch.rand(k) + 0.5).cuda()
    y1 = gemv_fused(w, EPI_STORE, xf=xf, gamma=gamma, eps=1e-6)
    y2 = gemv(w, rmsnorm(xf, gamma, 1e-6, w.k_pad), EPI_STORE)
    # different f16 rounding points (x*g vs x*rs*g): equal to f16 precision
    torch.testing.assert_close(y1, y2, rtol=2e-3, atol=2e-3 * float(y2.abs().max()))
    ref = _rs(xf.cpu(), 1e-6) * (_xg_f16(xf.cpu(), gamma.cpu()) @ deq.T)
    assert nmse(y1.cpu(), ref) < 1e-6


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q8_0])
@pytest.mark.parametrize("M", [1, 3])
def test_gemv_fused_swiglu_fused_norm(cuda, native, qt, M):
    from mipipe.ops.kernels import PackedWeight, gemv_fused, EPI_SWIGLU
    F, k = 72, 1024
    rng = np.random.default_rng(9)
    g = (rng.standard_normal((F, k)) / math.sqrt(k)).astype(np.float32)
    u = (rng.standard_normal((F, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(np.concatenate([g, u]), qt)
    deq = torch.from_numpy(Q.dequantize(raw, qt).reshape(2 * F, k))
    w = PackedWeight(raw, qt, 2 * F, k, gateup=True)
    xf = torch.randn(M, k)
    gamma = torch.rand(k) + 0.5
    h = gemv_fused(w, EPI_SWIGLU, xf=xf.cuda(), gamma=gamma.cuda(), eps=1e-5)
    xg, rs = _xg_f16(xf, gamma), _rs(xf, 1e-5)
    ref = torch.nn.functional.silu(rs * (xg @ deq[:F].T)) * (rs * (xg @ deq[F:].T))
    assert nmse(h.float().cpu(), ref) < 1e-5


def test_gemv_fused_nonmultiple_d_and_zero_fill(cuda, native):
    """d not a multiple of 256 (zero K tail) and the zero-fill side job (odd length)."""
    from mipipe.ops.kernels import PackedWeight, gemv_fused, EPI_STORE
    n, k = 48, 896
    raw, deq = _weights(Q.Q8_0, n, k, 21)
    w = PackedWeight(raw, Q.Q8_0, n, k)
    xf = torch.randn(2, k)
    gamma = torch.rand(k) + 0.5
    junk = torch.randn(12345).cuda()
    y = gemv_fused(w, EPI_STORE, xf=xf.cuda(), gamma=gamma.cuda(), eps=1e-5, zero=junk)
    ref = _rs(xf, 1e-5) * (_xg_f16(xf, gamma) @ deq.T)
    assert nmse(y.cpu(), ref) < 1e-5
    torch.cuda.synchronize()
    assert int((junk != 0).sum()) == 0


@pytest.mark.parametrize("M", [5, 40])
def test_gemv_bias_zero_any_m(cuda, native, M):
    """bias / zero-fill without the norm work at every row count."""
    from mipipe.ops.kernels import PackedWeight, gemv_fused, EPI_ATOMIC
    n, k = 64, 1024
    raw, deq = _weights(Q.Q4_K, n, k, 5)
    w = PackedWeight(raw, Q.Q4_K, n, k)
    xh = torch.zeros(M, w.k_pad, dtype=torch.float16)
    xh[:, :k] = torch.randn(M, k).half()
    bias = torch.randn(n)
    junk = torch.randn(777).cuda()
    y = gemv_fused(w, EPI_ATOMIC, x=xh.cuda(), bias=bias.cuda(), nsplit=3, zero=junk)
    assert nmse(y.cpu(), xh[:, :k].float() @ deq.T + bias) < 1e-5
    torch.cuda.synchronize()
    assert int((junk != 0).sum()) == 0


@pytest.mark.parametrize("M,n", [(1, 128256), (3, 32000), (64, 128256), (5, 100), (2, 7)])
def test_argmax_two_level(cuda, native, M, n):
    from mipipe.ops.kernels import argmax
    logits = torch.randn(M, n + 16).cuda()     # padded row stride like the engine's logits
    view = logits[:, :n]
    got = argmax(view).cpu()
    ref = view.cpu().argmax(-1).int()
    assert torch.equal(got, ref)
    # repeat: the arrival counters reset themselves
    assert torch.equal(argmax(view).cpu(), ref)


def test_argmax_ties_lowest_index(cuda, native):
    from mipipe.ops.kernels import argmax
    n = 50000
    logits = torch.zeros(3, n)
    logits[0, [7, 30000, 49999]] = 5.0
    logits[1, [40000, 2049]] = 1.0
    logits[2] = -1.0
    got = argmax(logits.cuda()).cpu().tolist()
    assert got == [7, 2049, 0]
    assert argmax(logits.cuda(), two_level=False).cpu().tolist() == [7, 2049, 0]
