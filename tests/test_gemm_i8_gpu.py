"""int8-activation GEMM prototype (csrc/kernels/gemm3.hip W3<P_I8>): per-row int8
activations x per-row int8 re-quantized weights on v_mfma_i32_16x16x64_i8.

The kernel is checked against the exact integer math (int64 dot products of the same int8 values,
times the two row scales: the int32 MFMA sums are exact, so only the f32 epilogue rounds), and its
end-to-end error against the fp32 product of the original (Q4_K / Q6_K-dequantized) weights is
recorded: the re-quantization is a lossy format change, which is why the engine keeps the f16 path."""
import math

import numpy as np
import pytest
import torch

from mipipe.utils import quants as Q

pytestmark = pytest.mark.gpu


def nmse(a, b):
    a, b = a.double(), b.double()
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def _setup(qt, n, k, M, seed):
    from mipipe.ops.kernels import PackedWeight, I8Weight
    rng = np.random.default_rng(seed)
    wf = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(wf, qt)
    deq = torch.from_numpy(Q.dequantize(raw, qt).reshape(n, k))
    w = PackedWeight(raw, qt, n, k)
    w8 = I8Weight(w)
    g = torch.Generator().manual_seed(seed)
    xh = torch.zeros(M, w.k_pad, dtype=torch.float16)
    xh[:, :k] = torch.randn(M, k, generator=g).half()
    return w, w8, deq, xh


def test_quant_rows_i8_matches_torch(cuda, native):
    from mipipe.ops.kernels import quant_rows_i8
    x = (torch.randn(37, 768) * torch.linspace(0.1, 10, 37)[:, None]).half()
    q, xs = quant_rows_i8(x.cuda())
    s = x.float().abs().amax(1) / 127
    assert torch.allclose(xs.cpu(), s, rtol=1e-6)
    ref = torch.round(x.float() / s[:, None])
    assert (q.cpu().float() - ref).abs().max() <= 1   # f32 reciprocal vs division at exact .5 ties


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K])
@pytest.mark.parametrize("M", [65, 256, 300])
def test_gemm_i8_exact_integer_math(cuda, native, qt, M):
    from mipipe.ops.kernels import gemm_i8, quant_rows_i8, EPI_STORE, EPI_ATOMIC, EPI_SWIGLU
    n, k = 512, 2048
    w, w8, deq, xh = _setup(qt, n, k, M, 31 + M + qt)
    q, xs = quant_rows_i8(xh.cuda())
    ref = (q.cpu().long() @ w8.q[:n].cpu().long().T).double() * xs.cpu().double()[:, None] * w8.ws[:n].cpu().double()
    y = gemm_i8(w8, xq=(q, xs), epi=EPI_STORE).cpu()
    assert nmse(y, ref) < 1e-12
    base = torch.randn(M, n)
    y2 = gemm_i8(w8, xq=(q, xs), epi=EPI_ATOMIC, y=base.clone().cuda()).cpu()
    assert nmse(y2 - base, ref) < 1e-10
    h = gemm_i8(w8, xq=(q, xs), epi=EPI_SWIGLU).cpu()
    gi = torch.tensor([16 * (o // 8) + (o % 8) for o in range(n // 2)])
    href = torch.nn.functional.silu(ref[:, gi]) * ref[:, gi + 8]
    assert nmse(h.float(), href) < 1e-5
    # the format change itself: per-row int8 x and w against the fp32 product of the K-quant weights
    full = xh[:, :k].float() @ deq.T
    err = nmse(y, full)
    print(f"int8 vs fp32 ({Q.TYPE_NAMES[qt]}, M={M}): NMSE {err:.2e}")
    assert err < 1e-3
