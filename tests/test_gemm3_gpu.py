"""GEMM v3 (csrc/kernels/gemm3.hip) against a plain PyTorch fp32 reference.

The v3 GEMM runs the wide (> 64-row) decode micro-batches and prompt chunks of 16-bit weights
(hip_stage.cpp HipStage::gemv picks it for F16 / BF16; quantized weights take gemm4), and
every type through prefill_gemm_v=3.  Besides small shapes in every quant type, tile shape and
epilogue, it is checked at the 70B widths (K = 8192 / 28672, split-K forced to 1, 4 and 8)."""
import math

import numpy as np
import pytest
import torch

from mipipe.utils import quants as Q

pytestmark = pytest.mark.gpu

TYPES = [Q.Q4_K, Q.Q5_K, Q.Q6_K, Q.Q8_0, Q.Q4_0, Q.F16, Q.BF16]
TILES = [(128, 128), (128, 256), (256, 128), (256, 256)]


def nmse(a, b):
    a, b = a.double(), b.double()
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def _weights(qt, n, k, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(x, qt)
    return raw, torch.from_numpy(Q.dequantize(raw, qt).reshape(n, k))


def _x(M, k, k_pad, seed):
    g = torch.Generator().manual_seed(seed)
    xh = torch.zeros(M, k_pad, dtype=torch.float16)
    xh[:, :k] = torch.randn(M, k, generator=g).half()
    return xh


@pytest.fixture
def tuning(native):
    from mipipe.ops.kernels import set_gemm3_tuning
    yield set_gemm3_tuning
    set_gemm3_tuning(0, 0, 0, 0)


@pytest.mark.parametrize("qt", TYPES)
@pytest.mark.parametrize("tile", TILES)
@pytest.mark.parametrize("M", [65, 200, 300])
def test_gemm3_tiles(cuda, tuning, qt, tile, M):
    """STORE / ATOMIC (auto split) / SwiGLU on 13 tiles (partial column group), 5 super-blocks
    (20 stages), partial row blocks, for every forced workgroup tile."""
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_STORE, EPI_ATOMIC, EPI_SWIGLU
    tuning(tile[0], tile[1], 0, 0)
    n, k = 208, 1280
    raw, deq = _weights(qt, n, k, 900 + qt + M)
    w = PackedWeight(raw, qt, n, k)
    xh = _x(M, k, w.k_pad, M)
    ref = xh[:, :k].float() @ deq.T
    y = gemm(w, xh.cuda(), EPI_STORE, v=3)
    assert nmse(y.cpu(), ref) < 1e-5
    base = torch.randn(M, n)
    y2 = gemm(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda(), v=3)
    assert nmse(y2.cpu(), ref + base) < 1e-5
    h = gemm(w, xh.cuda(), EPI_SWIGLU, v=3)
    gi = torch.tensor([16 * (o // 8) + (o % 8) for o in range(n // 2)])
    href = torch.nn.functional.silu(ref[:, gi]) * ref[:, gi + 8]
    assert nmse(h.float().cpu(), href) < 1e-4


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K, Q.Q8_0])
@pytest.mark.parametrize("shape", [(512, 8192), (256, 28672)])
@pytest.mark.parametrize("nsplit", [1, 4, 8])
@pytest.mark.parametrize("M", [65, 128, 256, 300])
def test_gemm3_headline_widths_split(cuda, tuning, qt, shape, nsplit, M):
    """The 70B headline path: K = 8192 (qkv / o / gate-up) and 28672 (down), ATOMIC epilogue with
    split-K forced to 1 / 4 / 8 over the 128 / 448 stages, added into a non-zero residual."""
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_ATOMIC
    tuning(0, 0, nsplit, 0)
    n, k = shape
    raw, deq = _weights(qt, n, k, 17 + qt)
    w = PackedWeight(raw, qt, n, k)
    xh = _x(M, k, w.k_pad, 5 + M)
    ref = xh[:, :k].float() @ deq.T
    base = torch.randn(M, n)
    y = gemm(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda(), v=3)
    assert nmse(y.cpu() - base, ref) < 1e-5


def test_gemm3_asymmetric_identity(cuda, native):
    """Layout check with exact integer data: W = [I | 2I | ...] style asymmetric pattern over f16
    weights; X rows distinct -- any row/column swap in the A/B/C maps shows as an exact mismatch."""
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_STORE
    n, k, M = 256, 512, 256
    w_np = np.zeros((n, k), np.float32)
    for j in range(n):
        w_np[j, j] = 1.0
        w_np[j, (3 * j + 7) % k] = 2.0
    w = PackedWeight(Q.quantize(w_np, Q.F16), Q.F16, n, k)
    x = torch.zeros(M, k, dtype=torch.float16)
    x[:, :] = (torch.arange(M)[:, None] * 3 + torch.arange(k)[None, :] % 17).half() % 64
    y = gemm(w, x.cuda(), EPI_STORE, v=3).cpu()
    ref = x.float() @ torch.from_numpy(w_np).T
    assert torch.equal(y, ref)


@pytest.mark.parametrize("M", [128, 256])
def test_gemm3_matches_gemv_bf16(cuda, native, M):
    """16-bit weights (packed image loaded straight into LDS, no dequant): the GEMM agrees with the
    decode GEMV on the same packed weights."""
    from mipipe.ops.kernels import PackedWeight, gemm, gemv, EPI_STORE
    n, k = 64, 256
    rng = np.random.default_rng(3)
    wf = (rng.standard_normal((n, k)) * 0.05).astype(np.float32)
    w = PackedWeight(Q.quantize(wf, Q.BF16), Q.BF16, n, k)
    xh = _x(M, k, w.k_pad, 9)
    y = gemm(w, xh.cuda(), EPI_STORE, v=3).cpu()
    y2 = torch.cat([gemv(w, xh[r:r + 64].cuda(), EPI_STORE).cpu() for r in range(0, M, 64)])
    assert nmse(y, y2) < 1e-6


@pytest.mark.parametrize("M", [1, 64, 128, 300])
def test_bf16_weights_keep_their_range(cuda, native, M):
    """BF16 weights run on the bf16 MFMA (activations rounded to bf16), never narrowed to f16: rows
    of magnitude 1e6 (past f16's 65504) and 1e-9 (below f16's subnormals) come out right in the
    decode GEMV (M <= 64) and in the GEMM (M > 64)."""
    from mipipe.ops.kernels import PackedWeight, gemm, gemv, gemv_small, EPI_STORE
    n, k = 64, 512
    rng = np.random.default_rng(11)
    wf = rng.standard_normal((n, k)).astype(np.float32)
    wf[:16] *= 1e6      # beyond f16
    wf[16:32] *= 1e-9   # below f16
    raw = Q.quantize(wf, Q.BF16)
    deq = torch.from_numpy(Q.dequantize(raw, Q.BF16).reshape(n, k))
    assert deq[:16].abs().max() > 65504 and deq[16:32].abs().max() < 6e-8
    w = PackedWeight(raw, Q.BF16, n, k)
    g = torch.Generator().manual_seed(M)
    xh = torch.zeros(M, w.k_pad, dtype=torch.float16)
    xh[:, :k] = (torch.randn(M, k, generator=g) * 1e-3).half()
    ref = xh[:, :k].bfloat16().float() @ deq.T
    ys = [(gemv(w, xh.cuda(), EPI_STORE) if M <= 64 else gemm(w, xh.cuda(), EPI_STORE, v=3)).cpu()]
    if M == 1:
        ys.append(gemv_small(w, EPI_STORE, x=xh.cuda()).cpu())   # the single-stream kernel (gemvs)
    for y in ys:
        for rows in (slice(0, 16), slice(16, 32), slice(32, 64)):
            assert torch.isfinite(y[:, rows]).all()
            assert nmse(y[:, rows], ref[:, rows]) < 1e-5, rows
