"""gemm2 (the quantized types' wide-decode / prompt GEMM, csrc/kernels/gemv2.hip) at the 70B
headline widths against a plain PyTorch fp32 reference: K = 8192 (qkv / o / gate-up) and 28672
(down), split-K chosen through the GEMM2_SPLIT_WG knob (unsplit, the default 256-workgroup target,
a deep split), both with float atomics and through per-split partial stores + the fixed-order
reduction the engine uses by default (gemm_splitk_store)."""
import math

import numpy as np
import pytest
import torch

from mipipe.utils import quants as Q

pytestmark = pytest.mark.gpu


def nmse(a, b):
    a, b = a.double(), b.double()
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


@pytest.fixture
def split_wg(native):
    from mipipe import _native as N
    yield lambda v: N.check(N.lib().mp_set_knob(b"GEMM2_SPLIT_WG", v), "knob")
    N.lib().mp_set_knob(b"GEMM2_SPLIT_WG", 256)


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K, Q.Q8_0])
@pytest.mark.parametrize("shape", [(512, 8192), (256, 28672)])
@pytest.mark.parametrize("wg", [16, 256, 2048])
@pytest.mark.parametrize("M", [65, 128, 256, 300])
def test_gemm2_headline_widths_split(cuda, split_wg, qt, shape, wg, M):
    from mipipe import _native as N
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_ATOMIC, _ptr, _stream
    split_wg(wg)
    n, k = shape
    rng = np.random.default_rng(31 + qt)
    xw = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(xw, qt)
    deq = torch.from_numpy(Q.dequantize(raw, qt).reshape(n, k))
    w = PackedWeight(raw, qt, n, k)
    g = torch.Generator().manual_seed(M)
    xh = torch.zeros(M, w.k_pad, dtype=torch.float16)
    xh[:, :k] = torch.randn(M, k, generator=g).half()
    ref = xh[:, :k].float() @ deq.T
    base = torch.randn(M, n)
    # float atomics (gemm2's own split)
    y = gemm(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda(), v=2)
    assert nmse(y.cpu() - base, ref) < 1e-5
    # partial stores + fixed-order reduction: same result, bitwise reproducible
    L = N.lib()
    ns = L.mp_gemm2_splits(w.ntiles, w.nsb, M)
    scratch = torch.empty(max(1, ns) * M * w.ntiles * 16, dtype=torch.float32, device="cuda")
    xd = xh.cuda()
    outs = []
    for _ in range(2):
        y2 = base.clone().cuda()
        r = N.check(L.mp_op_gemm2_splitk(w.ptype, _ptr(w.dev), w.ntiles, w.nsb, _ptr(xd), w.k_pad, M, _ptr(y2),
                                         y2.stride(0), n, _ptr(scratch), scratch.numel(), _stream()), "gemm2_splitk")
        assert r == (1 if ns > 1 else 0)
        if r == 0:
            break
        torch.cuda.synchronize()
        outs.append(y2.cpu())
    if outs:
        assert nmse(outs[0] - base, ref) < 1e-5
        assert torch.equal(outs[0], outs[1])
