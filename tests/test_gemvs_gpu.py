"""Small-M decode GEMV (gemvs.hip, M <= 4: the single-stream path) against a plain PyTorch fp32
reference of the same op: every packed type, every epilogue, the fused RMSNorm prologue, every
work split (tiles per workgroup G, in-workgroup k-slices, k-splits over the grid), bias, ragged
N / K, determinism of the single-owner residual add, and the engine-level switch."""
import math

import numpy as np
import pytest
import torch

from mipipe.utils import quants as Q

pytestmark = pytest.mark.gpu

TYPES = [Q.Q4_K, Q.Q5_K, Q.Q6_K, Q.Q8_0, Q.Q4_0, Q.F16]


def nmse(a, b):
    a, b = a.double(), b.double()
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def _weights(qt, n, k, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(x, qt)
    return raw, torch.from_numpy(Q.dequantize(raw, qt).reshape(n, k))


def _xn(xf, gamma, eps):
    # the rmsnorm kernel's rounding point: f16(x * rsqrt(mean(x^2) + eps) * gamma)
    rs = torch.rsqrt((xf * xf).mean(-1, keepdim=True) + eps)
    return (xf * rs * gamma).half().float()


def _xh(M, k, k_pad, seed):
    g = torch.Generator().manual_seed(seed)
    xh = torch.zeros(M, k_pad, dtype=torch.float16)
    xh[:, :k] = torch.randn(M, k, generator=g).half()
    return xh


@pytest.mark.parametrize("qt", TYPES)
@pytest.mark.parametrize("M", [1, 2, 3, 4])
def test_gemvs_store_norm_bias(cuda, native, qt, M):
    from mipipe.ops.kernels import PackedWeight, gemv_small, EPI_STORE
    n, k = 200, 1792            # 13 tiles (ragged last), 7 super-blocks (uneven k-slices)
    raw, deq = _weights(qt, n, k, 3 + qt)
    w = PackedWeight(raw, qt, n, k)
    xf = torch.randn(M, k) * 3
    gamma = torch.rand(k) + 0.5
    bias = torch.randn(n)
    y = gemv_small(w, EPI_STORE, xf=xf.cuda(), gamma=gamma.cuda(), eps=1e-5, bias=bias.cuda())
    ref = _xn(xf, gamma, 1e-5) @ deq.T + bias
    assert nmse(y.cpu(), ref) < 1e-5


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K, Q.Q8_0])
@pytest.mark.parametrize("G", [1, 2, 4, 8])
@pytest.mark.parametrize("M", [1, 4])
def test_gemvs_every_tile_grouping(cuda, native, qt, G, M):
    """G tiles per 8-wave workgroup: 8/G waves split each tile's k-range (reduced through LDS)."""
    from mipipe.ops.kernels import PackedWeight, gemv_small, EPI_STORE
    n, k = 136, 4096
    raw, deq = _weights(qt, n, k, 17)
    w = PackedWeight(raw, qt, n, k)
    xh = _xh(M, k, w.k_pad, 5)
    y = gemv_small(w, EPI_STORE, x=xh.cuda(), G=G)
    assert nmse(y.cpu(), xh[:, :k].float() @ deq.T) < 1e-5


@pytest.mark.parametrize("qt", TYPES)
@pytest.mark.parametrize("nsplit", [0, 1, 2, 3, 7])
def test_gemvs_residual_add(cuda, native, qt, nsplit):
    """ATOMIC: y += W x (single owner at one k-split, atomics when k is split over the grid)."""
    from mipipe.ops.kernels import PackedWeight, gemv_small, EPI_ATOMIC
    n, k, M = 96, 1792, 2
    raw, deq = _weights(qt, n, k, 29 + qt)
    w = PackedWeight(raw, qt, n, k)
    xh = _xh(M, k, w.k_pad, 8)
    base = torch.randn(M, n)
    y = gemv_small(w, EPI_ATOMIC, x=xh.cuda(), y=base.clone().cuda(), nsplit=nsplit)
    assert nmse(y.cpu(), base + xh[:, :k].float() @ deq.T) < 1e-5


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q5_K, Q.Q8_0])
@pytest.mark.parametrize("M", [1, 3])
def test_gemvs_swiglu_norm(cuda, native, qt, M):
    from mipipe.ops.kernels import PackedWeight, gemv_small, EPI_SWIGLU
    F, k = 72, 1024
    rng = np.random.default_rng(9)
    g = (rng.standard_normal((F, k)) / math.sqrt(k)).astype(np.float32)
    u = (rng.standard_normal((F, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(np.concatenate([g, u]), qt)
    deq = torch.from_numpy(Q.dequantize(raw, qt).reshape(2 * F, k))
    w = PackedWeight(raw, qt, 2 * F, k, gateup=True)
    xf = torch.randn(M, k)
    gamma = torch.rand(k) + 0.5
    h = gemv_small(w, EPI_SWIGLU, xf=xf.cuda(), gamma=gamma.cuda(), eps=1e-5)
    xn = _xn(xf, gamma, 1e-5)
    ref = torch.nn.functional.silu(xn @ deq[:F].T) * (xn @ deq[F:].T)
    assert nmse(h.float().cpu(), ref) < 1e-5


def test_gemvs_matches_rmsnorm_plus_gemv(cuda, native):
    """Fused norm prologue == standalone rmsnorm kernel + v2 GEMV (same f16 rounding point).  The
    single-row dot form takes q unrounded (the MFMA forms round each weight to f16), so the
    comparison runs the MFMA form (GEMVS_DOT 0); the dot form is checked against the oracle."""
    from mipipe import _native as N
    from mipipe.ops.kernels import PackedWeight, gemv, gemv_small, rmsnorm, EPI_STORE
    n, k, M = 256, 4096, 1
    raw, deq = _weights(Q.Q4_K, n, k, 41)
    w = PackedWeight(raw, Q.Q4_K, n, k)
    xf = (torch.randn(M, k) * 2).cuda()
    gamma = (torch.rand(k) + 0.5).cuda()
    N.check(N.lib().mp_set_knob(b"GEMVS_DOT", 0), "knob")
    try:
        y1 = gemv_small(w, EPI_STORE, xf=xf, gamma=gamma, eps=1e-6)
    finally:
        N.lib().mp_reset_knob(b"GEMVS_DOT")
    y2 = gemv(w, rmsnorm(xf, gamma, 1e-6, w.k_pad), EPI_STORE)
    torch.testing.assert_close(y1, y2, rtol=1e-4, atol=1e-4 * float(y2.abs().max()))


def test_gemvs_ragged_k_and_long_k(cuda, native):
    """K with a zero tail (896 -> 1024 padded) under the norm, and a long K (14336, the 8B down
    projection) whose k-range fills most of the x LDS image."""
    from mipipe.ops.kernels import PackedWeight, gemv_small, EPI_STORE, EPI_ATOMIC
    raw, deq = _weights(Q.Q8_0, 48, 896, 21)
    w = PackedWeight(raw, Q.Q8_0, 48, 896)
    xf = torch.randn(2, 896)
    gamma = torch.rand(896) + 0.5
    y = gemv_small(w, EPI_STORE, xf=xf.cuda(), gamma=gamma.cuda(), eps=1e-5)
    assert nmse(y.cpu(), _xn(xf, gamma, 1e-5) @ deq.T) < 1e-5
    raw, deq = _weights(Q.Q6_K, 64, 14336, 22)
    w = PackedWeight(raw, Q.Q6_K, 64, 14336)
    xh = _xh(4, 14336, w.k_pad, 3)
    base = torch.randn(4, 64)
    y = gemv_small(w, EPI_ATOMIC, x=xh.cuda(), y=base.clone().cuda())
    assert nmse(y.cpu(), base + xh[:, :14336].float() @ deq.T) < 1e-5


def test_gemvs_single_owner_add_is_deterministic(cuda, native):
    from mipipe.ops.kernels import PackedWeight, gemv_small, EPI_ATOMIC
    n, k = 512, 8192
    raw, _ = _weights(Q.Q4_K, n, k, 2)
    w = PackedWeight(raw, Q.Q4_K, n, k)
    xh = _xh(1, k, w.k_pad, 4).cuda()
    base = torch.randn(1, n).cuda()
    a = gemv_small(w, EPI_ATOMIC, x=xh, y=base.clone(), deterministic=True)
    b = gemv_small(w, EPI_ATOMIC, x=xh, y=base.clone(), deterministic=True)
    assert torch.equal(a, b)


def test_gemvs_rejects_bad_shapes(cuda, native):
    from mipipe.ops.kernels import PackedWeight, gemv_small, EPI_STORE
    raw, _ = _weights(Q.Q4_K, 32, 256, 1)
    w = PackedWeight(raw, Q.Q4_K, 32, 256)
    with pytest.raises(RuntimeError):
        gemv_small(w, EPI_STORE, x=_xh(5, 256, w.k_pad, 1).cuda())     # M > 4
    raw, _ = _weights(Q.Q4_K, 32, 1024, 1)
    w = PackedWeight(raw, Q.Q4_K, 32, 1024)
    with pytest.raises(RuntimeError):
        gemv_small(w, EPI_STORE, x=_xh(1, 1024, w.k_pad, 1).cuda(), nsplit=2)   # STORE cannot split K


@pytest.mark.parametrize("name,ftype", [("tiny-gqa", "Q4_K"), ("tiny-qwen2", "Q4_K"), ("tiny-moe", "Q4_K"),
                                        ("tiny-gqa", "Q4_K_M"), ("tiny-qwen2", "Q4_K_M")])
def test_engine_small_gemv_matches_v2_path(cuda, native, model_dir, name, ftype):
    """Single-stream engine logits with the gemvs path (default) vs the v2 GEMV + rmsnorm path.
    Q4_K_M: the layers whose attn_v is Q6_K take the two-segment q+k | v launch (gemvs2)."""
    from conftest import make_model
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, name, ftype)
    prompts = [[3, 4, 5, 6, 7], [9, 10]]
    outs = {}
    for sg in (True, False):
        with Engine(gguf=path, max_ctx=64, mb_size=2, small_gemv=sg) as eng:
            eng.start(prompts)
            lg = eng.logits(2).copy()
            toks, _ = eng.generate(prompts, 6)
        outs[sg] = (lg, toks)
    a, b = outs[True][0].astype(np.float64), outs[False][0].astype(np.float64)
    assert ((a - b) ** 2).sum() / (b ** 2).sum() < 1e-5
    assert outs[True][1] == outs[False][1]


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q5_K, Q.Q6_K, Q.Q8_0])
@pytest.mark.parametrize("case", ["store_norm", "atomic_split", "swiglu", "long_k"])
def test_gemvs_single_row_dot_form(cuda, native, qt, case):
    """M = 1 on the v_dot2 form (knob GEMVS_DOT, dequant.h dot1: biased magic pairs, per-sub-block
    bias correction from the staged x) against the fp32 oracle and against the MFMA form: every
    epilogue, k split over the grid (atomics), ragged N / K and a 14336-wide K."""
    from mipipe import _native as N
    from mipipe.ops.kernels import PackedWeight, gemv_small, EPI_STORE, EPI_ATOMIC, EPI_SWIGLU
    n, k = (200, 1792) if case != "long_k" else (72, 14336)
    if case == "swiglu":
        n = 144
    raw, deq = _weights(qt, n, k, 41 + qt)
    w = PackedWeight(raw, qt, n, k, gateup=case == "swiglu")
    xf = torch.randn(1, k) * 3
    gamma = torch.rand(k) + 0.5
    xh = _xh(1, k, w.k_pad, 13)
    base = torch.randn(1, n)
    outs = []
    try:
        for dot in (1, 0):
            N.check(N.lib().mp_set_knob(b"GEMVS_DOT", dot), "knob")
            if case == "store_norm":
                outs.append(gemv_small(w, EPI_STORE, xf=xf.cuda(), gamma=gamma.cuda(), eps=1e-5).cpu())
            elif case in ("atomic_split", "long_k"):
                outs.append(gemv_small(w, EPI_ATOMIC, x=xh.cuda(), y=base.clone().cuda(),
                                       nsplit=3 if case == "atomic_split" else 0).cpu() - base)
            else:
                outs.append(gemv_small(w, EPI_SWIGLU, xf=xf.cuda(), gamma=gamma.cuda(), eps=1e-5).float().cpu())
    finally:
        N.lib().mp_reset_knob(b"GEMVS_DOT")
    if case == "store_norm":
        ref = _xn(xf, gamma, 1e-5) @ deq.T
    elif case == "swiglu":
        xn = _xn(xf, gamma, 1e-5)
        F = n // 2
        ref = torch.nn.functional.silu(xn @ deq[:F].T) * (xn @ deq[F:].T)
    else:
        ref = xh[:, :k].float() @ deq.T
    assert torch.isfinite(outs[0]).all()
    assert nmse(outs[0], ref) < 1e-5, nmse(outs[0], ref)
    assert nmse(outs[0], outs[1]) < 1e-5
