"""GEMM v4 (csrc/kernels/gemm4.hip, gemm3's LDS-DMA stream on the 32x32x16 MFMA) against a plain
PyTorch fp32 reference (numpy dequant of the same GGUF blocks as the oracle).

Checked: every supported weight type, both row tiles (128 / 256), partial row and column blocks,
the three epilogues, split-K by atomics and by per-split partial stores + the fixed-order
reduction (the engine's wide-decode path for qkv / o / down), the Llama-3-70B headline widths
(K = 8192 / 28672) and an exact-integer layout probe of the A / B / C lane maps."""
import math

import numpy as np
import pytest
import torch

from mipipe.utils import quants as Q

pytestmark = pytest.mark.gpu

TYPES = [Q.Q4_K, Q.Q5_K, Q.Q6_K, Q.Q8_0, Q.F16, Q.BF16]


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


def _ref(xh, k, deq, qt):
    xa = xh[:, :k].float()
    if qt == Q.BF16:   # the bf16 MFMA rounds the activations to bf16
        xa = xh[:, :k].bfloat16().float()
    return xa @ deq.T


@pytest.fixture
def tuning(native):
    from mipipe.ops.kernels import set_gemm3_tuning
    yield set_gemm3_tuning
    set_gemm3_tuning(0, 0, 0, 0)


@pytest.mark.parametrize("qt", TYPES)
@pytest.mark.parametrize("bm", [0, 96, 128, 256])
@pytest.mark.parametrize("M", [65, 200, 300])
def test_gemm4_tiles(cuda, tuning, qt, bm, M):
    """STORE / ATOMIC (auto split) / SwiGLU on 13 tiles (a partial 256-column group), 5
    super-blocks (20 stages), partial row blocks, for every row tile (96: three 32-row fragments,
    two workgroups per CU; 16-bit weights keep 128)."""
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_STORE, EPI_ATOMIC, EPI_SWIGLU
    tuning(bm, 0, 0, 0)
    n, k = 208, 1280
    raw, deq = _weights(qt, n, k, 700 + qt + M)
    w = PackedWeight(raw, qt, n, k)
    xh = _x(M, k, w.k_pad, M + 1)
    ref = _ref(xh, k, deq, qt)
    y = gemm(w, xh.cuda(), EPI_STORE, v=4)
    assert nmse(y.cpu(), ref) < 1e-5
    base = torch.randn(M, n)
    y2 = gemm(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda(), v=4)
    assert nmse(y2.cpu(), ref + base) < 1e-5
    h = gemm(w, xh.cuda(), EPI_SWIGLU, v=4)
    gi = torch.tensor([16 * (o // 8) + (o % 8) for o in range(n // 2)])
    href = torch.nn.functional.silu(ref[:, gi]) * ref[:, gi + 8]
    assert nmse(h.float().cpu(), href) < 1e-4


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K])
@pytest.mark.parametrize("shape", [(512, 8192), (256, 28672)])
@pytest.mark.parametrize("nsplit", [1, 4, 8])
@pytest.mark.parametrize("M", [65, 256, 300])
def test_gemm4_headline_widths_split(cuda, tuning, qt, shape, nsplit, M):
    """The 70B headline widths: K = 8192 (qkv / o / gate-up) and 28672 (down), ATOMIC with split-K
    forced to 1 / 4 / 8, added into a non-zero residual."""
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_ATOMIC
    tuning(0, 0, nsplit, 0)
    n, k = shape
    raw, deq = _weights(qt, n, k, 31 + qt)
    w = PackedWeight(raw, qt, n, k)
    xh = _x(M, k, w.k_pad, 9 + M)
    ref = _ref(xh, k, deq, qt)
    base = torch.randn(M, n)
    y = gemm(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda(), v=4)
    assert nmse(y.cpu() - base, ref) < 1e-5


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K])
@pytest.mark.parametrize("M", [128, 256])
def test_gemm4_splitk_partial_stores(cuda, tuning, qt, M):
    """The engine's split-K for the narrow wide-decode GEMMs: every split stores its partial tile,
    the fixed-order reduction adds them into y.  Bitwise reproducible run to run."""
    from mipipe.ops.kernels import PackedWeight, gemm_splitk
    n, k = 1024, 8192
    raw, deq = _weights(qt, n, k, 77 + qt)
    w = PackedWeight(raw, qt, n, k)
    xh = _x(M, k, w.k_pad, 3 + M).cuda()
    ref = _ref(xh.cpu(), k, deq, qt)
    base = torch.randn(M, n)
    outs = []
    for _ in range(2):
        y = base.clone().cuda()
        ns = gemm_splitk(w, xh, y)
        assert ns >= 2
        outs.append(y.cpu())
    assert nmse(outs[0] - base, ref) < 1e-5
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("bm", [128, 256])
def test_gemm4_asymmetric_identity(cuda, tuning, bm):
    """Lane-map check with exact integer data (F16 weights with an asymmetric 0/1/2 pattern,
    distinct integer rows of x): any row / column / k swap in the 32x32x16 A, B or C maps is an
    exact mismatch."""
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_STORE
    tuning(bm, 0, 0, 0)
    n, k, M = 256, 512, 256
    w_np = np.zeros((n, k), np.float32)
    for j in range(n):
        w_np[j, j] = 1.0
        w_np[j, (3 * j + 7) % k] = 2.0
    w = PackedWeight(Q.quantize(w_np, Q.F16), Q.F16, n, k)
    x = ((torch.arange(M)[:, None] * 3 + torch.arange(k)[None, :] % 17) % 64).half()
    y = gemm(w, x.cuda(), EPI_STORE, v=4).cpu()
    ref = x.float() @ torch.from_numpy(w_np).T
    assert torch.equal(y, ref)


@pytest.mark.parametrize("M", [96, 256])
def test_gemm4_matches_gemm3_q4k(cuda, native, M):
    """Same packed Q4_K weights through the 32x32 GEMM and the 16x16 GEMM v3: equal up to f32
    summation order."""
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_STORE
    n, k = 512, 4096
    raw, _ = _weights(Q.Q4_K, n, k, 5)
    w = PackedWeight(raw, Q.Q4_K, n, k)
    xh = _x(M, k, w.k_pad, 8).cuda()
    assert nmse(gemm(w, xh, EPI_STORE, v=4).cpu(), gemm(w, xh, EPI_STORE, v=3).cpu()) < 1e-8


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K, Q.Q8_0])
@pytest.mark.parametrize("nw", [7, 8])
@pytest.mark.parametrize("M", [65, 256])
def test_gemm4_seven_wave_tiles(cuda, native, qt, nw, M):
    """224-column workgroups (7 compute waves; the x pieces round-robin over 7 waves with one
    duplicate load) against 256-column ones and the oracle: 40 tiles = two full 224-column groups
    plus a partial one, STORE and SwiGLU (unsplit launches are the ones that take 7 waves)."""
    from mipipe import _native as N
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_STORE, EPI_SWIGLU
    N.check(N.lib().mp_set_knob(b"GEMM4_NW", nw), "knob")
    try:
        n, k = 640, 2048
        raw, deq = _weights(qt, n, k, 400 + qt + M)
        w = PackedWeight(raw, qt, n, k)
        xh = _x(M, k, w.k_pad, M + 7)
        ref = _ref(xh, k, deq, qt)
        y = gemm(w, xh.cuda(), EPI_STORE, v=4)
        assert nmse(y.cpu(), ref) < 1e-5
        h = gemm(w, xh.cuda(), EPI_SWIGLU, v=4)
        gi = torch.tensor([16 * (o // 8) + (o % 8) for o in range(n // 2)])
        href = torch.nn.functional.silu(ref[:, gi]) * ref[:, gi + 8]
        assert nmse(h.float().cpu(), href) < 1e-4
    finally:
        N.lib().mp_set_knob(b"GEMM4_NW", 0)


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K, Q.Q8_0])
@pytest.mark.parametrize("form", ["tw4", "nw4", "w8x64", "w7x64"])
@pytest.mark.parametrize("k", [2048, 2304])
@pytest.mark.parametrize("M", [65, 256])
def test_gemm4_four_wave_tiles(cuda, tuning, qt, form, k, M):
    """The 64-column and 4-wave forms on every tile: 4 waves x 64 columns with the accumulators in
    AGPRs (GEMM4_TW4=2; the AGPR -> VGPR epilogue copies once landed on in-flight LDS reads at the
    loop's even exit), 32 columns per wave at two workgroups per CU (GEMM4_NW=4), and 8 / 7 waves x
    64 columns on 128-row tiles (GEMM4_TW4=4, GEMM4_NW=7 for the 448-column group: 40 tiles = one
    full group plus a partial one).  An even (32) and an odd (36) stage count, STORE / SwiGLU /
    split-K ATOMIC over a non-zero residual."""
    from mipipe import _native as N
    from mipipe.ops.kernels import PackedWeight, gemm, EPI_STORE, EPI_ATOMIC, EPI_SWIGLU
    knobs = {"tw4": [(b"GEMM4_TW4", 2)], "nw4": [(b"GEMM4_NW", 4)], "w8x64": [(b"GEMM4_TW4", 4)],
             "w7x64": [(b"GEMM4_TW4", 4), (b"GEMM4_NW", 7)]}[form]
    for name, val in knobs:
        N.check(N.lib().mp_set_knob(name, val), "knob")
    try:
        n = 640
        raw, deq = _weights(qt, n, k, 900 + qt + M + k)
        w = PackedWeight(raw, qt, n, k)
        xh = _x(M, k, w.k_pad, M + 11)
        ref = _ref(xh, k, deq, qt)
        y = gemm(w, xh.cuda(), EPI_STORE, v=4)
        assert torch.isfinite(y).all() and nmse(y.cpu(), ref) < 1e-5
        h = gemm(w, xh.cuda(), EPI_SWIGLU, v=4)
        gi = torch.tensor([16 * (o // 8) + (o % 8) for o in range(n // 2)])
        href = torch.nn.functional.silu(ref[:, gi]) * ref[:, gi + 8]
        assert nmse(h.float().cpu(), href) < 1e-4
        tuning(0, 0, 3, 0)   # 3 K splits: per-split stage counts 11 / 11 / 10 or 12 / 12 / 12
        base = torch.randn(M, n)
        y2 = gemm(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda(), v=4)
        assert nmse(y2.cpu() - base, ref) < 1e-5
    finally:
        for name, _ in knobs:
            N.lib().mp_reset_knob(name)


def _ref_gpu(xh, k, deq, qt):
    """fp32 reference on the GPU (the 70B-width shapes are ~20 GFLOP each)."""
    xa = xh[:, :k].float()
    if qt == Q.BF16:
        xa = xh[:, :k].bfloat16().float()
    return (xa.cuda() @ deq.cuda().T).cpu()


# Per-split stage counts of 1, 2, 3, 4 (= the 3-buffer ring + 1) and 5 at K = 8192 (128 stages):
# the forced split count and the stage count of its LAST split.  Odd counts run the kernel's odd
# tail stage (gemm4.hip `if (s < s_end) stage(...)`), whose next-stage LDS reads are never consumed
# (tools/isa_lint.py: their registers must stay pinned until the final lgkmcnt(0)).
TAIL_SPLITS = [(128, 1), (64, 2), (43, 2), (32, 4), (26, 3), (3, 42)]


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K])
@pytest.mark.parametrize("ns_last", TAIL_SPLITS, ids=[f"ns{a}" for a, _ in TAIL_SPLITS])
@pytest.mark.parametrize("M", [65, 129, 256])
def test_gemm4_splitk_tail_stage_counts(cuda, tuning, qt, ns_last, M):
    """Split-K at 70B width K = 8192 with every per-split stage count from 1 to 5 and the odd 43
    (3 splits): ATOMIC into a residual and the per-split partial stores over a NaN-filled scratch,
    both finite and at the oracle; partial stores bitwise equal over three runs."""
    from mipipe.ops.kernels import PackedWeight, gemm, gemm_splitk, EPI_ATOMIC
    ns, _ = ns_last
    tuning(0, 0, ns, 0)
    n, k = 512, 8192
    raw, deq = _weights(qt, n, k, 900 + qt)
    w = PackedWeight(raw, qt, n, k)
    xh = _x(M, k, w.k_pad, 17 + M)
    ref = _ref_gpu(xh, k, deq, qt)
    base = torch.randn(M, n)
    y = gemm(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda(), v=4).cpu()
    assert torch.isfinite(y).all()
    assert nmse(y - base, ref) < 1e-5
    outs = []
    for _ in range(3):
        y2 = base.clone().cuda()
        got = gemm_splitk(w, xh.cuda(), y2, max_splits=ns)
        assert got == ns
        outs.append(y2.cpu())
    assert torch.isfinite(outs[0]).all()
    assert nmse(outs[0] - base, ref) < 1e-5
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("M", [65, 129, 256])
def test_gemm4_splitk_qkv_width_three_splits(cuda, tuning, M):
    """The advisor's probe shape: 70B qkv N = 10240, K = 8192, 3 splits of 43 / 43 / 42 stages (the
    odd tail in two of them), per-split partial stores over a NaN scratch: finite, every row at the
    oracle."""
    from mipipe.ops.kernels import PackedWeight, gemm_splitk
    tuning(0, 0, 3, 0)
    n, k = 10240, 8192
    raw, deq = _weights(Q.Q4_K, n, k, 4242)
    w = PackedWeight(raw, Q.Q4_K, n, k)
    xh = _x(M, k, w.k_pad, 5 + M)
    ref = _ref_gpu(xh, k, deq, Q.Q4_K)
    y = torch.zeros(M, n).cuda()
    assert gemm_splitk(w, xh.cuda(), y, max_splits=3) == 3
    y = y.cpu()
    assert torch.isfinite(y).all()
    rows = ((y - ref) ** 2).sum(1) / (ref ** 2).sum(1)
    assert float(rows.max()) < 1e-5, f"worst row {int(rows.argmax())}: {float(rows.max()):.3e}"



@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K])
@pytest.mark.parametrize("ns_last", TAIL_SPLITS, ids=[f"ns{a}" for a, _ in TAIL_SPLITS])
@pytest.mark.parametrize("M", [65, 256])
def test_gemm4_w8x64_splitk_tails(cuda, tuning, qt, ns_last, M):
    """The 8-wave x 64-column form (GEMM4_TW4=4) on the split-K partial stores with every
    per-split stage count 1-5 and 43, over a NaN-filled scratch: finite, at the oracle, bitwise
    equal run to run; and the whole-K SwiGLU at the 70B gate/up K."""
    from mipipe import _native as N
    from mipipe.ops.kernels import PackedWeight, gemm, gemm_splitk, EPI_SWIGLU
    ns, _ = ns_last
    N.check(N.lib().mp_set_knob(b"GEMM4_TW4", 4), "knob")
    try:
        tuning(0, 0, ns, 0)
        n, k = 1024, 8192
        raw, deq = _weights(qt, n, k, 1900 + qt)
        w = PackedWeight(raw, qt, n, k)
        xh = _x(M, k, w.k_pad, 27 + M)
        ref = _ref_gpu(xh, k, deq, qt)
        base = torch.randn(M, n)
        outs = []
        for _ in range(2):
            y2 = base.clone().cuda()
            assert gemm_splitk(w, xh.cuda(), y2, max_splits=ns) == ns
            outs.append(y2.cpu())
        assert torch.isfinite(outs[0]).all()
        assert nmse(outs[0] - base, ref) < 1e-5
        assert torch.equal(outs[0], outs[1])
        if ns == 128:
            tuning(0, 0, 0, 0)
            h = gemm(w, xh.cuda(), EPI_SWIGLU, v=4)
            gi = torch.tensor([16 * (o // 8) + (o % 8) for o in range(n // 2)])
            href = torch.nn.functional.silu(ref[:, gi]) * ref[:, gi + 8]
            assert torch.isfinite(h.float()).all() and nmse(h.float().cpu(), href) < 1e-4
    finally:
        N.lib().mp_reset_knob(b"GEMM4_TW4")
