"""Grouped MoE dequant GEMM (csrc/kernels/gemm4.hip MoE mode) and the MoE router kernels
at Mixtral-8x7B widths (d 4096, d_ff 14336, 8 experts, top-2) against a plain PyTorch fp32 oracle.

The weights are random GGUF blocks (Q4_K gate/up, Q6_K down, as in Mixtral Q4_K_M), packed by the
engine's packer; the oracle dequantizes them with the unpack kernel (itself checked against the
numpy dequantizer in test_kernels_gpu.py) and runs fp32 matmuls per routed expert.  M covers a
65-token call (16 rows per expert), the 256-sequence decode micro-batch (64 rows per expert) and a
512-token prompt chunk (128 per expert), with the default 128-row tiles and the opt-in 64- and 96-row
ones (knob GEMM4_MOE64 1 / 2), plus a skewed routing."""
import numpy as np
import pytest
import torch

from mipipe.utils import quants as Q

pytestmark = pytest.mark.gpu

D, F, E, K_TOP = 4096, 14336, 8, 2


def nmse(a, b):
    a, b = a.double(), b.double()
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def _rand_blocks(qt, n, k, rng):
    """Random, finite GGUF blocks of type qt for an [n][k] matrix (scales ~1e-4: O(1) outputs)."""
    nb = n * k // 256
    if qt == Q.Q4_K:   # d, dmin (f16), 12 B of 6-bit scales / mins, 128 B of nibbles
        blk = rng.integers(0, 256, (nb, 144), dtype=np.uint8)
        blk[:, 0:2] = (rng.uniform(0.5, 1.0, nb) * 1e-4).astype(np.float16).view(np.uint8).reshape(nb, 2)
        blk[:, 2:4] = (rng.uniform(0.0, 1.0, nb) * 1e-4).astype(np.float16).view(np.uint8).reshape(nb, 2)
        return blk.reshape(n, -1)
    assert qt == Q.Q6_K   # ql 128, qh 64, int8 scales 16, d (f16)
    blk = rng.integers(0, 256, (nb, 210), dtype=np.uint8)
    blk[:, 208:210] = (rng.uniform(0.5, 1.0, nb) * 3e-5).astype(np.float16).view(np.uint8).reshape(nb, 2)
    return blk.reshape(n, -1)


DOWN_QT = int(__import__("os").environ.get("MOE_TEST_DOWN_QT", Q.Q6_K))


@pytest.fixture(scope="module")
def experts(native):
    from mipipe.ops.kernels import PackedWeight
    rng = np.random.default_rng(11)
    gu, dn = [], []
    for _ in range(E):
        gu.append(PackedWeight(_rand_blocks(Q.Q4_K, 2 * F, D, rng), Q.Q4_K, 2 * F, D, gateup=True))
        dn.append(PackedWeight(_rand_blocks(DOWN_QT, D, F, rng), DOWN_QT, D, F))
    gu_all = torch.cat([w.dev for w in gu])
    dn_all = torch.cat([w.dev for w in dn])
    return gu, dn, gu_all, dn_all


@pytest.fixture(params=[0, 1, 2], ids=["tile128", "tile64", "tile96"])
def moe64(request, native):
    from mipipe import _native as N
    N.check(N.lib().mp_set_knob(b"GEMM4_MOE64", request.param), "knob")
    yield request.param
    N.lib().mp_set_knob(b"GEMM4_MOE64", 0)


@pytest.mark.parametrize("M", [65, 256, 512, "256skew"])
def test_moe_grouped_gemm_mixtral_widths(cuda, experts, moe64, M):
    """("256skew": expert 0 favoured, so it gets several row blocks of any tile height, e.g. three
    of the 96-row tiles, while the others run short ones.)"""
    from mipipe.ops.kernels import moe_route, moe_gemm, EPI_SWIGLU, EPI_ATOMIC
    gu, dn, gu_all, dn_all = experts
    skew = M == "256skew"
    M = 256 if skew else M
    g = torch.Generator().manual_seed(M + skew)
    logits = torch.randn(M, E, generator=g)
    if skew:
        logits[:, 0] += 2.5
    logits = logits.cuda()
    counts, lists, weights = moe_route(logits, K_TOP)
    x = torch.randn(M, gu[0].k_pad, generator=g).half().cuda()
    h = torch.zeros(M * K_TOP, dn[0].k_pad, dtype=torch.float16, device="cuda")
    moe_gemm(gu_all, gu[0].dev.numel(), gu[0].ptype, gu[0].ntiles, gu[0].nsb, F, EPI_SWIGLU, x, M, E, K_TOP,
             counts, lists, weights, h=h)
    base = torch.randn(M, D, generator=g).cuda()
    y = base.clone()
    moe_gemm(dn_all, dn[0].dev.numel(), dn[0].ptype, dn[0].ntiles, dn[0].nsb, D, EPI_ATOMIC, h, M, E, K_TOP,
             counts, lists, weights, x_per_slot=True, y=y)
    torch.cuda.synchronize()

    # routing: every token's k slots are listed exactly once, with the renormalised top-k softmax
    cnt = counts.cpu().tolist()
    assert sum(cnt) == M * K_TOP
    slots = sorted(s for e in range(E) for s in lists[e, : cnt[e]].cpu().tolist())
    assert slots == list(range(M * K_TOP))
    top = torch.topk(logits.cpu(), K_TOP, dim=1)
    wref = torch.softmax(top.values, dim=1).reshape(-1)
    assert torch.allclose(weights.cpu(), wref, atol=1e-5)

    gi = torch.tensor([16 * (o // 8) + (o % 8) for o in range(F)], device="cuda")
    y_ref = base.clone().double()
    h_err, h_ref_sq = 0.0, 0.0
    for e in range(E):
        sl = lists[e, : cnt[e]].long()
        if sl.numel() == 0:
            continue
        tok = sl // K_TOP
        assert set(top.indices[tok.cpu(), (sl % K_TOP).cpu()].tolist()) == {e}
        wg = gu[e].unpack().float()
        G = x[tok, :D].float() @ wg.T
        href = torch.nn.functional.silu(G[:, gi]) * G[:, gi + 8]
        hk = h[sl, :F].float()
        h_err += float(((hk - href) ** 2).sum())
        h_ref_sq += float((href ** 2).sum())
        wd = dn[e].unpack().float()
        yd = hk @ wd.T   # the kernel's own h as the down input: isolates the down GEMM's error
        y_ref.index_add_(0, tok, (weights[sl][:, None] * yd).double())
        del wg, wd, G
    assert h_err / h_ref_sq < 1e-4
    err = ((y - base).double() - (y_ref - base.double())).abs()
    wrong = (err > 1e-3 * (y_ref - base.double()).abs().max()).nonzero().cpu()
    if len(wrong):   # diagnostics for an intermittent mismatch (r8e): which rows / columns / experts
        rows = sorted(set(wrong[:, 0].tolist()))
        cols = wrong[:, 1]
        own = {e: len(set((lists[e, : cnt[e]] // K_TOP).tolist()) & set(rows)) for e in range(E)}
        print(f"MISMATCH M={M}: {len(wrong)} entries, rows {rows[:16]} ({len(rows)}), cols {int(cols.min())}-"
              f"{int(cols.max())} ({len(set(cols.tolist()))} distinct, by 256-col group "
              f"{sorted(set((cols // 256).tolist()))}), experts {own}, counts {cnt}", flush=True)
    assert nmse((y - base).cpu(), (y_ref - base.double()).cpu()) < 1e-5


def test_router_logits_kernel(cuda, native):
    """Dense-router logits (fixed-order reduction: bitwise repeatable) against fp32, E in {8, 60}."""
    from mipipe.ops.kernels import router_logits
    g = torch.Generator().manual_seed(3)
    for e_n, M in ((8, 1), (8, 257), (60, 33)):
        x = torch.randn(M, D, generator=g).half().cuda()
        r = (torch.randn(e_n, D, generator=g) * 0.02).half().cuda()
        out = router_logits(x, r)
        ref = x.float() @ r.float().T
        assert nmse(out.cpu(), ref.cpu()) < 1e-8
        assert torch.equal(out, router_logits(x, r))
