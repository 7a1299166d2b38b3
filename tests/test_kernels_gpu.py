"""T1 kernel tests (test-backend-ops style): every HIP kernel vs a plain PyTorch fp32 reference."""
import math

import numpy as np
import pytest
import torch

from mipipe.utils import quants as Q

pytestmark = pytest.mark.gpu

QTYPES = [Q.F16, Q.BF16, Q.F32, Q.Q8_0, Q.Q4_0, Q.Q4_K, Q.Q5_K, Q.Q6_K]


def nmse(a, b):
    a, b = a.double(), b.double()
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def _weights(qt, n, k, seed):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((n, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(x, qt)
    deq = torch.from_numpy(Q.dequantize(raw, qt).reshape(n, k))
    return raw, deq


@pytest.mark.parametrize("qt", QTYPES)
def test_unpack_matches_dequant(cuda, native, qt):
    from mipipe.ops.kernels import PackedWeight
    n, k = 48, 768
    raw, deq = _weights(qt, n, k, qt)
    w = PackedWeight(raw, qt, n, k)
    got = w.unpack().float().cpu()
    # f16 products/rounding inside the dequantizer
    torch.testing.assert_close(got, deq, rtol=2e-3, atol=2e-3 * deq.abs().max().item())


@pytest.mark.parametrize("qt", QTYPES)
@pytest.mark.parametrize("M", [1, 3, 16, 17, 32, 45, 64, 70])
def test_gemv_store(cuda, native, qt, M):
    from mipipe.ops.kernels import PackedWeight, gemv, EPI_STORE
    n, k = 80, 1024
    raw, deq = _weights(qt, n, k, 100 + qt)
    w = PackedWeight(raw, qt, n, k)
    x = torch.randn(M, k)
    xh = torch.zeros(M, w.k_pad, dtype=torch.float16)
    xh[:, :k] = x.half()
    y = gemv(w, xh.cuda(), EPI_STORE)
    ref = xh[:, :k].float() @ deq.T
    assert nmse(y.cpu(), ref) < 1e-5


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q6_K, Q.Q8_0, Q.F16])
@pytest.mark.parametrize("nsplit", [1, 3, 8])
@pytest.mark.parametrize("M", [5, 29, 61])
def test_gemv_atomic_split(cuda, native, qt, nsplit, M):
    from mipipe.ops.kernels import PackedWeight, gemv, EPI_ATOMIC
    n, k = 64, 2048
    raw, deq = _weights(qt, n, k, 7)
    w = PackedWeight(raw, qt, n, k)
    xh = torch.randn(M, k).half()
    base = torch.randn(M, n)
    y = gemv(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda(), nsplit=nsplit)
    ref = base + xh.float() @ deq.T
    assert nmse(y.cpu(), ref) < 1e-5


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q5_K, Q.Q8_0])
@pytest.mark.parametrize("M", [4, 32, 48, 64])
def test_gemv_swiglu(cuda, native, qt, M):
    from mipipe.ops.kernels import PackedWeight, gemv, EPI_SWIGLU
    F, k = 40, 512
    rng = np.random.default_rng(5)
    g = (rng.standard_normal((F, k)) / math.sqrt(k)).astype(np.float32)
    u = (rng.standard_normal((F, k)) / math.sqrt(k)).astype(np.float32)
    raw = Q.quantize(np.concatenate([g, u]), qt)
    deq = torch.from_numpy(Q.dequantize(raw, qt).reshape(2 * F, k))
    w = PackedWeight(raw, qt, 2 * F, k, gateup=True)
    xh = torch.randn(M, k).half()
    h = gemv(w, xh.cuda(), EPI_SWIGLU)
    gg = xh.float() @ deq[:F].T
    uu = xh.float() @ deq[F:].T
    ref = torch.nn.functional.silu(gg) * uu
    assert nmse(h.float().cpu(), ref) < 1e-5


@pytest.mark.parametrize("M", [1, 64, 200])
def test_swiglu_saturates_instead_of_inf(cuda, native, M):
    """A gate/up pair whose SwiGLU product passes f16's 65504 (massive-activation channels):
    the f16 intermediate saturates at +-65504 instead of becoming inf (decode GEMV for M <= 64,
    prompt GEMM above); the in-range columns stay exact."""
    from mipipe.ops.kernels import PackedWeight, gemv, gemm, EPI_SWIGLU
    F, k = 16, 256
    g = np.zeros((F, k), np.float32)
    u = np.zeros((F, k), np.float32)
    g[:8, 0], u[:8, 0] = 60.0, 60.0          # 8 saturating outputs: silu(60 x) * 60 x >> 65504 for x = 10
    g[8:, 1], u[8:, 1] = 0.5, 0.25           # 8 ordinary outputs
    raw = Q.quantize(np.concatenate([g, u]), Q.F16)
    w = PackedWeight(raw, Q.F16, 2 * F, k, gateup=True)
    xh = torch.zeros(M, k, dtype=torch.float16)
    xh[:, 0], xh[:, 1] = 10.0, 2.0
    h = (gemv(w, xh.cuda(), EPI_SWIGLU) if M <= 64 else gemm(w, xh.cuda(), EPI_SWIGLU)).float().cpu()
    assert torch.isfinite(h).all()
    assert (h[:, :8] == 65504.0).all()
    ref = torch.nn.functional.silu(torch.tensor(1.0)) * 0.5
    torch.testing.assert_close(h[:, 8:], ref.expand(M, 8), rtol=2e-3, atol=1e-4)


def test_gemv_asymmetric_identity(cuda, native):
    """A = I style check with an asymmetric operand (catches transposed C writes)."""
    from mipipe.ops.kernels import PackedWeight, gemv
    n, k = 16, 256
    wmat = np.zeros((n, k), np.float32)
    for i in range(n):
        wmat[i, i] = 1.0 + i
        wmat[i, (7 * i + 3) % k] = -0.5 * i
    raw = Q.quantize(wmat, Q.F16)
    w = PackedWeight(raw, Q.F16, n, k)
    x = torch.zeros(16, k, dtype=torch.float16)
    for m in range(16):
        x[m, m] = 1.0
        x[m, 100 + m] = 2.0 * m
    y = gemv(w, x.cuda()).cpu()
    ref = x.float() @ torch.from_numpy(wmat).T
    torch.testing.assert_close(y, ref)


def test_rmsnorm(cuda, native):
    from mipipe.ops.kernels import rmsnorm
    x = torch.randn(7, 4096) * 3
    w = torch.rand(4096) + 0.5
    out = rmsnorm(x.cuda(), w.cuda(), 1e-5).float().cpu()[:, :4096]
    ref = x * torch.rsqrt((x * x).mean(-1, keepdim=True) + 1e-5) * w
    torch.testing.assert_close(out, ref, rtol=2e-3, atol=2e-3)
    out2 = rmsnorm(x[:, :288].contiguous().cuda(), w[:288].contiguous().cuda(), 1e-5).float().cpu()
    assert out2.shape[1] == 512 and (out2[:, 288:] == 0).all()


@pytest.mark.parametrize("qt", QTYPES)
def test_embed(cuda, native, qt):
    from mipipe.ops.kernels import embed
    V, d = 50, 512
    raw, deq = _weights(qt, V, d, 9)
    tok = torch.tensor([3, 0, 49, 17], dtype=torch.int32)
    x = embed(torch.from_numpy(raw).cuda(), qt, d, tok.cuda()).cpu()
    torch.testing.assert_close(x, deq[tok.long()], rtol=1e-5, atol=1e-6)


def test_argmax(cuda, native):
    from mipipe.ops.kernels import argmax
    x = torch.randn(5, 128256)
    x[2, 77777] = 100
    x[4, :] = 1.0          # ties -> lowest index
    out = argmax(x.cuda()).cpu()
    ref = x.argmax(-1).int()
    assert out.tolist() == ref.tolist()


def test_sample_distribution(cuda, native):
    from mipipe.ops.kernels import sample
    V = 1000
    logits = torch.full((1, V), -20.0)
    logits[0, [3, 10, 500]] = torch.tensor([2.0, 1.0, 0.0])
    cnt = {}
    for s in range(400):
        t = int(sample(logits.cuda(), temp=1.0, seed=s).item())
        cnt[t] = cnt.get(t, 0) + 1
    assert set(cnt) <= {3, 10, 500}
    p = torch.softmax(torch.tensor([2.0, 1.0, 0.0]), 0)
    assert abs(cnt.get(3, 0) / 400 - p[0].item()) < 0.1
    # top-k = 1 is greedy; top-p small keeps only the max
    assert int(sample(logits.cuda(), temp=1.0, top_k=1, seed=1).item()) == 3
    assert int(sample(logits.cuda(), temp=1.0, top_p=0.3, seed=2).item()) == 3
    assert int(sample(logits.cuda(), temp=0.0).item()) == 3


def test_sample_cut_order(cuda, native):
    """llama.cpp chain semantics: min-p / top-p cut the T = 1 distribution, the draw uses T."""
    from mipipe.ops.kernels import sample
    V = 1000
    logits = torch.full((1, V), -20.0)
    logits[0, [3, 10, 500]] = torch.tensor([2.0, 1.0, 0.0])
    cnt = {}
    for s in range(600):
        # T = 1 relative probs (1, .37, .14): min-p 0.3 drops token 500 even though at T = 2 it is .37
        t = int(sample(logits.cuda(), temp=2.0, min_p=0.3, seed=s).item())
        cnt[t] = cnt.get(t, 0) + 1
    assert set(cnt) <= {3, 10}
    p3 = 1.0 / (1.0 + math.exp(-0.5))            # softmax([2, 1] / 2)[0]
    assert abs(cnt.get(3, 0) / 600 - p3) < 0.08
    # top-p 0.6 at T = 1: the max alone holds .665 -> always token 3, whatever T
    assert {int(sample(logits.cuda(), temp=3.0, top_p=0.6, seed=s).item()) for s in range(40)} == {3}


def test_penalize_and_history(cuda, native):
    from mipipe.ops.kernels import penalize, hist_push
    M, V, L = 3, 300, 8
    g = torch.Generator().manual_seed(0)
    logits = torch.randn(M, V, generator=g) * 3
    hist = torch.full((M, L), -1, dtype=torch.int32)
    hist[0, :5] = torch.tensor([7, 7, 250, 3, 7], dtype=torch.int32)
    hist[1, :] = torch.tensor([1, 2, 3, 4, 1, 2, 1, 299], dtype=torch.int32)
    rep, fq, pr = 1.3, 0.25, 0.5
    ref = logits.clone()
    for m in range(M):
        toks = [int(t) for t in hist[m] if t >= 0]
        for t in set(toks):
            c = toks.count(t)
            l = float(ref[m, t])
            l = l / rep if l > 0 else l * rep
            ref[m, t] = l - c * fq - pr
    got = penalize(logits.cuda(), hist.cuda(), rep, fq, pr).cpu()
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-6)
    # ring append
    h = hist.cuda()
    cnt = torch.tensor([5, 8, 0], dtype=torch.int32, device="cuda")
    hist_push(h, cnt, torch.tensor([11, 12, 13], dtype=torch.int32, device="cuda"))
    h = h.cpu()
    assert int(h[0, 5]) == 11 and int(h[1, 0]) == 12 and int(h[2, 0]) == 13
    assert cnt.cpu().tolist() == [6, 9, 1]


def _ref_attention(q, k, v, kvlen):
    # q [M, Hq, hd], k/v [S, Hkv, hd]; row m attends keys [0, kvlen[m])
    M, Hq, hd = q.shape
    Hkv = k.shape[1]
    G = Hq // Hkv
    out = torch.zeros(M, Hq, hd)
    for m in range(M):
        L = int(kvlen[m])
        for h in range(Hq):
            s = (k[:L, h // G].double() @ q[m, h].double()) / math.sqrt(hd)
            p = torch.softmax(s, 0)
            out[m, h] = (p[:, None] * v[:L, h // G].double()).sum(0).float()
    return out


@pytest.mark.parametrize("hd,Hq,Hkv", [(128, 32, 8), (64, 32, 4), (48, 6, 6), (128, 64, 8)])
@pytest.mark.parametrize("mode", ["decode", "prefill"])
def test_rope_kv_attention(cuda, native, hd, Hq, Hkv, mode):
    from mipipe.ops.kernels import rope_kv, attention, rope_cs_table
    torch.manual_seed(hd + Hq)
    Dp = 64 if hd <= 64 else 128
    max_ctx, n_slots = 512, 3
    pages = max_ctx // 64
    bt = torch.arange(n_slots * pages, dtype=torch.int32).reshape(n_slots, pages)
    bt = bt[:, torch.randperm(pages)].contiguous()          # non-trivial page order
    kc = torch.zeros(n_slots * pages, Hkv, 64, Dp, dtype=torch.float16).cuda()
    vc = torch.zeros(n_slots * pages, Hkv, Dp, 64, dtype=torch.float16).cuda()
    cs = rope_cs_table(max_ctx, hd, 10000.0).cuda()
    slot_id = 1
    S = 300                                                   # tokens in the sequence
    qkv = torch.randn(S, (Hq + 2 * Hkv) * hd)
    pos = torch.arange(S, dtype=torch.int32)
    slot = torch.full((S,), slot_id, dtype=torch.int32)
    q = rope_kv(qkv.cuda(), pos.cuda(), slot.cuda(), bt.cuda(), cs, Hq, Hkv, hd, Dp, 1 / math.sqrt(hd), kc, vc)
    # reference rope
    inv = 10000.0 ** (-torch.arange(0, hd, 2, dtype=torch.float64) / hd)
    ang = pos.double()[:, None] * inv[None]
    c, s_ = torch.cos(ang).float(), torch.sin(ang).float()

    def rope(x):
        x0, x1 = x[..., 0::2], x[..., 1::2]
        o = torch.empty_like(x)
        o[..., 0::2] = x0 * c[:, None] - x1 * s_[:, None]
        o[..., 1::2] = x0 * s_[:, None] + x1 * c[:, None]
        return o
    qr = rope(qkv[:, :Hq * hd].view(S, Hq, hd))
    kr = rope(qkv[:, Hq * hd:(Hq + Hkv) * hd].view(S, Hkv, hd))
    vr = qkv[:, (Hq + Hkv) * hd:].view(S, Hkv, hd)
    torch.testing.assert_close(q.float().cpu()[:, :, :hd], qr / math.sqrt(hd), rtol=2e-3, atol=2e-3)
    assert (q.float().cpu()[:, :, hd:] == 0).all()
    # K/V pages hold the roped keys / values at the block-table positions
    kcc, vcc = kc.float().cpu(), vc.float().cpu()
    for p_ in [0, 63, 64, 200, 299]:
        page = bt[slot_id, p_ // 64]
        torch.testing.assert_close(kcc[page, :, p_ % 64, :hd], kr[p_], rtol=2e-3, atol=2e-3)
        torch.testing.assert_close(vcc[page, :, :hd, p_ % 64], vr[p_], rtol=2e-3, atol=2e-3)
    kref, vref = kr.half().float(), vr.half().float()
    if mode == "decode":
        # 4 sequences all in slot 1 at different lengths (decode rows of one micro-batch)
        lens = torch.tensor([1, 64, 257, 300], dtype=torch.int32)
        M = 4
        qd = q[lens.long() - 1].contiguous()
        for n_split, split_len in [(1, 512), (3, 128)]:
            out = attention(qd, lens.cuda(), torch.full((M,), slot_id, dtype=torch.int32).cuda(), bt.cuda(), kc, vc,
                            Hkv, hd, tq=1, split_len=split_len, n_split=n_split).float().cpu()
            ref = _ref_attention(qd.float().cpu()[:, :, :hd] * math.sqrt(hd), kref, vref, lens)
            torch.testing.assert_close(out.view(M, Hq, hd), ref, rtol=5e-3, atol=5e-3)
    else:
        G = Hq // Hkv
        tq = max(1, 16 // G)
        kvlen = pos + 1
        out = attention(q, kvlen.cuda(), slot.cuda(), bt.cuda(), kc, vc, Hkv, hd, tq=tq, split_len=512,
                        n_split=1).float().cpu()
        idx = torch.tensor([0, 1, 63, 64, 150, 299])
        ref = _ref_attention(q.float().cpu()[idx][:, :, :hd] * math.sqrt(hd), kref, vref, kvlen[idx])
        torch.testing.assert_close(out.view(S, Hq, hd)[idx], ref, rtol=5e-3, atol=5e-3)


@pytest.mark.parametrize("v", [1])
@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q5_K, Q.Q6_K, Q.Q8_0, Q.Q4_0, Q.F16])
@pytest.mark.parametrize("M", [17, 64, 100, 256, 300])
def test_gemm_prefill(cuda, native, qt, M, v):
    """Prefill MFMA dequant-GEMM vs torch fp32: STORE, ADD, SwiGLU.  v=1: 64x64 tiles (the fallback
    for the types gemm4 does not take, e.g. Q4_0; the 128-row v=2 form is retired)."""
    from mipipe.ops.kernels import PackedWeight, gemm as gemm_any, EPI_STORE, EPI_ATOMIC, EPI_SWIGLU
    gemm = lambda *a_, **kw: gemm_any(*a_, v=v, **kw)
    n, k = 208, 1280                     # 13 tiles (partial workgroup), 5 super-blocks
    raw, deq = _weights(qt, n, k, 300 + qt + M)
    w = PackedWeight(raw, qt, n, k)
    x = torch.randn(M, k)
    xh = torch.zeros(M, w.k_pad, dtype=torch.float16)
    xh[:, :k] = x.half()
    ref = xh[:, :k].float() @ deq.T
    y = gemm(w, xh.cuda(), EPI_STORE)
    assert nmse(y.cpu(), ref) < 1e-5
    base = torch.randn(M, n)
    y2 = gemm(w, xh.cuda(), EPI_ATOMIC, y=base.clone().cuda())
    assert nmse(y2.cpu(), ref + base) < 1e-5
    if qt in (Q.Q4_K, Q.Q8_0):
        # interleaved gate/up rows: tile rows 0-7 gate, 8-15 up of the same 8 outputs
        h = gemm(w, xh.cuda(), EPI_SWIGLU)
        gi = torch.tensor([16 * (o // 8) + (o % 8) for o in range(n // 2)])
        g, u = ref[:, gi], ref[:, gi + 8]
        href = torch.nn.functional.silu(g) * u
        assert nmse(h.float().cpu(), href) < 1e-4
