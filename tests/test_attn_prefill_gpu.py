"""Prefill flash attention (attn_prefill.hip) vs a plain PyTorch fp32 reference: causal masking,
GQA groups G = 1, 4, 7, 8, head dims 64/128 (and 48 padded to 64), chunks that start mid-sequence,
long contexts (4096) and packed chunks whose segments belong to different sequences / slots."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(q, K, V, pos):
    """q [R, Hq, hd] f32 (already scaled), K/V [S, Hkv, hd]; row r attends keys [0, pos[r]]."""
    R, Hq, hd = q.shape
    Hkv = K.shape[1]
    G = Hq // Hkv
    Ke = K.double().repeat_interleave(G, dim=1)   # [S, Hq, hd]
    Ve = V.double().repeat_interleave(G, dim=1)
    s = torch.einsum("rhd,shd->rhs", q.double(), Ke)
    keys = torch.arange(K.shape[0])
    s = s.masked_fill(keys[None, None, :] > pos[:, None, None], float("-inf"))
    return torch.einsum("rhs,shd->rhd", torch.softmax(s, -1), Ve).float()


def _setup(hd, Hq, Hkv, seqs, seed):
    """seqs: list of (slot, p0, T): prefill rows at positions p0..p0+T-1 of `slot` (KV of
    positions < p0 + T already in the cache).  Returns the kernel inputs and per-slot K/V."""
    g = torch.Generator().manual_seed(seed)
    Dp = 64 if hd <= 64 else 128
    n_slots = max(s for s, _, _ in seqs) + 1
    max_ctx = max(p0 + T for _, p0, T in seqs)
    max_ctx = (max_ctx + 63) // 64 * 64
    pages = max_ctx // 64
    perm = torch.randperm(n_slots * pages, generator=g)
    bt = perm[: n_slots * pages].reshape(n_slots, pages).to(torch.int32).contiguous()
    kc = torch.zeros(n_slots * pages, Hkv, 64, Dp, dtype=torch.float16)
    vc = torch.zeros(n_slots * pages, Hkv, Dp, 64, dtype=torch.float16)
    KV = {}
    for s, p0, T in seqs:
        S = p0 + T
        K = (torch.randn(S, Hkv, hd, generator=g)).half()
        V = (torch.randn(S, Hkv, hd, generator=g)).half()
        KV[s] = (K.float(), V.float())
        for p_ in range(S):
            page = int(bt[s, p_ // 64])
            kc[page, :, p_ % 64, :hd] = K[p_]
            vc[page, :, :hd, p_ % 64] = V[p_]
    M = sum(T for _, _, T in seqs)
    q = torch.zeros(M, Hq, Dp, dtype=torch.float16)
    q[:, :, :hd] = (torch.randn(M, Hq, hd, generator=g) / math.sqrt(hd)).half()
    pos = torch.cat([torch.arange(p0, p0 + T, dtype=torch.int32) for _, p0, T in seqs])
    slot = torch.cat([torch.full((T,), s, dtype=torch.int32) for s, _, T in seqs])
    segs, row = [], 0
    for _, _, T in seqs:
        segs.append((row, T))
        row += T
    return q, pos, slot, bt, kc, vc, KV, segs


@pytest.mark.parametrize("hd,Hq,Hkv", [(128, 32, 8), (128, 64, 8), (64, 32, 4), (128, 8, 8), (48, 6, 6),
                                       (128, 28, 4)])
@pytest.mark.parametrize("seqs", [[(0, 0, 1)], [(0, 0, 37)], [(1, 0, 300)], [(0, 200, 130)],
                                  [(2, 0, 20), (0, 100, 45), (1, 5, 3), (3, 0, 128)]])
@pytest.mark.parametrize("n_split", [1, 2])
def test_attn_prefill_matches_reference(cuda, native, hd, Hq, Hkv, seqs, n_split):
    from mipipe.ops.kernels import attn_prefill
    q, pos, slot, bt, kc, vc, KV, segs = _setup(hd, Hq, Hkv, seqs, seed=hd + Hq + len(seqs))
    pages = max(p0 + T - 1 for _, p0, T in seqs) // 64 + 1
    out = attn_prefill(q.cuda(), pos.cuda(), slot.cuda(), bt.cuda(), kc.cuda(), vc.cuda(), Hkv, hd, segs,
                       n_split=n_split, split_pages=-(-pages // n_split))
    out = out.float().cpu().view(-1, Hq, hd)
    row = 0
    for (s, p0, T), (r0, _) in zip(seqs, segs):
        K, V = KV[s]
        ref = _ref(q[r0:r0 + T, :, :hd].float(), K, V, pos[r0:r0 + T])
        torch.testing.assert_close(out[r0:r0 + T], ref, rtol=5e-3, atol=5e-3)


@pytest.mark.parametrize("hd,Hq,Hkv", [(128, 32, 8), (128, 64, 8)])
@pytest.mark.parametrize("n_split,split_pages", [(1, 1), (3, 22), (8, 8)])
def test_attn_prefill_long_context(cuda, native, hd, Hq, Hkv, n_split, split_pages):
    """A 512-row chunk at the end of a 4096-token sequence (causal page skipping over 64 pages),
    whole or KV-split over workgroups (incl. splits past the last page) + LSE merge."""
    from mipipe.ops.kernels import attn_prefill
    seqs = [(0, 3584, 512)]
    q, pos, slot, bt, kc, vc, KV, segs = _setup(hd, Hq, Hkv, seqs, seed=7)
    out = attn_prefill(q.cuda(), pos.cuda(), slot.cuda(), bt.cuda(), kc.cuda(), vc.cuda(), Hkv, hd, segs,
                       n_split=n_split, split_pages=split_pages)
    out = out.float().cpu().view(-1, Hq, hd)
    idx = torch.tensor([0, 1, 63, 64, 255, 300, 511])
    K, V = KV[0]
    ref = _ref(q[idx, :, :hd].float(), K, V, pos[idx])
    torch.testing.assert_close(out[idx], ref, rtol=5e-3, atol=5e-3)


def test_attn_prefill_matches_decode_shaped_kernel(cuda, native):
    """Same chunk through the old row-group kernel (attention.hip, tq tokens per group)."""
    from mipipe.ops.kernels import attn_prefill, attention
    seqs = [(1, 0, 300)]
    q, pos, slot, bt, kc, vc, KV, segs = _setup(128, 32, 8, seqs, seed=3)
    a = attn_prefill(q.cuda(), pos.cuda(), slot.cuda(), bt.cuda(), kc.cuda(), vc.cuda(), 8, 128, segs)
    b = attention(q.cuda(), (pos + 1).cuda(), slot.cuda(), bt.cuda(), kc.cuda(), vc.cuda(), 8, 128, tq=4,
                  split_len=512, n_split=1)
    torch.testing.assert_close(a.float(), b.float(), rtol=2e-3, atol=2e-3)
