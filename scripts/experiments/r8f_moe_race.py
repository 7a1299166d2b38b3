"""r8f: locate the intermittent grouped-MoE down-projection mismatch: the same inputs through the
down GEMM 12 times (BM 64 / 128 by knob), each result against the fp32 oracle; for a bad run, which
(token rows, output columns) are wrong and by how much."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from mipipe import _native as N  # noqa: E402
from mipipe.ops.kernels import PackedWeight, moe_route, moe_gemm, EPI_SWIGLU, EPI_ATOMIC  # noqa: E402
from mipipe.utils import quants as Q  # noqa: E402
from test_moe_gemm_gpu import _rand_blocks, D, F, E, K_TOP  # noqa: E402

N.build()
rng = np.random.default_rng(11)
qt = int(os.environ.get("QT", Q.Q6_K))
dn = [PackedWeight(_rand_blocks(qt, D, F, rng), qt, D, F) for _ in range(E)]
dn_all = torch.cat([w.dev for w in dn])
dense = [w.unpack().float() for w in dn]
for M in (65, 256):
    g = torch.Generator().manual_seed(M)
    logits = torch.randn(M, E, generator=g).cuda()
    counts, lists, weights = moe_route(logits, K_TOP)
    h = (torch.randn(M * K_TOP, F, generator=g) * 0.5).half().cuda()
    cnt = counts.cpu().tolist()
    y_ref = torch.zeros(M, D, dtype=torch.float64, device="cuda")
    for e in range(E):
        sl = lists[e, : cnt[e]].long()
        if sl.numel():
            y_ref.index_add_(0, sl // K_TOP, (weights[sl][:, None] * (h[sl].float() @ dense[e].T)).double())
    for bm in (0, 128):
        N.check(N.lib().mp_set_knob(b"GEMM3_BM", bm), "knob")
        bad = 0
        for it in range(12):
            y = torch.zeros(M, D, device="cuda")
            moe_gemm(dn_all, dn[0].dev.numel(), dn[0].ptype, dn[0].ntiles, dn[0].nsb, D, EPI_ATOMIC, h, M, E, K_TOP,
                     counts, lists, weights, x_per_slot=True, y=y)
            torch.cuda.synchronize()
            err = (y.double() - y_ref).abs()
            tol = 1e-3 * y_ref.abs().max()
            wrong = (err > tol).nonzero()
            if len(wrong):
                bad += 1
                rows = sorted(set(wrong[:, 0].tolist()))
                cols = wrong[:, 1]
                print(f"M={M} bm={bm} it={it}: {len(wrong)} wrong of {M * D}; rows {rows[:12]}{'...' if len(rows) > 12 else ''} "
                      f"({len(rows)}); cols {int(cols.min())}-{int(cols.max())} ({len(set(cols.tolist()))} distinct, "
                      f"col%32 {sorted(set((cols % 32).tolist()))[:8]}); max err {float(err.max()):.3g} vs |y| {float(y_ref.abs().max()):.3g}",
                      flush=True)
                # which experts own the wrong rows
                own = {}
                for e in range(E):
                    toks = set((lists[e, : cnt[e]] // K_TOP).tolist())
                    k = len(toks & set(rows))
                    if k:
                        own[e] = (k, cnt[e])
                print("   experts (wrong rows, rows of expert):", own, flush=True)
        print(f"M={M} bm={bm}: {bad}/12 runs wrong; counts {cnt}", flush=True)
N.lib().mp_set_knob(b"GEMM3_BM", 0)
