"""r8g: the grouped-MoE test body (gate/up -> down back to back, as in test_moe_gemm_gpu.py) 10 times per
variant: as in the test, with a device sync between the two GEMMs, and with h pre-filled by
a torch kernel; reports which slots / rows / columns are wrong when a run fails."""
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
gu = [PackedWeight(_rand_blocks(Q.Q4_K, 2 * F, D, rng), Q.Q4_K, 2 * F, D, gateup=True) for _ in range(E)]
dn = [PackedWeight(_rand_blocks(Q.Q6_K, D, F, rng), Q.Q6_K, D, F) for _ in range(E)]
gu_all = torch.cat([w.dev for w in gu])
dn_all = torch.cat([w.dev for w in dn])
dd = [w.unpack().float() for w in dn]
for M in (65, 256):
    g = torch.Generator().manual_seed(M)
    logits = torch.randn(M, E, generator=g).cuda()
    counts, lists, weights = moe_route(logits, K_TOP)
    x = torch.randn(M, gu[0].k_pad, generator=g).half().cuda()
    cnt = counts.cpu().tolist()
    for variant in ("test", "sync", "h-nan-fill"):
        bad = 0
        for it in range(10):
            h = torch.zeros(M * K_TOP, dn[0].k_pad, dtype=torch.float16, device="cuda")
            if variant == "h-nan-fill":
                h.fill_(float("nan"))
            moe_gemm(gu_all, gu[0].dev.numel(), gu[0].ptype, gu[0].ntiles, gu[0].nsb, F, EPI_SWIGLU, x, M, E, K_TOP,
                     counts, lists, weights, h=h)
            if variant == "sync":
                torch.cuda.synchronize()
            y = torch.zeros(M, D, device="cuda")
            moe_gemm(dn_all, dn[0].dev.numel(), dn[0].ptype, dn[0].ntiles, dn[0].nsb, D, EPI_ATOMIC, h, M, E, K_TOP,
                     counts, lists, weights, x_per_slot=True, y=y)
            torch.cuda.synchronize()
            y_ref = torch.zeros(M, D, dtype=torch.float64, device="cuda")
            for e in range(E):
                sl = lists[e, : cnt[e]].long()
                if sl.numel():
                    y_ref.index_add_(0, sl // K_TOP, (weights[sl][:, None] * (h[sl].float() @ dd[e].T)).double())
            err = (y.double() - y_ref).abs()
            wrong = (err > 1e-3 * y_ref.abs().max()).nonzero()
            if len(wrong) or not torch.isfinite(y).all():
                bad += 1
                rows = sorted(set(wrong[:, 0].tolist()))
                cols = wrong[:, 1]
                own = {}
                for e in range(E):
                    k = len(set((lists[e, : cnt[e]] // K_TOP).tolist()) & set(rows))
                    if k:
                        own[e] = (k, cnt[e])
                print(f"M={M} {variant} it={it}: {len(wrong)} wrong; rows {rows[:10]} ({len(rows)}); cols "
                      f"{int(cols.min()) if len(cols) else -1}-{int(cols.max()) if len(cols) else -1} "
                      f"({len(set(cols.tolist()))} distinct); max err {float(err.max()):.3g} / {float(y_ref.abs().max()):.3g}; "
                      f"experts {own}; nonfinite {int((~torch.isfinite(y)).sum())}", flush=True)
        print(f"M={M} {variant}: {bad}/10 wrong", flush=True)
