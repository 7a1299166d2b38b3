"""r8t: which rows go wrong with gemm4 on the split-K decode GEMMs (prefill_gemm_v=4) on the 2-layer
70B-width model: per-row logit NMSE after two decode rounds, v4 against v2 (v2 passes the fp32
oracle); then the kernel-level split-K partial-store GEMM at the decode shapes, all rows against fp32."""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mipipe import _native as N  # noqa: E402
from mipipe.engine import Engine  # noqa: E402
from mipipe.models.config import CONFIGS  # noqa: E402
from mipipe.models.synthetic import write_synthetic_gguf  # noqa: E402
from mipipe.ops.kernels import PackedWeight, gemm_splitk  # noqa: E402
from mipipe.utils import quants as Q  # noqa: E402

N.build()


def nmse(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


cfg = CONFIGS["llama3-70b"].scaled(n_layer=2, vocab=4096, name="l70w2")
path = "/tmp/l70w2-Q4_K.gguf"
if not os.path.exists(path):
    write_synthetic_gguf(path, cfg, "Q4_K", seed=3, fast_random_blocks=True)
rng = np.random.default_rng(5)
mb = 256
prompts = [[int(t) for t in rng.integers(3, cfg.vocab, int(n))] for n in rng.integers(4, 24, mb)]
res = {}
for v in (2, 4):
    with Engine(gguf=path, max_ctx=64, n_mb=1, mb_size=mb, prefill_chunk=512, prefill_gemm_v=v) as eng:
        eng.start(prompts)
        lg0 = eng.logits(rows=mb).copy()
        eng.decode(1)
        lg1 = eng.logits(rows=mb).copy()
        res[v] = (lg0, lg1, eng.tokens())
same_tok = sum(a == b for a, b in zip(res[2][2], res[4][2]))
e0 = [nmse(res[4][0][r], res[2][0][r]) for r in range(mb)]
e1 = [nmse(res[4][1][r], res[2][1][r]) for r in range(mb)]
bad = [r for r in range(mb) if e1[r] > 1e-5]
print(f"prefill logits max NMSE v4 vs v2 {max(e0):.2e}; after 1 decode round max {max(e1):.2e}; "
      f"rows > 1e-5: {len(bad)} {bad[:40]}; same tokens {same_tok}/{mb}", flush=True)
by_block = [sum(1 for r in bad if r // 64 == b) for b in range(4)]
print("bad rows per 64-row block:", by_block, flush=True)

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_moe_gemm_gpu import _rand_blocks  # noqa: E402
for (n, k) in ((1024, 8192), (8192, 8192), (8192, 28672), (10240, 8192)):
    raw = _rand_blocks(Q.Q4_K, n, k, np.random.default_rng(n + k))
    w = PackedWeight(raw, Q.Q4_K, n, k)
    deq = w.unpack().float()
    xh = torch.randn(256, w.k_pad).half().cuda()
    ref = xh.float() @ deq.T
    y = torch.zeros(256, n).cuda()
    ns = gemm_splitk(w, xh, y)
    rows = [nmse(y[r].cpu(), ref[r].cpu()) for r in range(256)]
    badr = [r for r in range(256) if rows[r] > 1e-5]
    print(f"gemm4 split-K partial stores N={n} K={k} M=256: splits {ns}, max row NMSE {max(rows):.2e}, bad rows {badr[:20]}",
          flush=True)
