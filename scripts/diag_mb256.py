#!/usr/bin/env python3
"""Diagnostic for test_70b_width_mb256_matches_reference: per-row NMSE of the engine's logits
(after the prompt and after two decode rounds) against the fp32 oracle for ALL 256 rows, plus a
second engine run to tell a deterministic defect from a race."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mipipe.engine import Engine  # noqa: E402
from mipipe.models.config import CONFIGS  # noqa: E402
from mipipe.models.reference import RefLlama  # noqa: E402
from mipipe.models.synthetic import write_synthetic_gguf  # noqa: E402


def nmse(a, b):
    return float(((a - b) ** 2).sum() / max((b ** 2).sum(), 1e-30))


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/diag"
    os.makedirs(out, exist_ok=True)
    cfg = CONFIGS["llama3-70b"].scaled(n_layer=2, vocab=4096, name="l70w2")
    path = os.path.join(out, "l70w2-Q4_K.gguf")
    if not os.path.exists(path):
        write_synthetic_gguf(path, cfg, "Q4_K", seed=3, fast_random_blocks=True)
    rng = np.random.default_rng(5)
    mb = 256
    prompts = [[int(t) for t in rng.integers(3, cfg.vocab, int(n))] for n in rng.integers(4, 24, mb)]
    extra = {}
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        extra[k] = int(v) if v.lstrip("-").isdigit() else {"true": True, "false": False}.get(v, v)
    runs = []
    for _ in range(2):
        with Engine(gguf=path, max_ctx=64, n_mb=1, mb_size=mb, prefill_chunk=512, **extra) as eng:
            eng.start(prompts)
            lg0 = eng.logits(rows=mb)
            eng.decode(2)
            lg2 = eng.logits(rows=mb)
            toks = eng.tokens()
        runs.append((lg0, lg2, toks))
    (a0, a2, at), (b0, b2, bt) = runs
    print("run-to-run: max nmse lg0 %.3g lg2 %.3g, token rows differing %d" % (
        max(nmse(a0[r], b0[r]) for r in range(mb)), max(nmse(a2[r], b2[r]) for r in range(mb)),
        sum(at[r][:3] != bt[r][:3] for r in range(mb))), flush=True)
    ref = RefLlama.from_gguf(path, device="cuda")
    bad0, bad2 = [], []
    for r in range(mb):
        ref.reset()
        rl = ref.forward(prompts[r], 0)[-1].float().cpu().numpy()
        e0 = nmse(a0[r], rl)
        pos = len(prompts[r])
        for t in at[r][:2]:
            rl = ref.forward([t], pos)[-1].float().cpu().numpy()
            pos += 1
        e2 = nmse(a2[r], rl)
        if e0 > 2e-4:
            bad0.append((r, len(prompts[r]), round(e0, 5)))
        if e2 > 2e-4:
            bad2.append((r, len(prompts[r]), len(at[r]), at[r][:3], round(e2, 5), round(nmse(b2[r], rl), 5)))
    print("prompt-logit failures (row, len, nmse):", bad0)
    print("decode-logit failures (row, len, ntok, toks, nmse run A, run B):", len(bad2))
    for b in bad2:
        print("  ", b)


if __name__ == "__main__":
    main()
