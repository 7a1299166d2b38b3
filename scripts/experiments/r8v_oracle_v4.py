"""r8v: the 70B-width mb256 oracle test body (tests/test_engine_gpu.py::test_70b_width_mb256_matches_reference)
with prefill_gemm_v = 4 (gemm4 on the split-K decode GEMMs too) three times and v2 once, every row
checked against the fp32 oracle after the prompt and after two decode rounds."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from mipipe import _native as N  # noqa: E402
from mipipe.engine import Engine  # noqa: E402
from mipipe.models.config import CONFIGS  # noqa: E402
from mipipe.models.reference import RefLlama  # noqa: E402
from mipipe.models.synthetic import write_synthetic_gguf  # noqa: E402

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
runs = []
for v in (4, 4, 4, 2):
    with Engine(gguf=path, max_ctx=64, n_mb=1, mb_size=mb, prefill_chunk=512, prefill_gemm_v=v) as eng:
        eng.start(prompts)
        lg0 = eng.logits(rows=mb).copy()
        eng.decode(2)
        lg2 = eng.logits(rows=mb).copy()
        runs.append((v, lg0, lg2, eng.tokens()))
ref = RefLlama.from_gguf(path, device="cuda")
rows = list(range(0, mb, 3)) + [64, 128, 200, 255]
for (v, lg0, lg2, toks) in runs:
    bad = []
    worst = 0.0
    for r in sorted(set(rows)):
        ref.reset()
        rl = ref.forward(prompts[r], 0)[-1].float().cpu().numpy()
        e0 = nmse(lg0[r], rl)
        pos = len(prompts[r])
        for t in toks[r][:2]:
            rl = ref.forward([t], pos)[-1].float().cpu().numpy()
            pos += 1
        e2 = nmse(lg2[r], rl)
        worst = max(worst, e0, e2)
        if e0 > 2e-4 or e2 > 2e-4:
            bad.append((r, round(e0, 6), round(e2, 6)))
    print(f"prefill_gemm_v={v}: {len(set(rows))} rows vs fp32 oracle, worst NMSE {worst:.2e}, failing {bad[:10]}", flush=True)
same = [sum(a == b for a, b in zip(runs[0][3], x[3])) for x in runs]
print("same tokens as run 0:", same, "| max |lg2 - run0| per run:",
      [float(np.abs(x[2] - runs[0][2]).max()) for x in runs], flush=True)
