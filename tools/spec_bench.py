#!/usr/bin/env python3
"""Speculative (prompt-lookup) vs plain greedy decoding on one engine: decode tok/s, verify rounds,
acceptance.  Random-init weights rarely repeat themselves, so the acceptance here is whatever the
model's greedy output happens to give; the cost side (one verify round vs one decode step) is the
measurement that carries over to real checkpoints."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mipipe.engine import Engine

MODELS = {
    "llama3-70b": dict(name="Llama-3-70B", n_layer=80, d_model=8192, n_head=64, n_head_kv=8, d_ff=28672,
                       vocab=128256, rope_base=500000.0),
    "llama3-8b": dict(name="Llama-3-8B", n_layer=32, d_model=4096, n_head=32, n_head_kv=8, d_ff=14336,
                      vocab=128256, rope_base=500000.0),
}

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="llama3-8b", choices=sorted(MODELS))
ap.add_argument("--ftype", default="Q4_K_M")
ap.add_argument("--n", type=int, default=64)
ap.add_argument("--draft-max", type=int, default=4)
ap.add_argument("--mb-size", type=int, default=1)
ap.add_argument("--repeat-prompt", action="store_true", help="prompt = one motif repeated (lookup-friendly)")
a = ap.parse_args()
g = torch.Generator().manual_seed(0)
motif = torch.randint(3, MODELS[a.model]["vocab"], (16,), generator=g).tolist()
prompts = [(motif * 8) if a.repeat_prompt else torch.randint(3, MODELS[a.model]["vocab"], (128,), generator=g).tolist()
           for _ in range(a.mb_size)]
with Engine(synthetic=MODELS[a.model], ftype=a.ftype, n_mb=1, mb_size=a.mb_size, max_ctx=512, prefill_chunk=256,
            seed=1234) as eng:
    eng.generate(prompts, 8)   # warm-up (graphs, kernels)
    ref, s0 = eng.generate(prompts, a.n)
    out, s1 = eng.spec_generate(prompts, a.n, draft_max=a.draft_max)
print(json.dumps({"model": a.model, "mb_size": a.mb_size, "n": a.n, "same_output": out == ref,
                  "greedy_decode_tok_s": round(s0["decode_tok_s"], 1), "spec_decode_tok_s": round(s1["decode_tok_s"], 1),
                  "verify_rounds": s1["verify_rounds"], "accepted": s1["accepted"], "drafted": s1["drafted"],
                  "ms_per_decode_step": round(s0["decode_ms"] / max(1, a.n - 1), 3),
                  "ms_per_verify_round": round(s1["decode_ms"] / max(1, s1["verify_rounds"]), 3)}))
