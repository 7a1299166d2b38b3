#!/usr/bin/env python3
"""Prompt-processing throughput of the engine (synthetic weights): n sequences x len-token prompts,
prefill through Engine.generate(..., 1); prints one JSON line (prompt tok/s from the engine stats).

    python tools/prefill_bench.py --model llama3-70b --ftype Q4_K --n 64 --len 512 [--set prefill_gemm_v=2]
"""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from bench import MODELS, parse_set
from mipipe.engine import Engine


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-70b", choices=sorted(MODELS))
    ap.add_argument("--ftype", default="Q4_K")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--len", type=int, default=512)
    ap.add_argument("--set", action="append", default=[])
    a = ap.parse_args()
    cfg = dict(synthetic=MODELS[a.model], ftype=a.ftype, n_mb=1, mb_size=a.n, max_ctx=((a.len + 8 + 63) // 64) * 64,
               prefill_chunk=512, seed=1)
    cfg.update(parse_set(a.set))
    g = torch.Generator().manual_seed(0)
    prompts = torch.randint(3, MODELS[a.model]["vocab"], (a.n, a.len), generator=g).tolist()
    with Engine(**cfg) as eng:
        eng.generate(prompts[:2], 1)   # warm-up (graphs, kernels)
        t0 = time.perf_counter()
        _, st = eng.generate(prompts, 1)
        wall = time.perf_counter() - t0
    print(json.dumps({"model": a.model, "ftype": a.ftype, "n": a.n, "len": a.len, "set": a.set,
                      "prompt_tok_s_wall": round(a.n * a.len / wall, 1),
                      "stats": {k: v for k, v in st.items() if not isinstance(v, list)}}), flush=True)


if __name__ == "__main__":
    main()
