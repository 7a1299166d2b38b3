#!/usr/bin/env python3
"""Real-GGUF load at scale: write a random-init GGUF of a real architecture (8B
Q4_K_M: ~4.9 GB) to local disk, load it through Engine(gguf=...) (mmap -> multithreaded T16 packing
into pinned double-buffered staging -> hipMemcpyAsync), report load GB/s, then compare decode tok/s
of the file-loaded engine with the on-GPU random-init engine of the same shape.

    python tools/load_bench.py --model llama3-8b --ftype Q4_K_M --out /tmp/m.gguf
Prints one JSON line."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ftype", default="Q4_K_M")
    ap.add_argument("--out", default="/tmp/mipipe_load_bench.gguf")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--keep", action="store_true")
    a = ap.parse_args()
    import torch  # noqa: F401  (before the native library)
    from mipipe.engine import Engine
    from mipipe.models.config import CONFIGS
    from mipipe.models.synthetic import write_synthetic_gguf

    cfg = CONFIGS[a.model]
    t0 = time.time()
    if not os.path.exists(a.out):
        write_synthetic_gguf(a.out, cfg, a.ftype, seed=1, fast_random_blocks=True, with_tokenizer=False)
    write_s = time.time() - t0
    size = os.path.getsize(a.out)
    # page the file into the page cache first, so the number is the engine's (pack + DMA), not the disk's
    t1 = time.time()
    with open(a.out, "rb") as f:
        while f.read(1 << 26):
            pass
    read_s = time.time() - t1
    res = {"model": a.model, "ftype": a.ftype, "gguf_bytes": size, "write_s": round(write_s, 2),
           "page_cache_read_GBps": round(size / read_s / 1e9, 2)}
    t2 = time.time()
    with Engine(gguf=a.out, max_ctx=256, prefill_chunk=128) as eng:
        load_s = time.time() - t2
        wb = eng.info["weight_bytes_local"]
        res.update(load_s=round(load_s, 3), engine_load_ms=round(eng.info["load_ms"], 1),
                   weight_bytes=wb, load_GBps=round(wb / (eng.info["load_ms"] / 1e3) / 1e9, 2))
        r = eng.bench(prompt_len=64, warmup=3, steps=a.steps)
        res["file_decode_tok_s"] = round(r["decode_tok_s"], 1)
    syn = dict(n_layer=cfg.n_layer, d_model=cfg.d_model, n_head=cfg.n_head, n_head_kv=cfg.n_head_kv, d_ff=cfg.d_ff,
               vocab=cfg.vocab, rope_base=cfg.rope_base)
    with Engine(synthetic=syn, ftype=a.ftype, max_ctx=256, prefill_chunk=128) as eng:
        r = eng.bench(prompt_len=64, warmup=3, steps=a.steps)
        res["synthetic_decode_tok_s"] = round(r["decode_tok_s"], 1)
    if not a.keep:
        os.remove(a.out)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
