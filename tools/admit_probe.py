#!/usr/bin/env python3
"""Continuous-batching cost probe: a full micro-batch of B sequences decoding while one slot per
round is released and re-admitted with a fresh short prompt (what the server does when requests
finish at different rounds).  Reports ms per plain decode round vs per admit() call."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--ftype", default="Q4_K_M")
    ap.add_argument("--mb-size", type=int, default=64)
    ap.add_argument("--rounds", type=int, default=40)
    a = ap.parse_args()
    import torch  # noqa: F401
    import bench as B
    from mipipe.engine import Engine
    rng = np.random.default_rng(0)
    V = B.MODELS[a.model]["vocab"]
    P = lambda n: [int(t) for t in rng.integers(3, V, n)]
    with Engine(synthetic=B.MODELS[a.model], ftype=a.ftype, n_mb=1, mb_size=a.mb_size, max_ctx=1024) as eng:
        eng.start([P(int(rng.integers(8, 64))) for _ in range(a.mb_size)])
        eng.decode(3)
        t0 = time.perf_counter()
        for _ in range(a.rounds):
            eng.decode(1)
        dec = (time.perf_counter() - t0) * 1e3 / a.rounds
        adm, rel = [], []
        for r in range(a.rounds):
            s = r % a.mb_size
            t1 = time.perf_counter()
            eng.release(s)
            t2 = time.perf_counter()
            eng.admit([s], [P(int(rng.integers(8, 64)))])
            t3 = time.perf_counter()
            eng.decode(1)
            rel.append((t2 - t1) * 1e3)
            adm.append((t3 - t2) * 1e3)
        print(json.dumps(dict(mb_size=a.mb_size, decode_ms=round(dec, 3), admit_ms_p50=round(float(np.median(adm)), 3),
                              admit_ms_max=round(float(np.max(adm)), 3), release_ms_p50=round(float(np.median(rel)), 3))),
              flush=True)


if __name__ == "__main__":
    main()
