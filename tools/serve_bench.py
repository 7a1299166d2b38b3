#!/usr/bin/env python3
"""Serving benchmark of the C++ orchestrator: concurrent SSE /chat clients, continuous batching vs
one batch per engine run (--no-continuous).

Each of C client threads sends R SSE /chat requests back to back. Prompt lengths and n_predict vary per
request, so requests finish at different rounds. Reported: aggregate generated tokens/s, and the
p50/p90 of time-to-first-token and of whole-request latency.

    python tools/serve_bench.py --synthetic llama3-8b --ftype Q4_K_M --clients 16 --requests 4
"""
import argparse
import asyncio
import json
import os
import random
import socket
import subprocess
import sys
import threading
import time

import httpx

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "distributed-llm-pipeline_amd", "bin")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def pct(v, p):
    v = sorted(v)
    return v[min(len(v) - 1, int(p * (len(v) - 1) + 0.5))] if v else 0.0


def run(args, continuous: bool):
    port = free_port()
    cmd = [os.path.join(BIN, "orchestrator"), "--host", "127.0.0.1", "--port", str(port), "--synthetic", args.synthetic,
           "--ftype", args.ftype, "--mb-size", str(args.mb_size), "--micro-batches", str(args.micro_batches),
           "-c", str(args.ctx), "-n", "64"]
    if args.ngl is not None:
        cmd += ["-ngl", str(args.ngl)]
    if not continuous:
        cmd.append("--no-continuous")
    proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    url = f"http://127.0.0.1:{port}"
    try:
        t0 = time.time()
        while True:
            try:
                httpx.get(url + "/health", timeout=1)
                break
            except Exception:
                if time.time() - t0 > 300 or proc.poll() is not None:
                    raise RuntimeError("orchestrator did not come up")
                time.sleep(0.2)
        ttft, lat, ntok = [], [], [0]
        lock = threading.Lock()
        words = "the quick brown fox jumps over a lazy dog while pipelines stream tokens".split()

        def client(ci):
            rng = random.Random(1000 + ci)
            for _ in range(args.requests):
                prompt = " ".join(rng.choice(words) for _ in range(rng.randint(4, args.max_prompt_words)))
                n = rng.randint(args.min_new, args.max_new)
                t_start = time.time()
                first = None
                toks = 0
                with httpx.stream("POST", url + "/chat", json={"prompt": prompt, "n_predict": n}, timeout=600) as r:
                    for line in r.iter_lines():
                        if line.startswith("data:") and '"token"' in line:
                            if first is None:
                                first = time.time()
                            toks += 1
                t_end = time.time()
                with lock:
                    ttft.append(((first or t_end) - t_start) * 1e3)
                    lat.append((t_end - t_start) * 1e3)
                    ntok[0] += n

        async def aclient(ci, ac):
            rng = random.Random(1000 + ci)
            for _ in range(args.requests):
                prompt = " ".join(rng.choice(words) for _ in range(rng.randint(4, args.max_prompt_words)))
                n = rng.randint(args.min_new, args.max_new)
                t_start = time.time()
                first = None
                async with ac.stream("POST", url + "/chat", json={"prompt": prompt, "n_predict": n}, timeout=600) as r:
                    async for line in r.aiter_lines():
                        if first is None and line.startswith("data:") and '"token"' in line:
                            first = time.time()
                t_end = time.time()
                ttft.append(((first or t_end) - t_start) * 1e3)
                lat.append((t_end - t_start) * 1e3)
                ntok[0] += n

        async def amain():
            limits = httpx.Limits(max_connections=args.clients + 4, max_keepalive_connections=args.clients + 4)
            async with httpx.AsyncClient(limits=limits) as ac:
                await asyncio.gather(*[aclient(i, ac) for i in range(args.clients)])

        t0 = time.time()
        if args.client == "async":   # one event loop: no GIL contention between 64 reader threads
            asyncio.run(amain())
        else:
            th = [threading.Thread(target=client, args=(i,)) for i in range(args.clients)]
            [t.start() for t in th]
            [t.join() for t in th]
        wall = time.time() - t0
        return dict(mode="continuous" if continuous else "batch-per-run", client=args.client, slots=args.mb_size,
                    clients=args.clients, requests=len(lat),
                    gen_tok_s=round(ntok[0] / wall, 1), wall_s=round(wall, 2),
                    ttft_p50_ms=round(pct(ttft, 0.5), 1), ttft_p90_ms=round(pct(ttft, 0.9), 1),
                    latency_p50_ms=round(pct(lat, 0.5), 1), latency_p90_ms=round(pct(lat, 0.9), 1))
    finally:
        proc.terminate()
        try:
            proc.wait(20)
        except subprocess.TimeoutExpired:
            proc.kill()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--synthetic", default="llama3-8b")
    ap.add_argument("--ftype", default="Q4_K_M")
    ap.add_argument("--mb-size", type=int, default=16)
    ap.add_argument("--micro-batches", type=int, default=1)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--ngl", type=int, default=None)
    ap.add_argument("--clients", type=int, default=16)
    ap.add_argument("--requests", type=int, default=4)
    ap.add_argument("--max-prompt-words", type=int, default=64)
    ap.add_argument("--min-new", type=int, default=16)
    ap.add_argument("--max-new", type=int, default=128)
    ap.add_argument("--modes", default="continuous,batch")
    ap.add_argument("--client", default="async", choices=["async", "threads"],
                    help="async: all streams on one asyncio loop (default); threads: one thread per client")
    args = ap.parse_args()
    for m in args.modes.split(","):
        print(json.dumps(run(args, m == "continuous")), flush=True)


if __name__ == "__main__":
    sys.exit(main())
