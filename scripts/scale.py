#!/usr/bin/env python3
"""Weak-scaling curve of the headline benchmark: bench.py at N = 1, 2, 4, 8 GPUs (PP = N) on one
node, printed as ONE JSON object, plus the agreement of the N = 1 point with the newest driver
record (BENCH_rNN.json) in the repo root.

    bash scripts/scale.sh                       # in-process pipelines (no launcher), N = 1 2 4 8
    bash scripts/scale.sh --launcher torchrun   # one rank per GPU, the driver's launch
    bash scripts/scale.sh --gpus 1,2 --same-device -- --model llama3-8b   # 1-GPU rehearsal

Every N runs as its own child process (nothing here touches the GPU), each under its own time limit;
the first failing N ends the sweep (its stderr tail is in the JSON).  N larger than the visible GPU
count is skipped unless --same-device.  Efficiency is value(N) / (N * value(1)).
"""
import argparse
import glob
import json
import os
import re
import socket
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def visible_gpus():
    # count devices without initialising HIP in this process (children do the GPU work)
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=300)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def last_bench_record():
    recs = sorted(glob.glob(os.path.join(REPO, "BENCH_r*.json")))
    if not recs:
        return None
    try:
        d = json.load(open(recs[-1]))
        tail = d["run"]["stdout_tail"]
        m = re.search(r"\{.*\}", tail)
        line = json.loads(m.group(0)) if m else None
        return {"file": os.path.basename(recs[-1]), "value": line["value"] if line else None}
    except (KeyError, ValueError, TypeError):
        return {"file": os.path.basename(recs[-1]), "value": None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--launcher", choices=["inproc", "torchrun"], default="inproc")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--same-device", action="store_true")
    ap.add_argument("--timeout", type=int, default=900, help="seconds per N")
    ap.add_argument("bench_args", nargs="*", help="extra bench.py arguments (after --)")
    a = ap.parse_args()
    ns = [int(x) for x in a.gpus.split(",") if x]
    have = visible_gpus()
    points, err = [], None
    for n in ns:
        if n > have and not (a.same_device and have >= 1):
            points.append({"n_gpus": n, "skipped": f"{have} visible GPU(s)"})
            continue
        bench = [os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", str(a.steps), "--warmup",
                 str(a.warmup), "--no-secondary"] + (["--same-device"] if a.same_device and n > 1 else []) + a.bench_args
        env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
        if a.launcher == "torchrun" and n > 1:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
                   "--master-addr", "127.0.0.1", "--master-port", str(free_port())] + bench
        else:
            cmd = [sys.executable] + bench
        print(f"scale: N={n}: {' '.join(cmd)}", file=sys.stderr, flush=True)
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, cwd=REPO, env=env)
        except subprocess.TimeoutExpired:
            err = {"n_gpus": n, "error": f"timed out after {a.timeout} s"}
            break
        lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or len(lines) != 1:
            err = {"n_gpus": n, "rc": r.returncode, "stderr_tail": r.stderr[-2000:]}
            break
        d = json.loads(lines[0])
        p = {"n_gpus": n, "value": d["value"], "ms_per_step": d["ms_per_step"], "p50_token_ms": d.get("p50_token_ms"),
             "global_batch": d["config"]["global_batch"], "parallelism": d["config"]["parallelism"]}
        if "link" in d:
            p["link"] = d["link"]
        points.append(p)
    base = next((p for p in points if p.get("n_gpus") == 1 and "value" in p), None)
    for p in points:
        if base and "value" in p:
            p["speedup"] = round(p["value"] / base["value"], 3)
            p["efficiency"] = round(p["value"] / (p["n_gpus"] * base["value"]), 3)
    out = {"metric": "decode tokens/sec (whole node) + p50/token", "launcher": a.launcher, "scaling": "weak",
           "visible_gpus": have, "points": points}
    # the driver's BENCH record is the default (headline) configuration: compare only that one
    rec = last_bench_record() if not any(x in a.bench_args for x in ("--model", "--ftype", "--mb-size")) else None
    if rec and base:
        out["n1_vs_bench_record"] = dict(rec, n1_value=base["value"],
                                         ratio=round(base["value"] / rec["value"], 3) if rec.get("value") else None)
    if err:
        out["error"] = err
    print(json.dumps(out), flush=True)
    sys.exit(1 if err else 0)


if __name__ == "__main__":
    main()
