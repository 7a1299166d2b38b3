#!/usr/bin/env python3
"""Headline benchmark: whole-node decode tokens/s (+ p50 per-token latency) of the MI355X-native
pipeline engine on Llama-3-70B Q4_K, PP = number of GPUs (BASELINE.json: "decode tokens/sec (whole
node) + p50/token, Llama-3-70B PP=8 and 8B PP=1"; reference headline 2-3 tok/s for 70B, PDF p.12).

    python bench.py --gpus 1 --steps 20 --warmup 5                  # PP=1 on one MI355X
    python bench.py --gpus 8 --steps 20 ...                          # PP=8 in ONE process (no launcher)
    torchrun --nproc-per-node 8 bench.py --gpus 8 --steps 20 ...     # PP=8, one rank per GPU

Weights are random-init directly in HBM with the exact Llama-3-70B architecture and Q4_K block
format (no network, no checkpoint).  Every stage owns one GPU (contiguous layer range,
cost-balanced split with the LM head on the last stage); activations move stage to stage over
xGMI as bf16; N + 1 micro-batches (N > 1) of `--mb-size` sequences circulate through the piped
ring.  Two launches, the same engine:
  * under torchrun (WORLD_SIZE set): one process per GPU, engine mode "mp", RCCL send/recv on a
    2-rank communicator per link direction (ids exchanged over torch.distributed);
  * without a launcher (`--gpus N`, no WORLD_SIZE): one process, engine mode "local", one host
    thread per GPU, links from ncclCommInitAll (`--link auto`/`rccl`) or, if RCCL refuses, peer-copy
    LocalLinks (one device copy per boundary, receiver-side xGMI read); `--same-device` puts every
    stage on GPU 0 (the 1-GPU rehearsal of the N-stage path).
Default 256 sequences per micro-batch, sized for 288 GB of HBM: above 64 rows the Q4_K decode
projections run on the dequant MFMA GEMMs (HipStage::gemv's auto choice: gate/up and the LM head
on gemm4's 32x32x16 MFMA tiles, the split-K qkv / o / down on gemm2 in gemv2.hip; gemm3 for 16-bit
weights).  Weak scaling: per-GPU work is fixed
(every stage streams its own weights once per micro-batch per round), global batch =
n_mb * mb_size sequences.  The timed region is exactly K decode rounds (every sequence emits one
token per round), bracketed by barrier + torch.cuda.synchronize() on both sides; the MAX over
ranks is reported.

At N > 1 (no replicas) it also measures BASELINE configs 3 and 5 on the same N-stage pipeline:
Llama-3-8B bf16 (64 sequences per micro-batch) and Mixtral 8x7B Q4_K_M (256), N + 1 micro-batches.
At N = 1 the same run also measures, with the same bracket, the other named BASELINE configs at
one GPU (Llama-3-8B Q4_K_M single stream, Mixtral 8x7B Q4_K_M at 256 sequences on the grouped MoE
GEMM, Llama-3-8B bf16 at 64 sequences), the round-1 like-for-like point (70B, 64 sequences) and the
headline shape at the reference's 2K context (256 sequences decoding at positions ~2000, after a
real prefill of their 1984-token prompts): "secondary" in the JSON line (--no-secondary skips them).  For N > 1 the line reports the data
plane the engine built ("link": transport kind, RCCL communicator sizes as ncclCommCount returns
them, bf16 wire bytes per token per boundary).
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_TOK_S = 2.5   # Llama-3-70B, 2-3 tok/s (PDF p.12) -> midpoint

MODELS = {
    "llama3-70b": dict(name="Llama-3-70B", n_layer=80, d_model=8192, n_head=64, n_head_kv=8, d_ff=28672,
                       vocab=128256, rope_base=500000.0),
    "llama3-8b": dict(name="Llama-3-8B", n_layer=32, d_model=4096, n_head=32, n_head_kv=8, d_ff=14336,
                      vocab=128256, rope_base=500000.0),
    "mixtral-8x7b": dict(name="Mixtral-8x7B", n_layer=32, d_model=4096, n_head=32, n_head_kv=8, d_ff=14336,
                         vocab=32000, rope_base=1000000.0, n_expert=8, n_expert_used=2),
    "tinyllama": dict(name="TinyLlama-1.1B", n_layer=22, d_model=2048, n_head=32, n_head_kv=4, d_ff=5632,
                      vocab=32000, rope_base=10000.0),
}

# (label, model, ftype, mb_size, extra engine options, prompt length or None for --prompt-len): the
# other named BASELINE configs at one GPU (8B Q4_K_M single stream; Mixtral 8x7B on the grouped MoE
# GEMM; 8B bf16), the round-1 like-for-like point (70B, 64 sequences) and the headline shape at the
# reference CLI's 2K context (-c 2048, main.rs:45-46): 256 sequences decoding at positions ~2000,
# with the f16 KV cache (its attention is HBM-bound: 2.15 GB per layer) and the fp8 one
SECONDARY = [("llama3-8b Q4_K_M pp1 mb1", "llama3-8b", "Q4_K_M", 1, {}, None),
             ("llama3-70b Q4_K pp1 mb64", "llama3-70b", "Q4_K", 64, {}, None),
             ("mixtral-8x7b Q4_K_M pp1 mb256", "mixtral-8x7b", "Q4_K_M", 256, {}, None),
             ("llama3-8b BF16 pp1 mb64", "llama3-8b", "BF16", 64, {}, None),
             ("llama3-70b Q4_K pp1 mb256 ctx2048", "llama3-70b", "Q4_K", 256, {}, 1984),
             ("llama3-70b Q4_K pp1 mb256 ctx2048 kv-fp8", "llama3-70b", "Q4_K", 256, {"kv_dtype": "fp8"}, 1984)]

# N > 1: BASELINE configs 3 (Llama-3-8B bf16, PP=4) and 5 (Mixtral 8x7B, PP=4) on the same pipeline
# as the headline (PP = N, N + 1 micro-batches): measured by the driver's multi-GPU runs too
SECONDARY_PP = [("llama3-8b BF16 pp{N} mb64", "llama3-8b", "BF16", 64),
                ("mixtral-8x7b Q4_K_M pp{N} mb256", "mixtral-8x7b", "Q4_K_M", 256)]


def parse_set(items):
    out = {}
    for kv in items:
        k, v = kv.split("=", 1)
        out[k] = {"true": True, "false": False}.get(v.lower(), int(v) if v.lstrip("-").isdigit() else v)
    return out


def run(eng_factory, vocab, n_seq, prompt_len, steps, warmup, world, pg_cpu, devices=(0,), dump_tokens=None,
        trace=None):
    """Start n_seq synthetic prompts, warm up, time exactly `steps` decode rounds; returns
    (ms, p50 ms, engine info) with ms and p50 the MAX over ranks.  dump_tokens: write the generated
    tokens (where the last stage lives) to that JSON file, after the timed region.  trace: after the
    timed region, 5 more rounds with the engine's span trace on, written there (Chrome JSON)."""
    eng = eng_factory()
    try:
        g = torch.Generator().manual_seed(0)
        prompts = torch.randint(3, vocab, (n_seq, prompt_len), generator=g).tolist()
        eng.start(prompts)
        if warmup:
            eng.decode(warmup)

        def bracket():
            if world > 1:
                dist.barrier()
            if torch.cuda.is_available():
                for d in devices:   # in-process PP: every GPU of the pipeline
                    torch.cuda.synchronize(d)

        bracket()
        t0 = time.perf_counter()
        st = eng.decode(steps)
        bracket()
        ms = (time.perf_counter() - t0) * 1e3
        tms = sorted(st.get("token_ms", []))
        p50 = tms[len(tms) // 2] if tms else 0.0
        vals = torch.tensor([ms, p50], dtype=torch.float64, device="cpu" if (pg_cpu or world == 1) else "cuda")
        if world > 1:
            dist.all_reduce(vals, op=dist.ReduceOp.MAX)   # p50 only non-zero on the last stage
        from mipipe import _native as N
        info = N.jcall(N.lib().mp_engine_info, eng._h, what="engine info")
        if dump_tokens:
            with open(dump_tokens, "w") as f:
                json.dump(eng.tokens(), f)
        if trace:
            eng.trace(True)
            eng.decode(5)
            eng.write_trace(trace)
        return float(vals[0]), float(vals[1]), info
    finally:
        eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="llama3-70b", choices=sorted(MODELS))
    ap.add_argument("--ftype", default="Q4_K")
    ap.add_argument("--mb-size", type=int, default=256,
                    help="sequences per micro-batch (<= 1024; > 64 runs the decode projections on the MFMA GEMM)")
    ap.add_argument("--n-mb", type=int, default=0,
                    help="micro-batches in flight (default: 1 at PP=1, pipeline depth + 1 above: one spare micro-batch "
                         "covers the token ring's hand-off latency, parallel/pipeline.py simulate_piped_ring)")
    ap.add_argument("--pp", type=int, default=0,
                    help="pipeline depth (default: = #GPUs); --pp P < N runs N/P data-parallel pipeline replicas")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--link", default="auto", choices=["auto", "rccl", "local", "tcp"],
                    help="stage-to-stage transport (N > 1). torchrun: rccl (auto) or tcp. In-process: rccl pairs "
                         "from ncclCommInitAll, falling back to peer-copy local links if RCCL refuses (auto: rccl "
                         "when every stage has its own GPU)")
    ap.add_argument("--same-device", action="store_true",
                    help="every stage on GPU 0: rehearses the N > 1 path on a 1-GPU box (in-process: local links; "
                         "torchrun: a gloo process group and TCP links, RCCL refuses two ranks of a communicator "
                         "on one GPU)")
    ap.add_argument("--no-secondary", action="store_true", help="N = 1: skip the secondary configs")
    ap.add_argument("--dump-tokens", default=None, metavar="PATH",
                    help="write the headline run's generated tokens to PATH (JSON; A/B of e.g. the bf16 wire)")
    ap.add_argument("--trace", default=None, metavar="PATH",
                    help="after the timed region: 5 traced decode rounds of the headline run, Chrome JSON to PATH")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="extra engine option (A/B runs), e.g. --set fused_norm=false")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # no launcher and --gpus N > 1: the whole N-stage pipeline in this process (engine mode "local",
    # one host thread per GPU); under torchrun every rank owns one stage (engine mode "mp")
    inproc = world == 1 and args.gpus > 1
    if world > 1 and world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    from mipipe.engine import Engine
    from mipipe.parallel import init_from_torchrun

    n_gpus = args.gpus if inproc else world
    pp = args.pp or n_gpus
    if n_gpus % pp or (inproc and pp != n_gpus):
        print(f"bench.py: --pp {pp} with {n_gpus} GPUs: {'in-process runs one pipeline over all GPUs (use torchrun for replicas)' if inproc else 'must divide the GPU count'}",
              file=sys.stderr)
        sys.exit(2)
    replicas = n_gpus // pp
    if inproc:
        devices = [0] * n_gpus if args.same_device else list(range(n_gpus))
        if not args.same_device and torch.cuda.device_count() < n_gpus:
            print(f"bench.py: --gpus {n_gpus} but {torch.cuda.device_count()} visible GPU(s) (--same-device rehearses "
                  "the pipeline on GPU 0)", file=sys.stderr)
            sys.exit(2)
        link = args.link if args.link != "tcp" else "auto"
    else:
        devices = [0]
        link = "tcp" if args.same_device else ("rccl" if args.link in ("auto", "local") else args.link)
    tr_kw = dict(device=0, pg_backend="gloo") if args.same_device and not inproc else {}
    pg_cpu = args.same_device and not inproc

    def factory(model, ftype, mb_size, n_mb, extra=None, prompt_len=None):
        max_ctx = (((prompt_len or args.prompt_len) + args.warmup + args.steps + 8 + 63) // 64) * 64
        cfg = dict(synthetic=MODELS[model], ftype=ftype, n_mb=n_mb, mb_size=mb_size, max_ctx=max_ctx,
                   prefill_chunk=512, graphs=not args.no_graphs, split="cost", seed=1234)
        cfg.update(parse_set(args.set))
        cfg.update(extra or {})
        if inproc:
            # every stage in this process: stage s on devices[s], one host thread per stage
            return lambda: Engine(mode="local", stages=pp, devices=devices, link=link, **cfg)
        # one stage per rank (mipipe.parallel.init_from_torchrun): link r = stage r -> stage (r+1) % N,
        # its sender (rank r) creates the RCCL unique id, exchanged over torch.distributed (RCCL)
        return lambda: init_from_torchrun(pp=pp, link=link, **tr_kw, **cfg)

    n_mb = args.n_mb or (pp + 1 if pp > 1 else 1)
    ms, p50, info = run(factory(args.model, args.ftype, args.mb_size, n_mb), MODELS[args.model]["vocab"],
                        n_mb * args.mb_size, args.prompt_len, args.steps, args.warmup, world, pg_cpu,
                        sorted(set(devices)),
                        dump_tokens=args.dump_tokens if rank == world - 1 else None,   # the last stage's rank
                        trace=(args.trace if world == 1 else f"{args.trace}.rank{rank}") if args.trace else None)
    n_tok = args.steps * n_mb * args.mb_size * replicas
    value = n_tok / (ms / 1e3)

    secondary = {}
    if n_gpus == 1 and not args.no_secondary:
        for label, model, ftype, mb, extra, plen in SECONDARY:
            plen = plen or args.prompt_len
            if model == args.model and ftype == args.ftype and mb == args.mb_size and not extra and plen == args.prompt_len:
                continue
            sms, sp50, _ = run(factory(model, ftype, mb, 1, extra, plen), MODELS[model]["vocab"], mb, plen,
                               args.steps, args.warmup, world, pg_cpu)
            secondary[label] = dict(tok_s=round(args.steps * mb / (sms / 1e3), 2), ms_per_round=round(sms / args.steps, 4),
                                    p50_token_ms=round(sp50, 4))

    elif n_gpus > 1 and replicas == 1 and not args.no_secondary:
        for label, model, ftype, mb in SECONDARY_PP:
            if model == args.model and ftype == args.ftype:
                continue
            sms, sp50, _ = run(factory(model, ftype, mb, n_mb), MODELS[model]["vocab"], n_mb * mb, args.prompt_len,
                               args.steps, args.warmup, world, pg_cpu, sorted(set(devices)))
            secondary[label.format(N=pp)] = dict(tok_s=round(args.steps * n_mb * mb / (sms / 1e3), 2),
                                                 ms_per_round=round(sms / args.steps, 4), p50_token_ms=round(sp50, 4),
                                                 micro_batches=n_mb, mb_size=mb)

    link_info = None
    if n_gpus > 1:
        links = info.get("links", [])
        link_info = dict(kind=sorted({l["kind"] for l in links}), comm_nranks=sorted({l["comm_nranks"] for l in links}),
                         links_per_rank=len(links), act_dtype=info.get("act_dtype"),
                         wire_bytes_per_token=info.get("wire_bytes_per_token"),
                         launcher="in-process" if inproc else "torchrun", engine_mode=info.get("mode"),
                         devices=sorted({s["device"] for s in info["stages"]}), same_device=args.same_device)
        if info.get("link_fallback"):
            link_info["fallback"] = info["link_fallback"]
        if world > 1:
            link_info.update(torch_pg_world=dist.get_world_size(), torch_pg_backend=dist.get_backend())

    if rank == 0:
        m = MODELS[args.model]
        line = {
            "metric": "decode tokens/sec (whole node) + p50/token",
            "value": round(value, 2),
            "unit": "tokens/s",
            "n_gpus": n_gpus,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms / args.steps, 4),
            "p50_token_ms": round(p50, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / BASELINE_TOK_S, 2) if args.model == "llama3-70b" else None,
            # like-for-like with the reference's single-stream figure: the rate EACH sequence sees
            "per_stream_tok_s": round(1e3 / (ms / args.steps), 2),
            "vs_baseline_per_stream": round(1e3 / (ms / args.steps) / BASELINE_TOK_S, 2) if args.model == "llama3-70b" else None,
            "dtype": "bf16-class: f16 MFMA on dequantized " + args.ftype + " weights, f32 accumulate",
            "data": "synthetic prompts, random-init weights (GGUF " + args.ftype + " blocks generated in HBM)",
            "config": {"model": f"{m['name']} {args.ftype}", "global_batch": n_mb * args.mb_size * replicas,
                       "seq_len": args.prompt_len,
                       "parallelism": f"pp{pp}" if replicas == 1 else f"dp{replicas}xpp{pp}",
                       "micro_batches": n_mb, "mb_size": args.mb_size, "max_ctx": info["max_ctx"],
                       "stages": info["stages"]},
        }
        if secondary:
            line["secondary"] = secondary
        if link_info:
            line["link"] = link_info
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
