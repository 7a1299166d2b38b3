"""Pipeline-parallel planning and launch helpers around the native engine.

The pipeline itself (stage workers, links, the micro-batched piped ring) is C++
(csrc/runtime/engine.cpp). This module exposes the parts a user plans with:

* plan_partition: the engine's own contiguous layer partitioner (model.cpp), called through the C
  API. It plays the part of llama.cpp's tensor_split and of the design report's Halda
  scheduler (PDF p.5, D2).
* simulate_piped_ring: an event model of the engine's decode schedule. Use it to choose the number
  of micro-batches for given per-stage and per-link times (D1, the piped ring).
* init_from_torchrun: one process per GPU. It reads torchrun's RANK, WORLD_SIZE and LOCAL_RANK,
  sets up the RCCL unique ids of the ring's links over torch.distributed, and builds an
  Engine(mode="mp"). This is the MI355X form of prima.cpp's --world/--rank launch (D11). With
  pp < world it runs world/pp data-parallel replicas of a pp-stage pipeline (SURVEY.md 2.4,
  "replica DP, e.g. 2 x PP4").
"""
from __future__ import annotations

import json
import os

from .. import _native as N


def plan_partition(layer_cost, n_stages: int | None = None, split: str = "cost", first_extra: float = 0.0,
                   last_extra: float = 0.0, device_speed=None) -> list[tuple[int, int]]:
    """Contiguous [begin, end) layer ranges for each stage.

    The split modes:

    * "even": equal layer counts.
    * "mem": balance the layer bytes only.
    * "cost": also charge first_extra (the embedding) to stage 0 and last_extra (the LM head) to
      the last stage.

    "mem" and "cost" minimise the slowest stage's cost divided by its device_speed.
    """
    speed = list(device_speed) if device_speed is not None else [1.0] * int(n_stages or 1)
    if n_stages is not None and len(speed) != n_stages:
        raise ValueError("device_speed needs one entry per stage")
    cfg = dict(layer_cost=[float(c) for c in layer_cost], device_speed=[float(s) for s in speed],
               first_extra=float(first_extra), last_extra=float(last_extra), split=split)
    out = N.jcall(N.lib().mp_plan_partition, N.cstr(json.dumps(cfg)), what="plan_partition")
    return [(int(a), int(b)) for a, b in out]


def simulate_piped_ring(stage_ms, n_mb: int, rounds: int = 16, link_ms: float = 0.0, ring_ms: float = 0.0) -> dict:
    """Event model of the engine's decode schedule.

    Every stage runs its items in (round, micro-batch) order. Item (r, m) on stage s starts when
    all of these hold:

    * stage s is free;
    * stage s-1 has finished (r, m), plus link_ms;
    * on stage 0 with r > 0: the last stage has finished (r-1, m), plus ring_ms (the sampled
      token coming back around the ring).

    Returns the steady-state ms per round (every sequence emits one token per round), the
    busy fraction of each stage, and the closed-form bound:
    max(n_mb * max(stage_ms), sum(stage_ms) + (S-1) * link_ms + ring_ms).
    """
    S = len(stage_ms)
    if S < 1 or n_mb < 1 or rounds < 2:
        raise ValueError("need >= 1 stage, >= 1 micro-batch, >= 2 rounds")
    free = [0.0] * S
    done = {}   # (s, r, m) -> finish time
    for r in range(rounds):
        for m in range(n_mb):
            for s in range(S):
                t = free[s]
                if s > 0:
                    t = max(t, done[(s - 1, r, m)] + link_ms)
                elif r > 0:
                    t = max(t, done[(S - 1, r - 1, m)] + ring_ms)
                done[(s, r, m)] = free[s] = t + stage_ms[s]
    # steady state from the second half of the rounds
    r0 = rounds // 2
    t0 = done[(S - 1, r0 - 1, n_mb - 1)]
    t1 = done[(S - 1, rounds - 1, n_mb - 1)]
    round_ms = (t1 - t0) / (rounds - r0)
    bound = max(n_mb * max(stage_ms), sum(stage_ms) + (S - 1) * link_ms + ring_ms)
    return dict(round_ms=round_ms, bound_ms=bound,
                stage_busy=[n_mb * c / round_ms for c in stage_ms],
                bubble=max(0.0, 1.0 - n_mb * max(stage_ms) / round_ms))


def init_from_torchrun(pp: int | None = None, device: int | None = None, pg_backend: str | None = None, **cfg):
    """Build this rank's Engine stage under torchrun, with one process per GPU.

    `pp` is the pipeline depth (default: the world size). The world splits into world // pp
    independent replicas of a pp-stage pipeline: data parallelism across replicas, pipeline
    parallelism within each. Replica g holds ranks [g*pp, (g+1)*pp). With pp = 1 every rank runs the
    whole model on its own GPU.

    Inside a replica the ring has one link per rank: stage r sends to stage (r+1) % pp. The sender
    of each link creates its RCCL unique id, and the ids are exchanged with torch.distributed
    (backend "nccl", which is RCCL on ROCm). Keyword arguments are engine config keys (see
    mipipe.engine).

    `device` overrides the GPU of this rank (default LOCAL_RANK) and `pg_backend` the
    torch.distributed backend (default: "nccl" for GPU stages, "gloo" for CPU stages).  Several
    ranks on ONE GPU (a rehearsal of the multi-rank path on a 1-GPU box) need device=0,
    pg_backend="gloo" and link="tcp": RCCL refuses two ranks of one communicator on one GPU.
    """
    import torch
    import torch.distributed as dist

    from ..engine import Engine, rccl_unique_id_hex

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    pp = int(pp or world)
    if pp < 1 or world % pp:
        raise ValueError(f"pipeline depth {pp} does not divide the world size {world}")
    group, stage = divmod(rank, pp)
    link = cfg.pop("link", "rccl")
    cpu = cfg.get("backend", "hip") == "cpu"
    if cpu:
        link = "tcp"   # RCCL moves device buffers; CPU stages talk over TCP
    dev = local_rank if device is None else int(device)
    if not cpu:
        torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        kw = {}
        restart = os.environ.get("TORCHELASTIC_RESTART_COUNT")
        if restart not in (None, "0") and os.environ.get("TORCHELASTIC_USE_AGENT_STORE", "").lower() == "true":
            # under torchrun the agent's store outlives a restart: key a restarted attempt's
            # rendezvous by the restart count, or its ranks read the dead attempt's peer addresses
            # (parallel/elastic.py)
            from datetime import timedelta
            base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]), world, False,
                                 timeout=timedelta(seconds=300))
            kw = dict(store=dist.PrefixStore(f"mipipe/attempt_{restart}", base), rank=rank, world_size=world)
        backend = pg_backend or ("gloo" if cpu else "nccl")
        if backend == "gloo":
            dist.init_process_group("gloo", **kw)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev), **kw)
    if pp == 1:
        cfg.setdefault("mode", "local")
        cfg.setdefault("stages", 1)
        cfg.setdefault("devices", [dev])
        return Engine(**cfg)
    if cfg.get("device_speed") == "probe":
        # Halda: every rank measures its own device, the list is gathered so all ranks of the
        # replica derive the same cost-balanced partition
        from ..engine import device_probe
        mine = device_probe(-1 if cpu else dev)["speed"]
        speeds = [None] * world
        if world > 1:
            dist.all_gather_object(speeds, mine)
        else:
            speeds = [mine]
        cfg["device_speed"] = speeds[group * pp:(group + 1) * pp]
    cfg.update(mode="mp", world=pp, rank=stage, device=dev, link=link)
    if link == "rccl":
        ids = [None] * world
        dist.all_gather_object(ids, rccl_unique_id_hex())
        cfg["rccl_ids"] = ids[group * pp:(group + 1) * pp]
    else:
        base = cfg.pop("base_port", int(os.environ.get("MASTER_PORT", "29500")) + 11)
        cfg["base_port"] = base + group * pp   # each replica's ring on its own ports
    return Engine(**cfg)
