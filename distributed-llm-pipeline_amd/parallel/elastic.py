"""Rank restart for multi-process pipelines (one process per stage / GPU).

The reference's design report restarts a dead worker and resumes (auto-healing, PDF p.6-7
§5.2-5.3).  A pipeline rank cannot be replaced on its own: its RCCL communicator
and the TCP / RCCL links of its neighbours die with it.  So recovery here is at the level of the
whole ring, the torchrun way:

  * every `every` decode rounds all ranks of a replica write a checkpoint together
    (`Engine.save_state`: each rank its own stage's KV shard, the last stage the sequences), then
    the replica's stage 0 marks it COMPLETE (after a barrier, so a checkpoint is either whole or
    ignored) and removes the older ones;
  * a rank that dies makes the torchrun elastic agent (`--max-restarts N`) stop the survivors and
    start every rank again;
  * the restarted ranks rebuild their stages, load the newest COMPLETE checkpoint and continue;
    greedy and seeded sampling resume token for token (`load_state` restores the sampler step).

    torchrun --nproc-per-node 8 --max-restarts 3 --master-addr 127.0.0.1 run.py
    # run.py:
    from mipipe.parallel.elastic import generate_elastic
    tokens = generate_elastic(prompts, 256, "/scratch/ckpt", every=32, synthetic=..., ftype="Q4_K")

Fault injection for tests: MIPIPE_ELASTIC_FAIL="rank,round" makes that global rank exit after
completing `round` decode rounds, on the first attempt only (TORCHELASTIC_RESTART_COUNT == 0).
"""
from __future__ import annotations

import os
import shutil

_MARK = "COMPLETE"


def _ckpt_name(rounds: int) -> str:
    return f"round_{rounds:08d}"


def latest_checkpoint(root: str) -> tuple[str | None, int]:
    """(path, rounds) of the newest COMPLETE checkpoint under `root`, or (None, 0)."""
    best, n = None, 0
    if os.path.isdir(root):
        for d in os.listdir(root):
            if d.startswith("round_") and os.path.exists(os.path.join(root, d, _MARK)):
                r = int(d[6:])
                if best is None or r > n:
                    best, n = os.path.join(root, d), r
    return best, n


def _maybe_fail(rank: int, rounds: int):
    spec = os.environ.get("MIPIPE_ELASTIC_FAIL")
    if not spec or os.environ.get("TORCHELASTIC_RESTART_COUNT", "0") != "0":
        return
    r, k = (int(v) for v in spec.split(","))
    if rank == r and rounds >= k:
        os._exit(17)   # a crash, not an exception: no cleanup, links left dangling


def generate_elastic(prompts, n_predict: int, ckpt_dir: str, every: int = 16, pp: int | None = None, **cfg):
    """Greedy / sampled generation of `prompts` (token id lists) for `n_predict` tokens on this
    torchrun rank's pipeline stage, checkpointed every `every` rounds under `ckpt_dir` and
    resumed from the newest complete checkpoint after a restart.  Returns the generated tokens on
    every rank of the replica (broadcast from its last stage)."""
    import torch.distributed as dist

    from .pipeline import init_from_torchrun

    if n_predict < 1 or every < 1:
        raise ValueError("n_predict and every must be >= 1")
    eng = init_from_torchrun(pp=pp, **cfg)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    pp = int(pp or world)
    group, stage = divmod(rank, pp)
    root = os.path.join(ckpt_dir, f"replica{group}")
    os.makedirs(root, exist_ok=True)
    # the barrier of this replica's ranks (one process group per replica, created on every rank)
    groups = [dist.new_group(list(range(g * pp, (g + 1) * pp))) for g in range(world // pp)] if world > 1 else None
    sync = (lambda: dist.barrier(group=groups[group])) if groups else (lambda: None)
    try:
        path, done = latest_checkpoint(root)
        if path:
            eng.load_state(path)
        else:
            eng.start(prompts)   # prefill + first token
            done = 0
        remaining = n_predict - 1 - done
        while remaining > 0:
            k = min(every, remaining)
            eng.decode(k)
            done += k
            remaining -= k
            _maybe_fail(rank, done)
            if remaining <= 0:
                break
            d = os.path.join(root, _ckpt_name(done))
            sync()
            eng.save_state(d)
            sync()
            if stage == 0:
                open(os.path.join(d, _MARK), "w").close()
                for old in os.listdir(root):
                    if old.startswith("round_") and old != _ckpt_name(done):
                        shutil.rmtree(os.path.join(root, old), ignore_errors=True)
            sync()
        # the last stage samples, so it holds every token; the replica's other ranks take its list
        toks = [[t[:n_predict] for t in eng.tokens()] if stage == pp - 1 else None]
        if groups:
            dist.broadcast_object_list(toks, src=group * pp + pp - 1, group=groups[group])
        return toks[0]
    finally:
        eng.close()
