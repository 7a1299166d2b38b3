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
    greedy and seeded sampling resume token for token (`load_state` restores the sampler step);
  * every checkpoint carries a digest of the run (prompts, n_predict, engine config): a later call
    with other prompts or settings on the same directory ignores it instead of resuming someone
    else's generation, and a run that finishes removes its checkpoints.

    torchrun --nproc-per-node 8 --max-restarts 3 --master-addr 127.0.0.1 run.py
    # run.py:
    from mipipe.parallel.elastic import generate_elastic
    tokens = generate_elastic(prompts, 256, "/scratch/ckpt", every=32, synthetic=..., ftype="Q4_K")

Fault injection for tests: MIPIPE_ELASTIC_FAIL="rank,round" makes that global rank exit after
completing `round` decode rounds, on the first attempt only (TORCHELASTIC_RESTART_COUNT == 0).
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil

_MARK = "COMPLETE"
_RUN = "RUN"   # digest of the run that wrote the checkpoint


def _ckpt_name(rounds: int, digest: str = "") -> str:
    return f"round_{rounds:08d}" + (f"_{digest[:12]}" if digest else "")


def run_digest(prompts, n_predict: int, cfg: dict) -> str:
    """Identity of a generation run: a checkpoint is resumed only by the run that wrote it."""
    blob = json.dumps(dict(prompts=[[int(t) for t in p] for p in prompts], n_predict=int(n_predict), cfg=cfg),
                      sort_keys=True, default=str)
    return hashlib.sha256(blob.encode()).hexdigest()


def _digest_of(d: str) -> str | None:
    try:
        with open(os.path.join(d, _RUN)) as f:
            return f.read().strip()
    except OSError:
        return None


def latest_checkpoint(root: str, digest: str | None = None) -> tuple[str | None, int]:
    """(path, rounds) of the newest COMPLETE checkpoint under `root` (written by the run `digest`,
    when given), or (None, 0)."""
    best, n = None, 0
    if os.path.isdir(root):
        for d in os.listdir(root):
            p = os.path.join(root, d)
            if d.startswith("round_") and os.path.exists(os.path.join(p, _MARK)):
                if digest is not None and _digest_of(p) != digest:
                    continue
                r = int(d[6:14])
                if best is None or r > n:
                    best, n = p, r
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
    digest = run_digest(prompts, n_predict, dict(cfg, pp=pp, every=every))
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
        path, done = latest_checkpoint(root, digest)
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
            d = os.path.join(root, _ckpt_name(done, digest))
            sync()
            eng.save_state(d)
            sync()
            if stage == 0:
                with open(os.path.join(d, _RUN), "w") as f:
                    f.write(digest)
                open(os.path.join(d, _MARK), "w").close()
                for old in os.listdir(root):   # this run's older checkpoints (not other runs')
                    if (old.startswith("round_") and old != _ckpt_name(done, digest)
                            and _digest_of(os.path.join(root, old)) in (digest, None)):
                        shutil.rmtree(os.path.join(root, old), ignore_errors=True)
            sync()
        # the last stage samples, so it holds every token; the replica's other ranks take its list
        toks = [[t[:n_predict] for t in eng.tokens()] if stage == pp - 1 else None]
        if groups:
            dist.broadcast_object_list(toks, src=group * pp + pp - 1, group=groups[group])
        # finished: this run's checkpoints are spent (every rank has its tokens)
        sync()
        if stage == 0:
            for old in os.listdir(root):
                if old.startswith("round_") and _digest_of(os.path.join(root, old)) == digest:
                    shutil.rmtree(os.path.join(root, old), ignore_errors=True)
        return toks[0]
    finally:
        eng.close()
