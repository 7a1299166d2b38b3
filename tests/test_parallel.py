"""mipipe.parallel: the native partitioner through the C API, the piped-ring schedule model, and the
torchrun launch helper (2 processes, CPU stages over TCP, gloo rendezvous)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import REPO, make_model


def test_plan_partition_modes(native):
    from mipipe.parallel import plan_partition
    cost = [1.0] * 10
    assert plan_partition(cost, 3, split="even") == [(0, 4), (4, 7), (7, 10)]
    # a heavy LM head pushes layers off the last stage under "cost", not under "mem"
    cst = plan_partition(cost, 2, split="cost", last_extra=4.0)
    mem = plan_partition(cost, 2, split="mem", last_extra=4.0)
    assert mem == [(0, 5), (5, 10)]
    assert cst == [(0, 7), (7, 10)]
    # a twice-as-fast device takes twice the layers
    assert plan_partition([1.0] * 9, device_speed=[2.0, 1.0]) == [(0, 6), (6, 9)]
    with pytest.raises(RuntimeError):
        plan_partition(cost, 11)


@pytest.mark.parametrize("stages,n_mb", [(1, 1), (2, 1), (2, 2), (4, 4), (4, 8), (8, 8)])
def test_piped_ring_model_matches_bound(stages, n_mb):
    from mipipe.parallel import simulate_piped_ring
    st = [1.0 + 0.1 * s for s in range(stages)]
    r = simulate_piped_ring(st, n_mb, rounds=24, link_ms=0.05, ring_ms=0.02)
    assert r["round_ms"] == pytest.approx(r["bound_ms"])
    if r["bound_ms"] == pytest.approx(n_mb * max(st)):   # throughput-bound: the slowest stage never idles
        assert r["stage_busy"][-1] == pytest.approx(1.0) and r["bubble"] == pytest.approx(0.0, abs=1e-9)
    assert 0.0 <= r["bubble"] < 1.0


def test_piped_ring_needs_micro_batches():
    """One micro-batch on 8 stages leaves each stage busy 1/8 of the time; 8 fill the ring."""
    from mipipe.parallel import simulate_piped_ring
    one = simulate_piped_ring([1.0] * 8, 1)
    eight = simulate_piped_ring([1.0] * 8, 8)
    assert one["round_ms"] == pytest.approx(8.0) and one["stage_busy"][0] == pytest.approx(1 / 8)
    assert eight["round_ms"] == pytest.approx(8.0) and eight["stage_busy"][0] == pytest.approx(1.0)


_SCRIPT = r"""
import json, sys
sys.path.insert(0, {repo!r})
from mipipe.parallel import init_from_torchrun
import torch.distributed as dist
eng = init_from_torchrun(pp={pp}, gguf={path!r}, backend="cpu", max_ctx=128, n_mb=2, mb_size=1, prefill_chunk=16,
                         split="even", base_port={port})
out, _ = eng.generate({prompts!r}, 6)
stages = eng.info["stages"]
last = eng.info["stages"][-1]["stage"]
eng.close()
dist.barrier()
print("OUT " + json.dumps(dict(rank=dist.get_rank(), out=out, stages=stages)), flush=True)
dist.destroy_process_group()
"""


@pytest.mark.parametrize("world,pp", [(2, 2), (4, 2), (2, 1)])
def test_init_from_torchrun_replicas(native, model_dir, tmp_path, world, pp):
    """world / pp data-parallel replicas of a pp-stage pipeline (CPU stages, TCP rings, gloo
    rendezvous): every replica's last stage produces the single-process tokens."""
    from mipipe.engine import Engine
    from test_engine_cpu import free_port
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    prompts = [[5, 6, 7, 8], [9, 10]]
    with Engine(gguf=path, backend="cpu", max_ctx=128, n_mb=2, mb_size=1, prefill_chunk=16) as eng:
        ref, _ = eng.generate(prompts, 6)
    script = tmp_path / "run.py"
    script.write_text(_SCRIPT.format(repo=REPO, path=path, prompts=prompts, port=free_port(), pp=pp))
    mport = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(mport), OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    res = {}
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
        d = json.loads([l for l in o.splitlines() if l.startswith("OUT ")][-1][4:])
        res[d["rank"]] = d
    for g in range(world // pp):
        last = res[g * pp + pp - 1]
        assert len(last["stages"]) == pp
        assert last["out"] == ref   # the replica's last stage holds the generated tokens


_ELASTIC = r"""
import json, os, sys
sys.path.insert(0, {repo!r})
from mipipe.parallel import generate_elastic
import torch.distributed as dist
out = generate_elastic({prompts!r}, {n!r}, {ckpt!r}, every=3, pp=2, gguf={path!r}, backend="cpu", max_ctx=128,
                       n_mb=2, mb_size=1, prefill_chunk=16, split="even", base_port={port})
# one file per (rank, attempt): torchrun merges the ranks' stdout, and two lines written at once can
# interleave mid-line
res = dict(rank=int(os.environ["RANK"]), restart=os.environ.get("TORCHELASTIC_RESTART_COUNT"), out=out)
with open(os.path.join({ckpt!r}, "..", "out_%d_%s.json" % (res["rank"], res["restart"])), "w") as f:
    json.dump(res, f)
dist.destroy_process_group()
"""


def test_elastic_rank_restart_resumes_from_checkpoint(native, model_dir, tmp_path):
    """A 2-stage multi-process pipeline under `torchrun --max-restarts 1`: rank 1 dies after 7
    decode rounds; torchrun restarts both ranks, they resume from the round-6 checkpoint and the
    generation equals the uninterrupted single-process one."""
    from mipipe.engine import Engine
    from test_engine_cpu import free_port
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    prompts, n = [[5, 6, 7, 8], [9, 10]], 12
    with Engine(gguf=path, backend="cpu", max_ctx=128, n_mb=2, mb_size=1, prefill_chunk=16) as eng:
        ref, _ = eng.generate(prompts, n)
    ckpt = tmp_path / "ckpt"
    script = tmp_path / "run.py"
    script.write_text(_ELASTIC.format(repo=REPO, path=path, prompts=prompts, n=n, ckpt=str(ckpt), port=free_port()))
    env = dict(os.environ, OMP_NUM_THREADS="2", MIPIPE_ELASTIC_FAIL="1,7")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2", "--max-restarts", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), str(script)]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-3000:])
    outs = [json.loads(f.read_text()) for f in sorted(tmp_path.glob("out_*.json"))]
    assert len(outs) == 2, (outs, p.stdout[-2000:])
    assert {o["restart"] for o in outs} == {"1"}, outs       # only the restarted attempt finished
    assert all(o["out"] == ref for o in outs)
    assert not list((ckpt / "replica0").glob("round_*"))   # a finished run removes its checkpoints


def test_elastic_checkpoint_of_another_run_is_ignored(native, model_dir, tmp_path):
    """A checkpoint left by one run (other prompts / n_predict) on the same directory is not resumed
    by the next run: the next run generates its own prompts from scratch."""
    from mipipe.engine import Engine
    from mipipe.parallel import elastic as E
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    kw = dict(gguf=path, backend="cpu", max_ctx=128, prefill_chunk=16)
    root = tmp_path / "ckpt"
    # a stale, COMPLETE checkpoint of an older run (other prompts) in replica 0's directory
    with Engine(**kw) as eng:
        eng.start([[11, 12, 13]])
        eng.decode(4)
        d = root / "replica0" / "round_00000004"
        d.parent.mkdir(parents=True)
        eng.save_state(str(d))
        (d / "RUN").write_text(E.run_digest([[11, 12, 13]], 20, dict(kw, pp=None, every=4)))
        (d / "COMPLETE").write_text("")
    prompts = [[5, 6, 7, 8]]
    with Engine(**kw) as eng:
        ref, _ = eng.generate(prompts, 9)
    out = E.generate_elastic(prompts, 9, str(root), every=4, **kw)
    assert out == ref
    assert (root / "replica0" / "round_00000004").exists()   # another run's checkpoint is left alone


_SPEC = r"""
import json, sys
sys.path.insert(0, {repo!r})
from mipipe.parallel import init_from_torchrun
import torch.distributed as dist
eng = init_from_torchrun(pp={pp}, gguf={path!r}, backend="cpu", max_ctx=128, n_mb=2, mb_size=2, prefill_chunk=32,
                         split="even", base_port={port})
out, st = eng.spec_generate({prompts!r}, {n}, draft_max=4, ngram=2)
eng.close()
dist.barrier()
print("OUT " + json.dumps(dict(rank=dist.get_rank(), out=out, stats=st)), flush=True)
dist.destroy_process_group()
"""


@pytest.mark.parametrize("pp", [2, 3])
def test_spec_generate_across_processes(native, model_dir, tmp_path, pp):
    """Speculative decoding (prompt lookup) with one process per stage: after every verify pass the
    last stage's tokens travel the ring to every rank, so all ranks draft the same next chunk; every
    rank's output equals single-process greedy decoding (the design report's
    distributed speculative decoding, PDF p.12)."""
    from mipipe.engine import Engine
    from test_engine_cpu import free_port
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    # repetitive prompts so lookup drafts exist (the acceptance itself depends on the model)
    prompts = [[5, 6, 7, 8, 5, 6, 7, 8, 5, 6], [9, 10, 11, 9, 10, 11, 9], [20, 21, 22, 23, 20, 21], [40, 41, 40, 41]]
    n = 10
    with Engine(gguf=path, backend="cpu", max_ctx=128, n_mb=2, mb_size=2, prefill_chunk=32) as eng:
        ref, _ = eng.generate(prompts, n)
    script = tmp_path / "spec.py"
    script.write_text(_SPEC.format(repo=REPO, path=path, prompts=prompts, n=n, port=free_port(), pp=pp))
    mport = free_port()
    procs = []
    for r in range(pp):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(pp), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(mport), OMP_NUM_THREADS="2")
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=240) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
        d = json.loads([l for l in o.splitlines() if l.startswith("OUT ")][-1][4:])
        assert d["out"] == ref, (d["rank"], d["out"], ref)
        assert d["stats"]["verify_rounds"] >= 1 and d["stats"]["drafted"] >= 1
