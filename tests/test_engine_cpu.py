"""CPU-backend engine tests (no GPU): the CpuStage model against the torch fp32 oracle, the
pipeline runtime (multi-stage in one process over HostLinks, multi-process over TCP links),
micro-batch invariance and seeded sampling.  These exercise the same scheduler/ring code the
GPU path uses (engine.cpp), so the pipeline logic is covered on every CPU test run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import REPO, make_model


def nmse(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("name,ftype", [("stories15m", "F32"), ("tiny-gqa", "Q8_0"), ("tiny-gqa", "Q4_K_M"),
                                        ("tiny-l3", "Q6_K"), ("tiny-moe", "Q5_K_M"), ("tiny-gqa", "BF16"),
                                        ("tiny-qwen2", "Q4_K_M")])
@pytest.mark.parametrize("act", ["f32", "q8"])
def test_cpu_engine_matches_reference(native, model_dir, name, ftype, act):
    """cpu_act f32 (dequantized weights, f32 dots): the fp32 oracle to 1e-8.  cpu_act q8 (the default:
    integer dots against int8 activation blocks, cpu_qdot.cpp): within the int8 rounding of the
    activations, and the oracle's greedy token wherever its top-2 margin is clear."""
    from mipipe.engine import Engine
    from mipipe.models.reference import RefLlama
    path, cfg = make_model(model_dir, name, ftype)
    ref = RefLlama.from_gguf(path)
    rng = np.random.default_rng(0)
    prompt = [int(t) for t in rng.integers(3, cfg.vocab, 21)]
    tol = 1e-8 if act == "f32" else 2e-3
    with Engine(gguf=path, backend="cpu", max_ctx=128, prefill_chunk=16, threads=4, cpu_act=act) as eng:
        eng.start([prompt])
        lg = eng.logits()[0]
        ref.reset()
        rl = ref.forward(prompt, 0)[-1].numpy()
        assert nmse(lg, rl) < tol, nmse(lg, rl)
        pos = len(prompt)
        for step in range(4):
            tok = eng.tokens()[0][-1]
            top2 = np.sort(rl)[-2:]
            if act == "f32" or top2[1] - top2[0] > 0.05 * (abs(top2).max() + 1):
                assert tok == int(rl.argmax()), step
            eng.decode(1)
            lg = eng.logits()[0]
            rl = ref.forward([tok], pos)[-1].numpy()
            pos += 1
            assert nmse(lg, rl) < tol, (step, nmse(lg, rl))


@pytest.mark.parametrize("stages,n_mb", [(2, 2), (3, 3), (4, 1)])
def test_cpu_pipeline_matches_pp1(native, model_dir, stages, n_mb):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    rng = np.random.default_rng(1)
    prompts = [[int(t) for t in rng.integers(3, cfg.vocab, n)] for n in (9, 40, 3, 17, 5, 2)[: 2 * n_mb]]
    with Engine(gguf=path, backend="cpu", max_ctx=128, n_mb=1, mb_size=len(prompts), prefill_chunk=16) as eng:
        ref_out, _ = eng.generate(prompts, 7)
    with Engine(gguf=path, backend="cpu", max_ctx=128, n_mb=n_mb, mb_size=2, prefill_chunk=16,
                stages=stages, split="even") as eng:
        assert len(eng.info["stages"]) == stages
        out, _ = eng.generate(prompts, 7)
        # a second generation on the same engine (ring drained, KV slots reused)
        out2, _ = eng.generate(prompts[:1], 5)
    assert out == ref_out
    assert out2[0] == ref_out[0][:5]


def test_cpu_microbatch_invariance(native, model_dir):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-moe", "Q8_0")
    prompts = [[11, 12, 13], [400, 5, 6, 7, 8, 9, 10], [42]]
    singles = []
    with Engine(gguf=path, backend="cpu", max_ctx=64) as eng:
        for p in prompts:
            o, _ = eng.generate([p], 6)
            singles.append(o[0])
    with Engine(gguf=path, backend="cpu", max_ctx=64, n_mb=2, mb_size=2) as eng:
        o, _ = eng.generate(prompts, 6)
    assert o == singles


def test_cpu_microbatch_over_64_rows(native, model_dir):
    """mb_size > 64 (decode projections on the prompt GEMM on the HIP backend): the runtime's
    slot bookkeeping, token ring and pager take micro-batches wider than one GEMV row block."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    rng = np.random.default_rng(72)
    prompts = [[int(t) for t in rng.integers(3, cfg.vocab, size=int(rng.integers(1, 6)))] for _ in range(72)]
    with Engine(gguf=path, backend="cpu", max_ctx=64) as eng:
        singles = [eng.generate([p], 4)[0][0] for p in (prompts[0], prompts[65], prompts[71])]
    with Engine(gguf=path, backend="cpu", max_ctx=64, n_mb=1, mb_size=72) as eng:
        o, _ = eng.generate(prompts, 4)
    assert [o[0], o[65], o[71]] == singles


def test_cpu_sampling_seeded(native, model_dir):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    prompts = [[5, 6, 7], [8, 9, 10, 11]]
    outs = []
    for seed in (7, 7, 8):
        with Engine(gguf=path, backend="cpu", max_ctx=64, mb_size=2, temp=1.5, top_k=40, top_p=0.9,
                    min_p=0.01, seed=seed) as eng:
            o, _ = eng.generate(prompts, 12)
            outs.append(o)
    assert outs[0] == outs[1] and outs[0] != outs[2]
    assert all(0 <= t < cfg.vocab for seq in outs[0] for t in seq)


def test_cpu_synthetic_bench(native):
    from mipipe.engine import Engine
    syn = dict(n_layer=2, d_model=256, n_head=4, n_head_kv=2, d_ff=512, vocab=1024)
    with Engine(synthetic=syn, backend="cpu", ftype="Q4_K_M", max_ctx=128, n_mb=2, mb_size=2, stages=2) as eng:
        r = eng.bench(prompt_len=8, warmup=1, steps=4)
    assert r["decode_tok_s"] > 0 and r["p50_ms"] > 0


def test_bench_py_inprocess_pipeline_cpu():
    """`python bench.py --gpus 2` with no launcher (no WORLD_SIZE) runs a 2-stage pipeline in ONE
    process (engine mode "local"), here on the CPU backend: one JSON line with 2 stages, N + 1
    micro-batches, and the data plane the engine reports."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--same-device", "--model", "tinyllama",
           "--ftype", "Q4_K_M", "--steps", "1", "--warmup", "0", "--mb-size", "1", "--prompt-len", "4",
           "--set", "backend=cpu", "--set", "threads=4", "--no-secondary"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["parallelism"] == "pp2"
    assert d["config"]["micro_batches"] == 3 and len(d["config"]["stages"]) == 2
    assert d["link"]["launcher"] == "in-process" and d["link"]["engine_mode"] == "local"
    assert d["link"]["kind"] == ["host"] and d["link"]["links_per_rank"] == 4


def test_bench_py_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], capture_output=True,
                       text=True, timeout=120, cwd=REPO, env=env)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


_MP_SCRIPT = r"""
import json, sys
sys.path.insert(0, {repo!r})
from mipipe.engine import Engine
cfg = json.loads(sys.argv[1])
with Engine(**cfg) as eng:
    out, _ = eng.generate({prompts!r}, 7)
    print("OUT " + json.dumps(out if cfg["rank"] == cfg["world"] - 1 else None), flush=True)
"""


@pytest.mark.parametrize("world", [2, 3])
def test_cpu_multiprocess_tcp_pipeline(native, model_dir, world):
    """One process per stage (the torchrun layout of bench.py / mi-cli --world/--rank), TCP ring."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q4_K_M")
    prompts = [[3, 4, 5, 6], [7, 8], [9, 10, 11]]
    with Engine(gguf=path, backend="cpu", max_ctx=64, n_mb=3, mb_size=1) as eng:
        ref_out, _ = eng.generate(prompts, 7)
    port = free_port()
    script = _MP_SCRIPT.format(repo=REPO, prompts=prompts)
    procs = []
    for r in range(world):
        c = dict(gguf=path, backend="cpu", mode="mp", world=world, rank=r, link="tcp", base_port=port,
                 max_ctx=64, n_mb=3, mb_size=1, split="even", threads=2)
        procs.append(subprocess.Popen([sys.executable, "-c", script, json.dumps(c)], stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True, cwd=REPO))
    outs = []
    for p in procs:
        o, _ = p.communicate(timeout=240)
        assert p.returncode == 0, o[-3000:]
        outs.append(o)
    last = [l for l in outs[-1].splitlines() if l.startswith("OUT ")]
    assert last and json.loads(last[0][4:]) == ref_out


def test_fault_injection_fail_and_health(native, model_dir):
    """A stage that throws mid-run aborts the links; the error surfaces with its cause and the
    engine health turns not-ok."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with Engine(gguf=path, backend="cpu", max_ctx=64, n_mb=2, mb_size=1, stages=2, split="even",
                fault={"stage": 1, "fail_at": 5}) as eng:
        assert eng.health()["ok"]
        with pytest.raises(RuntimeError, match="injected fault"):
            eng.generate([[3, 4, 5], [6, 7]], 8)
        assert not eng.health()["ok"]


def test_fault_injection_dropped_message_times_out(native, model_dir):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with Engine(gguf=path, backend="cpu", max_ctx=64, n_mb=1, mb_size=1, stages=2, split="even",
                link_timeout_s=1.5, fault={"stage": 0, "drop_send_at": 3}) as eng:
        with pytest.raises(RuntimeError, match="timed out|aborted"):
            eng.generate([[3, 4, 5]], 8)


def test_fault_delay_and_trace(native, model_dir, tmp_path):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with Engine(gguf=path, backend="cpu", max_ctx=64, n_mb=2, mb_size=1, stages=2, split="even",
                fault={"stage": 0, "delay_ms": 5}) as eng:
        eng.trace(True)
        out, _ = eng.generate([[3, 4, 5], [6, 7]], 6)
        h = eng.health()
        eng.write_trace(str(tmp_path / "t.json"))
    assert h["ok"] and all(s["items_done"] > 0 for s in h["stages"])
    assert h["stages"][0]["bytes_sent"] > 0
    ev = json.load(open(tmp_path / "t.json"))["traceEvents"]
    spans = [e for e in ev if e["ph"] == "X"]
    assert {e["pid"] for e in spans} == {0, 1}
    dec0 = [e for e in spans if e["pid"] == 0 and e["name"].startswith("decode")]
    assert dec0 and all(e["dur"] >= 0 for e in dec0)


def _penalize(lg, window, rep, fq, pr):
    lg = lg.copy()
    for t in set(window):
        c = window.count(t)
        l = lg[t]
        lg[t] = (l / rep if l > 0 else l * rep) - c * fq - pr
    return lg


def test_cpu_repetition_penalties_match_reference(native, model_dir):
    """Greedy decoding with llama.cpp-style penalties over the last n accepted tokens (prompt
    included) against the torch oracle with the penalties applied in Python."""
    from mipipe.engine import Engine
    from mipipe.models.reference import RefLlama
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    ref = RefLlama.from_gguf(path)
    prompt = [5, 9, 5, 17, 30, 9]
    rep, fq, pr, last_n = 1.8, 0.3, 0.4, 8
    with Engine(gguf=path, backend="cpu", cpu_act="f32", max_ctx=64, repeat_penalty=rep, frequency_penalty=fq,
                presence_penalty=pr, repeat_last_n=last_n) as eng:
        out, _ = eng.generate([prompt], 10)
    ref.reset()
    seq = list(prompt)
    lg = ref.forward(prompt, 0)[-1].numpy()
    want = []
    for step in range(10):
        tok = int(_penalize(lg, seq[-last_n:], rep, fq, pr).argmax())
        want.append(tok)
        lg = ref.forward([tok], len(seq))[-1].numpy()
        seq.append(tok)
    assert out[0] == want
    with Engine(gguf=path, backend="cpu", max_ctx=64) as eng:
        plain, _ = eng.generate([prompt], 10)
    assert plain[0] != want   # the penalties changed the greedy path


@pytest.mark.parametrize("stages,n_mb,mb_size", [(1, 1, 1), (1, 2, 2), (2, 2, 2)])
def test_cpu_speculative_lookup_matches_greedy(native, model_dir, stages, n_mb, mb_size):
    """Prompt-lookup speculative decoding reproduces plain greedy decoding exactly,
    across micro-batches and pipeline stages, and accepts drafts on repetitive context."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    rng = np.random.default_rng(3)
    motif = [int(t) for t in rng.integers(3, cfg.vocab, 6)]
    prompts = [motif * 4, [int(t) for t in rng.integers(3, cfg.vocab, 11)], motif * 2 + [7, 8], [42, 43, 44]]
    prompts = prompts[: n_mb * mb_size]
    kw = dict(gguf=path, backend="cpu", max_ctx=128, n_mb=n_mb, mb_size=mb_size, prefill_chunk=32,
              stages=stages, split="even")
    with Engine(**kw) as eng:
        ref, _ = eng.generate(prompts, 24)
    with Engine(**kw) as eng:
        out, st = eng.spec_generate(prompts, 24, draft_max=5, ngram=3)
        # the engine stays usable for plain generation afterwards
        again, _ = eng.generate(prompts[:1], 6)
    assert out == ref
    assert again[0] == ref[0][:6]
    assert st["verify_rounds"] <= 23
    assert st["drafted"] >= st["accepted"] >= 0


def test_cpu_speculative_lookup_accepts_repeats(native, model_dir):
    """Greedy decoding of stories15m (random init) falls into a repeated-token run that prompt
    lookup drafts and the verifier accepts: fewer verify rounds than tokens, same output."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "stories15m", "F32")
    rng = np.random.default_rng(3)
    prompt = [int(t) for t in rng.integers(3, cfg.vocab, 6)] * 4
    with Engine(gguf=path, backend="cpu", max_ctx=256) as eng:
        ref, _ = eng.generate([prompt], 60)
        out, st = eng.spec_generate([prompt], 60, draft_max=5, ngram=3)
    assert out == ref
    assert st["accepted"] > 0 and st["verify_rounds"] < 59, st
    assert st["n_decode_tokens"] == 59


def test_cpu_speculative_rejects_sampling(native, model_dir):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with Engine(gguf=path, backend="cpu", max_ctx=64, temp=0.8) as eng:
        with pytest.raises(RuntimeError, match="greedy"):
            eng.spec_generate([[5, 6, 7]], 4)


@pytest.mark.parametrize("stages,n_mb,sampling", [(1, 1, False), (2, 2, False), (3, 3, True)])
def test_cpu_checkpoint_resume(native, model_dir, tmp_path, stages, n_mb, sampling):
    """save_state between decode rounds, load into a fresh engine: the resumed generation equals
    the uninterrupted one token for token (greedy, and seeded sampling with penalties)."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    rng = np.random.default_rng(3)
    prompts = [[int(t) for t in rng.integers(3, cfg.vocab, n)] for n in (9, 70, 3, 17, 5, 2)[: 2 * n_mb]]
    kw = dict(gguf=path, backend="cpu", max_ctx=128, n_mb=n_mb, mb_size=2, prefill_chunk=16, stages=stages,
              split="even")
    if sampling:
        kw.update(temp=1.2, top_k=30, top_p=0.95, seed=11, repeat_penalty=1.3, repeat_last_n=16)
    with Engine(**kw) as eng:
        eng.start(prompts)
        eng.decode(3)
        r = eng.save_state(str(tmp_path / "st"))
        assert r["rounds_done"] == 3 and r["sequences"] == len(prompts)
        eng.decode(6)
        full = eng.tokens()
    assert (tmp_path / "st" / "session.json").exists()
    assert all((tmp_path / "st" / f"stage{k}.bin").exists() for k in range(stages))
    with Engine(**kw) as eng:
        eng.load_state(str(tmp_path / "st"))
        assert eng.tokens() == [t[:4] for t in full]
        eng.decode(6)
        resumed = eng.tokens()
    assert resumed == full


def test_cpu_checkpoint_rejects_other_shape(native, model_dir, tmp_path):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with Engine(gguf=path, backend="cpu", max_ctx=64, mb_size=2) as eng:
        eng.start([[5, 6, 7], [8, 9]])
        eng.decode(2)
        eng.save_state(str(tmp_path / "st"))
    with Engine(gguf=path, backend="cpu", max_ctx=64, mb_size=1, n_mb=2) as eng:
        with pytest.raises(RuntimeError):
            eng.load_state(str(tmp_path / "st"))


def test_cpu_released_slot_not_reused_after_load_state(native, model_dir, tmp_path):
    """after start / release / save / load, a prompt sharing the released slot's old
    prefix must not reuse its (never restored) KV: the output equals a fresh engine's."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    rng = np.random.default_rng(21)
    A = [int(t) for t in rng.integers(3, cfg.vocab, 27)]
    B = [int(t) for t in rng.integers(3, cfg.vocab, 9)]
    kw = dict(gguf=path, backend="cpu", max_ctx=128, mb_size=2, prefill_chunk=16)
    A2 = A + [int(t) for t in rng.integers(3, cfg.vocab, 4)]
    with Engine(**kw) as eng:
        fresh, _ = eng.generate([A2, B], 6)
    with Engine(**kw) as eng:
        eng.start([A, B])
        eng.decode(3)
        eng.release(0)
        eng.save_state(str(tmp_path / "st"))
    with Engine(**kw) as eng:
        eng.load_state(str(tmp_path / "st"))
        out, _ = eng.generate([A2, B], 6)
    assert out[0] == fresh[0]


def test_cpu_load_state_rejects_corrupt_session(native, model_dir, tmp_path):
    """session.json / stage files are untrusted: bad sizes, lengths and ids fail cleanly."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    kw = dict(gguf=path, backend="cpu", max_ctx=64, mb_size=2, prefill_chunk=16)
    with Engine(**kw) as eng:
        eng.start([[5, 6, 7], [8, 9]])
        eng.decode(2)
        eng.save_state(str(tmp_path / "st"))
    good = json.loads((tmp_path / "st" / "session.json").read_text())

    def corrupt(fn):
        j = json.loads(json.dumps(good))
        fn(j)
        (tmp_path / "st" / "session.json").write_text(json.dumps(j))
        with Engine(**kw) as eng:
            with pytest.raises(RuntimeError, match="load_state"):
                eng.load_state(str(tmp_path / "st"))

    corrupt(lambda j: j.update(active=[1]))                       # size mismatch
    corrupt(lambda j: j.update(base_round=[0, 0, 0]))
    corrupt(lambda j: j["prompts"].__setitem__(0, list(range(3, 3 + 70))))   # longer than max_ctx
    corrupt(lambda j: j["prompts"].__setitem__(1, [8, cfg.vocab + 5]))      # id out of range
    corrupt(lambda j: j["generated"].__setitem__(0, [-1, 2, 3]))
    corrupt(lambda j: j["prompts"].__setitem__(0, [5, 6, 7, 8]))            # KV length disagrees
    corrupt(lambda j: j.update(base_round=[5, 0]))                           # admitted in the future
    (tmp_path / "st" / "session.json").write_text(json.dumps(good))
    with Engine(**kw) as eng:
        eng.load_state(str(tmp_path / "st"))


@pytest.mark.parametrize("stages", [1, 2])
def test_cpu_prefix_cache_multiturn(native, model_dir, stages):
    """Multi-turn: the second request re-sends prompt + reply + new text; with the prefix cache the
    slot's KV is reused (only the new tail is prefilled) and the output equals a cold engine's."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    rng = np.random.default_rng(5)
    p1 = [int(t) for t in rng.integers(3, cfg.vocab, 37)]
    kw = dict(gguf=path, backend="cpu", max_ctx=256, prefill_chunk=16, stages=stages, split="even")
    with Engine(**kw) as eng:
        o1, _ = eng.generate([p1], 9)
        p2 = p1 + o1[0] + [int(t) for t in rng.integers(3, cfg.vocab, 11)]
        o2, _ = eng.generate([p2], 9)
        reused = eng.health()["prefix_reused_tokens"]
    # KV of p1 + the 8 generated tokens that went through decode
    assert reused == len(p1) + 8
    with Engine(prefix_cache=False, **kw) as eng:
        c2, _ = eng.generate([p2], 9)
        assert eng.health()["prefix_reused_tokens"] == 0
    assert o2 == c2


def test_cpu_max_ctx_auto(native, model_dir):
    """max_ctx 0 (llama.cpp -c 0): sized from memory, capped by the model's training context."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with Engine(gguf=path, backend="cpu", max_ctx=0, mb_size=2) as eng:
        assert eng.info["max_ctx"] == cfg.n_ctx_train
        out, _ = eng.generate([[5, 6, 7]], 4)
        assert len(out[0]) == 4


@pytest.mark.parametrize("stages", [1, 2])
def test_cpu_continuous_batching(native, model_dir, stages):
    """Sequences admitted into free slots between decode rounds (and a released slot re-used)
    generate exactly what each would generate alone."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    rng = np.random.default_rng(11)
    P = [[int(t) for t in rng.integers(3, cfg.vocab, n)] for n in (9, 30, 5, 17, 12)]
    alone = []
    with Engine(gguf=path, backend="cpu", max_ctx=128, prefill_chunk=16) as eng:
        for p in P:
            o, _ = eng.generate([p], 10)
            alone.append(o[0])
    with Engine(gguf=path, backend="cpu", max_ctx=128, n_mb=2, mb_size=2, prefill_chunk=16, stages=stages,
                split="even") as eng:
        eng.start([P[0], P[1]])                 # slots 0, 1
        eng.decode(3)
        eng.admit([2, 3], [P[2], P[3]])         # mid-stream, other micro-batch
        eng.decode(5)
        t = eng.tokens()
        assert t[0][:9] == alone[0][:9] and t[1][:9] == alone[1][:9]
        assert t[2][:6] == alone[2][:6] and t[3][:6] == alone[3][:6]
        eng.release(0)
        eng.admit([0], [P[4]])                  # re-use a slot whose neighbour (slot 1) keeps going
        eng.decode(4)
        t = eng.tokens()
        assert t[0][:5] == alone[4][:5]
        assert t[1][:10] == alone[1][:10] and t[2][:10] == alone[2][:10]
        with pytest.raises(RuntimeError):
            eng.admit([1], [P[0]])              # busy slot


def test_cpu_gpu_mem_sums_stages_sharing_a_device(native, model_dir):
    """--gpu-mem is per GPU, so stages emulated on one device add up."""
    import re
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    kw = dict(gguf=path, backend="cpu", max_ctx=256, mb_size=2, stages=2, split="even")

    def need(devices, gib):
        try:
            with Engine(devices=devices, gpu_mem_gib=gib, **kw):
                return None
        except RuntimeError as e:
            m = re.search(r"GPU (\d+) \(stage ([\d,]+)\) needs ([\d.]+) MiB", str(e))
            assert m, str(e)
            return m.group(2), float(m.group(3))

    stages, total = need([0, 0], 1e-9)
    assert stages == "0,1"
    s0, a0 = need([0, 1], 1e-9)
    assert s0 == "0" and a0 < total
    budget_mib = max(a0, total - a0) * 1.02
    assert budget_mib < total
    assert need([0, 1], budget_mib / 1024) is None      # each GPU fits alone
    assert need([0, 0], budget_mib / 1024)[0] == "0,1"  # together they do not


@pytest.mark.parametrize("source", ["synthetic", "gguf"])
def test_int8_gemm_copies_count_in_memory_budget(native, model_dir, source):
    """int8_gemm keeps an int8 copy of every quantized non-MoE projection (1 B per padded
    weight + a float row scale); --gpu-mem (and the max_ctx auto KV budget, same accounting) must
    see those bytes.  The check runs before any stage is built, so it is testable without a GPU."""
    import re
    from mipipe.engine import Engine
    if source == "gguf":
        path, cfg = make_model(model_dir, "tiny-gqa", "Q4_K_M")
        kw = dict(gguf=path)
        n_layer, d, f, hq, hkv = cfg.n_layer, cfg.d_model, cfg.d_ff, cfg.n_head, cfg.n_head_kv
        hd = d // hq
    else:
        syn = dict(n_layer=3, d_model=512, n_head=8, n_head_kv=2, d_ff=1536, vocab=2048)
        kw = dict(synthetic=syn, ftype="Q4_K")
        n_layer, d, f, hq, hkv, hd = 3, 512, 1536, 8, 2, 64

    def weights_mib(**extra):
        with pytest.raises(RuntimeError) as ei:
            Engine(max_ctx=128, gpu_mem_gib=1e-9, **kw, **extra)
        m = re.search(r"weights ([\d.]+) \+ KV", str(ei.value))
        assert m, str(ei.value)
        return float(m.group(1))

    pad = lambda n: (n + 15) // 16 * 16
    padk = lambda k: (k + 255) // 256 * 256
    mats = [(hq * hd, d), (hkv * hd, d), (hkv * hd, d), (d, hq * hd), (f, d), (f, d), (d, f)]
    expect = n_layer * sum(pad(n) * padk(k) + pad(n) * 4 for n, k in mats) / 1048576.0
    extra = weights_mib(int8_gemm=True) - weights_mib()
    assert abs(extra - expect) < 0.01, (extra, expect)


def test_cpu_device_speed_probe_partition(native, model_dir):
    """Halda-style partitioning from MEASURED device speed (device_speed="probe"): every stage gets
    a positive speed, the split stays contiguous and generation matches PP=1."""
    from mipipe.engine import Engine, device_probe
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    host = device_probe(-1)
    assert host["hbm_read_gbps"] > 0.1 and host["speed"] == host["hbm_read_gbps"]
    prompts = [[5, 6, 7, 8], [9, 10]]
    with Engine(gguf=path, backend="cpu", max_ctx=128, mb_size=2) as eng:
        ref, _ = eng.generate(prompts, 6)
    with Engine(gguf=path, backend="cpu", max_ctx=128, mb_size=2, stages=2, device_speed="probe") as eng:
        sp = eng.info["device_speed"]
        assert len(sp) == 2 and all(v > 0 for v in sp)
        st = eng.info["stages"]
        assert st[0]["layer_begin"] == 0 and st[0]["layer_end"] == st[1]["layer_begin"]
        out, _ = eng.generate(prompts, 6)
    assert out == ref


def test_fp8_kv_needs_hip_backend(native, model_dir):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with pytest.raises(RuntimeError, match="kv_dtype fp8"):
        Engine(gguf=path, backend="cpu", max_ctx=128, kv_dtype="fp8")
    with pytest.raises(RuntimeError, match="kv_dtype must be"):
        Engine(gguf=path, backend="cpu", max_ctx=128, kv_dtype="int4")


def test_hybrid_split_needs_local_mode(model_dir):
    """gpu_layers < n_layer (a CPU stage in front of the GPU stages) is a single-process layout."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with pytest.raises(Exception, match="needs mode local"):
        Engine(gguf=path, max_ctx=64, mode="mp", world=2, rank=0, gpu_layers=2)
