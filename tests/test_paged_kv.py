"""Paged KV cache (kvpager.h): one pool of 64-token pages per stage shared by every
sequence slot, pages granted on admission / decode and returned on release.  A pool smaller than
n_slots x max_ctx must run any mix of sequences whose LIVE tokens fit, and give the same tokens as
an engine where every slot owns max_ctx."""
import numpy as np
import pytest

from conftest import make_model


def _prompts(cfg, lens, seed=5):
    rng = np.random.default_rng(seed)
    return [[int(t) for t in rng.integers(3, cfg.vocab, n)] for n in lens]


@pytest.mark.parametrize("stages", [1, 2])
def test_cpu_oversubscribed_pool_matches_static(native, model_dir, stages):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    P = _prompts(cfg, (300, 10, 7, 12))
    kw = dict(gguf=path, backend="cpu", max_ctx=512, n_mb=1, mb_size=4, prefill_chunk=64, stages=stages, split="even")
    with Engine(**kw) as eng:
        static, _ = eng.generate(P, 40)
    # 10 pages = 640 tokens for 4 slots of max_ctx 512: the 340-token sequence alone needs 6 pages,
    # more than a 640 / 4 = 160-token static share
    with Engine(kv_pool_tokens=640, **kw) as eng:
        assert eng.info["kv_pages"] == 10
        paged, _ = eng.generate(P, 40)
    assert paged == static


def test_cpu_pool_exhaustion_raises(native, model_dir):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    with Engine(gguf=path, backend="cpu", max_ctx=512, mb_size=2, kv_pool_tokens=192) as eng:
        eng.start(_prompts(cfg, (100, 60)))          # 2 + 1 pages of 3
        with pytest.raises(RuntimeError, match="KV page pool exhausted"):
            eng.decode(40)                            # slot 1 would cross into a 4th page


def test_cpu_release_returns_pages_and_admit_reuses_them(native, model_dir):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    P = _prompts(cfg, (150, 20, 200), seed=9)
    with Engine(gguf=path, backend="cpu", max_ctx=512, prefill_chunk=64) as eng:
        alone = eng.generate([P[2]], 8)[0][0]
    with Engine(gguf=path, backend="cpu", max_ctx=512, mb_size=2, prefill_chunk=64, kv_pool_tokens=320) as eng:
        eng.start([P[0], P[1]])                        # 3 + 1 of 5 pages
        eng.decode(4)
        assert eng.kv_stats()["kv_free_pages"] == 1
        with pytest.raises(RuntimeError, match="exhausted"):
            eng.decode(200)                            # slot 0 cannot grow to 6 pages
        eng.release(0)
        assert eng.kv_stats()["kv_free_pages"] == 4
        eng.admit([0], [P[2]])                         # 4 pages: only fits with slot 0's pages back
        eng.decode(7)
        assert eng.tokens()[0][:8] == alone


def test_cpu_paged_checkpoint_resume(native, model_dir, tmp_path):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    P = _prompts(cfg, (90, 33), seed=2)
    kw = dict(gguf=path, backend="cpu", max_ctx=256, mb_size=2, prefill_chunk=32, kv_pool_tokens=384)
    with Engine(**kw) as eng:
        ref, _ = eng.generate(P, 20)
    with Engine(**kw) as eng:
        eng.start(P)
        eng.decode(9)
        eng.save_state(str(tmp_path))
    with Engine(**kw) as eng:
        eng.load_state(str(tmp_path))
        eng.decode(10)
        assert eng.tokens() == ref


@pytest.mark.gpu
def test_gpu_64_slots_oversubscribed_pool(cuda, native, model_dir):
    """64 slots whose sum fits the pool while the longest sequence exceeds pool / 64 run to
    completion with the tokens of the static layout."""
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q4_K_M")
    lens = [1000] + [int(n) for n in np.random.default_rng(4).integers(8, 40, 63)]
    P = _prompts(cfg, lens, seed=8)
    kw = dict(gguf=path, max_ctx=2048, n_mb=1, mb_size=64, prefill_chunk=256)
    with Engine(**kw) as eng:
        static, _ = eng.generate(P, 20)
    # 128 pages = 8192 tokens = 128 per slot on average; slot 0 needs 16 pages
    with Engine(kv_pool_tokens=64 * 128, **kw) as eng:
        assert eng.info["kv_pages"] == 128
        paged, _ = eng.generate(P, 20)
    assert paged == static


@pytest.mark.gpu
def test_gpu_paged_continuous_batching(cuda, native, model_dir):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    P = _prompts(cfg, (130, 30, 70, 12), seed=6)
    alone = []
    with Engine(gguf=path, max_ctx=512, prefill_chunk=64) as eng:
        for p in P:
            alone.append(eng.generate([p], 10)[0][0])
    with Engine(gguf=path, max_ctx=512, n_mb=2, mb_size=2, prefill_chunk=64, kv_pool_tokens=512) as eng:
        eng.start([P[0], P[1]])
        eng.decode(3)
        eng.admit([2], [P[2]])
        eng.decode(6)
        t = eng.tokens()
        assert t[0][:10] == alone[0] and t[1][:10] == alone[1] and t[2][:7] == alone[2][:7]
        eng.release(0)
        eng.admit([0], [P[3]])
        eng.decode(9)
        assert eng.tokens()[0][:10] == alone[3]
