"""Deterministic reduction mode: with `deterministic=True` the split-K GEMVs store
per-split partials that one kernel adds in a fixed order, and the MoE down projection stores per-slot
outputs combined in expert-rank order; no float atomic ever adds into a shared output.  Logits must
then be bitwise identical across runs and between PP=1 and a PP=2 emulation on one GPU."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# 70B-width, 2 layers (d 8192, 64 q / 8 kv heads, d_ff 28672); small vocab keeps the head cheap
WIDE = dict(n_layer=2, d_model=8192, n_head=64, n_head_kv=8, d_ff=28672, vocab=32000, rope_base=500000.0)
MOE = dict(n_layer=2, d_model=1024, n_head=8, n_head_kv=2, d_ff=2816, vocab=4096, n_expert=8, n_expert_used=2)


def _run(syn, ftype, mb, stages=1, **kw):
    from mipipe.engine import Engine
    extra = dict(stages=stages, devices=[0] * stages, link="local", split="even") if stages > 1 else {}
    rng = np.random.default_rng(3)
    prompts = [[int(t) for t in rng.integers(3, syn["vocab"], int(n))] for n in rng.integers(5, 40, mb)]
    with Engine(synthetic=syn, ftype=ftype, max_ctx=128, n_mb=1, mb_size=mb, prefill_chunk=64, seed=7, **extra,
                **kw) as eng:
        eng.start(prompts)
        eng.decode(3)
        return eng.logits(rows=mb), eng.tokens()


@pytest.mark.parametrize("mb", [1, 16, 64, 128, 256])
def test_deterministic_bitwise_runs_and_pp2(cuda, native, mb):
    """mb > 64 runs the decode projections on the GEMMs: the split-K ones (qkv / o / down, gemm4)
    store per-split partials that a fixed-order reduction adds (`gemm_splitk_store`, the default);
    the whole-K ones (gate/up, the LM head, gemm4) have one writer per output element."""
    a, ta = _run(WIDE, "Q4_K", mb, deterministic=True)
    b, tb = _run(WIDE, "Q4_K", mb, deterministic=True)
    assert np.array_equal(a, b), float(np.abs(a - b).max())
    assert ta == tb
    c, tc = _run(WIDE, "Q4_K", mb, stages=2, deterministic=True)
    assert np.array_equal(a, c), float(np.abs(a - c).max())
    assert ta == tc


@pytest.mark.parametrize("ftype,mb,sk", [("Q4_K", 128, False), ("BF16", 128, True), ("BF16", 256, False)])
def test_deterministic_wide_paths(cuda, native, ftype, mb, sk):
    """The other wide-batch paths of deterministic mode: split-K partial stores off (the GEMMs then
    run unsplit) and 16-bit weights (gemm3, unsplit in deterministic mode)."""
    a, ta = _run(WIDE, ftype, mb, deterministic=True, gemm_splitk_store=sk)
    b, tb = _run(WIDE, ftype, mb, deterministic=True, gemm_splitk_store=sk)
    assert np.array_equal(a, b), float(np.abs(a - b).max())
    assert ta == tb


def test_deterministic_close_to_default(cuda, native):
    """The fixed-order reduction changes only the summation order of the split-K partials."""
    a, _ = _run(WIDE, "Q4_K", 4, deterministic=True)
    b, _ = _run(WIDE, "Q4_K", 4)
    err = np.abs(a - b).max() / (np.abs(b).max() + 1e-9)
    assert err < 1e-3, err


def test_deterministic_moe_bitwise(cuda, native):
    a, ta = _run(MOE, "Q4_K_M", 8, deterministic=True)
    b, tb = _run(MOE, "Q4_K_M", 8, deterministic=True)
    assert np.array_equal(a, b)
    assert ta == tb
    c, _ = _run(MOE, "Q4_K_M", 8)
    assert np.abs(a - c).max() / (np.abs(c).max() + 1e-9) < 1e-3
