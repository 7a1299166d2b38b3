"""MALL prefetch side stream (knob PREFETCH, hip_stage.cpp prefetch_layer / prefetch_join): the
single-stream decode with a prefetch branch forked per layer and joined per step -- captured into
the decode hipGraph as a parallel branch -- generates exactly what it generates without it, in graph
and eager mode."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graphs", [True, False])
def test_prefetch_matches_default(cuda, native, model_dir, graphs):
    from conftest import make_model
    from mipipe import _native as N
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, "tiny-gqa", "Q4_K_M")
    rng = np.random.default_rng(11)
    prompts = [[int(t) for t in rng.integers(3, cfg.vocab, 9)]]
    kw = dict(gguf=path, max_ctx=128, graphs=graphs)
    with Engine(**kw) as eng:
        ref, _ = eng.generate(prompts, 16)
    N.check(N.lib().mp_set_knob(b"PREFETCH", 256), "knob")
    try:
        with Engine(**kw) as eng:
            out, _ = eng.generate(prompts, 16)
    finally:
        N.lib().mp_set_knob(b"PREFETCH", 0)
    assert out == ref
