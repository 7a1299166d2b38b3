"""Wave-level decode attention (attention.hip attn_decode_wave_kernel: one wave per (token, kv head,
split), chunks streamed with two in flight, no cross-wave merge) against the workgroup kernel and
the fp32 oracle: head dims 64 / 128, f16 and fp8 KV pages, one split and several (long contexts
with a short split: the last-arriving wave merges), paged block tables with mixed lengths."""
import numpy as np
import pytest

from conftest import make_model

pytestmark = pytest.mark.gpu


def nmse(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def _knob(native, name, v):
    from mipipe import _native as N
    N.check(N.lib().mp_set_knob(name.encode(), int(v)), "set_knob")


@pytest.fixture
def wave_knob(native):
    yield lambda v: _knob(native, "ATTN_WAVE", v)
    _knob(native, "ATTN_WAVE", 2)


@pytest.mark.parametrize("name,ftype,kv", [("tiny-gqa", "Q8_0", "f16"), ("tiny-l3", "Q6_K", "f16"),
                                           ("tiny-l3", "Q6_K", "fp8"), ("tiny-qwen2", "Q4_K_M", "f16")])
@pytest.mark.parametrize("split", [0, 128])
def test_wave_attention_matches_workgroup_kernel(cuda, wave_knob, model_dir, name, ftype, kv, split):
    from mipipe.engine import Engine
    path, cfg = make_model(model_dir, name, ftype)
    rng = np.random.default_rng(9)
    prompts = [[int(t) for t in rng.integers(3, cfg.vocab, n)] for n in (300, 7, 129, 64, 191, 1)]
    res = {}
    for mode in (1, 0):
        wave_knob(mode)
        kw = dict(gguf=path, max_ctx=512, n_mb=2, mb_size=3, prefill_chunk=128, kv_dtype=kv, attn_split_len=split)
        with Engine(**kw) as eng:
            eng.start(prompts)
            eng.decode(3)
            lg = [eng.logits(rows=3).copy()]
            eng.decode(2)
            lg.append(eng.logits(rows=3).copy())
            res[mode] = (eng.tokens(), lg)
    assert res[1][0] == res[0][0]
    # e4m3 pages: a 1e-7 difference in a new K / V value can round to the neighbouring fp8 code
    tol = 1e-4 if kv == "fp8" else 1e-6
    for a, b in zip(res[1][1], res[0][1]):
        assert nmse(a, b) < tol


def test_wave_attention_matches_reference(cuda, wave_knob, model_dir):
    """Forced wave kernel, single stream with splits, against the fp32 oracle step by step."""
    from mipipe.engine import Engine
    from mipipe.models.reference import RefLlama
    wave_knob(1)
    path, cfg = make_model(model_dir, "tiny-l3", "Q6_K")
    ref = RefLlama.from_gguf(path)
    prompt = [int(t) for t in np.random.default_rng(3).integers(3, cfg.vocab, 200)]
    with Engine(gguf=path, max_ctx=512, prefill_chunk=64, attn_split_len=128) as eng:
        eng.start([prompt])
        ref.reset()
        rl = ref.forward(prompt, 0)[-1].numpy()
        pos = len(prompt)
        for step in range(5):
            tok = eng.tokens()[0][-1]
            eng.decode(1)
            rl = ref.forward([tok], pos)[-1].numpy()
            pos += 1
            assert nmse(eng.logits()[0], rl) < 2e-4, (step, nmse(eng.logits()[0], rl))
