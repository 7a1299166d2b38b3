"""Packed prefill (several sequences per prefill chunk, one GEMM per projection) must give the same
results as one-sequence-per-chunk prefill, on the CPU backend (always) and on the GPU."""
import numpy as np
import pytest

from conftest import make_model


def nmse(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(((a - b) ** 2).sum() / ((b ** 2).sum() + 1e-30))


def _run(path, packed, **kw):
    from mipipe.engine import Engine
    rng = np.random.default_rng(11)
    prompts = [[int(t) for t in rng.integers(3, 2000, n)] for n in (37, 5, 70, 1, 20, 9)]
    with Engine(gguf=path, n_mb=2, mb_size=3, max_ctx=256, prefill_chunk=48, packed_prefill=packed, **kw) as eng:
        out, _ = eng.generate(prompts, 6)
        return out, eng.logits(rows=3)


@pytest.mark.parametrize("stages", [1, 2])
def test_packed_prefill_cpu(native, model_dir, stages):
    path, cfg = make_model(model_dir, "tiny-gqa", "Q8_0")
    a = _run(path, False, backend="cpu", stages=stages, split="even")
    b = _run(path, True, backend="cpu", stages=stages, split="even")
    assert a[0] == b[0]
    assert nmse(b[1], a[1]) < 1e-9


@pytest.mark.gpu
@pytest.mark.parametrize("name,ftype", [("tiny-gqa", "Q4_K_M"), ("tiny-moe", "Q8_0")])
def test_packed_prefill_gpu(cuda, native, model_dir, name, ftype):
    path, cfg = make_model(model_dir, name, ftype)
    a = _run(path, False)
    b = _run(path, True)
    assert a[0] == b[0]
    assert nmse(b[1], a[1]) < 1e-5
