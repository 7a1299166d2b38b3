"""T0 format tests (CPU): quant round-trips, GGUF round-trip, native GGUF reader, T16 packer."""
import json
import os

import numpy as np
import pytest

from mipipe.utils import quants as Q
from mipipe.utils.gguf import GGUFWriter, GGUFReader, U32, STRING, F32T
from mipipe.utils.t16 import unpack_t16, PACK_OF

ALL = [Q.F32, Q.F16, Q.BF16, Q.Q8_0, Q.Q4_0, Q.Q4_K, Q.Q5_K, Q.Q6_K]
# worst-case relative RMS error of quantize->dequantize on gaussian data
TOL = {Q.F32: 0, Q.F16: 1e-3, Q.BF16: 5e-3, Q.Q8_0: 0.01, Q.Q4_0: 0.2, Q.Q4_K: 0.12, Q.Q5_K: 0.06, Q.Q6_K: 0.03}


@pytest.mark.parametrize("qt", ALL)
def test_quant_roundtrip(qt):
    rng = np.random.default_rng(qt)
    x = rng.standard_normal(256 * 8).astype(np.float32)
    b = Q.quantize(x, qt)
    assert b.nbytes == Q.tensor_bytes(qt, x.shape)
    y = Q.dequantize(b, qt)
    rel = np.sqrt(np.mean((x - y) ** 2) / np.mean(x ** 2))
    assert rel <= TOL[qt] + 1e-7, rel


def test_scale_min_pack_roundtrip():
    rng = np.random.default_rng(0)
    sc = rng.integers(0, 64, (100, 8)).astype(np.uint8)
    mn = rng.integers(0, 64, (100, 8)).astype(np.uint8)
    s2, m2 = Q.unpack_scale_min_k4(Q.pack_scale_min_k4(sc, mn))
    assert (s2 == sc).all() and (m2 == mn).all()


@pytest.mark.parametrize("qt", ALL)
def test_native_dequant_row_matches_numpy(native, qt):
    rng = np.random.default_rng(7 + qt)
    K = 512
    b = Q.quantize(rng.standard_normal(K).astype(np.float32), qt)
    ref = Q.dequantize(b, qt)
    out = np.zeros(K, np.float32)
    assert native.mp_dequant_row(qt, b.ctypes.data, out.ctypes.data, K) == 0
    np.testing.assert_allclose(out, ref, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q5_K, Q.Q6_K, Q.Q8_0])
def test_native_dequant_row_random_bits(native, qt):
    """Every quant / scale / high-bit field exercised (random block bytes, 6-bit scales up to 63):
    the native row dequantizer (CPU backend, per-sub-block scales hoisted) against numpy."""
    rng = np.random.default_rng(11 + qt)
    K = 1024
    b = Q.random_blocks(rng, qt, 1, K, 0.05)
    ref = Q.dequantize(b, qt).reshape(-1)
    out = np.zeros(K, np.float32)
    assert native.mp_dequant_row(qt, b.ctypes.data, out.ctypes.data, K) == 0
    np.testing.assert_allclose(out, ref, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("qt", [Q.Q4_K, Q.Q5_K, Q.Q6_K, Q.Q8_0])
def test_random_blocks_finite(qt):
    rng = np.random.default_rng(1)
    b = Q.random_blocks(rng, qt, 4, 512, 0.05)
    y = Q.dequantize(b, qt)
    assert np.isfinite(y).all() and 0.005 < y.std() < 0.5


def test_gguf_roundtrip(tmp_path, native):
    p = str(tmp_path / "t.gguf")
    w = GGUFWriter(p)
    w.add("general.architecture", "llama")
    w.add("llama.block_count", 3, U32)
    w.add("some.float", 0.25, F32T)
    w.add("some.list", ["a", "bb", "ccc"], elem_type=STRING)
    w.add("some.ints", [1, 2, 3])
    rng = np.random.default_rng(0)
    x = rng.standard_normal((4, 256)).astype(np.float32)
    w.add_tensor("a.weight", Q.quantize(x, Q.Q4_K), Q.Q4_K, (256, 4))
    w.add_tensor("b.weight", x[0], Q.F32, (256,))
    w.write()
    r = GGUFReader(p)
    assert r.kv["llama.block_count"] == 3 and r.kv["some.list"] == ["a", "bb", "ccc"]
    assert abs(r.kv["some.float"] - 0.25) < 1e-9
    np.testing.assert_allclose(r.tensor_f32("b.weight"), x[0])
    np.testing.assert_allclose(r.tensor_f32("a.weight"), Q.dequantize(Q.quantize(x, Q.Q4_K), Q.Q4_K).reshape(4, 256))
    # native (mmap) reader agrees on metadata and tensor offsets
    h = native.mp_gguf_open(p.encode())
    assert h
    j = json.loads(native.mp_gguf_json(h).decode())
    native.mp_gguf_close(h)
    assert j["version"] == 3 and j["kv"]["llama.block_count"] == 3
    assert j["kv"]["some.list"]["array_len"] == 3
    t = {d["name"]: d for d in j["tensors"]}
    assert t["a.weight"]["ne"] == [256, 4] and t["a.weight"]["type"] == Q.Q4_K
    assert t["a.weight"]["offset"] == r.tensors["a.weight"].offset
    assert t["b.weight"]["nbytes"] == 1024


def test_gguf_rejects_garbage(tmp_path, native):
    p = tmp_path / "bad.gguf"
    p.write_bytes(b"GGUF\x03\x00\x00\x00" + b"\xff" * 40)
    assert not native.mp_gguf_open(str(p).encode())
    assert b"gguf" in native.mp_last_error()


@pytest.mark.parametrize("qt", ALL)
def test_t16_pack_layout(native, qt):
    """The C++ packer + the kernel's indexing (numpy mirror) reproduce the dequantized weights."""
    from mipipe.ops.kernels import pack_t16
    rng = np.random.default_rng(11 + qt)
    n, k = 32, 512
    if qt in (Q.F32, Q.F16, Q.BF16, Q.Q8_0, Q.Q4_0):
        k = 288          # exercise K padding (stories15M shape)
    x = rng.standard_normal((n, k)).astype(np.float32)
    raw = Q.quantize(x, qt)
    ref = Q.dequantize(raw, qt).reshape(n, k)
    packed = pack_t16(raw, qt, n, k)
    got = unpack_t16(packed, PACK_OF[qt], n, k)
    tol = 1e-3 if qt == Q.F32 else 1e-6   # BF16 stays bf16 (P_BF16): exact
    np.testing.assert_allclose(got, ref, rtol=tol, atol=tol * np.abs(ref).max())


def test_t16_gateup_interleave(native):
    from mipipe.ops.kernels import pack_t16
    rng = np.random.default_rng(3)
    F, k = 16, 256
    g = rng.standard_normal((F, k)).astype(np.float32)
    u = rng.standard_normal((F, k)).astype(np.float32)
    raw = Q.quantize(np.concatenate([g, u]), Q.Q8_0)
    packed = pack_t16(raw, Q.Q8_0, 2 * F, k, gateup=True)
    got = unpack_t16(packed, PACK_OF[Q.Q8_0], 2 * F, k)
    deq = Q.dequantize(raw, Q.Q8_0).reshape(2 * F, k)
    for t in range(2 * F // 16):
        np.testing.assert_allclose(got[16 * t:16 * t + 8], deq[8 * t:8 * t + 8], rtol=1e-6)
        np.testing.assert_allclose(got[16 * t + 8:16 * t + 16], deq[F + 8 * t:F + 8 * t + 8], rtol=1e-6)


@pytest.mark.parametrize("qt", [Q.Q8_0, Q.Q4_0, Q.Q4_K, Q.Q5_K, Q.Q6_K])
def test_cpu_integer_dot_matches_dequant(native, qt):
    """CPU stage integer dots (cpu_qdot.cpp): quantized weight rows x int8 activation blocks.  The
    AVX2 form equals the scalar one (same integer sums, f32 order aside), and both stay within the
    int8 rounding of x of the f32 dot of the dequantized row (numpy oracle)."""
    import ctypes
    rng = np.random.default_rng(31 + qt)
    N, K = 24, 1024
    w = rng.standard_normal((N, K)).astype(np.float32) * 0.05
    b = np.concatenate([Q.quantize(w[n], qt) for n in range(N)])
    wd = np.stack([Q.dequantize(Q.quantize(w[n], qt), qt) for n in range(N)])
    x = rng.standard_normal(K).astype(np.float32)
    x[::97] *= 20.0   # a few outliers per 32-block
    y = np.zeros(N, np.float32)
    ys = np.zeros(N, np.float32)
    assert native.mp_qdot_rows(qt, b.ctypes.data, N, K, x.ctypes.data, y.ctypes.data, ys.ctypes.data) == 1
    ref = wd.astype(np.float64) @ x.astype(np.float64)
    np.testing.assert_allclose(y, ys, rtol=1e-5, atol=1e-5 * np.abs(ref).max())
    # exact up to f32 rounding against the dequantized row times the int8-rounded activations
    xb = x.reshape(-1, 32).astype(np.float32)
    d = np.abs(xb).max(1, keepdims=True) / np.float32(127)
    x8 = (np.clip(np.rint(xb / np.where(d > 0, d, 1)), -127, 127) * d).reshape(-1)
    ref8 = wd.astype(np.float64) @ x8.astype(np.float64)
    np.testing.assert_allclose(y, ref8, rtol=2e-5, atol=2e-5 * np.abs(ref8).max())
    rel = np.sqrt(((y - ref) ** 2).mean() / (ref ** 2).mean())
    assert rel < 2e-2, rel   # the int8 rounding of x (outlier-heavy blocks)
