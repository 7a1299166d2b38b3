"""Reference quantizers / dequantizers for the ggml block formats (numpy).

These are the test oracle for every HIP dequant kernel and the writer side of the
synthetic-GGUF generator.  The block layouts follow the GGUF/ggml spec recorded in
SURVEY.md §2.8 (the reference delegates these formats to its llama.cpp submodule,
`.gitmodules:1-3`, which is not in the mount; the spec is reconstructed there).

Formats: F32, F16, BF16, Q8_0, Q4_0, Q4_K, Q5_K, Q6_K.  Quantizers are simple
(min/max based) but produce valid blocks; dequantizers are exact implementations of
the block math, so `dequant(bytes)` is the ground truth a kernel must reproduce.
"""
from __future__ import annotations

import numpy as np

# ggml type ids
F32, F16, Q4_0, Q4_1, Q5_0, Q5_1, Q8_0, Q8_1 = 0, 1, 2, 3, 6, 7, 8, 9
Q2_K, Q3_K, Q4_K, Q5_K, Q6_K, Q8_K = 10, 11, 12, 13, 14, 15
BF16 = 30

QK_K = 256

TYPE_NAMES = {F32: "F32", F16: "F16", BF16: "BF16", Q8_0: "Q8_0", Q4_0: "Q4_0",
              Q4_K: "Q4_K", Q5_K: "Q5_K", Q6_K: "Q6_K"}
NAME_TO_TYPE = {v: k for k, v in TYPE_NAMES.items()}

# (block_elems, block_bytes)
BLOCK = {
    F32: (1, 4), F16: (1, 2), BF16: (1, 2),
    Q8_0: (32, 34), Q4_0: (32, 18),
    Q4_K: (256, 144), Q5_K: (256, 176), Q6_K: (256, 210),
}


def row_bytes(qtype: int, n: int) -> int:
    be, bb = BLOCK[qtype]
    assert n % be == 0, (qtype, n)
    return n // be * bb


def tensor_bytes(qtype: int, shape) -> int:
    n = int(np.prod(shape))
    be, bb = BLOCK[qtype]
    assert n % be == 0
    return n // be * bb


# ----------------------------------------------------------------------------- bf16
def f32_to_bf16_bits(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = ((u >> 16) & 1) + 0x7FFF
    return ((u + r) >> 16).astype(np.uint16)


def bf16_bits_to_f32(b: np.ndarray) -> np.ndarray:
    return (b.astype(np.uint32) << 16).view(np.float32)


# ----------------------------------------------------------------------------- Q8_0
def quantize_q8_0(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32).reshape(-1, 32)
    amax = np.abs(x).max(axis=1)
    d = amax / 127.0
    inv = np.where(d > 0, 1.0 / np.where(d > 0, d, 1), 0.0)
    q = np.clip(np.rint(x * inv[:, None]), -127, 127).astype(np.int8)
    out = np.zeros((x.shape[0], 34), np.uint8)
    out[:, 0:2] = d.astype(np.float16).reshape(-1, 1).view(np.uint8)
    out[:, 2:] = q.view(np.uint8)
    return out.reshape(-1)


def dequantize_q8_0(b: np.ndarray) -> np.ndarray:
    b = np.asarray(b, np.uint8).reshape(-1, 34)
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
    q = b[:, 2:].view(np.int8).astype(np.float32)
    return (d * q).reshape(-1)


# ----------------------------------------------------------------------------- Q4_0
def quantize_q4_0(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32).reshape(-1, 32)
    idx = np.abs(x).argmax(axis=1)
    mx = x[np.arange(x.shape[0]), idx]
    d = mx / -8.0
    inv = np.where(d != 0, 1.0 / np.where(d != 0, d, 1), 0.0)
    q = np.clip(np.floor(x * inv[:, None] + 8.5), 0, 15).astype(np.uint8)
    out = np.zeros((x.shape[0], 18), np.uint8)
    out[:, 0:2] = d.astype(np.float16).reshape(-1, 1).view(np.uint8)
    out[:, 2:] = q[:, :16] | (q[:, 16:] << 4)
    return out.reshape(-1)


def dequantize_q4_0(b: np.ndarray) -> np.ndarray:
    b = np.asarray(b, np.uint8).reshape(-1, 18)
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
    qs = b[:, 2:]
    lo = (qs & 15).astype(np.float32) - 8
    hi = (qs >> 4).astype(np.float32) - 8
    return (d * np.concatenate([lo, hi], axis=1)).reshape(-1)


# ----------------------------------------------------------------------------- K-quant scale packing
def pack_scale_min_k4(sc: np.ndarray, mn: np.ndarray) -> np.ndarray:
    """Pack 8 six-bit scales and mins per block into the 12-byte ggml layout."""
    sc = sc.astype(np.uint8)
    mn = mn.astype(np.uint8)
    s = np.zeros((sc.shape[0], 12), np.uint8)
    for j in range(4):
        s[:, j] = (sc[:, j] & 63) | ((sc[:, j + 4] >> 4) << 6)
        s[:, j + 4] = (mn[:, j] & 63) | ((mn[:, j + 4] >> 4) << 6)
        s[:, j + 8] = (sc[:, j + 4] & 15) | ((mn[:, j + 4] & 15) << 4)
    return s


def unpack_scale_min_k4(s: np.ndarray):
    """Inverse of pack_scale_min_k4 == ggml get_scale_min_k4 for j = 0..7."""
    s = s.astype(np.uint8)
    sc = np.zeros((s.shape[0], 8), np.uint8)
    mn = np.zeros((s.shape[0], 8), np.uint8)
    for j in range(8):
        if j < 4:
            sc[:, j] = s[:, j] & 63
            mn[:, j] = s[:, j + 4] & 63
        else:
            sc[:, j] = (s[:, j + 4] & 15) | ((s[:, j - 4] >> 6) << 4)
            mn[:, j] = (s[:, j + 4] >> 4) | ((s[:, j] >> 6) << 4)
    return sc, mn


def _kquant_affine(x: np.ndarray, nmax: int):
    """Per 32-weight sub-block affine quantization with 6-bit super-block scales.

    x: [nb, 8, 32].  Returns (d, dmin, sc6, mn6, q) with q in [0, nmax].
    """
    mn = np.minimum(x.min(axis=2), 0.0)              # [nb, 8] (<= 0)
    mx = x.max(axis=2)
    scale = (mx - mn) / nmax                          # [nb, 8]
    mins = -mn                                        # >= 0
    d = scale.max(axis=1) / 63.0
    dmin = mins.max(axis=1) / 63.0
    d16 = d.astype(np.float16).astype(np.float32)
    dmin16 = dmin.astype(np.float16).astype(np.float32)
    inv_d = np.where(d16 > 0, 1.0 / np.where(d16 > 0, d16, 1), 0.0)
    inv_dm = np.where(dmin16 > 0, 1.0 / np.where(dmin16 > 0, dmin16, 1), 0.0)
    sc6 = np.clip(np.rint(scale * inv_d[:, None]), 0, 63).astype(np.uint8)
    mn6 = np.clip(np.rint(mins * inv_dm[:, None]), 0, 63).astype(np.uint8)
    eff_s = d16[:, None] * sc6.astype(np.float32)     # [nb, 8]
    eff_m = dmin16[:, None] * mn6.astype(np.float32)
    inv_s = np.where(eff_s > 0, 1.0 / np.where(eff_s > 0, eff_s, 1), 0.0)
    q = np.clip(np.rint((x + eff_m[:, :, None]) * inv_s[:, :, None]), 0, nmax).astype(np.uint8)
    return d16, dmin16, sc6, mn6, q


# ----------------------------------------------------------------------------- Q4_K
def quantize_q4_k(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32).reshape(-1, 8, 32)
    nb = x.shape[0]
    d, dmin, sc6, mn6, q = _kquant_affine(x, 15)
    q = q.reshape(nb, 256)
    out = np.zeros((nb, 144), np.uint8)
    out[:, 0:2] = d.astype(np.float16).reshape(-1, 1).view(np.uint8)
    out[:, 2:4] = dmin.astype(np.float16).reshape(-1, 1).view(np.uint8)
    out[:, 4:16] = pack_scale_min_k4(sc6, mn6)
    qs = np.zeros((nb, 128), np.uint8)
    for c in range(4):
        qs[:, 32 * c:32 * c + 32] = q[:, 64 * c:64 * c + 32] | (q[:, 64 * c + 32:64 * c + 64] << 4)
    out[:, 16:] = qs
    return out.reshape(-1)


def dequantize_q4_k(b: np.ndarray) -> np.ndarray:
    b = np.asarray(b, np.uint8).reshape(-1, 144)
    nb = b.shape[0]
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
    dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)
    sc, mn = unpack_scale_min_k4(b[:, 4:16])
    qs = b[:, 16:]
    y = np.zeros((nb, 256), np.float32)
    for c in range(4):
        q = qs[:, 32 * c:32 * c + 32]
        s1 = d * sc[:, 2 * c:2 * c + 1]
        m1 = dmin * mn[:, 2 * c:2 * c + 1]
        s2 = d * sc[:, 2 * c + 1:2 * c + 2]
        m2 = dmin * mn[:, 2 * c + 1:2 * c + 2]
        y[:, 64 * c:64 * c + 32] = s1 * (q & 15) - m1
        y[:, 64 * c + 32:64 * c + 64] = s2 * (q >> 4) - m2
    return y.reshape(-1)


# ----------------------------------------------------------------------------- Q5_K
def quantize_q5_k(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32).reshape(-1, 8, 32)
    nb = x.shape[0]
    d, dmin, sc6, mn6, q = _kquant_affine(x, 31)
    q = q.reshape(nb, 256)
    out = np.zeros((nb, 176), np.uint8)
    out[:, 0:2] = d.astype(np.float16).reshape(-1, 1).view(np.uint8)
    out[:, 2:4] = dmin.astype(np.float16).reshape(-1, 1).view(np.uint8)
    out[:, 4:16] = pack_scale_min_k4(sc6, mn6)
    qh = np.zeros((nb, 32), np.uint8)
    qs = np.zeros((nb, 128), np.uint8)
    for c in range(4):
        lo = q[:, 64 * c:64 * c + 32]
        hi = q[:, 64 * c + 32:64 * c + 64]
        qs[:, 32 * c:32 * c + 32] = (lo & 15) | ((hi & 15) << 4)
        qh |= ((lo >> 4) & 1) << (2 * c)
        qh |= ((hi >> 4) & 1) << (2 * c + 1)
    out[:, 16:48] = qh
    out[:, 48:] = qs
    return out.reshape(-1)


def dequantize_q5_k(b: np.ndarray) -> np.ndarray:
    b = np.asarray(b, np.uint8).reshape(-1, 176)
    nb = b.shape[0]
    d = b[:, 0:2].copy().view(np.float16).astype(np.float32)
    dmin = b[:, 2:4].copy().view(np.float16).astype(np.float32)
    sc, mn = unpack_scale_min_k4(b[:, 4:16])
    qh = b[:, 16:48]
    qs = b[:, 48:]
    y = np.zeros((nb, 256), np.float32)
    for c in range(4):
        ql = qs[:, 32 * c:32 * c + 32]
        lo = (ql & 15) + (((qh >> (2 * c)) & 1) << 4)
        hi = (ql >> 4) + (((qh >> (2 * c + 1)) & 1) << 4)
        y[:, 64 * c:64 * c + 32] = d * sc[:, 2 * c:2 * c + 1] * lo - dmin * mn[:, 2 * c:2 * c + 1]
        y[:, 64 * c + 32:64 * c + 64] = d * sc[:, 2 * c + 1:2 * c + 2] * hi - dmin * mn[:, 2 * c + 1:2 * c + 2]
    return y.reshape(-1)


# ----------------------------------------------------------------------------- Q6_K
def quantize_q6_k(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32).reshape(-1, 16, 16)
    nb = x.shape[0]
    amax_idx = np.abs(x).argmax(axis=2)
    mx = np.take_along_axis(x, amax_idx[:, :, None], axis=2)[:, :, 0]   # signed max-magnitude
    scale = mx / -32.0                                                   # [nb, 16]
    amax_s = np.abs(scale).max(axis=1)
    d = amax_s / 127.0
    d16 = d.astype(np.float16).astype(np.float32)
    inv_d = np.where(d16 > 0, 1.0 / np.where(d16 > 0, d16, 1), 0.0)
    sc = np.clip(np.rint(scale * inv_d[:, None]), -128, 127).astype(np.int8)
    eff = d16[:, None] * sc.astype(np.float32)
    inv = np.where(eff != 0, 1.0 / np.where(eff != 0, eff, 1), 0.0)
    q = (np.clip(np.rint(x * inv[:, :, None]), -32, 31) + 32).astype(np.uint8).reshape(nb, 256)
    ql = np.zeros((nb, 128), np.uint8)
    qh = np.zeros((nb, 64), np.uint8)
    for n in range(2):
        qq = q[:, 128 * n:128 * n + 128]
        l = np.arange(32)
        q1, q2, q3, q4 = qq[:, l], qq[:, l + 32], qq[:, l + 64], qq[:, l + 96]
        ql[:, 64 * n + l] = (q1 & 15) | ((q3 & 15) << 4)
        ql[:, 64 * n + 32 + l] = (q2 & 15) | ((q4 & 15) << 4)
        qh[:, 32 * n + l] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
    out = np.zeros((nb, 210), np.uint8)
    out[:, 0:128] = ql
    out[:, 128:192] = qh
    out[:, 192:208] = sc.view(np.uint8)
    out[:, 208:210] = d16.astype(np.float16).reshape(-1, 1).view(np.uint8)
    return out.reshape(-1)


def dequantize_q6_k(b: np.ndarray) -> np.ndarray:
    b = np.asarray(b, np.uint8).reshape(-1, 210)
    nb = b.shape[0]
    ql = b[:, 0:128]
    qh = b[:, 128:192]
    sc = b[:, 192:208].view(np.int8).astype(np.float32)
    d = b[:, 208:210].copy().view(np.float16).astype(np.float32)
    y = np.zeros((nb, 256), np.float32)
    for n in range(2):
        l = np.arange(32)
        L = ql[:, 64 * n:64 * n + 64]
        H = qh[:, 32 * n:32 * n + 32]
        S = sc[:, 8 * n:8 * n + 8]
        q1 = ((L[:, l] & 15) | (((H[:, l] >> 0) & 3) << 4)).astype(np.int32) - 32
        q2 = ((L[:, l + 32] & 15) | (((H[:, l] >> 2) & 3) << 4)).astype(np.int32) - 32
        q3 = ((L[:, l] >> 4) | (((H[:, l] >> 4) & 3) << 4)).astype(np.int32) - 32
        q4 = ((L[:, l + 32] >> 4) | (((H[:, l] >> 6) & 3) << 4)).astype(np.int32) - 32
        isx = l // 16
        y[:, 128 * n + l] = d * S[:, isx] * q1
        y[:, 128 * n + 32 + l] = d * S[:, isx + 2] * q2
        y[:, 128 * n + 64 + l] = d * S[:, isx + 4] * q3
        y[:, 128 * n + 96 + l] = d * S[:, isx + 6] * q4
    return y.reshape(-1)


# ----------------------------------------------------------------------------- dispatch
def quantize(x: np.ndarray, qtype: int) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    if qtype == F32:
        return x.reshape(-1).view(np.uint8).copy()
    if qtype == F16:
        return x.astype(np.float16).reshape(-1).view(np.uint8).copy()
    if qtype == BF16:
        return f32_to_bf16_bits(x.reshape(-1)).view(np.uint8).copy()
    return {Q8_0: quantize_q8_0, Q4_0: quantize_q4_0, Q4_K: quantize_q4_k,
            Q5_K: quantize_q5_k, Q6_K: quantize_q6_k}[qtype](x)


def dequantize(b: np.ndarray, qtype: int, shape=None) -> np.ndarray:
    b = np.ascontiguousarray(b, np.uint8).reshape(-1)
    if qtype == F32:
        y = b.view(np.float32).copy()
    elif qtype == F16:
        y = b.view(np.float16).astype(np.float32)
    elif qtype == BF16:
        y = bf16_bits_to_f32(b.view(np.uint16))
    else:
        y = {Q8_0: dequantize_q8_0, Q4_0: dequantize_q4_0, Q4_K: dequantize_q4_k,
             Q5_K: dequantize_q5_k, Q6_K: dequantize_q6_k}[qtype](b)
    return y.reshape(shape) if shape is not None else y


def random_blocks(rng: np.random.Generator, qtype: int, n_rows: int, n_cols: int,
                  scale: float = 0.02) -> np.ndarray:
    """Random-init weights of a given ggml type WITHOUT going through float quantization
    (fast path for large synthetic models): random quant bits + sane block scales."""
    be, bb = BLOCK[qtype]
    nblk = n_rows * n_cols // be
    if qtype in (F32, F16, BF16):
        w = (rng.standard_normal(n_rows * n_cols, dtype=np.float32) * scale)
        return quantize(w, qtype)
    raw = rng.integers(0, 256, size=(nblk, bb), dtype=np.uint8)
    if qtype == Q8_0:
        raw[:, 0:2] = np.full((nblk, 1), scale / 64.0, np.float16).view(np.uint8)
    elif qtype == Q4_0:
        raw[:, 0:2] = np.full((nblk, 1), scale / 4.0, np.float16).view(np.uint8)
    elif qtype in (Q4_K, Q5_K):
        nmax = 15 if qtype == Q4_K else 31
        d = scale * 2.0 / (nmax * 40.0)
        raw[:, 0:2] = np.full((nblk, 1), d, np.float16).view(np.uint8)
        raw[:, 2:4] = np.full((nblk, 1), scale / 40.0, np.float16).view(np.uint8)
        sc = rng.integers(24, 56, size=(nblk, 8)).astype(np.uint8)
        mn = rng.integers(24, 56, size=(nblk, 8)).astype(np.uint8)
        raw[:, 4:16] = pack_scale_min_k4(sc, mn)
    elif qtype == Q6_K:
        raw[:, 192:208] = rng.integers(40, 100, size=(nblk, 16)).astype(np.int8).view(np.uint8)
        raw[:, 208:210] = np.full((nblk, 1), scale / (32.0 * 70.0), np.float16).view(np.uint8)
    return raw.reshape(-1)
