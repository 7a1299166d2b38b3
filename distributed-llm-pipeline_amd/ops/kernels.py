"""Thin torch wrappers over the HIP kernels (used by the T1 kernel tests and tools).

Every op launches the hand-written gfx950 kernel on torch's current HIP stream.  There is no
PyTorch fallback: if `libmipipe.so` is missing the import of the library raises.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import _native as N
from ..utils import quants as Q

EPI_STORE, EPI_ATOMIC, EPI_SWIGLU = 0, 1, 2
P_F16, P_Q8_0, P_Q4_K, P_Q5_K, P_Q6_K, P_Q4_0, P_BF16, P_I8 = 0, 1, 2, 3, 4, 5, 6, 7


def _ptr(t: torch.Tensor | None):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def pack_type(ggml_type: int) -> int:
    return N.lib().mp_pack_type(ggml_type)


def packed_dims(ggml_type: int, n: int, k: int):
    n_pad = (n + 15) // 16 * 16
    k_pad = (k + 255) // 256 * 256
    return n_pad, k_pad, n_pad // 16, k_pad // 256


def pack_t16(raw: np.ndarray, ggml_type: int, n: int, k: int, gateup: bool = False) -> np.ndarray:
    """Pack a GGUF-native [n][k] tensor (bytes) into the T16 device layout (host, C++ packer)."""
    raw = np.ascontiguousarray(raw, dtype=np.uint8)
    nbytes = N.lib().mp_packed_bytes(ggml_type, n, k)
    out = np.empty(nbytes, np.uint8)
    rb = Q.row_bytes(ggml_type, k)
    N.check(N.lib().mp_pack_t16(ggml_type, n, k, raw.ctypes.data, rb, out.ctypes.data, int(gateup)), "pack_t16")
    return out


class PackedWeight:
    """A T16-packed weight resident on the GPU."""

    def __init__(self, raw: np.ndarray, ggml_type: int, n: int, k: int, device="cuda", gateup=False):
        self.ggml_type, self.n, self.k = ggml_type, n, k
        self.ptype = pack_type(ggml_type)
        self.n_pad, self.k_pad, self.ntiles, self.nsb = packed_dims(ggml_type, n, k)
        self.host = pack_t16(raw, ggml_type, n, k, gateup)
        self.dev = torch.from_numpy(self.host).to(device)

    @classmethod
    def random(cls, ggml_type: int, n: int, k: int, seed: int = 0, scale: float | None = None, device="cuda"):
        """Random-init blocks of the type generated on the device (mp_init_packed, the synthetic
        models' weights): no host copy."""
        self = cls.__new__(cls)
        self.ggml_type, self.n, self.k = ggml_type, n, k
        self.ptype = pack_type(ggml_type)
        self.n_pad, self.k_pad, self.ntiles, self.nsb = packed_dims(ggml_type, n, k)
        self.host = None
        nbytes = N.lib().mp_packed_bytes(ggml_type, n, k)
        self.dev = torch.empty(nbytes, dtype=torch.uint8, device=device)
        N.check(N.lib().mp_init_packed(_ptr(self.dev), nbytes, self.ptype, scale if scale else 1.0 / k ** 0.5, seed,
                                       _stream()), "init_packed")
        return self

    def unpack(self) -> torch.Tensor:
        out = torch.zeros(self.n_pad, self.k_pad, dtype=torch.float16, device=self.dev.device)
        N.check(N.lib().mp_op_unpack(self.ptype, _ptr(self.dev), self.ntiles, self.nsb, _ptr(out), self.k_pad,
                                     _stream()), "unpack")
        return out[: self.n, : self.k]


def gemv(w: PackedWeight, x: torch.Tensor, epi: int = EPI_STORE, y: torch.Tensor | None = None,
         nsplit: int = 1, n_valid: int | None = None) -> torch.Tensor:
    """x: f16 [M][K_pad] (zero tail). Returns f32 [M][n] (STORE/ATOMIC) or f16 [M][n/2] (SWIGLU)."""
    assert x.dtype == torch.float16 and x.shape[1] == w.k_pad and x.is_contiguous()
    M = x.shape[0]
    if epi == EPI_SWIGLU:
        F = w.n // 2
        h = torch.zeros(M, F, dtype=torch.float16, device=x.device) if y is None else y
        N.check(N.lib().mp_op_gemv(w.ptype, epi, _ptr(w.dev), w.ntiles, w.nsb, _ptr(x), w.k_pad, M, None, 0,
                                   _ptr(h), h.stride(0), F if n_valid is None else n_valid, 1, _stream()), "gemv")
        return h
    if y is None:
        y = torch.zeros(M, w.n, dtype=torch.float32, device=x.device)
    N.check(N.lib().mp_op_gemv(w.ptype, epi, _ptr(w.dev), w.ntiles, w.nsb, _ptr(x), w.k_pad, M, _ptr(y),
                               y.stride(0), None, 0, w.n if n_valid is None else n_valid, nsplit, _stream()),
            "gemv")
    return y


def gemv_small(w: PackedWeight, epi: int = EPI_STORE, *, x: torch.Tensor | None = None,
               xf: torch.Tensor | None = None, gamma: torch.Tensor | None = None, eps: float = 1e-5,
               bias: torch.Tensor | None = None, y: torch.Tensor | None = None, G: int = 0, nsplit: int = 0,
               deterministic: bool = False) -> torch.Tensor:
    """Small-M decode GEMV (gemvs.hip, M <= 4), the engine's single-stream path.
    xf/gamma: fused RMSNorm -- the GEMV runs on f16(xf * rsqrt(mean(xf^2) + eps) * gamma), the
    standalone rmsnorm kernel's rounding.  ATOMIC adds into `y`.  G (tiles per workgroup) and nsplit
    (k-splits over the grid, ATOMIC only) override the launcher's plan (0 = auto)."""
    if xf is not None:
        assert xf.dtype == torch.float32 and xf.is_contiguous()
        M, d = xf.shape
    else:
        assert x.dtype == torch.float16 and x.shape[1] == w.k_pad and x.is_contiguous()
        M, d = x.shape[0], 0
    F = w.n // 2
    if epi == EPI_SWIGLU:
        h = torch.zeros(M, F, dtype=torch.float16, device=w.dev.device) if y is None else y
        Y, ldy, H, ldh, nv = None, 0, h, h.stride(0), F
    else:
        y = torch.zeros(M, w.n, dtype=torch.float32, device=w.dev.device) if y is None else y
        Y, ldy, H, ldh, nv = y, y.stride(0), None, 0, w.n
    N.check(N.lib().mp_op_gemvs(w.ptype, epi, _ptr(w.dev), w.ntiles, w.nsb, _ptr(x), w.k_pad if x is not None else 0,
                                M, _ptr(Y), ldy, _ptr(H), ldh, nv, _ptr(xf), d, _ptr(gamma), eps, d, _ptr(bias),
                                G, nsplit, int(deterministic), _stream()), "gemv_small")
    return h if epi == EPI_SWIGLU else y


def gemm(w: PackedWeight, x: torch.Tensor, epi: int = EPI_STORE, y: torch.Tensor | None = None,
         n_valid: int | None = None, v: int = 3, allow_split: bool = True) -> torch.Tensor:
    """Prefill / wide-decode GEMM (any M): x f16 [M][K_pad]. Same outputs as gemv (ATOMIC adds).
    v=3: BM x BN in {128, 256}^2 workgroup tiles, weights dequantized once per workgroup into LDS
    (launch_gemm3; ATOMIC may split K over workgroups unless allow_split is False); v=4: the 32x32x16
    MFMA GEMM (launch_gemm4); v=1: the 64 x 64 tile GEMM.  (v=2, the 128-row form of the decode GEMV,
    is retired.)"""
    assert x.dtype == torch.float16 and x.shape[1] == w.k_pad and x.is_contiguous()
    M = x.shape[0]
    L = N.lib()
    if v == 3:
        fn = lambda *a: L.mp_op_gemm3(*a[:-1], int(allow_split), a[-1])
    elif v == 4:
        fn = lambda *a: L.mp_op_gemm4(*a[:-1], int(allow_split), a[-1])
    else:
        assert v == 1, "gemm: v must be 1, 3 or 4 (the v=2 form is retired)"
        fn = L.mp_op_gemm
    if epi == EPI_SWIGLU:
        F = w.n // 2
        h = torch.zeros(M, F, dtype=torch.float16, device=x.device) if y is None else y
        N.check(fn(w.ptype, epi, _ptr(w.dev), w.ntiles, w.nsb, _ptr(x), w.k_pad, M, None, 0,
                   _ptr(h), h.stride(0), F if n_valid is None else n_valid, _stream()), "gemm")
        return h
    if y is None:
        y = torch.zeros(M, w.n, dtype=torch.float32, device=x.device)
    N.check(fn(w.ptype, epi, _ptr(w.dev), w.ntiles, w.nsb, _ptr(x), w.k_pad, M, _ptr(y),
               y.stride(0), None, 0, w.n if n_valid is None else n_valid, _stream()), "gemm")
    return y


def gemm_splitk(w: PackedWeight, x: torch.Tensor, y: torch.Tensor, v: int = 4, max_splits: int = 16) -> int:
    """Split-K through per-split partial stores and the fixed-order reduction added into y (the
    engine's wide-decode path for qkv / o / down, gemm_splitk_store); returns the split count (0:
    the shape did not split, y untouched).  The scratch starts as NaN, so a partial element the
    kernel never writes poisons y instead of reading as a plausible value."""
    assert x.dtype == torch.float16 and x.shape[1] == w.k_pad and x.is_contiguous() and v == 4
    M = x.shape[0]
    scratch = torch.full((max_splits * M * w.ntiles * 16,), float("nan"), dtype=torch.float32, device=x.device)
    return N.check(N.lib().mp_op_gemm4_splitk(w.ptype, _ptr(w.dev), w.ntiles, w.nsb, _ptr(x), w.k_pad, M, _ptr(y),
                                               y.stride(0), w.n, _ptr(scratch), scratch.numel(), _stream()),
                   "gemm_splitk")


def moe_route(logits: torch.Tensor, k: int, list_cap: int | None = None):
    """Top-k routing of router logits [M][E] (f32, contiguous): returns (counts [E], lists [E][list_cap]
    of token-slot ids t * k + j, renormalised top-k weights [M * k])."""
    M, E = logits.shape
    list_cap = list_cap or M * k
    counts = torch.zeros(E, dtype=torch.int32, device=logits.device)
    lists = torch.full((E, list_cap), -1, dtype=torch.int32, device=logits.device)
    weights = torch.zeros(M * k, dtype=torch.float32, device=logits.device)
    N.check(N.lib().mp_op_moe_route(_ptr(logits), logits.stride(0), M, E, k, _ptr(counts), _ptr(lists), list_cap,
                                    _ptr(weights), _stream()), "moe_route")
    return counts, lists, weights


def moe_gemm(w_dev: torch.Tensor, estride: int, ptype: int, ntiles: int, nsb: int, n_valid: int, epi: int,
             x: torch.Tensor, M: int, E: int, k: int, counts, lists, weights=None, *, x_per_slot: bool = False,
             h: torch.Tensor | None = None, y: torch.Tensor | None = None) -> None:
    """Grouped expert GEMM (gemm4 MoE mode, K13) over E packed matrices estride bytes apart:
    EPI_SWIGLU writes h[slot] = SwiGLU(x[slot // k] W_e^T) for every routed slot; EPI_ATOMIC adds
    weights[slot] * (x[slot] W_e^T) into y[slot // k] (x_per_slot: x rows are slots)."""
    assert x.dtype == torch.float16 and x.is_contiguous()
    N.check(N.lib().mp_op_moe_gemm4(ptype, epi, _ptr(w_dev), estride, ntiles, nsb, _ptr(x), x.stride(0),
                                    int(x_per_slot), M, E, k, _ptr(counts), _ptr(lists), lists.shape[1],
                                    _ptr(weights), _ptr(y), y.stride(0) if y is not None else 0, _ptr(h),
                                    h.stride(0) if h is not None else 0, n_valid, _stream()), "moe_gemm4")


def router_logits(x: torch.Tensor, r_dense: torch.Tensor) -> torch.Tensor:
    """logits [M][E] f32 = x [M][K] f16 . r_dense [E][K]^T (the dense-router kernel, E <= 64)."""
    M, K = x.shape[0], r_dense.shape[1]
    E = r_dense.shape[0]
    out = torch.zeros(M, 64, dtype=torch.float32, device=x.device)
    N.check(N.lib().mp_op_router_logits(_ptr(x), x.stride(0), _ptr(r_dense.contiguous()), K, E, M, _ptr(out), 64,
                                        _stream()), "router_logits")
    return out[:, :E]


class I8Weight:
    """Per-row int8 re-quantization of a packed weight for the int8-activation GEMM prototype
    (SURVEY K15): w8[n][k] = round(w[n][k] / ws[n]), ws[n] = max_k |w[n][k]| / 127, packed into P_I8
    chunks (csrc/kernels/gemm3.hip W3<P_I8>: byte ((2 st + kk) * 64 + 16 g + r) * 16 + j of chunk
    (tile t, super-block sb) is row 16 t + r, k = 256 sb + 128 st + 64 kk + 16 g + j)."""

    ptype = P_I8

    def __init__(self, w: PackedWeight):
        dense = w.unpack().float()
        n, k = dense.shape
        self.n, self.k, self.n_pad, self.k_pad, self.ntiles, self.nsb = n, k, w.n_pad, w.k_pad, w.ntiles, w.nsb
        ws = dense.abs().amax(1).clamp_min(1e-30) / 127.0
        q = torch.zeros(self.n_pad, self.k_pad, dtype=torch.int8, device=dense.device)
        q[:n, :k] = torch.round(dense / ws[:, None]).clamp(-127, 127).to(torch.int8)
        self.ws = torch.ones(self.n_pad, dtype=torch.float32, device=dense.device)
        self.ws[:n] = ws
        self.q = q
        v = q.view(self.ntiles, 16, self.nsb, 2, 2, 4, 16)           # t, r, sb, st, kk, g, j
        self.dev = v.permute(0, 2, 3, 4, 5, 1, 6).contiguous().view(-1)   # t, sb, st, kk, g, r, j


def quant_rows_i8(x: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """f16 [M][K] -> (int8 [M][K], f32 row scales [M]): q = round(x / s), s = max|x| / 127 per row."""
    assert x.dtype == torch.float16 and x.is_contiguous()
    M, K = x.shape
    q = torch.empty(M, K, dtype=torch.int8, device=x.device)
    xs = torch.empty(M, dtype=torch.float32, device=x.device)
    N.check(N.lib().mp_op_quant_i8(_ptr(x), K, M, K, _ptr(q), K, _ptr(xs), _stream()), "quant_i8")
    return q, xs


def gemm_i8(w: I8Weight, x: torch.Tensor | None = None, epi: int = EPI_STORE, y: torch.Tensor | None = None,
            xq: tuple[torch.Tensor, torch.Tensor] | None = None, allow_split: bool = True) -> torch.Tensor:
    """int8-activation GEMM prototype: x f16 [M][K_pad] quantized per row (or xq = quant_rows_i8(x)
    given), v_mfma_i32_16x16x64_i8 against I8Weight, y = xs[m] ws[n] sum_k xq wq (exact int32 sums)."""
    q, xs = xq if xq is not None else quant_rows_i8(x)
    assert q.shape[1] == w.k_pad
    M = q.shape[0]
    L = N.lib()
    if epi == EPI_SWIGLU:
        F = w.n // 2
        h = torch.zeros(M, F, dtype=torch.float16, device=q.device) if y is None else y
        N.check(L.mp_op_gemm3_i8(epi, _ptr(w.dev), w.ntiles, w.nsb, _ptr(q), w.k_pad, M, None, 0, _ptr(h), h.stride(0),
                                 F, _ptr(xs), _ptr(w.ws), int(allow_split), _stream()), "gemm_i8")
        return h
    if y is None:
        y = torch.zeros(M, w.n, dtype=torch.float32, device=q.device)
    N.check(L.mp_op_gemm3_i8(epi, _ptr(w.dev), w.ntiles, w.nsb, _ptr(q), w.k_pad, M, _ptr(y), y.stride(0), None, 0,
                             w.n, _ptr(xs), _ptr(w.ws), int(allow_split), _stream()), "gemm_i8")
    return y


def set_gemm3_tuning(bm: int = 0, bn: int = 0, nsplit: int = 0, split_wg: int = 0) -> None:
    """Force the v3 GEMM's tile rows / columns (128 | 256) and ATOMIC split-K factor (0 = auto);
    split_wg: workgroup target of the automatic split.  0 restores a knob to the process's own value
    (its MIPIPE_* environment variable, else the default)."""
    N.check(N.lib().mp_set_gemm3_tuning(bm, bn, nsplit, split_wg), "set_gemm3_tuning")


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, k_pad: int | None = None) -> torch.Tensor:
    M, d = x.shape
    k_pad = k_pad or (d + 255) // 256 * 256
    out = torch.zeros(M, k_pad, dtype=torch.float16, device=x.device)
    N.check(N.lib().mp_op_rmsnorm(_ptr(x), x.stride(0), _ptr(w), d, eps, _ptr(out), k_pad, M, _stream()), "rmsnorm")
    return out


def embed(raw_table: torch.Tensor, ggml_type: int, d: int, tokens: torch.Tensor) -> torch.Tensor:
    M = tokens.numel()
    x = torch.empty(M, d, dtype=torch.float32, device=tokens.device)
    rb = Q.row_bytes(ggml_type, d)
    N.check(N.lib().mp_op_embed(ggml_type, _ptr(raw_table), rb, d, _ptr(tokens), M, _ptr(x), d, _stream()), "embed")
    return x


def attn_prefill(q, pos, slot, block_table, k_cache, v_cache, Hkv, hd, segs=None, n_split=1, split_pages=1):
    """Prefill flash attention (attn_prefill.hip): q [M][Hq][Dp] f16 (q_scale applied), rows in
    `segs` = [(row0, T), ...] runs of consecutive positions of one sequence each (default: one run);
    n_split > 1 splits every tile's pages (split_pages each) over workgroups, merged by attn_combine."""
    M, Hq, Dp = q.shape
    segs = segs or [(0, M)]
    sa = np.asarray(segs, np.int32).reshape(-1)
    out = torch.zeros(M, Hq * hd, dtype=torch.float16, device=q.device)
    op = ml = None
    if n_split > 1:
        op = torch.full((n_split, M * Hq, Dp), float("nan"), dtype=torch.float32, device=q.device)
        ml = torch.full((n_split, M * Hq, 2), float("nan"), dtype=torch.float32, device=q.device)
    N.check(N.lib().mp_op_attn_prefill(_ptr(q), _ptr(pos), _ptr(slot), _ptr(block_table), block_table.shape[1],
                                       _ptr(k_cache), _ptr(v_cache), Hq, Hkv, hd, Dp,
                                       sa.ctypes.data, len(segs), _ptr(out), out.stride(0), n_split, split_pages,
                                       _ptr(op), _ptr(ml), M, _stream()), "attn_prefill")
    return out


ARGMAX_CHUNKS = 64


def argmax(logits: torch.Tensor, two_level: bool = True) -> torch.Tensor:
    """Greedy token per row (lowest index on ties).  two_level: (chunk, row) grid + last-arriver
    reduce (the engine's path); otherwise one workgroup per row."""
    M, n = logits.shape
    out = torch.empty(M, dtype=torch.int32, device=logits.device)
    part = cnt = None
    if two_level:
        part = torch.empty(M, ARGMAX_CHUNKS, 2, dtype=torch.float32, device=logits.device)
        cnt = torch.zeros(M, dtype=torch.int32, device=logits.device)
    N.check(N.lib().mp_op_argmax(_ptr(logits), logits.stride(0), n, M, _ptr(out), _ptr(part), _ptr(cnt),
                                 _stream()), "argmax")
    if cnt is not None:
        assert int(cnt.abs().sum()) == 0, "argmax arrival counters did not reset"
    return out


def gemv_fused(w: PackedWeight, epi: int = EPI_STORE, *, x: torch.Tensor | None = None,
               xf: torch.Tensor | None = None, gamma: torch.Tensor | None = None, eps: float = 1e-5,
               bias: torch.Tensor | None = None, y: torch.Tensor | None = None, nsplit: int = 1,
               zero: torch.Tensor | None = None, ssq: torch.Tensor | None = None) -> torch.Tensor:
    """Decode GEMV (gemv2.hip) with the fusions the engine uses at single-stream decode.
    xf/gamma: deferred RMSNorm of the f32 rows xf (M <= 4, x unused) -- the GEMV runs on
    f16(xf * gamma); STORE/SWIGLU outputs are scaled by rsqrt(mean(xf^2) + eps), ATOMIC outputs are
    left unscaled and sum(xf^2) per row is added into `ssq` (f32 [M]).  bias: added once per output.
    zero: f32 tensor cleared after the GEMV."""
    if xf is not None:
        assert xf.dtype == torch.float32 and xf.is_contiguous()
        M, d = xf.shape
    else:
        assert x.dtype == torch.float16 and x.shape[1] == w.k_pad and x.is_contiguous()
        M, d = x.shape[0], 0
    F = w.n // 2
    if epi == EPI_SWIGLU:
        h = torch.zeros(M, F, dtype=torch.float16, device=w.dev.device) if y is None else y
        Y, ldy, H, ldh, nv = None, 0, h, h.stride(0), F
    else:
        y = torch.zeros(M, w.n, dtype=torch.float32, device=w.dev.device) if y is None else y
        Y, ldy, H, ldh, nv = y, y.stride(0), None, 0, w.n
    N.check(N.lib().mp_op_gemv_fused(w.ptype, epi, _ptr(w.dev), w.ntiles, w.nsb, _ptr(x), w.k_pad if x is not None else 0,
                                     M, _ptr(Y), ldy, _ptr(H), ldh, nv, nsplit, _ptr(xf), d, _ptr(gamma), eps, d,
                                     _ptr(ssq), _ptr(bias), _ptr(zero), 0 if zero is None else zero.numel(), _stream()),
            "gemv_fused")
    return H if epi == EPI_SWIGLU else Y


def sample(logits: torch.Tensor, temp: float, top_k: int = 0, top_p: float = 1.0, min_p: float = 0.0,
           seed: int = 0, step: torch.Tensor | None = None) -> torch.Tensor:
    M, n = logits.shape
    out = torch.empty(M, dtype=torch.int32, device=logits.device)
    N.check(N.lib().mp_op_sample(_ptr(logits), logits.stride(0), n, M, temp, top_k, top_p, min_p, seed, _ptr(step),
                                 _ptr(out), _stream()), "sample")
    return out


def penalize(logits: torch.Tensor, hist: torch.Tensor, repeat: float = 1.0, freq: float = 0.0,
             presence: float = 0.0) -> torch.Tensor:
    """In-place repetition penalties: logits f32 [M][n], hist int32 [M][last_n] (-1 = empty)."""
    M, n = logits.shape
    assert hist.dtype == torch.int32 and hist.shape[0] == M and hist.is_contiguous()
    N.check(N.lib().mp_op_penalize(_ptr(logits), logits.stride(0), n, M, _ptr(hist), hist.shape[1], repeat, freq,
                                   presence, _stream()), "penalize")
    return logits


def hist_push(hist: torch.Tensor, cnt: torch.Tensor, tokens: torch.Tensor) -> None:
    """hist[m][cnt[m] % last_n] = tokens[m]; cnt[m] += 1 (int32 device tensors)."""
    M, last_n = hist.shape
    N.check(N.lib().mp_op_hist_push(_ptr(hist), _ptr(cnt), last_n, _ptr(tokens), M, _stream()), "hist_push")


def rope_cs_table(max_pos: int, hd: int, base: float, freq_factors=None) -> torch.Tensor:
    inv = base ** (-np.arange(0, hd, 2, dtype=np.float64) / hd)
    if freq_factors is not None:
        inv = inv / np.asarray(freq_factors, np.float64)
    ang = np.outer(np.arange(max_pos, dtype=np.float64), inv)
    cs = np.stack([np.cos(ang), np.sin(ang)], -1).astype(np.float32)   # [pos][hd/2][2]
    return torch.from_numpy(cs)


def rope_kv(qkv, pos, slot, block_table, rope_cs, Hq, Hkv, hd, Dp, q_scale, k_cache, v_cache):
    M = qkv.shape[0]
    q_out = torch.zeros(M, Hq, Dp, dtype=torch.float16, device=qkv.device)
    N.check(N.lib().mp_op_rope_kv(_ptr(qkv), qkv.stride(0), M, Hq, Hkv, hd, Dp, _ptr(pos), _ptr(slot),
                                  _ptr(block_table), block_table.shape[1], _ptr(rope_cs), q_scale, _ptr(q_out),
                                  _ptr(k_cache), _ptr(v_cache), _stream()), "rope_kv")
    return q_out


def attention(q, kvlen, slot, block_table, k_cache, v_cache, Hkv, hd, tq=1, split_len=256, n_split=1):
    M, Hq, Dp = q.shape
    out = torch.zeros(M, Hq * hd, dtype=torch.float16, device=q.device)
    o_part = torch.zeros(max(n_split, 1), M * Hq, Dp, dtype=torch.float32, device=q.device)
    ml_part = torch.zeros(max(n_split, 1), M * Hq, 2, dtype=torch.float32, device=q.device)
    N.check(N.lib().mp_op_attention(_ptr(q), _ptr(kvlen), _ptr(slot), _ptr(block_table), block_table.shape[1],
                                    _ptr(k_cache), _ptr(v_cache), M, Hq, Hkv, hd, Dp, tq, split_len, n_split,
                                    _ptr(o_part), _ptr(ml_part), _ptr(out), out.stride(0), _stream()), "attention")
    return out
