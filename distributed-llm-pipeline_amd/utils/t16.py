"""Numpy reference of the T16 packed-weight layout (csrc/runtime/qtypes.h, csrc/kernels/dequant.h).

`unpack_t16(packed, ptype, n, k)` decodes the packed bytes exactly the way the HIP dequantizers
index them (lane l = 16g + r, half h, MFMA step s, element j -> k = 64g + 32h + 8s + j), in f32.  It is the CPU-side oracle
that the C++ packer is tested against (the GPU unpack kernel is tested against the same function).
"""
from __future__ import annotations

import numpy as np

from . import quants as Q

P_F16, P_Q8_0, P_Q4_K, P_Q5_K, P_Q6_K, P_Q4_0, P_BF16 = 0, 1, 2, 3, 4, 5, 6
CHUNK = {P_F16: 8192, P_Q8_0: 4352, P_Q4_K: 2304, P_Q5_K: 2816, P_Q6_K: 3360, P_Q4_0: 2304, P_BF16: 8192}
PACK_OF = {Q.F32: P_F16, Q.F16: P_F16, Q.BF16: P_BF16, Q.Q8_0: P_Q8_0, Q.Q4_0: P_Q4_0,
           Q.Q4_K: P_Q4_K, Q.Q5_K: P_Q5_K, Q.Q6_K: P_Q6_K}


def _f16(b2):
    return np.frombuffer(np.ascontiguousarray(b2).tobytes(), np.float16).astype(np.float32)


def _bf16(b2):
    u = np.frombuffer(np.ascontiguousarray(b2).tobytes(), np.uint16).astype(np.uint32) << 16
    return u.view(np.float32)


def unpack_t16(packed: np.ndarray, ptype: int, n: int, k: int) -> np.ndarray:
    n_pad = (n + 15) // 16 * 16
    k_pad = (k + 255) // 256 * 256
    ntiles, nsb = n_pad // 16, k_pad // 256
    cb = CHUNK[ptype]
    P = np.asarray(packed, np.uint8).reshape(ntiles, nsb, cb)
    out = np.zeros((n_pad, k_pad), np.float32)
    lane = np.arange(64)
    g, r = lane >> 4, lane & 15
    for t in range(ntiles):
        for sb in range(nsb):
            c = P[t, sb]
            for h in range(2):
                for s in range(4):
                    for j in range(8):
                        kk = sb * 256 + 64 * g + 32 * h + 8 * s + j           # [64]
                        row = 16 * t + r
                        pos = (j & 1) * 4 + (j >> 1)                          # nibble position
                        if ptype in (P_Q4_K, P_Q5_K, P_Q6_K, P_Q4_0):
                            dw = c[h * 1024 + lane * 16 + s * 4 + pos // 2]
                            q = (dw >> ((pos & 1) * 4)) & 15
                        if ptype in (P_Q4_K, P_Q5_K):
                            hdr0 = 2048 if ptype == P_Q4_K else 2560
                            hdr = np.stack([c[hdr0 + 16 * rr: hdr0 + 16 * rr + 16] for rr in r])
                            d = _f16(hdr[:, 0:2])
                            dmin = _f16(hdr[:, 2:4])
                            # per lane group g: v = sc(2g) | m(2g) << 6 | sc(2g+1) << 12 | m(2g+1) << 18,
                            # byte b of v at header byte 4 + 4b + g
                            v = sum(hdr[lane, 4 + 4 * b + g].astype(np.int64) << (8 * b) for b in range(3))
                            sh = 12 * h
                            sc, mn = (v >> sh) & 63, (v >> (sh + 6)) & 63
                            if ptype == P_Q5_K:
                                qh = c[2048 + h * 256 + lane * 4 + (8 * s + pos) // 8]
                                q = q + (((qh >> ((8 * s + pos) % 8)) & 1) << 4)
                            v = d * sc * q - dmin * mn
                        elif ptype == P_Q6_K:
                            i = j >> 1
                            bit = 16 * s + ((8 + 2 * i) if (j & 1) else 2 * i)
                            qh = c[2048 + h * 512 + lane * 8 + bit // 8]
                            q = q + (((qh >> (bit % 8)) & 3) << 4)
                            scl = np.stack([c[3072 + 16 * rr: 3072 + 16 * rr + 16] for rr in r]).view(np.int8)
                            d = _f16(np.stack([c[3328 + 2 * rr: 3328 + 2 * rr + 2] for rr in r]))
                            sub = 4 * g + 2 * h + (s >> 1)
                            v = d * scl[np.arange(64), sub].astype(np.float32) * (q.astype(np.float32) - 32)
                        elif ptype == P_Q4_0:
                            blk = 2 * g + h
                            d = _f16(np.stack([c[2048 + 16 * rr + 2 * bb: 2048 + 16 * rr + 2 * bb + 2] for rr, bb in zip(r, blk)]))
                            v = d * (q.astype(np.float32) - 8)
                        elif ptype == P_Q8_0:
                            u = c[h * 2048 + lane * 32 + s * 8 + j].astype(np.float32)
                            blk = 2 * g + h
                            d = _f16(np.stack([c[4096 + 16 * rr + 2 * bb: 4096 + 16 * rr + 2 * bb + 2] for rr, bb in zip(r, blk)]))
                            v = d * (u - 128)
                        else:  # F16 / BF16 (same layout)
                            b2 = np.stack([c[h * 4096 + s * 1024 + l * 16 + 2 * j: h * 4096 + s * 1024 + l * 16 + 2 * j + 2]
                                           for l in lane])
                            v = _bf16(b2) if ptype == P_BF16 else _f16(b2)
                        out[row, kk] = v
    return out[:n, :k]
