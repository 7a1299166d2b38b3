// Per-packed-type register dequantizers for the T16 layout (see csrc/runtime/qtypes.h).
//
// For one (tile, 256-k super-block) chunk, lane l = 16g + r loads `Raw` (its row r's share) and
// `dequant<h>` turns half h (k in [128h, 128h+128)) into the four f16 B-operand fragments of
// v_mfma_f32_16x16x32_f16: b[s] holds W[row r][k = 128h + 32s + 8g + j], j = 0..7.
// Integer->f16 uses the 1024-magic (0x6400 | q == 1024 + q, exact), one v_pk_add_f16 to remove the
// offset (exact) and one v_pk_fma/mul_f16 with the block scale (single rounding).
#pragma once
#include "kcommon.h"
#include "../runtime/qtypes.h"

namespace mpk {
using namespace mp;

__device__ __forceinline__ half2_t h2splat(float v) { f16 h = (f16)v; return half2_t{h, h}; }

template <int PT> struct Deq;

// ------------------------------------------------------------------ Q4_K (144 B / 256 w)
template <> struct Deq<P_Q4_K> {
  static constexpr int CB = chunk_bytes(P_Q4_K);
  struct Raw { u32x4 q0, q1, hdr; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) {
    r.q0 = ld16_nt(c + lane * 16);
    r.q1 = ld16_nt(c + 1024 + lane * 16);
    r.hdr = ld16(c + 2048 + (lane & 15) * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
    const half2_t dm = as_h2(r.hdr.x);
    const float d = (float)dm.x, dmin = (float)dm.y;
    const uint32_t S0 = r.hdr.y, S1 = r.hdr.z, S2 = r.hdr.w;
    uint32_t sc, mn;
    if (H == 0) { sc = S0 & 0x3F3F3F3Fu; mn = S1 & 0x3F3F3F3Fu; }
    else {
      sc = (S2 & 0x0F0F0F0Fu) | ((S0 >> 2) & 0x30303030u);
      mn = ((S2 >> 4) & 0x0F0F0F0Fu) | ((S1 >> 2) & 0x30303030u);
    }
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const half2_t off = {(f16)1024.0f, (f16)1024.0f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half2_t S = h2splat(d * (float)((sc >> (8 * s)) & 0xFF));
      const half2_t M = h2splat(-dmin * (float)((mn >> (8 * s)) & 0xFF));
      const uint32_t qd = q[s];
      uint32_t w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        half2_t v = as_h2(((qd >> (4 * i)) & 0x000F000Fu) | 0x64006400u) - off;
        w[i] = as_u32(__builtin_elementwise_fma(v, S, M));
      }
      b[s] = pack8(w[0], w[1], w[2], w[3]);
    }
  }
};

// ------------------------------------------------------------------ Q5_K (176 B / 256 w)
template <> struct Deq<P_Q5_K> {
  static constexpr int CB = chunk_bytes(P_Q5_K);
  struct Raw { u32x4 q0, q1, hdr; uint32_t qh0, qh1; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) {
    r.q0 = ld16_nt(c + lane * 16);
    r.q1 = ld16_nt(c + 1024 + lane * 16);
    r.qh0 = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(c + 2048 + lane * 4));
    r.qh1 = __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(c + 2048 + 256 + lane * 4));
    r.hdr = ld16(c + 2560 + (lane & 15) * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
    const half2_t dm = as_h2(r.hdr.x);
    const float d = (float)dm.x, dmin = (float)dm.y;
    const uint32_t S0 = r.hdr.y, S1 = r.hdr.z, S2 = r.hdr.w;
    uint32_t sc, mn;
    if (H == 0) { sc = S0 & 0x3F3F3F3Fu; mn = S1 & 0x3F3F3F3Fu; }
    else {
      sc = (S2 & 0x0F0F0F0Fu) | ((S0 >> 2) & 0x30303030u);
      mn = ((S2 >> 4) & 0x0F0F0F0Fu) | ((S1 >> 2) & 0x30303030u);
    }
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const uint32_t qh = H == 0 ? r.qh0 : r.qh1;
    const half2_t off = {(f16)1024.0f, (f16)1024.0f};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half2_t S = h2splat(d * (float)((sc >> (8 * s)) & 0xFF));
      const half2_t M = h2splat(-dmin * (float)((mn >> (8 * s)) & 0xFF));
      const uint32_t qd = q[s];
      const uint32_t hb = (qh >> (8 * s)) & 0xFFu;
      const uint32_t x = hb | (hb << 12);
      uint32_t w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t hi = ((x >> i) << 4) & 0x00100010u;
        half2_t v = as_h2(((qd >> (4 * i)) & 0x000F000Fu) | hi | 0x64006400u) - off;
        w[i] = as_u32(__builtin_elementwise_fma(v, S, M));
      }
      b[s] = pack8(w[0], w[1], w[2], w[3]);
    }
  }
};

// ------------------------------------------------------------------ Q6_K (210 B / 256 w)
template <> struct Deq<P_Q6_K> {
  static constexpr int CB = chunk_bytes(P_Q6_K);
  struct Raw { u32x4 q0, q1, sc; u32x2 qh0, qh1; uint32_t d; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) {
    r.q0 = ld16_nt(c + lane * 16);
    r.q1 = ld16_nt(c + 1024 + lane * 16);
    r.qh0 = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(c + 2048 + lane * 8));
    r.qh1 = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(c + 2048 + 512 + lane * 8));
    r.sc = ld16(c + 3072 + (lane & 15) * 16);
    r.d = *reinterpret_cast<const uint16_t*>(c + 3328 + (lane & 15) * 2);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
    const float d = h2f((uint16_t)r.d);
    const int gb = (lane >> 5) & 1;          // (g >> 1)
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const u32x2 qh = H == 0 ? r.qh0 : r.qh1;
    const half2_t off = {(f16)1056.0f, (f16)1056.0f};   // 1024 magic + 32 zero-point
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // sub-block (16 weights) index = 8H + 2s + gb  -> dword 2H + (s>>1), byte 2(s&1) + gb
      const uint32_t scw = r.sc[2 * H + (s >> 1)];
      const int scv = (int)(int8_t)((scw >> (8 * (2 * (s & 1) + gb))) & 0xFF);
      const half2_t S = h2splat(d * (float)scv);
      const uint32_t qd = q[s];
      const uint32_t h16 = (qh[s >> 1] >> (16 * (s & 1))) & 0xFFFFu;
      const uint32_t e = h16 | (h16 << 8);
      uint32_t w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t hi = ((e >> (2 * i)) << 4) & 0x00300030u;
        half2_t v = as_h2(((qd >> (4 * i)) & 0x000F000Fu) | hi | 0x64006400u) - off;
        w[i] = as_u32(v * S);
      }
      b[s] = pack8(w[0], w[1], w[2], w[3]);
    }
  }
};

// ------------------------------------------------------------------ Q8_0 (34 B / 32 w)
template <> struct Deq<P_Q8_0> {
  static constexpr int CB = chunk_bytes(P_Q8_0);
  struct Raw { u32x4 a0, a1, b0, b1, dd; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) {
    r.a0 = ld16_nt(c + lane * 32);
    r.a1 = ld16_nt(c + lane * 32 + 16);
    r.b0 = ld16_nt(c + 2048 + lane * 32);
    r.b1 = ld16_nt(c + 2048 + lane * 32 + 16);
    r.dd = ld16(c + 4096 + (lane & 15) * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
    const half2_t off = {(f16)1152.0f, (f16)1152.0f};   // 1024 magic + 128 (bytes stored q+128)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int blk = 4 * H + s;
      const uint32_t dw = r.dd[blk >> 1];
      const f16 dh = __builtin_bit_cast(f16, (uint16_t)(dw >> (16 * (blk & 1))));
      const half2_t S = {dh, dh};
      const u32x4 src = H == 0 ? (s < 2 ? r.a0 : r.a1) : (s < 2 ? r.b0 : r.b1);
      const uint32_t lo = src[2 * (s & 1)], hi = src[2 * (s & 1) + 1];
      uint32_t w[4];
      w[0] = as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, lo, 0x04010400u)) - off) * S);
      w[1] = as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, lo, 0x04030402u)) - off) * S);
      w[2] = as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, hi, 0x04010400u)) - off) * S);
      w[3] = as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, hi, 0x04030402u)) - off) * S);
      b[s] = pack8(w[0], w[1], w[2], w[3]);
    }
  }
};

// ------------------------------------------------------------------ Q4_0 (18 B / 32 w)
template <> struct Deq<P_Q4_0> {
  static constexpr int CB = chunk_bytes(P_Q4_0);
  struct Raw { u32x4 q0, q1, dd; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) {
    r.q0 = ld16_nt(c + lane * 16);
    r.q1 = ld16_nt(c + 1024 + lane * 16);
    r.dd = ld16(c + 2048 + (lane & 15) * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
    const half2_t off = {(f16)1032.0f, (f16)1032.0f};
    const u32x4 q = H == 0 ? r.q0 : r.q1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int blk = 4 * H + s;
      const uint32_t dw = r.dd[blk >> 1];
      const f16 dh = __builtin_bit_cast(f16, (uint16_t)(dw >> (16 * (blk & 1))));
      const half2_t S = {dh, dh};
      const uint32_t qd = q[s];
      uint32_t w[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        w[i] = as_u32((as_h2(((qd >> (4 * i)) & 0x000F000Fu) | 0x64006400u) - off) * S);
      b[s] = pack8(w[0], w[1], w[2], w[3]);
    }
  }
};

// ------------------------------------------------------------------ F16 (plain)
template <> struct Deq<P_F16> {
  static constexpr int CB = chunk_bytes(P_F16);
  struct Raw { u32x4 v[8]; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = ld16_nt(c + i * 1024 + lane * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
#pragma unroll
    for (int s = 0; s < 4; ++s) b[s] = __builtin_bit_cast(half8_t, r.v[4 * H + s]);
  }
};

}  // namespace mpk
