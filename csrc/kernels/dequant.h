// Per-packed-type register dequantizers for the T16 layout (see csrc/runtime/qtypes.h).
//
// For one (tile, 256-k super-block) chunk, lane l = 16g + r loads `Raw` (its row r's share) and
// `dequant<h>` turns half h (k in [128h, 128h+128)) into the four f16 B-operand fragments of
// v_mfma_f32_16x16x32_f16: b[s] holds W[row r][k = 128h + 32s + 8g + j], j = 0..7.
//
// Integer -> f16 by exponent magic, no shifts per pair.  A dword holds 8 nibbles (j = 2i at bit
// 4i, j = 2i+1 at bit 16+4i).  (w & 0x000F000F) | 0x64006400 is the f16 pair (1024 + q) for
// j = {0,1} (mantissa unit 1 at exponent 2^10); (w & 0x00F000F0) | 0x54005400 is (64 + q) for
// j = {2,3}: at exponent 2^6 the mantissa unit is 1/16, so the nibble sitting at bits 4..7 reads
// as q exactly.  The same two masks on (w >> 8) give j = {4,5} and {6,7}.  High bits of Q5_K/Q6_K
// are OR-ed in at +16 (bit 4 / bit 8 respectively).  Per f16 pair: one v_and_or_b32 (masks kept
// in VGPRs: GFX9 VOP3 takes no literals), one v_pk_add_f16 removing the exact offset, and one
// v_pk_fma/mul_f16 applying the block scale (single rounding on the final weight).
#pragma once
#include "kcommon.h"
#include "../runtime/qtypes.h"

namespace mpk {
using namespace mp;

__device__ __forceinline__ half2_t h2lo(half2_t v) { return half2_t{v.x, v.x}; }
__device__ __forceinline__ half2_t h2hi(half2_t v) { return half2_t{v.y, v.y}; }
__device__ __forceinline__ half2_t h2splat(float v) { f16 h = (f16)v; return half2_t{h, h}; }
__device__ __forceinline__ half2_t h2c(float v) { return half2_t{(f16)v, (f16)v}; }

template <int PT> struct Deq;

struct Consts { uint32_t mlo, mhi, mag_hi, mag_lo; };
__device__ __forceinline__ Consts make_consts() {
  Consts c;
  asm("v_mov_b32 %0, 0x000f000f" : "=v"(c.mlo));
  asm("v_mov_b32 %0, 0x00f000f0" : "=v"(c.mhi));
  asm("v_mov_b32 %0, 0x64006400" : "=v"(c.mag_hi));   // 1024 + q
  asm("v_mov_b32 %0, 0x54005400" : "=v"(c.mag_lo));   // 64 + q   (q at mantissa bits 4..7)
  return c;
}
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t m, uint32_t c) {
  uint32_t d;
  asm("v_and_or_b32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(m), "v"(c));
  return d;
}

// four 6/8-bit scale bytes -> (s0, s2), (s1, s3) as f16 pairs times `mul`
__device__ __forceinline__ void bytes4_to_h2(uint32_t v, half2_t mul, half2_t& s02, half2_t& s13) {
  s02 = (as_h2((v & 0x00FF00FFu) | 0x64006400u) - h2c(1024.f)) * mul;
  s13 = (as_h2(((v >> 8) & 0x00FF00FFu) | 0x64006400u) - h2c(1024.f)) * mul;
}
__device__ __forceinline__ half2_t pick(half2_t s02, half2_t s13, int s) {
  return s == 0 ? h2lo(s02) : s == 1 ? h2lo(s13) : s == 2 ? h2hi(s02) : h2hi(s13);
}

// 6-bit Q4_K/Q5_K scales of half H: bytes j = sub-blocks 4H .. 4H+3
template <int H>
__device__ __forceinline__ void kscales(const u32x4& hdr, uint32_t& sc, uint32_t& mn) {
  const uint32_t S0 = hdr.y, S1 = hdr.z, S2 = hdr.w;
  if (H == 0) { sc = S0 & 0x3F3F3F3Fu; mn = S1 & 0x3F3F3F3Fu; }
  else {
    sc = (S2 & 0x0F0F0F0Fu) | ((S0 >> 2) & 0x30303030u);
    mn = ((S2 >> 4) & 0x0F0F0F0Fu) | ((S1 >> 2) & 0x30303030u);
  }
}

// ------------------------------------------------------------------ Q4_K (144 B / 256 w)
template <> struct Deq<P_Q4_K> {
  static constexpr int CB = chunk_bytes(P_Q4_K);
  struct Raw { u32x4 q0, q1, hdr; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) {
    r.q0 = ld16_nt(c + lane * 16);
    r.q1 = ld16_nt(c + 1024 + lane * 16);
    r.hdr = ld16(c + 2048 + (lane & 15) * 16);
  }
  // Min-free dequant: B = fma(x_magic, S, T) with T = -offset * S EXACT (power-of-two multiple of
  // an f16), i.e. B = q * S rounded once; the "- dmin * m" term of every 32-weight sub-block is
  // left to one extra MFMA per 4 super-blocks against the sub-block sums of x (mins() below):
  // 2 VALU ops per f16 pair instead of 3.
  // mins of the 8 sub-blocks of this super-block as the B fragment of that MFMA: -dmin * m_j
  __device__ static __forceinline__ half8_t mins(const Raw& r) {
    const half2_t dm = as_h2(r.hdr.x);
    const uint32_t S0 = r.hdr.y, S1 = r.hdr.z, S2 = r.hdr.w;
    (void)S0;
    const uint32_t m03 = S1 & 0x3F3F3F3Fu;
    const uint32_t m47 = ((S2 >> 4) & 0x0F0F0F0Fu) | ((S1 >> 2) & 0x30303030u);
    const half2_t nd = -h2hi(dm), c = h2hi(dm) * h2c(1024.f);   // exact: power-of-two multiple
    const Consts k = make_consts();
    auto cv = [&](uint32_t v) { return as_u32(__builtin_elementwise_fma(as_h2(and_or(v, 0x00FF00FFu, k.mag_hi)), nd, c)); };
    // pairs (m0,m2),(m1,m3) -> reorder to m0..m7 in j order
    const half2_t a02 = as_h2(cv(m03)), a13 = as_h2(cv(m03 >> 8)), b02 = as_h2(cv(m47)), b13 = as_h2(cv(m47 >> 8));
    half8_t o;
    o[0] = a02.x; o[1] = a13.x; o[2] = a02.y; o[3] = a13.y;
    o[4] = b02.x; o[5] = b13.x; o[6] = b02.y; o[7] = b13.y;
    return o;
  }
  template <int H>
  __device__ static __forceinline__ void dequant_fast(const Raw& r, half8_t b[4], int lane) {
    const half2_t dm = as_h2(r.hdr.x);
    uint32_t sc, mn;
    kscales<H>(r.hdr, sc, mn);
    const Consts k = make_consts();
    const half2_t d2 = h2lo(dm);
    const half2_t nd = d2 * h2c(-1024.f);
    const half2_t S02 = __builtin_elementwise_fma(as_h2(and_or(sc, 0x00FF00FFu, k.mag_hi)), d2, nd);
    const half2_t S13 = __builtin_elementwise_fma(as_h2(and_or(sc >> 8, 0x00FF00FFu, k.mag_hi)), d2, nd);
    const half2_t T02 = S02 * h2c(-1024.f), T13 = S13 * h2c(-1024.f);
    const half2_t U02 = S02 * h2c(-64.f), U13 = S13 * h2c(-64.f);
    const u32x4 q = H == 0 ? r.q0 : r.q1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half2_t S = pick(S02, S13, s), T = pick(T02, T13, s), U = pick(U02, U13, s);
      const uint32_t w = q[s], t = w >> 8;
      b[s] = pack8(as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mlo, k.mag_hi)), S, T)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mhi, k.mag_lo)), S, U)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mlo, k.mag_hi)), S, T)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mhi, k.mag_lo)), S, U)));
    }
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
    const half2_t dm = as_h2(r.hdr.x);
    uint32_t sc, mn;
    kscales<H>(r.hdr, sc, mn);
    half2_t S02, S13, M02, M13;
    bytes4_to_h2(sc, h2lo(dm), S02, S13);
    bytes4_to_h2(mn, -h2hi(dm), M02, M13);
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const Consts k = make_consts();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half2_t S = pick(S02, S13, s), M = pick(M02, M13, s);
      const uint32_t w = q[s], t = w >> 8;
      b[s] = pack8(as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mlo, k.mag_hi)) - h2c(1024.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mhi, k.mag_lo)) - h2c(64.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mlo, k.mag_hi)) - h2c(1024.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mhi, k.mag_lo)) - h2c(64.f), S, M)));
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
    uint32_t sc, mn;
    kscales<H>(r.hdr, sc, mn);
    half2_t S02, S13, M02, M13;
    bytes4_to_h2(sc, h2lo(dm), S02, S13);
    bytes4_to_h2(mn, -h2hi(dm), M02, M13);
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const uint32_t qh = H == 0 ? r.qh0 : r.qh1;
    const Consts k = make_consts();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half2_t S = pick(S02, S13, s), M = pick(M02, M13, s);
      const uint32_t w = q[s], t = w >> 8;
      const uint32_t hb = (qh >> (8 * s)) & 0xFFu;
      const uint32_t x = hb | (hb << 12);   // (x >> i): hi(2i) at bit 0, hi(2i+1) at bit 16
      // +16: bit 4/20 in the 1024-exponent words, bit 8/24 in the 64-exponent words
      const uint32_t h0 = ((x << 4) & 0x00100010u) | k.mag_hi, h1 = ((x << 7) & 0x01000100u) | k.mag_lo;
      const uint32_t h2 = ((x << 2) & 0x00100010u) | k.mag_hi, h3 = ((x << 5) & 0x01000100u) | k.mag_lo;
      b[s] = pack8(as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mlo, h0)) - h2c(1024.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mhi, h1)) - h2c(64.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mlo, h2)) - h2c(1024.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mhi, h3)) - h2c(64.f), S, M)));
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
    const f16 dh = __builtin_bit_cast(f16, (uint16_t)r.d);
    const float d = (float)dh;
    const int gb = (lane >> 5) & 1;          // (g >> 1)
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const u32x2 qh = H == 0 ? r.qh0 : r.qh1;
    const Consts k = make_consts();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // sub-block (16 weights) = 8H + 2s + gb -> dword 2H + (s>>1), byte 2(s&1) + gb
      const uint32_t scw = r.sc[2 * H + (s >> 1)];
      const int scv = (int)(int8_t)((scw >> (8 * (2 * (s & 1) + gb))) & 0xFF);
      const half2_t S = h2splat(d * (float)scv);
      const uint32_t w = q[s], t = w >> 8;
      const uint32_t h16 = (qh[s >> 1] >> (16 * (s & 1))) & 0xFFFFu;
      const uint32_t e = h16 | (h16 << 8);   // (e >> 2i): hi(2i) at bits 0-1, hi(2i+1) at 16-17
      const uint32_t h0 = ((e << 4) & 0x00300030u) | k.mag_hi, h1 = ((e << 6) & 0x03000300u) | k.mag_lo;
      const uint32_t h2 = (e & 0x00300030u) | k.mag_hi, h3 = ((e << 2) & 0x03000300u) | k.mag_lo;
      b[s] = pack8(as_u32((as_h2(and_or(w, k.mlo, h0)) - h2c(1056.f)) * S),   // 1024 + 32 zero point
                   as_u32((as_h2(and_or(w, k.mhi, h1)) - h2c(96.f)) * S),     // 64 + 32
                   as_u32((as_h2(and_or(t, k.mlo, h2)) - h2c(1056.f)) * S),
                   as_u32((as_h2(and_or(t, k.mhi, h3)) - h2c(96.f)) * S));
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
    const half2_t off = h2c(1152.f);   // 1024 magic + 128 (bytes stored q+128)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int blk = 4 * H + s;
      const half2_t dd = as_h2(r.dd[blk >> 1]);
      const half2_t S = (blk & 1) ? h2hi(dd) : h2lo(dd);
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
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const Consts k = make_consts();
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int blk = 4 * H + s;
      const half2_t dd = as_h2(r.dd[blk >> 1]);
      const half2_t S = (blk & 1) ? h2hi(dd) : h2lo(dd);
      const uint32_t w = q[s], t = w >> 8;
      b[s] = pack8(as_u32((as_h2(and_or(w, k.mlo, k.mag_hi)) - h2c(1032.f)) * S),   // 1024 + 8
                   as_u32((as_h2(and_or(w, k.mhi, k.mag_lo)) - h2c(72.f)) * S),     // 64 + 8
                   as_u32((as_h2(and_or(t, k.mlo, k.mag_hi)) - h2c(1032.f)) * S),
                   as_u32((as_h2(and_or(t, k.mhi, k.mag_lo)) - h2c(72.f)) * S));
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
