// Per-packed-type register dequantizers for the T16 layout (see csrc/runtime/qtypes.h).
//
// k-mapping.  For one (16-row tile, 256-k super-block) chunk, lane l = 16g + r holds row r, and
// MFMA i = 4h + s (h = 0..1, s = 0..3) of the super-block covers, for lane group g, element j:
//     k = 64 g + 32 h + 8 s + j  =  t16_xoff(g, i) + j
// so lane group g owns the 64-wide quarter [64g, 64g + 64): the 32-wide sub-blocks 2g (h = 0) and
// 2g + 1 (h = 1) of Q4_K/Q5_K (whose nibbles share the same GGUF bytes), the blocks 2g, 2g+1 of
// Q8_0/Q4_0 and the 16-wide sub-blocks 4g..4g+3 of Q6_K.  Each lane therefore decodes only the
// scales of its own quarter (a quarter of the work of a k = 128h + 32s + 8g + j mapping, measured
// 7-16 us of a 58-72 us 70B gate/up GEMV: profiles/r1d_gemv_cost_probes.txt).  `dequant<h>` gives
// the four B fragments b[s] (MFMA i = 4h + s): b[s][j] = W[row r][k(g, h, s, j)]; the A (x)
// fragment of MFMA i for lane (g, m) is x[m][t16_xoff(g, i) + j].
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

__device__ __forceinline__ constexpr int t16_xoff(int g, int i) { return 64 * g + 8 * i; }
// LDS x tiles (16 B-chunked rows of 256 k, padded to 264 f16): the k-quarters of rows 8..15 (mod 16)
// are stored swapped in pairs so that an A-fragment ds_read_b128 is bank-conflict free (gemv2.hip)
__device__ __forceinline__ constexpr int x_qswap(int row) { return ((row >> 3) & 1) << 6; }

__device__ __forceinline__ half2_t h2lo(half2_t v) { return half2_t{v.x, v.x}; }
__device__ __forceinline__ half2_t h2hi(half2_t v) { return half2_t{v.y, v.y}; }
__device__ __forceinline__ half2_t h2splat(float v) { f16 h = (f16)v; return half2_t{h, h}; }
__device__ __forceinline__ half2_t h2c(float v) { return half2_t{(f16)v, (f16)v}; }

// Weight sources for Deq<PT>::load (offsets in bytes from the chunk start).
//   PtrSrc: flat global loads.
//   BufSrc: raw buffer loads through a wave-uniform descriptor over [base, base + num_records):
//           a load past the range returns zeros WITHOUT touching memory, so a fixed-depth
//           prefetch ring can run past the end of a wave's super-block range at no HBM cost
//           (the loads stay unconditional: path-independent vmcnt).
struct PtrSrc {
  const uint8_t* p;
  __device__ __forceinline__ u32x4 q16nt(int o) const { return ld16_nt(p + o); }
  __device__ __forceinline__ u32x4 q16(int o) const { return ld16(p + o); }
  __device__ __forceinline__ uint32_t q4nt(int o) const { return __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p + o)); }
  __device__ __forceinline__ uint32_t q4(int o) const { return *reinterpret_cast<const uint32_t*>(p + o); }
  __device__ __forceinline__ u32x2 q8nt(int o) const { return __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p + o)); }
  __device__ __forceinline__ uint32_t q2(int o) const { return *reinterpret_cast<const uint16_t*>(p + o); }
};
struct BufSrc {
  __amdgpu_buffer_rsrc_t r;
  int base;   // chunk offset within the descriptor's range
  __device__ __forceinline__ u32x4 q16nt(int o) const { return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, base + o, 0, 2)); }
  __device__ __forceinline__ u32x4 q16(int o) const { return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, base + o, 0, 0)); }
  __device__ __forceinline__ uint32_t q4nt(int o) const { return __builtin_amdgcn_raw_buffer_load_b32(r, base + o, 0, 2); }
  __device__ __forceinline__ uint32_t q4(int o) const { return __builtin_amdgcn_raw_buffer_load_b32(r, base + o, 0, 0); }
  __device__ __forceinline__ u32x2 q8nt(int o) const { return __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(r, base + o, 0, 2)); }
  __device__ __forceinline__ uint32_t q2(int o) const { return __builtin_amdgcn_raw_buffer_load_b16(r, base + o, 0, 0); }
};
//   LdsSrc: a chunk already copied to LDS (the fused attention + o-projection kernel)
struct LdsSrc {
  const uint8_t* p;
  __device__ __forceinline__ u32x4 q16nt(int o) const { return *reinterpret_cast<const u32x4*>(p + o); }
  __device__ __forceinline__ u32x4 q16(int o) const { return *reinterpret_cast<const u32x4*>(p + o); }
  __device__ __forceinline__ uint32_t q4nt(int o) const { return *reinterpret_cast<const uint32_t*>(p + o); }
  __device__ __forceinline__ uint32_t q4(int o) const { return *reinterpret_cast<const uint32_t*>(p + o); }
  __device__ __forceinline__ u32x2 q8nt(int o) const { return *reinterpret_cast<const u32x2*>(p + o); }
  __device__ __forceinline__ uint32_t q2(int o) const { return *reinterpret_cast<const uint16_t*>(p + o); }
};
// gfx9 raw-buffer descriptor word 3 (DATA_FORMAT 32, no swizzle)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}

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
// plain C (the compiler emits v_and_or_b32 with the VGPR-resident masks and sees its hazards:
// the inline-asm form cost an s_nop after most of them and re-materialised the masks per call)
__device__ __forceinline__ uint32_t and_or(uint32_t a, uint32_t m, uint32_t c) { return (a & m) | c; }

// Q4_K / Q5_K super-block header as packed (csrc/runtime/pack.cpp): dword 0 = (d, dmin) f16, then
// 12 bytes holding, for each lane group g, the 24-bit word
//     v_g = sc(2g) | m(2g) << 6 | sc(2g+1) << 12 | m(2g+1) << 18      (6-bit GGUF scales/mins)
// with byte b of v_g at header byte 4 + 4b + g.  Returns (d sc(2g), d sc(2g+1)) and
// (-dmin m(2g), -dmin m(2g+1)) as f16 pairs, each rounded once (same values as GGUF math in f16).
__device__ __forceinline__ void kquarter_scales(const u32x4& hdr, int lane, half2_t& S, half2_t& M) {
  const uint32_t g = (uint32_t)lane >> 4;
  const uint32_t lo = __builtin_amdgcn_perm(hdr.z, hdr.y, g | ((g + 4) << 8) | 0x0C0C0000u);
  const uint32_t v = __builtin_amdgcn_perm(hdr.w, lo, 0x0C000100u | ((g + 4) << 16));
  const uint32_t a = ((v << 4) & 0x003F0000u) | (v & 0x3Fu) | 0x64006400u;           // 1024 + sc
  const uint32_t b = ((v >> 2) & 0x003F0000u) | ((v >> 6) & 0x3Fu) | 0x64006400u;    // 1024 + m
  const half2_t dm = as_h2(hdr.x);
  const half2_t d2 = h2lo(dm), n2 = -h2hi(dm);
  S = __builtin_elementwise_fma(as_h2(a), d2, d2 * h2c(-1024.f));   // -1024 d exact (power of two)
  M = __builtin_elementwise_fma(as_h2(b), n2, n2 * h2c(-1024.f));
}

// ------------------------------------------------------------------ Q4_K (144 B / 256 w)
template <> struct Deq<P_Q4_K> {
  static constexpr int CB = chunk_bytes(P_Q4_K);
  struct Raw { u32x4 q0, q1, hdr; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) { load(r, PtrSrc{c}, lane); }
  template <class S>
  __device__ static __forceinline__ void load(Raw& r, const S& c, int lane) {
    r.q0 = c.q16nt(lane * 16);
    r.q1 = c.q16nt(1024 + lane * 16);
    r.hdr = c.q16(2048 + (lane & 15) * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) { dequant<H>(r, b, lane, make_consts()); }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane, const Consts& k) {
    half2_t S2, M2;
    kquarter_scales(r.hdr, lane, S2, M2);   // shared by H = 0 / 1 (CSE)
    const half2_t S = H ? h2hi(S2) : h2lo(S2), M = H ? h2hi(M2) : h2lo(M2);
    const u32x4 q = H == 0 ? r.q0 : r.q1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
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
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) { load(r, PtrSrc{c}, lane); }
  template <class S>
  __device__ static __forceinline__ void load(Raw& r, const S& c, int lane) {
    r.q0 = c.q16nt(lane * 16);
    r.q1 = c.q16nt(1024 + lane * 16);
    r.qh0 = c.q4nt(2048 + lane * 4);
    r.qh1 = c.q4nt(2048 + 256 + lane * 4);
    r.hdr = c.q16(2560 + (lane & 15) * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) { dequant<H>(r, b, lane, make_consts()); }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane, const Consts& k) {
    half2_t S2, M2;
    kquarter_scales(r.hdr, lane, S2, M2);
    const half2_t S = H ? h2hi(S2) : h2lo(S2), M = H ? h2hi(M2) : h2lo(M2);
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const uint32_t qh = H == 0 ? r.qh0 : r.qh1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
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
  struct Raw { u32x4 q0, q1; u32x2 qh0, qh1; uint32_t sc, d; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) { load(r, PtrSrc{c}, lane); }
  template <class S>
  __device__ static __forceinline__ void load(Raw& r, const S& c, int lane) {
    r.q0 = c.q16nt(lane * 16);
    r.q1 = c.q16nt(1024 + lane * 16);
    r.qh0 = c.q8nt(2048 + lane * 8);
    r.qh1 = c.q8nt(2048 + 512 + lane * 8);
    // int8 scales of this lane's 16-wide sub-blocks 4g..4g+3: dword g of the row's 16 scales
    r.sc = c.q4(3072 + (lane & 15) * 16 + 4 * (lane >> 4));
    r.d = c.q2(3328 + (lane & 15) * 2);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) { dequant<H>(r, b, lane, make_consts()); }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane, const Consts& k) {
    const f16 dh = __builtin_bit_cast(f16, (uint16_t)r.d);
    // sub-block of MFMA (H, s) = 4g + 2H + (s >> 1): bytes 2H, 2H+1 of r.sc; int8 -> f16 by the
    // exponent magic on (byte ^ 0x80) = sc + 128, minus 1152 (exact), times d (one rounding)
    const uint32_t u = r.sc ^ 0x80808080u;
    const half2_t S2 = (as_h2(__builtin_amdgcn_perm(0x64646464u, u, H ? 0x04030402u : 0x04010400u)) - h2c(1152.f)) *
                       half2_t{dh, dh};
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const u32x2 qh = H == 0 ? r.qh0 : r.qh1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const half2_t S = (s >> 1) ? h2hi(S2) : h2lo(S2);
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
  struct Raw { u32x4 a0, a1, b0, b1; uint32_t dd; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) { load(r, PtrSrc{c}, lane); }
  template <class S>
  __device__ static __forceinline__ void load(Raw& r, const S& c, int lane) {
    r.a0 = c.q16nt(lane * 32);
    r.a1 = c.q16nt(lane * 32 + 16);
    r.b0 = c.q16nt(2048 + lane * 32);
    r.b1 = c.q16nt(2048 + lane * 32 + 16);
    r.dd = c.q4(4096 + (lane & 15) * 16 + 4 * (lane >> 4));   // d(2g), d(2g+1)
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane, const Consts&) { dequant<H>(r, b, lane); }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
    const half2_t off = h2c(1152.f);   // 1024 magic + 128 (bytes stored q+128)
    const half2_t S = H ? h2hi(as_h2(r.dd)) : h2lo(as_h2(r.dd));   // block 2g + H
#pragma unroll
    for (int s = 0; s < 4; ++s) {
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
  struct Raw { u32x4 q0, q1; uint32_t dd; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) { load(r, PtrSrc{c}, lane); }
  template <class S>
  __device__ static __forceinline__ void load(Raw& r, const S& c, int lane) {
    r.q0 = c.q16nt(lane * 16);
    r.q1 = c.q16nt(1024 + lane * 16);
    r.dd = c.q4(2048 + (lane & 15) * 16 + 4 * (lane >> 4));   // d(2g), d(2g+1)
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) { dequant<H>(r, b, lane, make_consts()); }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane, const Consts& k) {
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const half2_t S = H ? h2hi(as_h2(r.dd)) : h2lo(as_h2(r.dd));   // block 2g + H
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t w = q[s], t = w >> 8;
      b[s] = pack8(as_u32((as_h2(and_or(w, k.mlo, k.mag_hi)) - h2c(1032.f)) * S),   // 1024 + 8
                   as_u32((as_h2(and_or(w, k.mhi, k.mag_lo)) - h2c(72.f)) * S),     // 64 + 8
                   as_u32((as_h2(and_or(t, k.mlo, k.mag_hi)) - h2c(1032.f)) * S),
                   as_u32((as_h2(and_or(t, k.mhi, k.mag_lo)) - h2c(72.f)) * S));
    }
  }
};

// bf16 pair (low, high halves of w) -> f16 pair (dense unpack only: the GEMV/GEMM kernels keep bf16):
// exact inside f16's normal range; v_cvt_pkrtz rounds toward zero, so a bf16 beyond 65504 becomes
// +-65504 (saturation) instead of an infinity
__device__ __forceinline__ uint32_t bf2_to_h2(uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)));
}
__device__ __forceinline__ half8_t bf8_to_h8(const u32x4& v) {
  return pack8(bf2_to_h2(v.x), bf2_to_h2(v.y), bf2_to_h2(v.z), bf2_to_h2(v.w));
}

// ------------------------------------------------------------------ F16 (plain)
template <> struct Deq<P_F16> {
  static constexpr int CB = chunk_bytes(P_F16);
  struct Raw { u32x4 v[8]; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) { load(r, PtrSrc{c}, lane); }
  template <class S>
  __device__ static __forceinline__ void load(Raw& r, const S& c, int lane) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = c.q16nt(i * 1024 + lane * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane, const Consts&) { dequant<H>(r, b, lane); }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
#pragma unroll
    for (int s = 0; s < 4; ++s) b[s] = __builtin_bit_cast(half8_t, r.v[4 * H + s]);
  }
};

// ------------------------------------------------------------------ BF16 (F16 layout, bf16 bits)
template <> struct Deq<P_BF16> {
  static constexpr int CB = chunk_bytes(P_BF16);
  struct Raw { u32x4 v[8]; };
  __device__ static __forceinline__ void load(Raw& r, const uint8_t* c, int lane) { load(r, PtrSrc{c}, lane); }
  template <class S>
  __device__ static __forceinline__ void load(Raw& r, const S& c, int lane) {
#pragma unroll
    for (int i = 0; i < 8; ++i) r.v[i] = c.q16nt(i * 1024 + lane * 16);
  }
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane, const Consts&) { dequant<H>(r, b, lane); }
  // the bf16 bits themselves: every consumer runs mma<true> on them (kcommon.h)
  template <int H>
  __device__ static __forceinline__ void dequant(const Raw& r, half8_t b[4], int lane) {
#pragma unroll
    for (int s = 0; s < 4; ++s) b[s] = __builtin_bit_cast(half8_t, r.v[4 * H + s]);
  }
};

// ------------------------------------------------------------------ single-row dot forms (gemvs M = 1)
// For ONE activation row the MFMA path wastes 15 of its 16 rows, and the dequant dominates the
// kernel's VALU (profiles/r11d_gemvs_probe.txt: dequant + MFMA 1.2-4 us of a 5.7-16.7 us GEMV).
// Here the exponent-magic pairs are used BIASED, straight as v_dot2_f32_f16 operands: a Q4_K pair
// reads (1024 + q) or (64 + q) exactly, so sum (1024 + q_j) x_j = sum q_j x_j + 1024 sum x_j and the
// bias term -- the same for every output column -- comes out of a per-(super-block, lane group)
// table the workgroup builds once from its staged x (DotCorr).  Per 8 weights: one shift, 4
// v_and_or, 4 v_dot2 (the MFMA form: shift, 4 v_and_or, 4 v_pk_add, 4 v_pk_fma, 2 MFMA); the scale
// and min are applied once per sub-block in f32, and q enters the dot unrounded (the MFMA form
// rounds each weight q S + M to f16).
//   xq: the lane group's x of the super-block in LDS (fragment i = 4h + s at xq + 8 i: t16_xoff),
//       read just before use (8 fragments held at once cost 32 VGPRs: occupancy 6 -> 4, r11f)
//   c: the lane group's 4 correction floats (DotCorr<PT>::make)
template <int PT> struct DotCorr;   // per (super-block, lane group g): 4 floats from that quarter's 64 x
// a[i] = x_j0 + x_j1 + x_j4 + x_j5, b[i] = x_j2 + x_j3 + x_j6 + x_j7 of fragment i (the positions the
// 1024- and 64-exponent magic words carry)
template <> struct DotCorr<P_Q4_K> {   // (C_h0, C_h1, X_h0, X_h1): C = 1024 a + 64 b over the half, X = sum x
  __device__ static __forceinline__ float4 make(const float (&a)[8], const float (&b)[8]) {
    float c[2] = {0.f, 0.f}, x[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) { c[i >> 2] += 1024.f * a[i] + 64.f * b[i]; x[i >> 2] += a[i] + b[i]; }
    return make_float4(c[0], c[1], x[0], x[1]);
  }
};
template <> struct DotCorr<P_Q5_K> : DotCorr<P_Q4_K> {};
template <> struct DotCorr<P_Q6_K> {   // C per 16-wide sub-block (h, s >> 1): 1056 a + 96 b (zero point 32)
  __device__ static __forceinline__ float4 make(const float (&a)[8], const float (&b)[8]) {
    float c[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i >> 1] += 1056.f * a[i] + 96.f * b[i];
    return make_float4(c[0], c[1], c[2], c[3]);
  }
};
template <> struct DotCorr<P_Q8_0> {   // C per 32-block h: 1152 (a + b) (bytes stored q + 128)
  __device__ static __forceinline__ float4 make(const float (&a)[8], const float (&b)[8]) {
    float c[2] = {0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i >> 2] += 1152.f * (a[i] + b[i]);
    return make_float4(c[0], c[1], 0.f, 0.f);
  }
};
template <int PT> constexpr bool dot1_supported() {
  return PT == P_Q4_K || PT == P_Q5_K || PT == P_Q6_K || PT == P_Q8_0;
}

__device__ __forceinline__ float d2(uint32_t w, uint32_t x, float acc) {
  return __builtin_amdgcn_fdot2(as_h2(w), as_h2(x), acc, false);
}

// sum over the lane's 64 weights of W x for one super-block (Q4_K / Q5_K)
__device__ __forceinline__ u32x4 xfrag(const f16* xq, int i) { return *reinterpret_cast<const u32x4*>(xq + 8 * i); }

template <bool Q5, class Raw>
__device__ __forceinline__ float dot1_q45k(const Raw& r, const f16* xq, const float4 c, int lane, const Consts& k) {
  half2_t S2, M2;
  kquarter_scales(r.hdr, lane, S2, M2);
  float acc[2] = {0.f, 0.f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const u32x4 q = h == 0 ? r.q0 : r.q1;
    uint32_t qh = 0;
    if constexpr (Q5) qh = h == 0 ? r.qh0 : r.qh1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t w = q[s], t = w >> 8;
      uint32_t h0 = k.mag_hi, h1 = k.mag_lo, h2 = k.mag_hi, h3 = k.mag_lo;
      if constexpr (Q5) {
        const uint32_t hb = (qh >> (8 * s)) & 0xFFu;
        const uint32_t xx = hb | (hb << 12);
        h0 = ((xx << 4) & 0x00100010u) | k.mag_hi; h1 = ((xx << 7) & 0x01000100u) | k.mag_lo;
        h2 = ((xx << 2) & 0x00100010u) | k.mag_hi; h3 = ((xx << 5) & 0x01000100u) | k.mag_lo;
      }
      const u32x4 xv = xfrag(xq, 4 * h + s);
      float a = acc[h];
      a = d2(and_or(w, k.mlo, h0), xv.x, a);
      a = d2(and_or(w, k.mhi, h1), xv.y, a);
      a = d2(and_or(t, k.mlo, h2), xv.z, a);
      a = d2(and_or(t, k.mhi, h3), xv.w, a);
      acc[h] = a;
    }
  }
  return (float)S2.x * (acc[0] - c.x) + (float)M2.x * c.z + (float)S2.y * (acc[1] - c.y) + (float)M2.y * c.w;
}

template <class Raw>
__device__ __forceinline__ float dot1_q6k(const Raw& r, const f16* xq, const float4 c, int lane, const Consts& k) {
  const float dh = (float)__builtin_bit_cast(f16, (uint16_t)r.d);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int H = 0; H < 2; ++H) {
    const u32x4 q = H == 0 ? r.q0 : r.q1;
    const u32x2 qh = H == 0 ? r.qh0 : r.qh1;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const uint32_t w = q[s], t = w >> 8;
      const uint32_t h16 = (qh[s >> 1] >> (16 * (s & 1))) & 0xFFFFu;
      const uint32_t e = h16 | (h16 << 8);
      const uint32_t h0 = ((e << 4) & 0x00300030u) | k.mag_hi, h1 = ((e << 6) & 0x03000300u) | k.mag_lo;
      const uint32_t h2 = (e & 0x00300030u) | k.mag_hi, h3 = ((e << 2) & 0x03000300u) | k.mag_lo;
      const u32x4 xv = xfrag(xq, 4 * H + s);
      float a = acc[2 * H + (s >> 1)];
      a = d2(and_or(w, k.mlo, h0), xv.x, a);
      a = d2(and_or(w, k.mhi, h1), xv.y, a);
      a = d2(and_or(t, k.mlo, h2), xv.z, a);
      a = d2(and_or(t, k.mhi, h3), xv.w, a);
      acc[2 * H + (s >> 1)] = a;
    }
  }
  // int8 scales of the lane's 16-wide sub-blocks 4g + 2H + (s >> 1): bytes 0..3 of r.sc
  const int32_t sc = (int32_t)r.sc;
  const float s0 = (float)(int8_t)(sc & 0xFF), s1 = (float)(int8_t)((sc >> 8) & 0xFF);
  const float s2 = (float)(int8_t)((sc >> 16) & 0xFF), s3 = (float)(int8_t)(sc >> 24);
  return dh * (s0 * (acc[0] - c.x) + s1 * (acc[1] - c.y) + s2 * (acc[2] - c.z) + s3 * (acc[3] - c.w));
}

template <class Raw>
__device__ __forceinline__ float dot1_q80(const Raw& r, const f16* xq, const float4 c, int lane) {
  const half2_t S = as_h2(r.dd);   // d(2g), d(2g + 1)
  float acc[2] = {0.f, 0.f};
#pragma unroll
  for (int H = 0; H < 2; ++H) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const u32x4 src = H == 0 ? (s < 2 ? r.a0 : r.a1) : (s < 2 ? r.b0 : r.b1);
      const uint32_t lo = src[2 * (s & 1)], hi = src[2 * (s & 1) + 1];
      const u32x4 xv = xfrag(xq, 4 * H + s);
      float a = acc[H];
      a = d2(__builtin_amdgcn_perm(0x64646464u, lo, 0x04010400u), xv.x, a);
      a = d2(__builtin_amdgcn_perm(0x64646464u, lo, 0x04030402u), xv.y, a);
      a = d2(__builtin_amdgcn_perm(0x64646464u, hi, 0x04010400u), xv.z, a);
      a = d2(__builtin_amdgcn_perm(0x64646464u, hi, 0x04030402u), xv.w, a);
      acc[H] = a;
    }
  }
  return (float)S.x * (acc[0] - c.x) + (float)S.y * (acc[1] - c.y);
}

template <int PT, class Raw>
__device__ __forceinline__ float dot1(const Raw& r, const f16* xq, const float4 c, int lane, const Consts& k) {
  if constexpr (PT == P_Q4_K) return dot1_q45k<false>(r, xq, c, lane, k);
  else if constexpr (PT == P_Q5_K) return dot1_q45k<true>(r, xq, c, lane, k);
  else if constexpr (PT == P_Q6_K) return dot1_q6k(r, xq, c, lane, k);
  else return dot1_q80(r, xq, c, lane);
}

}  // namespace mpk
