// Dequant GEMM v3 (M >= 128: wide decode micro-batches and prompt chunks).
//
// Y[M][N] (+)= X[M][K] W[N][K]^T with W in the T16 packed quant layout (csrc/runtime/qtypes.h).
// Workgroup tile BM x BN (BM 128 | 256 rows, BN 128 | 256 columns = 8 | 16 T16 tiles), 8 waves,
// K in stages of 64.  Unlike gemm2 (each wave dequantizes its own two 16-column tiles in registers,
// 3.5 VALU per MFMA at 2 waves/SIMD, 39 % MFMA busy: profiles/r5f_gemm2_m256_pmc.txt), every weight
// element is dequantized ONCE per workgroup, into an f16 LDS image that all waves read:
//
//   stage s (64 k):  X rows  --global_load_lds-->  A[s&1]  (f16, [BM][64], swizzled)
//                    W quant --global_load_lds-->  R[s&1]  (raw bytes of the stage, per-type image)
//                    R  --ds_read, VALU dequant, ds_write-->  B[s&1]  (f16, [BN][64], swizzled)
//
// Iteration s: issue the loads of A(s+1) and R(s+2), run the 2 FM FN MFMAs per wave of stage s
// from A(s&1)/B(s&1) (v_mfma_f32_16x16x32_f16, wave tile 16FM x 16FN, accumulators in registers),
// and dequantize R(s+1) into B((s+1)&1) (VALU).  The dequant of a stage and the MFMAs of the
// previous one are independent, so the two pipes overlap inside every wave; one barrier per stage.
//
// LDS images: rows (A) / columns (B) of 128 B = 8 chunks of 16 B (8 consecutive k); chunk c of row
// r sits at chunk c ^ ((r >> 1) & 7), which makes every ds_read_b128 of an MFMA operand (16 rows x
// 8 chunk groups) bank-conflict free.  global_load_lds writes lane-linear, so the swizzle is applied
// to the per-lane SOURCE address (cdna_hip_programming.md rule 21).  Dequant threads own column
// perm(r) = ((r & 7) << 1) | (r >> 3) of their tile so that each 8-lane ds_write_b128 group hits 8
// distinct chunks.
//
// Workgroups are mapped XCD-aware (blocks b, b + 8, ... share an XCD; consecutive logical ids =
// the row blocks of one column group, whose weight reads after the first then hit that XCD's L2).
// EPI_ATOMIC splits the stage range over blockIdx.y.
#include "kcommon.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"
#include "../runtime/tuning.h"

#include <algorithm>

namespace mpk {
using namespace mp;

typedef __attribute__((address_space(3))) void lds_t;

__device__ __forceinline__ int g3_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int g3_off(int row, int c) { return row * 128 + ((c ^ g3_swz(row)) << 4); }
__device__ __forceinline__ int g3_perm(int r) { return ((r & 7) << 1) | (r >> 3); }

// global -> LDS DMA of SZ (16 | 4) bytes per lane (LDS destination: wave-uniform base + lane * SZ;
// the sub-dword forms are not used: they land a dword per lane); the size must be a literal
template <int SZ>
__device__ __forceinline__ void glds(const void* g, char* lds) {
  static_assert(SZ == 16 || SZ == 4, "glds: 16 or 4 bytes per lane");
  if constexpr (SZ == 16) __builtin_amdgcn_global_load_lds(g, (lds_t*)lds, 16, 0, 0);
  else __builtin_amdgcn_global_load_lds(g, (lds_t*)lds, 4, 0, 0);
}

// Q4_K / Q5_K scale words of quarter g (= stage q of the super-block): (d sc(2g), d sc(2g+1)),
// (-dmin m(2g), -dmin m(2g+1)) as f16 pairs (dequant.h kquarter_scales with an explicit quarter)
__device__ __forceinline__ void kq_scales(const u32x4& hdr, uint32_t g, half2_t& S, half2_t& M) {
  const uint32_t lo = __builtin_amdgcn_perm(hdr.z, hdr.y, g | ((g + 4) << 8) | 0x0C0C0000u);
  const uint32_t v = __builtin_amdgcn_perm(hdr.w, lo, 0x0C000100u | ((g + 4) << 16));
  const uint32_t a = ((v << 4) & 0x003F0000u) | (v & 0x3Fu) | 0x64006400u;
  const uint32_t b = ((v >> 2) & 0x003F0000u) | ((v >> 6) & 0x3Fu) | 0x64006400u;
  const half2_t dm = as_h2(hdr.x);
  const half2_t d2 = h2lo(dm), n2 = -h2hi(dm);
  S = __builtin_elementwise_fma(as_h2(a), d2, d2 * h2c(-1024.f));
  M = __builtin_elementwise_fma(as_h2(b), n2, n2 * h2c(-1024.f));
}

// word j of the dwords [part * NS, part * NS + NS) of v (part wave-uniform)
template <int NS>
__device__ __forceinline__ uint32_t g3_word(const u32x4& v, int part, int j) {
  if constexpr (NS == 4) return v[j];
  else return part ? v[2 + j] : v[j];
}

// ---------------------------------------------------------------------------------------------
// Per-type raw stage image + dequant.  A stage of NT T16 tiles covers, per tile, quarter q of one
// super-block.  Dequant entry e (< 32 NT): h = e / (16 NT) (k half of the quarter: wave-uniform),
// tile T = (e >> 4) % NT, column perm(e & 15); dequant<NS> produces its 8-k chunks part * NS + j,
// j < NS (NS = 4: one thread per entry; NS = 2: two, part wave-uniform).  Segments are filled by 1-KB wave pieces
// (64 lanes x 16 B, or 64 x 4 B for the small fields), entry i of a segment at i * ES.
template <int PT> struct G3;
// how a stage's weights reach the f16 B image:
//   G3_RAW_LDS: raw quant bytes by global_load_lds into R, dequantized LDS -> VALU -> LDS
//   G3_DIRECT:  the packed f16 bytes by global_load_lds straight into B (16-bit f16 weights)
//   G3_REG:     16-B loads into registers one stage ahead, converted and written (bf16 weights:
//               their raw bytes are as large as the f16 image, too big for an LDS raw buffer)
enum { G3_RAW_LDS = 0, G3_DIRECT = 1, G3_REG = 2 };

struct G3Ctx {           // per-stage source addressing (wave-uniform)
  const uint8_t* W;      // packed matrix
  int t0, ntiles, nsb, sb, q;
  __device__ __forceinline__ const uint8_t* chunk(int T, int CB) const {
    const int t = min(t0 + T, ntiles - 1);
    return W + ((size_t)t * nsb + sb) * CB;
  }
};

// issue the global_load_lds pieces of one segment: n entries of ES bytes, pieces of 64 entries
// dealt round-robin over the 8 waves; src(i) = source of entry i
template <int ES, class F>
__device__ __forceinline__ void g3_segment(char* dst, int n, int wave, int lane, F src) {
  const int pieces = n / 64;
  for (int pc = wave; pc < pieces; pc += 8) glds<ES>(src(pc * 64 + lane), dst + pc * 64 * ES);
}

template <> struct G3<P_Q4_K> {
  static constexpr int CB = chunk_bytes(P_Q4_K);
  static constexpr int MODE = G3_RAW_LDS;
  static constexpr int raw_bytes(int NT) { return NT * 512 + NT * 256; }
  __device__ static __forceinline__ void issue(char* R, const G3Ctx& c, int NT, int wave, int lane) {
    g3_segment<16>(R, 32 * NT, wave, lane, [&](int i) {
      const int h = i / (16 * NT), T = (i >> 4) % NT, r = g3_perm(i & 15);
      return c.chunk(T, CB) + h * 1024 + (16 * c.q + r) * 16;
    });
    g3_segment<16>(R + NT * 512, 16 * NT, wave, lane, [&](int i) { return c.chunk(i >> 4, CB) + 2048 + (i & 15) * 16; });
  }
  template <int NS>
  __device__ static __forceinline__ void dequant(const char* R, int NT, int e, int part, int q, const Consts& k, half8_t* b) {
    const int h = e / (16 * NT), T = (e >> 4) % NT, r = g3_perm(e & 15);
    const u32x4 w4 = *reinterpret_cast<const u32x4*>(R + e * 16);
    const u32x4 hdr = *reinterpret_cast<const u32x4*>(R + NT * 512 + (T * 16 + r) * 16);
    half2_t S2, M2;
    kq_scales(hdr, (uint32_t)q, S2, M2);
    const half2_t S = h ? h2hi(S2) : h2lo(S2), M = h ? h2hi(M2) : h2lo(M2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint32_t w = g3_word<NS>(w4, part, s), t = w >> 8;
      b[s] = pack8(as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mlo, k.mag_hi)) - h2c(1024.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mhi, k.mag_lo)) - h2c(64.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mlo, k.mag_hi)) - h2c(1024.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mhi, k.mag_lo)) - h2c(64.f), S, M)));
    }
  }
};

template <> struct G3<P_Q5_K> {
  static constexpr int CB = chunk_bytes(P_Q5_K);
  static constexpr int MODE = G3_RAW_LDS;
  static constexpr int raw_bytes(int NT) { return NT * 512 + NT * 128 + NT * 256; }
  __device__ static __forceinline__ void issue(char* R, const G3Ctx& c, int NT, int wave, int lane) {
    g3_segment<16>(R, 32 * NT, wave, lane, [&](int i) {
      const int h = i / (16 * NT), T = (i >> 4) % NT, r = g3_perm(i & 15);
      return c.chunk(T, CB) + h * 1024 + (16 * c.q + r) * 16;
    });
    g3_segment<4>(R + NT * 512, 32 * NT, wave, lane, [&](int i) {
      const int h = i / (16 * NT), T = (i >> 4) % NT, r = g3_perm(i & 15);
      return c.chunk(T, CB) + 2048 + h * 256 + (16 * c.q + r) * 4;
    });
    g3_segment<16>(R + NT * 640, 16 * NT, wave, lane, [&](int i) { return c.chunk(i >> 4, CB) + 2560 + (i & 15) * 16; });
  }
  template <int NS>
  __device__ static __forceinline__ void dequant(const char* R, int NT, int e, int part, int q, const Consts& k, half8_t* b) {
    const int h = e / (16 * NT), T = (e >> 4) % NT, r = g3_perm(e & 15);
    const u32x4 w4 = *reinterpret_cast<const u32x4*>(R + e * 16);
    const uint32_t qh = *reinterpret_cast<const uint32_t*>(R + NT * 512 + e * 4) >> (8 * NS * part);
    const u32x4 hdr = *reinterpret_cast<const u32x4*>(R + NT * 640 + (T * 16 + r) * 16);
    half2_t S2, M2;
    kq_scales(hdr, (uint32_t)q, S2, M2);
    const half2_t S = h ? h2hi(S2) : h2lo(S2), M = h ? h2hi(M2) : h2lo(M2);
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint32_t w = g3_word<NS>(w4, part, s), t = w >> 8;
      const uint32_t hb = (qh >> (8 * s)) & 0xFFu;
      const uint32_t x = hb | (hb << 12);
      const uint32_t h0 = ((x << 4) & 0x00100010u) | k.mag_hi, h1 = ((x << 7) & 0x01000100u) | k.mag_lo;
      const uint32_t h2 = ((x << 2) & 0x00100010u) | k.mag_hi, h3 = ((x << 5) & 0x01000100u) | k.mag_lo;
      b[s] = pack8(as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mlo, h0)) - h2c(1024.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mhi, h1)) - h2c(64.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mlo, h2)) - h2c(1024.f), S, M)),
                   as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mhi, h3)) - h2c(64.f), S, M)));
    }
  }
};

template <> struct G3<P_Q6_K> {
  static constexpr int CB = chunk_bytes(P_Q6_K);
  static constexpr int MODE = G3_RAW_LDS;
  // quants 16 B, high bits 8 B (two 4-B entries), int8 scales 4 B per row, and per row the dword
  // holding its f16 d (rows 2i, 2i+1 share one; the sub-dword LDS-DMA forms write a dword per lane)
  static constexpr int raw_bytes(int NT) { return NT * 512 + NT * 256 + NT * 64 + NT * 64; }
  __device__ static __forceinline__ void issue(char* R, const G3Ctx& c, int NT, int wave, int lane) {
    g3_segment<16>(R, 32 * NT, wave, lane, [&](int i) {
      const int h = i / (16 * NT), T = (i >> 4) % NT, r = g3_perm(i & 15);
      return c.chunk(T, CB) + h * 1024 + (16 * c.q + r) * 16;
    });
    g3_segment<4>(R + NT * 512, 64 * NT, wave, lane, [&](int i) {
      const int e = i >> 1, h = e / (16 * NT), T = (e >> 4) % NT, r = g3_perm(e & 15);
      return c.chunk(T, CB) + 2048 + h * 512 + (16 * c.q + r) * 8 + 4 * (i & 1);
    });
    g3_segment<4>(R + NT * 768, 16 * NT, wave, lane, [&](int i) { return c.chunk(i >> 4, CB) + 3072 + (i & 15) * 16 + 4 * c.q; });
    g3_segment<4>(R + NT * 832, 16 * NT, wave, lane, [&](int i) { return c.chunk(i >> 4, CB) + 3328 + ((i & 15) >> 1) * 4; });
  }
  template <int NS>
  __device__ static __forceinline__ void dequant(const char* R, int NT, int e, int part, int q, const Consts& k, half8_t* b) {
    const int h = e / (16 * NT), T = (e >> 4) % NT, r = g3_perm(e & 15);
    const u32x4 w4 = *reinterpret_cast<const u32x4*>(R + e * 16);
    const u32x2 qh = *reinterpret_cast<const u32x2*>(R + NT * 512 + e * 8);
    const uint32_t sc = *reinterpret_cast<const uint32_t*>(R + NT * 768 + (T * 16 + r) * 4);
    const uint32_t dw = *reinterpret_cast<const uint32_t*>(R + NT * 832 + (T * 16 + r) * 4);
    const uint16_t dd = (uint16_t)((r & 1) ? dw >> 16 : dw);
    const f16 dh = __builtin_bit_cast(f16, dd);
    const uint32_t u = sc ^ 0x80808080u;
    const half2_t S2 = (as_h2(__builtin_amdgcn_perm(0x64646464u, u, h ? 0x04030402u : 0x04010400u)) - h2c(1152.f)) *
                       half2_t{dh, dh};
#pragma unroll
    for (int j = 0; j < NS; ++j) {
      const int hi = NS == 4 ? (j >> 1) : part;   // sub-block (16 k) of chunk part * NS + j
      const half2_t S = hi ? h2hi(S2) : h2lo(S2);
      const uint32_t w = g3_word<NS>(w4, part, j), t = w >> 8;
      const uint32_t h16 = ((hi ? qh[1] : qh[0]) >> (16 * (j & 1))) & 0xFFFFu;
      const uint32_t x = h16 | (h16 << 8);
      const uint32_t h0 = ((x << 4) & 0x00300030u) | k.mag_hi, h1 = ((x << 6) & 0x03000300u) | k.mag_lo;
      const uint32_t h2 = (x & 0x00300030u) | k.mag_hi, h3 = ((x << 2) & 0x03000300u) | k.mag_lo;
      b[j] = pack8(as_u32((as_h2(and_or(w, k.mlo, h0)) - h2c(1056.f)) * S),
                   as_u32((as_h2(and_or(w, k.mhi, h1)) - h2c(96.f)) * S),
                   as_u32((as_h2(and_or(t, k.mlo, h2)) - h2c(1056.f)) * S),
                   as_u32((as_h2(and_or(t, k.mhi, h3)) - h2c(96.f)) * S));
    }
  }
};

template <> struct G3<P_Q8_0> {
  static constexpr int CB = chunk_bytes(P_Q8_0);
  static constexpr int MODE = G3_RAW_LDS;
  static constexpr int raw_bytes(int NT) { return NT * 1024 + NT * 64; }
  __device__ static __forceinline__ void issue(char* R, const G3Ctx& c, int NT, int wave, int lane) {
    g3_segment<16>(R, 64 * NT, wave, lane, [&](int i) {
      const int e = i >> 1, h = e / (16 * NT), T = (e >> 4) % NT, r = g3_perm(e & 15);
      return c.chunk(T, CB) + h * 2048 + (16 * c.q + r) * 32 + 16 * (i & 1);
    });
    g3_segment<4>(R + NT * 1024, 16 * NT, wave, lane, [&](int i) { return c.chunk(i >> 4, CB) + 4096 + (i & 15) * 16 + 4 * c.q; });
  }
  template <int NS>
  __device__ static __forceinline__ void dequant(const char* R, int NT, int e, int part, int q, const Consts&, half8_t* b) {
    const int h = e / (16 * NT), T = (e >> 4) % NT, r = g3_perm(e & 15);
    const u32x4 a0 = *reinterpret_cast<const u32x4*>(R + e * 32 + (NS == 4 ? 0 : 16 * part));
    const u32x4 a1 = NS == 4 ? *reinterpret_cast<const u32x4*>(R + e * 32 + 16) : a0;
    const uint32_t dd = *reinterpret_cast<const uint32_t*>(R + NT * 1024 + (T * 16 + r) * 4);
    const half2_t off = h2c(1152.f);
    const half2_t S = h ? h2hi(as_h2(dd)) : h2lo(as_h2(dd));
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const u32x4 src = s < 2 ? a0 : a1;
      const uint32_t lo = src[2 * (s & 1)], hi = src[2 * (s & 1) + 1];
      b[s] = pack8(as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, lo, 0x04010400u)) - off) * S),
                   as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, lo, 0x04030402u)) - off) * S),
                   as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, hi, 0x04010400u)) - off) * S),
                   as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, hi, 0x04030402u)) - off) * S));
    }
  }
};

template <> struct G3<P_Q4_0> {
  static constexpr int CB = chunk_bytes(P_Q4_0);
  static constexpr int MODE = G3_RAW_LDS;
  static constexpr int raw_bytes(int NT) { return NT * 512 + NT * 64; }
  __device__ static __forceinline__ void issue(char* R, const G3Ctx& c, int NT, int wave, int lane) {
    g3_segment<16>(R, 32 * NT, wave, lane, [&](int i) {
      const int h = i / (16 * NT), T = (i >> 4) % NT, r = g3_perm(i & 15);
      return c.chunk(T, CB) + h * 1024 + (16 * c.q + r) * 16;
    });
    g3_segment<4>(R + NT * 512, 16 * NT, wave, lane, [&](int i) { return c.chunk(i >> 4, CB) + 2048 + (i & 15) * 16 + 4 * c.q; });
  }
  template <int NS>
  __device__ static __forceinline__ void dequant(const char* R, int NT, int e, int part, int q, const Consts& k, half8_t* b) {
    const int h = e / (16 * NT), T = (e >> 4) % NT, r = g3_perm(e & 15);
    const u32x4 w4 = *reinterpret_cast<const u32x4*>(R + e * 16);
    const uint32_t dd = *reinterpret_cast<const uint32_t*>(R + NT * 512 + (T * 16 + r) * 4);
    const half2_t S = h ? h2hi(as_h2(dd)) : h2lo(as_h2(dd));
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint32_t w = g3_word<NS>(w4, part, s), t = w >> 8;
      b[s] = pack8(as_u32((as_h2(and_or(w, k.mlo, k.mag_hi)) - h2c(1032.f)) * S),
                   as_u32((as_h2(and_or(w, k.mhi, k.mag_lo)) - h2c(72.f)) * S),
                   as_u32((as_h2(and_or(t, k.mlo, k.mag_hi)) - h2c(1032.f)) * S),
                   as_u32((as_h2(and_or(t, k.mhi, k.mag_lo)) - h2c(72.f)) * S));
    }
  }
};

// 16-bit weights: the stage's B image is loaded directly (no raw image, no dequant)
template <> struct G3<P_F16> {
  static constexpr int CB = chunk_bytes(P_F16);
  static constexpr int MODE = G3_DIRECT;
  static constexpr int raw_bytes(int) { return 0; }
  // B image bytes [col][128 B]: piece of 1 KB = 8 columns; lane l -> column 8 pc + (l >> 3), image
  // chunk l & 7 = source chunk c ^ swz(col); source chunk c (k = 8c..8c+7 of the quarter) is packed
  // element i = c (4H + s) of lane (q, r) of the T16 chunk: byte c * 1024 + (16 q + r) * 16
  __device__ static __forceinline__ void issue_b(char* B, const G3Ctx& c, int NT, int wave, int lane) {
    for (int pc = wave; pc < 2 * NT; pc += 8) {
      const int col = 8 * pc + (lane >> 3);
      const int ch = (lane & 7) ^ g3_swz(col);
      glds<16>(c.chunk(col >> 4, CB) + ch * 1024 + (16 * c.q + (col & 15)) * 16, B + pc * 1024);
    }
  }
};

// bf16 weights (F16 chunk layout, bf16 bits): entry e's chunks 4h + part NS + j of the quarter
// (k = 8 c .. 8 c + 7 of column perm(r)) are element i = c of lane (q, r): byte c * 1024 + (16 q + r) * 16
template <> struct G3<P_BF16> {
  static constexpr int CB = chunk_bytes(P_BF16);
  static constexpr int MODE = G3_REG;
  static constexpr int raw_bytes(int) { return 0; }
  template <int NS>
  __device__ static __forceinline__ void load(const G3Ctx& c, int NT, int e, int part, u32x4* v) {
    const int h = e / (16 * NT), T = (e >> 4) % NT, r = g3_perm(e & 15);
    const uint8_t* src = c.chunk(T, CB) + (16 * c.q + r) * 16;
#pragma unroll
    for (int j = 0; j < NS; ++j) v[j] = ld16_nt(src + (4 * h + NS * part + j) * 1024);
  }
  template <int NS>
  __device__ static __forceinline__ void convert(const u32x4* v, half8_t* b) {
#pragma unroll
    for (int j = 0; j < NS; ++j) b[j] = bf8_to_h8(v[j]);
  }
};

// PROBE (timing probes only, never in the engine): bit 0 skips the MFMAs (operand reads kept
// live), bit 1 the dequant, bit 2 all global->LDS staging
template <int PT, int EPI, int BM, int BN, int PROBE = 0>
__global__ __launch_bounds__(512) void gemm3_kernel(const GemvParams p, const int n_mb, const int st_per_split,
                                                    const int n_stages) {
  using Q = G3<PT>;
  constexpr int NT = BN / 16;
  constexpr int WN = BN == 256 ? 4 : (BM == 256 ? 2 : 4);
  constexpr int WM = 8 / WN;
  constexpr int FM = BM / (16 * WM), FN = BN / (16 * WN);
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, R_BYTES = Q::raw_bytes(NT);
  constexpr int A_PER_WAVE = BM / 64;   // 1-KB pieces (8 rows) per wave per stage
  static_assert(FM >= 1 && FN >= 1 && 16 * FM * WM == BM && 16 * FN * WN == BN, "tile");
  __shared__ __attribute__((aligned(16))) char smem[2 * A_BYTES + 2 * B_BYTES + 2 * R_BYTES];
  char* const As = smem;
  char* const Bs = smem + 2 * A_BYTES;
  char* const Rs = Bs + 2 * B_BYTES;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware logical id (bijective for any grid size): blocks b = x (mod 8) share an XCD and get
  // consecutive logical ids, i.e. the row blocks of one column group
  const int nwg = gridDim.x, bx = blockIdx.x;
  const int xcd = bx & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bx >> 3);
  const int cg = lid / n_mb, mb = lid - cg * n_mb;
  const int m0 = mb * BM;
  const int s_begin = blockIdx.y * st_per_split;
  const int s_end = min(s_begin + st_per_split, n_stages);
  if (s_begin >= s_end) return;   // uniform over the workgroup
  const int M = p.M;

  G3Ctx ctx;
  ctx.W = p.W; ctx.t0 = cg * NT; ctx.ntiles = p.ntiles; ctx.nsb = p.nsb;

  // A (x) stage: piece pc (8 rows) of this wave; lane -> row 8 pc + (l >> 3), image chunk l & 7
  auto issue_a = [&](int s, int buf) {
    if constexpr (PROBE & 4) return;
    const int k0 = s * 64;
#pragma unroll
    for (int i = 0; i < A_PER_WAVE; ++i) {
      const int pc = wave * A_PER_WAVE + i;
      const int row = 8 * pc + (lane >> 3);
      const int ch = (lane & 7) ^ g3_swz(row);
      const int gr = min(m0 + row, M - 1);
      glds<16>(p.X + (size_t)gr * p.ldx + k0 + 8 * ch, As + buf * A_BYTES + pc * 1024);
    }
  };
  // all 512 threads dequantize: NT = 16 one entry each; NT = 8 half an entry each, waves 2k and
  // 2k + 1 sharing the entries of lanes 64 k .. (part = wave parity; h stays wave-uniform)
  constexpr int DQ_NS = 32 * NT == 512 ? 4 : 2;
  const int dq_part = DQ_NS == 4 ? 0 : (wave & 1);
  const int dq_e = DQ_NS == 4 ? tid : (lane | ((wave >> 1) << 6));
  const int dq_h = dq_e / (16 * NT);
  const int dq_col = 16 * ((dq_e >> 4) % NT) + g3_perm(dq_e & 15);
  u32x4 breg[G3<PT>::MODE == G3_REG ? DQ_NS : 1];   // G3_REG: raw of the next stage to convert
  auto issue_b = [&](int s, int buf) {
    if constexpr (PROBE & 4) return;
    ctx.sb = s >> 2; ctx.q = s & 3;
    if constexpr (Q::MODE == G3_DIRECT) Q::issue_b(Bs + buf * B_BYTES, ctx, NT, wave, lane);
    else if constexpr (Q::MODE == G3_RAW_LDS) Q::issue(Rs + buf * R_BYTES, ctx, NT, wave, lane);
  };
  auto load_breg = [&](int s, u32x4* v) {
    if constexpr (Q::MODE == G3_REG) {
      ctx.sb = s >> 2; ctx.q = s & 3;
      Q::template load<DQ_NS>(ctx, NT, dq_e, dq_part, v);
    }
  };
  const Consts kc = make_consts();
  auto store_b = [&](const half8_t* b, int buf) {
    char* B = Bs + buf * B_BYTES;
#pragma unroll
    for (int j = 0; j < DQ_NS; ++j) *reinterpret_cast<half8_t*>(B + g3_off(dq_col, 4 * dq_h + DQ_NS * dq_part + j)) = b[j];
  };
  auto dequant = [&](int s, int buf) {   // raw R[buf] (registers for G3_REG) of stage s -> B[buf]
    if constexpr (PROBE & 2) return;
    half8_t b[DQ_NS];
    if constexpr (Q::MODE == G3_RAW_LDS) {
      Q::template dequant<DQ_NS>(Rs + buf * R_BYTES, NT, dq_e, dq_part, s & 3, kc, b);
      store_b(b, buf);
    } else if constexpr (Q::MODE == G3_REG) {
      Q::template convert<DQ_NS>(breg, b);
      store_b(b, buf);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // prologue: A(0), B/raw(0), raw(1) -> dequant(0)
  issue_a(s_begin, 0);
  issue_b(s_begin, 0);
  if constexpr (Q::MODE == G3_RAW_LDS) {
    if (s_begin + 1 < s_end) issue_b(s_begin + 1, 1);
    __syncthreads();
    dequant(s_begin, 0);
  } else if constexpr (Q::MODE == G3_REG) {
    load_breg(s_begin, breg);
    dequant(s_begin, 0);
    load_breg(min(s_begin + 1, s_end - 1), breg);
  }
  __syncthreads();

  const int wm = wave / WN, wn = wave % WN;
  const int rbase = wm * FM * 16 + (lane & 15), cbase = wn * FN * 16 + (lane & 15);
  const int g = lane >> 4;
  for (int s = s_begin; s < s_end; ++s) {
    const int t = s - s_begin, cur = t & 1;
    // A(s+1) -> A[cur^1] and raw(s+2) -> R[cur] (or, 16-bit weights, B(s+1) -> B[cur^1]): both
    // buffers were last read in iteration s-1
    // (unconditional, stage clamped to the range: the loop body stays one basic block, so the
    // scheduler can interleave the dequant VALU with the MFMAs; past-the-end loads re-read the last
    // stage into buffers nobody reads, the last dequant converts stale bytes into an unread buffer)
    const int s1 = min(s + 1, s_end - 1);
    issue_a(s1, cur ^ 1);
    if constexpr (Q::MODE == G3_DIRECT) issue_b(s1, cur ^ 1);
    else issue_b(min(s + 2, s_end - 1), cur);
    u32x4 bnext[Q::MODE == G3_REG ? DQ_NS : 1];   // G3_REG: raw(s+2), loaded while stage s computes
    load_breg(min(s + 2, s_end - 1), bnext);
    const char* Ab = As + cur * A_BYTES;
    const char* Bb = Bs + cur * B_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      half8_t a[FM], b[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) a[i] = *reinterpret_cast<const half8_t*>(Ab + g3_off(rbase + 16 * i, 4 * kk + g));
#pragma unroll
      for (int j = 0; j < FN; ++j) b[j] = *reinterpret_cast<const half8_t*>(Bb + g3_off(cbase + 16 * j, 4 * kk + g));
      if constexpr (PROBE & 1) {
#pragma unroll
        for (int i = 0; i < FM; ++i) asm volatile("" ::"v"(a[i]));
#pragma unroll
        for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(b[j]));
      } else {
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32(a[i], b[j], acc[i][j]);
      }
    }
    // dequant raw(s+1) -> B[cur^1] (landed at the end of iteration s-1).  Placed AFTER the MFMA
    // code: its ds_writes may not move above the operand ds_reads (the compiler cannot separate the
    // two B buffers), so written first it would serialise the whole dequant ahead of the first
    // MFMA; written here, its VALU is free to fill the MFMA stream and only the 4 stores trail it.
    dequant(s + 1, cur ^ 1);
    if constexpr (Q::MODE == G3_REG) {
#pragma unroll
      for (int j = 0; j < DQ_NS; ++j) breg[j] = bnext[j];
    }
    __syncthreads();
  }

  // epilogue: lane holds C[row 16 i + 4 g + v][col 16 j + r] of the wave tile
  const int r = lane & 15;
  const int row0 = m0 + wm * FM * 16 + 4 * g;
  const int col0 = cg * BN + wn * FN * 16;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = col0 + 16 * j + r;
    if constexpr (EPI == EPI_SWIGLU) {
      const int o = (n >> 4) * 8 + r;   // tile rows 0-7 gate, 8-15 up of the same 8 outputs
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const float other = __shfl_xor(acc[i][j][v], 8);
          const int m = row0 + 16 * i + v;
          if (r < 8 && m < M && o < p.n_valid) p.H[(size_t)m * p.ldh + o] = sat_f16(silu(acc[i][j][v]) * other);
        }
    } else {
      if (n < p.n_valid) {
        const float bias = (p.bias && blockIdx.y == 0) ? p.bias[n] : 0.f;
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int m = row0 + 16 * i + v;
            if (m < M) {
              float* dst = p.Y + (size_t)blockIdx.y * p.split_stride + (size_t)m * p.ldy + n;
              if constexpr (EPI == EPI_ATOMIC) unsafeAtomicAdd(dst, acc[i][j][v] + bias);
              else *dst = acc[i][j][v] + bias;
            }
          }
      }
    }
  }
}

}  // namespace mpk

namespace mp {

static int g3_force_bm = 0, g3_force_bn = 0, g3_force_split = 0, g3_split_wg = 256;
void set_gemm3_tuning(int bm, int bn, int nsplit, int split_wg) {
  g3_force_bm = bm; g3_force_bn = bn; g3_force_split = nsplit; g3_split_wg = split_wg > 0 ? split_wg : 256;
}

template <int PT, int EPI, int BM, int BN>
static void gemm3_go(GemvParams p, bool allow_split, hipStream_t st) {
  constexpr int NT = BN / 16;
  const int n_cg = (p.ntiles + NT - 1) / NT;
  const int n_mb = (p.M + BM - 1) / BM;
  const int n_stages = p.nsb * 4;
  const int wgs = n_cg * n_mb;
  int nsplit = 1;
  if (EPI == EPI_ATOMIC && allow_split) {
    if (g3_force_split > 0) nsplit = g3_force_split;
    else if (wgs < g3_split_wg) nsplit = std::max(1, std::min(g3_split_wg / wgs, n_stages / 16));
  }
  nsplit = std::max(1, std::min(nsplit, n_stages));
  const int per = (n_stages + nsplit - 1) / nsplit;
  nsplit = (n_stages + per - 1) / per;
  if constexpr (PT == P_Q4_K && EPI == EPI_SWIGLU && BM == 256 && BN == 256) {
    switch (knob(KNOB_GEMM3_PROBE)) {   // timing probes (tools/gemv_bench.py --knob GEMM3_PROBE=k)
      case 1: hipLaunchKernelGGL((mpk::gemm3_kernel<PT, EPI, BM, BN, 1>), dim3(wgs, nsplit), dim3(512), 0, st, p, n_mb, per, n_stages); return;
      case 2: hipLaunchKernelGGL((mpk::gemm3_kernel<PT, EPI, BM, BN, 2>), dim3(wgs, nsplit), dim3(512), 0, st, p, n_mb, per, n_stages); return;
      case 3: hipLaunchKernelGGL((mpk::gemm3_kernel<PT, EPI, BM, BN, 3>), dim3(wgs, nsplit), dim3(512), 0, st, p, n_mb, per, n_stages); return;
      case 4: hipLaunchKernelGGL((mpk::gemm3_kernel<PT, EPI, BM, BN, 4>), dim3(wgs, nsplit), dim3(512), 0, st, p, n_mb, per, n_stages); return;
      case 6: hipLaunchKernelGGL((mpk::gemm3_kernel<PT, EPI, BM, BN, 6>), dim3(wgs, nsplit), dim3(512), 0, st, p, n_mb, per, n_stages); return;
      default: break;
    }
  }
  hipLaunchKernelGGL((mpk::gemm3_kernel<PT, EPI, BM, BN>), dim3(wgs, nsplit), dim3(512), 0, st, p, n_mb, per, n_stages);
}

template <int PT, int BM, int BN>
static constexpr bool g3_fits() {
  return 2 * (BM * 128 + BN * 128 + mpk::G3<PT>::raw_bytes(BN / 16)) <= 160 * 1024;
}

template <int PT, int EPI>
static void gemm3_shape(GemvParams p, bool allow_split, hipStream_t st) {
  // BM: 128 rows when one 128-row block holds M; BN: 256 columns unless that leaves fewer than
  // half the CUs with a workgroup and the epilogue cannot split K
  const int bm = g3_force_bm ? g3_force_bm : (p.M <= 128 ? 128 : 256);
  const int wg256 = (p.ntiles + 15) / 16 * ((p.M + bm - 1) / bm);
  const bool splits = EPI == EPI_ATOMIC && allow_split;
  const int bn = g3_force_bn ? g3_force_bn : (!splits && wg256 < 128 ? 128 : 256);
  if (bm == 128) {
    if (bn == 128) gemm3_go<PT, EPI, 128, 128>(p, allow_split, st);
    else gemm3_go<PT, EPI, 128, 256>(p, allow_split, st);
  } else {
    // Q8_0's 32-B raw quants: 256 x 256 does not fit 160 KB of LDS double-buffered
    if constexpr (g3_fits<PT, 256, 256>()) {
      if (bn == 256) return gemm3_go<PT, EPI, 256, 256>(p, allow_split, st);
    }
    gemm3_go<PT, EPI, 256, 128>(p, allow_split, st);
  }
}

template <int PT>
static void gemm3_pt(int epi, const GemvParams& p, bool allow_split, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return gemm3_shape<PT, EPI_STORE>(p, allow_split, st);
    case EPI_ATOMIC: return gemm3_shape<PT, EPI_ATOMIC>(p, allow_split, st);
    case EPI_SWIGLU: return gemm3_shape<PT, EPI_SWIGLU>(p, allow_split, st);
  }
}

void launch_gemm3(int ptype, int epi, GemvParams p, hipStream_t st, bool allow_split) {
  switch (ptype) {
    case P_Q4_K: gemm3_pt<P_Q4_K>(epi, p, allow_split, st); break;
    case P_Q5_K: gemm3_pt<P_Q5_K>(epi, p, allow_split, st); break;
    case P_Q6_K: gemm3_pt<P_Q6_K>(epi, p, allow_split, st); break;
    case P_Q8_0: gemm3_pt<P_Q8_0>(epi, p, allow_split, st); break;
    case P_Q4_0: gemm3_pt<P_Q4_0>(epi, p, allow_split, st); break;
    case P_F16: gemm3_pt<P_F16>(epi, p, allow_split, st); break;
    case P_BF16: gemm3_pt<P_BF16>(epi, p, allow_split, st); break;
  }
}

}  // namespace mp
