// Dequant GEMM v4: gemm3's LDS-DMA pipeline on the 32x32x16 MFMA (M > 64: wide decode micro-batches
// and prompt chunks).
//
// Y[M][N] (+)= X[M][K] W[N][K]^T with W in the T16 packed quant layout (csrc/runtime/qtypes.h).
// Workgroup tile BM (128 | 256) rows x 256 columns, 8 waves; every wave OWNS 32 columns (two T16
// tiles) for all BM rows and runs v_mfma_f32_32x32x16_f16 on them: per 64-k stage BM/32 x 4
// MFMAs, each fed by ONE A-fragment ds_read_b128 and one register B fragment.
//
// Why 32x32x16 (gemm3 runs 16x16x32, the same FLOP per A byte): an MFMA of this shape occupies its
// SIMD for 32 cycles and blocks vector issue for 8 of them (MI355X_MICROARCH.md, issue-cost row),
// so per FLOP there are 1.5x the free issue cycles of the 16x16x32 form, and half the MFMA, wait and
// A-read instructions.  gemm3's PMC (profiles/r6b) shows the wave stream issue-bound (39 % of wave
// cycles waiting on issue, MFMA busy 46 %) with the Q4_K dequant and the A reads competing for the
// 8 free cycles of every 16-cycle MFMA.
//
// Lane mapping of the 32x32x16 operands (lane l, h = l >> 5, c = l & 31):
//   A (x):        row c of the 32-row fragment, k = 64 q + 32 kk + 16 h + 8 e + j  (t = 2 kk + e)
//   B (weights):  column c = tile (c >> 4), row (c & 15) of that tile, the same k: dword 2 h + e of
//                 the T16 piece (kk, row) -- so one ds_read_b64 fetches both MFMAs' quants of a kk
//   C:            column c, row 8 (v >> 2) + 4 h + (v & 3) of the 16 accumulators v
// The k permutation inside a 32-k half (A and B index it the same way) is all a dot product needs,
// and the sub-block scale of MFMA t (k-half kk) is uniform over the lanes.
//
// The x image, the raw weight images and the 3-stage counted-vmcnt / counted-lgkmcnt stream are
// gemm3's (gemm_lds.h); see gemm3.hip for the pipeline's invariants.
#include "gemm_lds.h"
#include "../runtime/tuning.h"

#include <algorithm>
#include <stdexcept>

namespace mpk {
using namespace mp;

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <bool BF>
__device__ __forceinline__ f32x16 mma32(half8_t a, half8_t b, f32x16 c) {
  if constexpr (BF)
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

// dword P of a B fragment register
template <int P>
__device__ __forceinline__ void set_dw(half8_t& f, uint32_t v) {
  u32x4 u = __builtin_bit_cast(u32x4, f);
  u[P] = v;
  f = __builtin_bit_cast(half8_t, u);
}

// Per-type reads of one wave's raw stage image (W3<PT>::issue layout, TW tiles) in the 32x32
// mapping: column pair `pair` = tiles 2 pair, 2 pair + 1 (32 columns, one MFMA B operand).
template <int PT> struct W4;

template <> struct W4<P_Q4_K> {
  static constexpr int NR = 3;   // LDS reads per stage per lane
  struct Raw { u32x4 hdr; u32x2 q[2]; };
  struct Prep { half2_t S2, M2; };
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, int pair, Raw& w) {
    const int c = lane & 31, u = 2 * pair + (c >> 4), r = c & 15, h = lane >> 5;
    ds_b128(w.hdr, R + TW * 512 + (u * 16 + r) * 16);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) ds_b64(w.q[kk], R + ((u * 2 + kk) * 16 + r) * 16 + 8 * h);
  }
  __device__ static __forceinline__ Prep prep(const Raw& w, int q) {
    Prep p;
    kq_scales(w.hdr, (uint32_t)q, p.S2, p.M2);
    return p;
  }
  __device__ static __forceinline__ half8_t frag(const Raw& w, const Prep& p, int t, int, const Consts& k) {
    const int kk = t >> 1, e = t & 1;
    return nib8(w.q[kk][e], kk ? h2hi(p.S2) : h2lo(p.S2), kk ? h2hi(p.M2) : h2lo(p.M2), k);
  }
  // dword P of frag() (nib8's four independent pairs), so a fragment's dequant can be spread over
  // the gaps between one wave's MFMAs instead of one 13-instruction VALU burst
  static constexpr bool kParts = true;
  template <int P>
  __device__ static __forceinline__ uint32_t fragp(const Raw& w, const Prep& p, int t, int, const Consts& k) {
    const int kk = t >> 1, e = t & 1;
    const uint32_t v = P >= 2 ? w.q[kk][e] >> 8 : w.q[kk][e];
    const half2_t S = kk ? h2hi(p.S2) : h2lo(p.S2), Mh = kk ? h2hi(p.M2) : h2lo(p.M2);
    if constexpr (P & 1) return as_u32(__builtin_elementwise_fma(as_h2(and_or(v, k.mhi, k.mag_lo)) - h2c(64.f), S, Mh));
    else return as_u32(__builtin_elementwise_fma(as_h2(and_or(v, k.mlo, k.mag_hi)) - h2c(1024.f), S, Mh));
  }
};

// Q6_K: quants [u][h][r] 16 B (dwords 2h, 2h+1 = one b64), high bits [u][kk][r] 8 B (the 2-bit
// pairs of dword g live in its 16-bit half g & 1... of dword g >> 1: one b32 per kk), int8 scales
// [u][r] (dword q), d [u][r]
template <> struct W4<P_Q6_K> {
  static constexpr int NR = 6;
  static constexpr bool kParts = true;
  struct Raw { uint32_t sc, d; u32x2 q[2]; uint32_t qd[2]; };
  struct Prep { uint32_t sc; f16 d; };
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, int pair, Raw& w) {
    const int c = lane & 31, u = 2 * pair + (c >> 4), r = c & 15, h = lane >> 5;
    ds_b32(w.sc, R + TW * 768 + (u * 16 + r) * 4);
    ds_u16(w.d, R + TW * 832 + (u * 16 + r) * 2);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      ds_b64(w.q[kk], R + ((u * 2 + kk) * 16 + r) * 16 + 8 * h);
      // high bits of dwords g = 2h, 2h+1: the 16-bit halves 0, 1 of dword (g >> 1) = h
      ds_b32(w.qd[kk], R + TW * 512 + ((u * 2 + kk) * 16 + r) * 8 + 4 * h);
    }
  }
  __device__ static __forceinline__ Prep prep(const Raw& w, int) {
    return Prep{w.sc ^ 0x80808080u, __builtin_bit_cast(f16, (uint16_t)w.d)};
  }
  __device__ static __forceinline__ half8_t frag(const Raw& w, const Prep& p, int t, int h, const Consts& k) {
    const int kk = t >> 1, e = t & 1;   // dword g = 2h + e: high bits in half e of qd[kk]
    const uint32_t h16 = (w.qd[kk] >> (16 * e)) & 0xFFFFu;
    // int8 scale of sub-block 4q + 2kk + (g >> 1) = 4q + 2kk + h: byte 2kk + h of the dword
    const uint32_t sb = (p.sc >> (8 * (2 * kk + h))) & 0xFFu;
    const f16 sf = (as_h2(0x6400u | sb).x - (f16)1152.f) * p.d;
    const half2_t S = half2_t{sf, sf};
    const uint32_t x = h16 | (h16 << 8);
    const uint32_t v = w.q[kk][e], tt = v >> 8;
    const uint32_t h0 = ((x << 4) & 0x00300030u) | k.mag_hi, h1 = ((x << 6) & 0x03000300u) | k.mag_lo;
    const uint32_t h2 = (x & 0x00300030u) | k.mag_hi, h3 = ((x << 2) & 0x03000300u) | k.mag_lo;
    return pack8(as_u32((as_h2(and_or(v, k.mlo, h0)) - h2c(1056.f)) * S),
                 as_u32((as_h2(and_or(v, k.mhi, h1)) - h2c(96.f)) * S),
                 as_u32((as_h2(and_or(tt, k.mlo, h2)) - h2c(1056.f)) * S),
                 as_u32((as_h2(and_or(tt, k.mhi, h3)) - h2c(96.f)) * S));
  }
  // dword P of frag() (the scale and high-bit words are shared: the compiler keeps them between steps)
  template <int P>
  __device__ static __forceinline__ uint32_t fragp(const Raw& w, const Prep& p, int t, int h, const Consts& k) {
    const int kk = t >> 1, e = t & 1;
    const uint32_t h16 = (w.qd[kk] >> (16 * e)) & 0xFFFFu;
    const uint32_t sb = (p.sc >> (8 * (2 * kk + h))) & 0xFFu;
    const f16 sf = (as_h2(0x6400u | sb).x - (f16)1152.f) * p.d;
    const half2_t S = half2_t{sf, sf};
    const uint32_t x = h16 | (h16 << 8);
    const uint32_t v = P >= 2 ? w.q[kk][e] >> 8 : w.q[kk][e];
    if constexpr (P == 0) return as_u32((as_h2(and_or(v, k.mlo, ((x << 4) & 0x00300030u) | k.mag_hi)) - h2c(1056.f)) * S);
    if constexpr (P == 1) return as_u32((as_h2(and_or(v, k.mhi, ((x << 6) & 0x03000300u) | k.mag_lo)) - h2c(96.f)) * S);
    if constexpr (P == 2) return as_u32((as_h2(and_or(v, k.mlo, (x & 0x00300030u) | k.mag_hi)) - h2c(1056.f)) * S);
    return as_u32((as_h2(and_or(v, k.mhi, ((x << 2) & 0x03000300u) | k.mag_lo)) - h2c(96.f)) * S);
  }
};

// Q5_K: quants as Q4_K, high-bit dword [u][kk][r] (byte g = dword g's 8 high bits), header [u][r]
template <> struct W4<P_Q5_K> {
  static constexpr int NR = 5;
  static constexpr bool kParts = false;
  template <int P, class RW, class PR>   // (unused: kParts false) the whole fragment's dword P
  __device__ static __forceinline__ uint32_t fragp(const RW& w, const PR& p, int t, int h, const Consts& k) {
    return __builtin_bit_cast(u32x4, frag(w, p, t, h, k))[P];
  }
  struct Raw { u32x4 hdr; u32x2 q[2]; uint32_t qh[2]; };
  struct Prep { half2_t S2, M2; };
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, int pair, Raw& w) {
    const int c = lane & 31, u = 2 * pair + (c >> 4), r = c & 15, h = lane >> 5;
    ds_b128(w.hdr, R + TW * 640 + (u * 16 + r) * 16);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      ds_b64(w.q[kk], R + ((u * 2 + kk) * 16 + r) * 16 + 8 * h);
      ds_b32(w.qh[kk], R + TW * 512 + ((u * 2 + kk) * 16 + r) * 4);
    }
  }
  __device__ static __forceinline__ Prep prep(const Raw& w, int q) {
    Prep p;
    kq_scales(w.hdr, (uint32_t)q, p.S2, p.M2);
    return p;
  }
  __device__ static __forceinline__ half8_t frag(const Raw& w, const Prep& p, int t, int h, const Consts& k) {
    const int kk = t >> 1, e = t & 1, g = 2 * h + e;
    const uint32_t hb = (w.qh[kk] >> (8 * g)) & 0xFFu;
    const uint32_t x = hb | (hb << 12);
    const half2_t S = kk ? h2hi(p.S2) : h2lo(p.S2), M = kk ? h2hi(p.M2) : h2lo(p.M2);
    const uint32_t v = w.q[kk][e], tt = v >> 8;
    const uint32_t h0 = ((x << 4) & 0x00100010u) | k.mag_hi, h1 = ((x << 7) & 0x01000100u) | k.mag_lo;
    const uint32_t h2 = ((x << 2) & 0x00100010u) | k.mag_hi, h3 = ((x << 5) & 0x01000100u) | k.mag_lo;
    return pack8(as_u32(__builtin_elementwise_fma(as_h2(and_or(v, k.mlo, h0)) - h2c(1024.f), S, M)),
                 as_u32(__builtin_elementwise_fma(as_h2(and_or(v, k.mhi, h1)) - h2c(64.f), S, M)),
                 as_u32(__builtin_elementwise_fma(as_h2(and_or(tt, k.mlo, h2)) - h2c(1024.f), S, M)),
                 as_u32(__builtin_elementwise_fma(as_h2(and_or(tt, k.mhi, h3)) - h2c(64.f), S, M)));
  }
};

// Q8_0: piece (u, kk, r) = 32 int8 (+128) at R + ((u*2 + kk)*16 + r)*32; bytes 16h .. 16h+15 hold
// dwords g = 2h, 2h+1 of the 16x16 map (one b128 per kk); block scales [u][r] = (d(2q), d(2q+1))
template <> struct W4<P_Q8_0> {
  static constexpr int NR = 3;
  static constexpr bool kParts = false;
  template <int P, class RW, class PR>   // (unused: kParts false) the whole fragment's dword P
  __device__ static __forceinline__ uint32_t fragp(const RW& w, const PR& p, int t, int h, const Consts& k) {
    return __builtin_bit_cast(u32x4, frag(w, p, t, h, k))[P];
  }
  struct Raw { uint32_t dd; u32x4 v[2]; };
  struct Prep { uint32_t dd; };
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, int pair, Raw& w) {
    const int c = lane & 31, u = 2 * pair + (c >> 4), r = c & 15, h = lane >> 5;
    ds_b32(w.dd, R + TW * 1024 + (u * 16 + r) * 4);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) ds_b128(w.v[kk], R + ((u * 2 + kk) * 16 + r) * 32 + 16 * h);
  }
  __device__ static __forceinline__ Prep prep(const Raw& w, int) { return Prep{w.dd}; }
  __device__ static __forceinline__ half8_t frag(const Raw& w, const Prep& p, int t, int, const Consts&) {
    const int kk = t >> 1, e = t & 1;
    const uint32_t lo = e ? w.v[kk].z : w.v[kk].x, hi = e ? w.v[kk].w : w.v[kk].y;
    const half2_t off = h2c(1152.f);
    const half2_t S = kk ? h2hi(as_h2(p.dd)) : h2lo(as_h2(p.dd));
    return pack8(as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, lo, 0x04010400u)) - off) * S),
                 as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, lo, 0x04030402u)) - off) * S),
                 as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, hi, 0x04010400u)) - off) * S),
                 as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, hi, 0x04030402u)) - off) * S));
  }
};

// 16-bit weights: the raw image holds [u][kk][lane16] 16-B fragment pieces of the 16x16 mapping
// (element 4 kk + g of lane (q, r)): piece g of (u, kk, r) = k 32 kk + 8 g + j -- the 32x32 lane
// (h, c) of MFMA t needs piece g = 2h + e of (u, kk, r)
template <int PT> struct W4_16 {
  static constexpr int NR = 4;
  static constexpr bool kParts = false;
  template <int P, class RW, class PR>   // (unused: kParts false) the whole fragment's dword P
  __device__ static __forceinline__ uint32_t fragp(const RW& w, const PR& p, int t, int h, const Consts& k) {
    return __builtin_bit_cast(u32x4, frag(w, p, t, h, k))[P];
  }
  struct Raw { u32x4 v[4]; };
  struct Prep {};
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, int pair, Raw& w) {
    const int c = lane & 31, u = 2 * pair + (c >> 4), r = c & 15, h = lane >> 5;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int kk = t >> 1, g = 2 * h + (t & 1);
      ds_b128(w.v[t], R + (u * 2 + kk) * 1024 + (16 * g + r) * 16);
    }
  }
  __device__ static __forceinline__ Prep prep(const Raw&, int) { return Prep{}; }
  __device__ static __forceinline__ half8_t frag(const Raw& w, const Prep&, int t, int, const Consts&) {
    return __builtin_bit_cast(half8_t, w.v[t]);
  }
};
template <> struct W4<P_F16> : W4_16<P_F16> {};
template <> struct W4<P_BF16> : W4_16<P_BF16> {};

template <int PT> constexpr bool g4_supported() {
  return PT == P_Q4_K || PT == P_Q5_K || PT == P_Q6_K || PT == P_Q8_0 || PT == P_F16 || PT == P_BF16;
}

// MoE mode (grouped GEMM over the routed experts): blockIdx.z = expert e, whose rows are
// the token slots the router listed for it (lists[e][0 .. counts[e])); row blocks past counts[e]
// exit at once.  The A staging gathers those rows (LDS-DMA addresses are per lane, so the gather
// costs nothing), the weights are expert e's, and the epilogues scatter by slot: SwiGLU into
// H[slot], down weighted by the router weight into Y[token] (atomics; per-slot rows in the
// deterministic mode, combined in slot order by launch_moe_combine).
struct G4Moe {
  const int32_t* counts = nullptr;
  const int32_t* lists = nullptr;
  int list_cap = 0;
  size_t estride = 0;
  int k = 1, x_per_slot = 0;
  const float* weights = nullptr;
  float* Yslot = nullptr;
};

// NWV compute waves (8, or 7: BN = 224 columns, so a 57344-column gate/up gives 256 workgroups
// for the 256 CUs instead of 224); the x rows are staged round-robin by all of them
template <int PT, int BM, int NWV, int TW = 2>
struct G4Geom {
  static constexpr int A_BYTES = BM * 128;                    // x rows of one 64-k stage
  static constexpr int R_WAVE = W3<PT>::RAW(TW);             // one wave's raw bytes of one stage
  static constexpr int STAGE = A_BYTES + NWV * R_WAVE;
  // stage buffers (x issued NB - 1 stages ahead, weights NB; the kernel handles 3-5)
  // (4-5 buffers for the 128-row tiles measured slower: MoE gate/up 454 -> 454 us at 128 rows, 499
  // -> 713 at 64 rows, where 5 buffers also cost the second workgroup per CU; r8j)
  static constexpr int NB = 3;
  static constexpr int NP = BM / 8;                           // 1-KB A pieces (8 rows) per stage
  static constexpr int A_INSTR = (NP + NWV - 1) / NWV;        // per wave (uniform: vmcnt accounting)
};

// FL (compile-time flags): bits 0-1 LDS-DMA spread mode, bit 2 non-temporal weights; bits 3-5 timing
// probes (probe builds only, wrong results): 3 raw bits as B fragments (no dequant VALU), 4 no MFMAs
// (operands kept live), 5 no LDS-DMA (the stage images keep stale bytes).  Compile-time
// because every weight DMA of a stage branched on them at run time: the 2-stage loop body of the MoE
// gate/up kernel carried 485 scalar instructions (36 of them 64-bit compares, 44 s_nop) against 32
// MFMAs.
// TW (tiles per wave): 2 (32 columns, one MFMA column block) or 4 (64 columns: two column pairs
// share every A fragment; the 64-row MoE tile, where 32-column waves left half the MFMAs of a
// 128-row tile on padding rows)
template <int PT, int EPI, int BM, bool MOE, int NWV = 8, int FL = 0, int TW = 2>
__global__ __launch_bounds__(64 * NWV) __attribute__((amdgpu_waves_per_eu(NWV == 4 && TW == 2 ? 2 : 1))) void gemm4_kernel(const GemvParams p, const int n_mb, const int st_per_split,
                                                    const int n_stages, const G4Moe mo) {
  static_assert(TW == 2 || TW == 4, "gemm4: 2 or 4 tiles per wave");
  constexpr int NPR = TW / 2;   // 32-column pairs per wave
  using Q3 = W3<PT>;
  using Q = W4<PT>;
  using G = G4Geom<PT, BM, NWV, TW>;
  constexpr bool PR_NODQ = (FL & 8) != 0, PR_NOMMA = (FL & 16) != 0, PR_NODMA = (FL & 32) != 0;
  constexpr int NB = G::NB, FR = BM / 32, BN = 16 * TW * NWV;
  constexpr bool BF = PT == P_BF16;
  static_assert(NB >= 3 && NB <= 5, "gemm4: 3-5 stage buffers");
  __shared__ __attribute__((aligned(16))) char smem[NB * G::STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware logical id (bijective for any grid size): consecutive ids (the row blocks of one
  // column group) share an XCD and its L2
  const int nwg = gridDim.x, bx = blockIdx.x;
  const int xcd = bx & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bx >> 3);
  const int cg = lid / n_mb, mb = lid - cg * n_mb;
  const int m0 = mb * BM;
  const int s_begin = blockIdx.y * st_per_split;
  const int s_end = min(s_begin + st_per_split, n_stages);
  if (s_begin >= s_end) return;   // uniform over the workgroup
  int M = p.M;
  int fr_live = FR;   // 32-row fragments holding rows < M (MoE: uniform per expert tile)
  const int32_t* list = nullptr;
  const uint8_t* Wbase = p.W;
  if constexpr (MOE) {
    const int e = blockIdx.z;
    M = mo.counts[e];
    if (m0 >= M) return;   // uniform: this expert has fewer routed rows
    fr_live = min(FR, (M - m0 + 31) >> 5);
    list = mo.lists + (size_t)e * mo.list_cap;
    Wbase += (size_t)e * mo.estride;
  }

  W3Src src;
  src.W = Wbase; src.t0 = cg * (BN / 16) + wave * TW; src.ntiles = p.ntiles; src.nsb = p.nsb;
  src.nt = (FL & 4) != 0;
  auto stage_a = [&](int b) { return smem + b * G::STAGE; };
  auto stage_r = [&](int b) { return smem + b * G::STAGE + G::A_BYTES + wave * G::R_WAVE; };
  // A piece pc = 8 rows; lane -> row 8 pc + (l >> 3), chunk l & 7 (swizzled on the source side):
  // each lane's source row pointers are fixed for the whole K loop (MoE: the gathered rows).
  // Pieces go round-robin over the NWV waves; a wave whose last slot is past the NP pieces re-loads
  // another wave's piece into that piece's place (identical bytes), so every wave issues A_INSTR.
  // All DMA addresses in the saddr form (glds_s): a wave-uniform base per stage plus a per-lane
  // 32-bit offset fixed for the whole K loop (x rows: the host checks they stay under 4 GiB)
  int apc[G::A_INSTR];
  uint32_t xoff[G::A_INSTR];
#pragma unroll
  for (int i = 0; i < G::A_INSTR; ++i) {
    const int pc0 = wave + NWV * i;
    apc[i] = pc0 < G::NP ? pc0 : pc0 - G::NP;
    const int row = 8 * apc[i] + (lane >> 3);
    const int ch = (lane & 7) ^ g3_swz(row);
    int gr = min(m0 + row, M - 1);
    if constexpr (MOE) {
      const int slot = list[gr];
      gr = mo.x_per_slot ? slot : slot / mo.k;
    }
    xoff[i] = (uint32_t)gr * (uint32_t)p.ldx * 2u + 16u * ch;
  }
  const uint8_t* const xbase = reinterpret_cast<const uint8_t*>(p.X);
  auto issue_a = [&](int s, int b) {
    if constexpr (PR_NODMA) return;
    const uint8_t* sb = uniform_ptr(xbase + (size_t)s * 128);
#pragma unroll
    for (int i = 0; i < G::A_INSTR; ++i) glds_s<16>(false, sb, xoff[i], stage_a(b) + apc[i] * 1024);
  };
  auto issue_a1 = [&](int i, int s, int b) {
    if constexpr (PR_NODMA) return;
    const uint8_t* sb = uniform_ptr(xbase + (size_t)s * 128);
#pragma unroll
    for (int ii = 0; ii < G::A_INSTR; ++ii)
      if (ii == i) glds_s<16>(false, sb, xoff[ii], stage_a(b) + apc[ii] * 1024);
  };
  // LDS-DMA issue schedule after the stage barrier: burst (spread == 0: every piece at the barrier,
  // so the two waves of a SIMD both stop issuing MFMAs for the whole burst), or one piece per MFMA
  // step (1), with waves 4-7 (the second wave of each SIMD) two steps later (2)
  const int dma_shift = (FL & 3) == 2 && wave >= 4 ? 2 : 0;
  // weight DMA: per-lane offsets from Wbase recorded once at (sb, q) = (0, 0) (EmitRecord), each
  // stage's scalar base from lane 0's address (EmitSaddr); the host checks the matrix < 4 GiB
  constexpr int NIB = Q3::NI(TW);
  uint32_t boff[NIB], boff0[NIB];
  {
    W3Src c0 = src;
    c0.sb = 0; c0.q = 0;
    Q3::template issue<TW>(smem, c0, EmitRecord<NIB>{Wbase, lane, boff, boff0});
  }
  auto issue_b = [&](int s, int b) {
    if constexpr (PR_NODMA) return;
    src.sb = s / 4; src.q = s % 4;
    Q3::template issue<TW>(stage_r(b), src, EmitSaddr<NIB>{src.nt, lane, boff, boff0});
  };

  f32x16 acc[FR][NPR];
#pragma unroll
  for (int i = 0; i < FR; ++i)
#pragma unroll
    for (int pp = 0; pp < NPR; ++pp)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[i][pp][v] = 0.f;
  const Consts kc = make_consts();
  const int h = lane >> 5, cl = lane & 31;
  // per-lane byte offset of A fragment (t, row cl) inside a stage image; row 32 i + cl adds 4096 i
  uint32_t aoff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) aoff[t] = (uint32_t)g3_off(cl, 4 * (t >> 1) + 2 * h + (t & 1));

  // A fragments read AD steps ahead (8; half the stage's NA fragments for the 64-row MoE tile)
  constexpr int NA = 4 * FR, AD = NA >= 16 ? 8 : NA / 2, NR = Q::NR * NPR, JB = NA - AD - 1;
  // B fragment t + 1 is dequantized at step i = IB of fragment t (behind the first MFMAs of t)
  // B fragment t + 1 is dequantized right behind fragment t's first MFMA (FR - 1 steps of slack
  // for its VALU chain), and the next stage's scales + first B fragment three steps after its raw
  // bytes were read (JP), not on the last step: the stage's first MFMA no longer waits for them
  constexpr int IB = FR >= 4 ? 1 : 0;
  static_assert(JB > FR / 2 && NA - AD > JB, "gemm4: barrier step");
  constexpr int JP = JB + 3 < NA - 2 ? JB + 3 : NA - 2;   // next stage's prep step (bf[.][0] of this stage: last use at FR - 1 < JB)
  static_assert((FL & 3) == 0 || JB + G::A_INSTR + 2 < NA, "gemm4: the spread LDS-DMA issue must end inside the stage");
  using RawT = typename Q::Raw;
  using PrepT = typename Q::Prep;
  // probes: a raw dword / raw fragment instead of the dequantized one
  struct RawDw { uint32_t d[sizeof(RawT) / 4]; };
  auto raw_dw = [&](const RawT& w, int k) { return __builtin_bit_cast(RawDw, w).d[k % (sizeof(RawT) / 4)]; };
  auto fragx = [&](const RawT& w, const PrepT& prp, int t) -> half8_t {
    if constexpr (PR_NODQ) {
      const u32x4 u = {raw_dw(w, t), raw_dw(w, t + 1), raw_dw(w, t + 2), raw_dw(w, t + 3)};
      return __builtin_bit_cast(half8_t, u);
    } else {
      return Q::frag(w, prp, t, h, kc);
    }
  };
  auto fragpx = [&](auto pc, const RawT& w, const PrepT& prp, int t) -> uint32_t {
    constexpr int P = decltype(pc)::value;
    if constexpr (PR_NODQ) return raw_dw(w, t + P);
    else return Q::template fragp<P>(w, prp, t, h, kc);
  };
  RawT raw[NPR];
  PrepT pr[NPR];
  half8_t bf[NPR][4];
  u32x4 af[NA];
  auto read_a = [&](auto jc, u32x4& dst, int b) {
    constexpr int j = decltype(jc)::value;
    ds_b128o<(j % FR) * 4096>(dst, lds_addr(stage_a(b)) + aoff[j / FR]);
  };

  // prologue: x of stages 0 .. NB-2 and weights of 0 .. NB-1 in flight (issue order x0 w0 x1 w1 ..
  // w(NB-1)); then stage 0's raw, first AD fragments, frag 0
  static_for<NB - 1>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    issue_a(min(s_begin + i, s_end - 1), i);
    issue_b(min(s_begin + i, s_end - 1), i);
  });
  issue_b(min(s_begin + NB - 1, s_end - 1), NB - 1);
  wait_vmcnt<(NB - 2) * (G::A_INSTR + NIB) + NIB>();
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int pp = 0; pp < NPR; ++pp) Q::template load<TW>(stage_r(0), lane, pp, raw[pp]);
  static_for<AD>([&](auto jc) { read_a(jc, af[decltype(jc)::value], 0); });
  wait_lgkm<AD>();   // raw in (the oldest reads)
#pragma unroll
  for (int pp = 0; pp < NPR; ++pp) {
    pr[pp] = Q::prep(raw[pp], s_begin & 3);
    bf[pp][0] = fragx(raw[pp], pr[pp], 0);
  }

  // One stage.  LAST (the split's final stage, compile-time) issues nothing for a next stage: no
  // LDS-DMA, no barrier, no raw_n / af_n reads -- so no LDS read is ever left unconsumed.  (A read
  // whose result is dead frees its destination VGPRs to the register allocator at once, while the
  // data is still in flight; whatever the compiler puts there next is overwritten when it lands:
  // tools/isa_lint.py "clobber".)  The counted waits count exactly the reads each form issues.
  auto stage = [&](auto lastc, const int s, const int b, u32x4 (&af)[NA], u32x4 (&af_n)[NA], RawT (&raw)[NPR],
                   RawT (&raw_n)[NPR], PrepT (&pr)[NPR], PrepT (&pr_n)[NPR]) {
    constexpr bool LAST = decltype(lastc)::value;
    // buffers of stages s+1 and s-1 (= s+NB-1, the next x issue); weights of s+NB go to b itself
    const int b1 = b + 1 == NB ? 0 : b + 1, b2 = b == 0 ? NB - 1 : b - 1;
    static_for<NA>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      constexpr int t = j / FR, i = j % FR;
      constexpr int later = (NA - 1 - j < AD - 1 ? NA - 1 - j : AD - 1) + (!LAST && j > JB ? NR + (j - JB - 1) : 0);
      wait_lgkm<(later < 15 ? later : 15)>();
      // MoE: no MFMAs on 32-row fragments past the expert's rows (their A reads stay: the counted
      // lgkmcnt waits assume every read issued)
      if (i == 0 || !MOE || i < fr_live) {
        const half8_t a = x_op<BF>(__builtin_bit_cast(half8_t, af[j]));
#pragma unroll
        for (int pp = 0; pp < NPR; ++pp) {
          if constexpr (PR_NOMMA) asm volatile("" :: "v"(a), "v"(bf[pp][t]));
          else acc[i][pp] = mma32<BF>(a, bf[pp][t], acc[i][pp]);
        }
      }
      if constexpr (j + AD < NA) read_a(std::integral_constant<int, j + AD>{}, af[j + AD], b);
      // B fragment t + 1, behind the first MFMAs of fragment t (its last use of the previous
      // stage's value was FR steps ago)
      if constexpr (Q::kParts && t < 3) {
        // fragment t + 1 one dword per step (steps 0-3 of fragment t; 0, 0, 1, 1 at two row fragments)
        static_for<4>([&](auto pc) {
          constexpr int P = decltype(pc)::value;
          if constexpr (i == (FR >= 4 ? P : P / 2)) {
#pragma unroll
            for (int pp = 0; pp < NPR; ++pp) set_dw<P>(bf[pp][t + 1], fragpx(pc, raw[pp], pr[pp], t + 1));
          }
        });
      } else if constexpr (i == IB && t < 3) {
#pragma unroll
        for (int pp = 0; pp < NPR; ++pp) bf[pp][t + 1] = fragx(raw[pp], pr[pp], t + 1);
      }
      if constexpr (!LAST) {
        if constexpr (j == JB) {
          // x(s+1) and w(s+1) in: w(s+2) (issued with x(s+1)) and the NB - 3 later stages' x and w may
          // be in flight
          wait_vmcnt<NIB + (NB - 3) * (G::A_INSTR + NIB)>();
          __builtin_amdgcn_s_barrier();
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (!(FL & 3)) {
            issue_a(min(s + NB - 1, s_end - 1), b2);
            issue_b(min(s + NB, s_end - 1), b);
          }
#pragma unroll
          for (int pp = 0; pp < NPR; ++pp) Q::template load<TW>(stage_r(b1), lane, pp, raw_n[pp]);
        }
        if constexpr (j >= JB && j < JB + G::A_INSTR + 3) {   // spread issue (uniform branches)
          if constexpr ((FL & 3) != 0) {
            const int slot = j - JB - dma_shift;
            if (slot >= 0 && slot < G::A_INSTR) issue_a1(slot, min(s + NB - 1, s_end - 1), b2);
            if (slot == G::A_INSTR) issue_b(min(s + NB, s_end - 1), b);
          }
        }
        if constexpr (j > JB) read_a(std::integral_constant<int, j - JB - 1>{}, af_n[j - JB - 1], b1);
        constexpr bool split0 = Q::kParts && JP + 4 < NA;   // bf[.][0] of stage s+1 one dword per step after JP
        if constexpr (j == JP) {   // stage s+1's raw bytes: the j - JB fragment reads after them may be in flight
          wait_lgkm<(j - JB < 15 ? j - JB : 15)>();
#pragma unroll
          for (int pp = 0; pp < NPR; ++pp) {   // (bf[.][0] of stage s: last use at j = FR - 1)
            pr_n[pp] = Q::prep(raw_n[pp], (s + 1) & 3);
            if constexpr (!split0) bf[pp][0] = fragx(raw_n[pp], pr_n[pp], 0);
          }
        }
        if constexpr (split0 && j > JP && j <= JP + 4) {
          constexpr int P = j - JP - 1;
#pragma unroll
          for (int pp = 0; pp < NPR; ++pp) set_dw<P>(bf[pp][0], fragpx(std::integral_constant<int, P>{}, raw_n[pp], pr_n[pp], 0));
        }
      }
    });
  };
  using F_ = std::false_type;
  using T_ = std::true_type;
  u32x4 afB[NA];
  RawT rawB[NPR];
  PrepT prB[NPR];
  int s = s_begin, b = 0;
  // pairs of stages, then an odd last stage as LAST (its next-stage reads would be dead).  After
  // an even count the loop's final next-stage reads are dead too, but live up to the loop exit (the
  // back edge uses them), and the exit goes straight to the lgkmcnt(0) below
  for (; s + 1 < s_end; s += 2) {
    stage(F_{}, s, b, af, afB, raw, rawB, pr, prB);
    b = b + 1 == NB ? 0 : b + 1;
    stage(F_{}, s + 1, b, afB, af, rawB, raw, prB, pr);
    b = b + 1 == NB ? 0 : b + 1;
  }
  // every LDS read retired BEFORE the even / odd exits join: with the accumulators in AGPRs (TW = 4)
  // the register allocator puts their AGPR -> VGPR copies for the epilogue at the top of the join
  // block, ahead of a wait placed there -- onto the destinations of the even exit's dead
  // next-stage reads (tools/isa_lint.py "clobber").  (The odd tail over-waits for its first reads.)
  wait_lgkm<0>();
  if (s < s_end) stage(T_{}, s, b, af, afB, raw, rawB, pr, prB);
  wait_vmcnt<0>();   // the clamped tail loads: drained before the workgroup's LDS is released
  wait_lgkm<0>();

  // epilogue: lane holds C[row 32 i + 8 (v >> 2) + 4 h + (v & 3)][col cl] of each of the wave's
  // 32-column pairs
  const int rowb = m0 + 4 * h;
#pragma unroll
  for (int pp = 0; pp < NPR; ++pp) {
  const int n = cg * BN + wave * 16 * TW + 32 * pp + cl;
  if constexpr (EPI == EPI_SWIGLU) {
    const int o = (n >> 4) * 8 + (cl & 15);   // tile rows 0-7 gate, 8-15 up of the same 8 outputs
#pragma unroll
    for (int i = 0; i < FR; ++i)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const float other = __shfl_xor(acc[i][pp][v], 8);
        const int m = rowb + 32 * i + 8 * (v >> 2) + (v & 3);
        if ((cl & 8) == 0 && m < M && o < p.n_valid) {
          const int hr = MOE ? list[m] : m;   // MoE: the slot's row of H
          p.H[(size_t)hr * p.ldh + o] = sat_f16(silu(acc[i][pp][v]) * other);
        }
      }
  } else {
    if (n < p.n_valid) {
      const float bias = (p.bias && blockIdx.y == 0) ? p.bias[n] : 0.f;
      float* Y = p.Y + (size_t)blockIdx.y * p.split_stride + n;
#pragma unroll
      for (int i = 0; i < FR; ++i)
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int m = rowb + 32 * i + 8 * (v >> 2) + (v & 3);
          if (m < M) {
            if constexpr (MOE) {   // down projection: weighted into the slot's token (or its own row)
              const int slot = list[m];
              const float wv = mo.weights[slot] * acc[i][pp][v];
              if (mo.Yslot) mo.Yslot[(size_t)slot * p.ldy + n] = wv;
              else unsafeAtomicAdd(p.Y + (size_t)(slot / mo.k) * p.ldy + n, wv);
            } else if constexpr (EPI == EPI_ATOMIC) {
              unsafeAtomicAdd(Y + (size_t)m * p.ldy, acc[i][pp][v] + bias);
            } else {
              Y[(size_t)m * p.ldy] = acc[i][pp][v] + bias;
            }
          }
        }
    }
  }
  }   // column pairs
}

}  // namespace mpk

namespace mp {

bool gemm4_supported(int ptype);

// K splits of a gemm4 launch: enough workgroups for one round over the 256 CUs (one 8-wave
// workgroup per CU: the 3-stage LDS ring takes ~130 KB), >= 16 stages (1024 k) per split
static int g4_splits(int wgs, int n_stages, int per_cu = 1) {
  const int target = knob(KNOB_GEMM2_SPLIT_WG) * per_cu;
  if (wgs >= target) return 1;
  return std::max(1, std::min(target / wgs, n_stages / 16));
}

template <int PT, int EPI, int BM, bool MOE = false, int NWV = 8, int TW = 2>
static void gemm4_go(GemvParams p, int nsplit, hipStream_t st, const mpk::G4Moe& mo = mpk::G4Moe{}, int E = 1) {
  const int n_cg = (p.ntiles + TW * NWV - 1) / (TW * NWV);
  const int n_mb = (p.M + BM - 1) / BM;   // MoE: p.M = the most rows one expert can get
  const int n_stages = p.nsb * 4;
  nsplit = std::max(1, std::min(nsplit, n_stages));
  const int per = (n_stages + nsplit - 1) / nsplit;
  nsplit = (n_stages + per - 1) / per;
  // non-temporal weight DMA where one row block reads each weight (GEMM4_WNT 0 = auto, 1 on, 2 off):
  // 70B gate/up 322 -> 287 us cold, +0.8 % / +1.4 % tok/s on 70B mb256 / Mixtral in the engine; with
  // two row blocks per column group (8B gate/up at M = 256) the second read needs the L2 copy (86.5
  // -> 89.7 us): profiles/r8k_wnt_ab.txt
  // the kernel's DMA offsets are 32-bit per lane: the weight matrix (one expert's) and the x rows
  // it addresses must stay under 4 GiB
  if ((size_t)p.ntiles * p.nsb * mpk::W3<PT>::CB >= (size_t(1) << 32) ||
      (size_t)std::max(p.M * std::max(1, mo.k), 1) * p.ldx * 2 >= (size_t(1) << 32))
    throw std::runtime_error("gemm4: operand over 4 GiB (32-bit DMA offsets)");
  const int wk = knob(KNOB_GEMM4_WNT);
  const bool wnt = wk == 1 || (wk == 0 && (MOE || n_mb == 1));
  const dim3 grid(n_cg * n_mb, nsplit, E), block(64 * NWV);
#define G4_LAUNCH(F) hipLaunchKernelGGL((mpk::gemm4_kernel<PT, EPI, BM, MOE, NWV, F, TW>), grid, block, 0, st, p, n_mb, per, n_stages, mo)
#ifdef MIPIPE_TIMING_PROBES
  // timing probes (knob GEMM4_PROBE): Q4_K dense gate/up (SwiGLU, 256 rows) and split-K stores
  if constexpr (PT == P_Q4_K && ((!MOE && ((EPI == EPI_SWIGLU && BM == 256) || (EPI == EPI_STORE && BM == 128))) ||
                                 (MOE && EPI == EPI_SWIGLU && BM == 128 && NWV == 8))) {
    const int pk = knob(KNOB_GEMM4_PROBE);
    if (pk) {
      const int w4 = wnt ? 4 : 0;
      switch (pk) {
        case 1: if (w4) G4_LAUNCH(4 | 8); else G4_LAUNCH(8); return;
        case 2: if (w4) G4_LAUNCH(4 | 16); else G4_LAUNCH(16); return;
        case 3: if (w4) G4_LAUNCH(4 | 24); else G4_LAUNCH(24); return;
        case 4: if (w4) G4_LAUNCH(4 | 32); else G4_LAUNCH(32); return;
        case 5: if (w4) G4_LAUNCH(4 | 40); else G4_LAUNCH(40); return;
        case 6: if (w4) G4_LAUNCH(4 | 48); else G4_LAUNCH(48); return;
        default: if (w4) G4_LAUNCH(4 | 56); else G4_LAUNCH(56); return;
      }
    }
  }
  // the LDS-DMA spread schedules (knob GEMM4_SPREAD, measured no faster: PERFORMANCE.md) exist in
  // the probe build only
  if constexpr (NWV >= 7) {   // (the 4-wave forms issue more DMA per wave than a stage's spread slots)
    switch (knob(KNOB_GEMM4_SPREAD) | (wnt ? 4 : 0)) {
      case 1: G4_LAUNCH(1); return;
      case 2: G4_LAUNCH(2); return;
      case 5: G4_LAUNCH(5); return;
      case 6: G4_LAUNCH(6); return;
      default: break;
    }
  }
#endif
  if (wnt) G4_LAUNCH(4);
  else G4_LAUNCH(0);
#undef G4_LAUNCH
}

// rows per workgroup: 256 unless one 128-row block holds M, or 256-row tiles leave most of the 256
// CUs idle (8B gate/up at M = 256: 112 workgroups of 256 rows, 112 us, against 224 of 128 rows,
// 78 us: profiles/r8a_gemm_microbench.txt).  16-bit weights: always 128, their raw stage images
// leave no room for three 256-row x images in LDS
// 8 waves x 64 columns on 128-row tiles (GEMM4_TW4 4: every dense shape, 5: the whole-K SwiGLU
// gate/up only, 6: the split-K shapes only): a 128 x 512 workgroup tile whose A fragments each feed
// two MFMAs (half the A-fragment LDS reads per MFMA of the 8 x 32 form) at two waves per SIMD (128
// accumulators + ~110 registers: 237 VGPRs, no spills)
// (A 7-wave 128-row tile at two workgroups per CU -- 81408 B of LDS fits, but the 128-register
// cap it needs spilled VGPRs that hold in-flight asm LDS reads: tools/isa_lint.py, 82 findings.
// Not shipped; the 96-row MoE tile reaches two per CU within its registers, r12i.)
static bool g4_w8x64(int ptype, int epi) {
  const int k = knob(KNOB_GEMM4_TW4);
  return !is16(ptype) && (k == 4 || (k == 5 && epi == EPI_SWIGLU) || (k == 6 && epi != EPI_SWIGLU));
}

static int g4_bm(int ptype, int M, int ntiles, int epi = -1) {
  if (is16(ptype)) return 128;
  if (knob(KNOB_GEMM3_BM)) return knob(KNOB_GEMM3_BM);
  if (epi >= 0 && g4_w8x64(ptype, epi)) return 128;
  if (M <= 128) return 128;
  const int cgs = (ntiles + 15) / 16;
  return cgs * ((M + 255) / 256) < 192 && cgs * ((M + 127) / 128) <= 512 ? 128 : 256;
}

// workgroups resident per CU: 2 for the 64-row tiles and for 4-wave 128-row tiles (GEMM4_NW=4)
static int g4_per_cu(int ptype, int bm) {
  return bm == 64 || bm == 96 || (bm == 128 && !is16(ptype) && knob(KNOB_GEMM4_NW) == 4) ? 2 : 1;
}

// compute waves per workgroup for an unsplit launch: 7 (224 columns) when that fills more of the
// 256 CUs in whole rounds (70B gate/up at M = 256: 224 -> 256 workgroups), else 8; knob GEMM4_NW
static int g4_nwv(int ntiles, int n_mb) {
  if (knob(KNOB_GEMM4_NW)) return knob(KNOB_GEMM4_NW);
  auto util = [&](int nw) {
    const long w = (long)(ntiles + 2 * nw - 1) / (2 * nw) * n_mb;
    const long rounds = (w + 255) / 256;
    return (double)w / (rounds * 256);
  };
  return util(7) > util(8) + 0.05 ? 7 : 8;
}

// T16 tiles per workgroup column group
static int g4_tpc(int ptype, int bm, int epi) {
  if (g4_w8x64(ptype, epi)) return 32;
  return g4_per_cu(ptype, bm) == 2 && bm == 128 ? 8 : 16;   // (bm 96: 8 waves x 32 columns, 16 tiles)
}

template <int PT, int EPI>
static void gemm4_bm(GemvParams p, int nsplit, hipStream_t st, int epi_sel = EPI) {
  const int bm = g4_bm(PT, p.M, p.ntiles, epi_sel);
  const bool nw7 = nsplit == 1 && g4_nwv(p.ntiles, (p.M + bm - 1) / bm) == 7;
  if constexpr (is16(PT)) {
    gemm4_go<PT, EPI, 128>(p, nsplit, st);
  } else if (g4_w8x64(PT, epi_sel)) {
    // 7 waves (448 columns) when that fills more of the 256 CUs in whole rounds
    const int n_mb = (p.M + 127) / 128;
    auto util = [&](int nw) {
      const long w = (long)(p.ntiles + 4 * nw - 1) / (4 * nw) * n_mb * nsplit;
      return (double)w / (((w + 255) / 256) * 256);
    };
    const int nwk = knob(KNOB_GEMM4_NW);
    if (nwk == 7 || (nwk == 0 && util(7) > util(8) + 0.05)) gemm4_go<PT, EPI, 128, false, 7, 4>(p, nsplit, st);
    else gemm4_go<PT, EPI, 128, false, 8, 4>(p, nsplit, st);
  } else if (((knob(KNOB_GEMM4_TW4) & 1) && bm == 256) || (knob(KNOB_GEMM4_TW4) == 2 && bm >= 128)) {
    // 4 waves of 64 columns (one per SIMD): every A fragment read from LDS feeds two MFMAs (half the
    // LDS A traffic of 8 waves x 32 columns); the same 256-column workgroup tile and grid
    if (bm == 128) gemm4_go<PT, EPI, 128, false, 4, 4>(p, nsplit, st);
    else gemm4_go<PT, EPI, 256, false, 4, 4>(p, nsplit, st);
  } else if (bm == 96) {   // (GEMM3_BM=96, A/B) ~72 KB of LDS: two 8-wave workgroups per CU
    if (nw7) gemm4_go<PT, EPI, 96, false, 7>(p, nsplit, st);
    else gemm4_go<PT, EPI, 96>(p, nsplit, st);
  } else if (bm == 64) {   // 60 KB of LDS: two workgroups per CU
    if (nw7) gemm4_go<PT, EPI, 64, false, 7>(p, nsplit, st);
    else gemm4_go<PT, EPI, 64>(p, nsplit, st);
  } else if (bm == 128) {
    // GEMM4_NW=4: 4 waves x 32 columns (64 KB of LDS, <= 256 registers): two independent workgroups
    // per CU, so one's stage barrier and DMA waits overlap the other's MFMAs
    if (knob(KNOB_GEMM4_NW) == 4) gemm4_go<PT, EPI, 128, false, 4>(p, nsplit, st);
    else if (nw7) gemm4_go<PT, EPI, 128, false, 7>(p, nsplit, st);
    else gemm4_go<PT, EPI, 128>(p, nsplit, st);
  } else {
    if (nw7) gemm4_go<PT, EPI, 256, false, 7>(p, nsplit, st);
    else gemm4_go<PT, EPI, 256>(p, nsplit, st);
  }
}

template <int PT>
static bool gemm4_pt(int epi, GemvParams p, bool allow_split, hipStream_t st, float* scratch, size_t scratch_n,
                     int* nsplit_out) {
  if constexpr (!mpk::g4_supported<PT>()) {
    return false;
  } else {
    const int esel = scratch ? EPI_ATOMIC : epi;   // split-K partial stores: the accumulating shapes
    const int bm = g4_bm(PT, p.M, p.ntiles, esel);
    const int tpc = g4_tpc(PT, bm, esel);   // T16 tiles per column group
    const int wgs = (p.ntiles + tpc - 1) / tpc * ((p.M + bm - 1) / bm);
    const int n_stages = p.nsb * 4;
    int ns = 1;
    if (scratch) {   // split-K partial stores: split s writes scratch + s * M * ldp
      ns = knob(KNOB_GEMM3_SPLIT) > 0 ? knob(KNOB_GEMM3_SPLIT) : g4_splits(wgs, n_stages, g4_per_cu(PT, bm));
      const int per = (n_stages + ns - 1) / ns;
      ns = (n_stages + per - 1) / per;
      const int ldp = p.ntiles * 16;
      if (ns < 2 || (size_t)ns * p.M * ldp > scratch_n) return false;
      p.Y = scratch; p.ldy = ldp; p.split_stride = (int64_t)p.M * ldp;
      *nsplit_out = ns;
      gemm4_bm<PT, EPI_STORE>(p, ns, st, EPI_ATOMIC);
      return true;
    }
    if (epi == EPI_ATOMIC && allow_split)
      ns = knob(KNOB_GEMM3_SPLIT) > 0 ? knob(KNOB_GEMM3_SPLIT) : g4_splits(wgs, n_stages, g4_per_cu(PT, bm));
    switch (epi) {
      case EPI_STORE: gemm4_bm<PT, EPI_STORE>(p, 1, st); break;
      case EPI_ATOMIC: gemm4_bm<PT, EPI_ATOMIC>(p, ns, st); break;
      case EPI_SWIGLU: gemm4_bm<PT, EPI_SWIGLU>(p, 1, st); break;
    }
    return true;
  }
}

static bool gemm4_dispatch(int ptype, int epi, const GemvParams& p, bool allow_split, hipStream_t st, float* scratch,
                           size_t scratch_n, int* ns) {
  switch (ptype) {
    case P_Q4_K: return gemm4_pt<P_Q4_K>(epi, p, allow_split, st, scratch, scratch_n, ns);
    case P_Q5_K: return gemm4_pt<P_Q5_K>(epi, p, allow_split, st, scratch, scratch_n, ns);
    case P_Q8_0: return gemm4_pt<P_Q8_0>(epi, p, allow_split, st, scratch, scratch_n, ns);
    case P_Q6_K: return gemm4_pt<P_Q6_K>(epi, p, allow_split, st, scratch, scratch_n, ns);
    case P_F16: return gemm4_pt<P_F16>(epi, p, allow_split, st, scratch, scratch_n, ns);
    case P_BF16: return gemm4_pt<P_BF16>(epi, p, allow_split, st, scratch, scratch_n, ns);
    default: return false;
  }
}

int gemm4_splits(int ptype, int ntiles, int nsb, int M) {
  if (!gemm4_supported(ptype)) return 1;
  const int bm = g4_bm(ptype, M, ntiles, EPI_ATOMIC);
  const int tpc = g4_tpc(ptype, bm, EPI_ATOMIC);
  const int wgs = (ntiles + tpc - 1) / tpc * ((M + bm - 1) / bm);
  const int n_stages = nsb * 4;
  int ns = knob(KNOB_GEMM3_SPLIT) > 0 ? knob(KNOB_GEMM3_SPLIT) : g4_splits(wgs, n_stages, g4_per_cu(ptype, bm));
  ns = std::max(1, std::min(ns, n_stages));
  const int per = (n_stages + ns - 1) / ns;
  return (n_stages + per - 1) / per;
}

bool gemm4_supported(int ptype) {
  return ptype == P_Q4_K || ptype == P_Q5_K || ptype == P_Q6_K || ptype == P_Q8_0 || ptype == P_F16 || ptype == P_BF16;
}

bool launch_gemm4(int ptype, int epi, GemvParams p, hipStream_t st, bool allow_split) {
  int ns = 0;
  return gemm4_dispatch(ptype, epi, p, allow_split, st, nullptr, 0, &ns);
}

// Grouped MoE GEMM (K13): p.M = tokens of the call (the most rows one expert can receive)
template <int PT, int EPI>
static void moe4_go(const MoeGemvParams& q, hipStream_t st) {
  GemvParams p{};
  p.W = q.W; p.X = q.X; p.ldx = q.ldx; p.M = q.M; p.Y = q.Y; p.ldy = q.ldy; p.H = q.H; p.ldh = q.ldh;
  p.ntiles = q.ntiles; p.nsb = q.nsb; p.n_valid = q.n_valid;
  mpk::G4Moe mo;
  mo.counts = q.counts; mo.lists = q.lists; mo.list_cap = q.list_cap; mo.estride = q.estride; mo.k = q.k;
  mo.x_per_slot = q.x_per_slot; mo.weights = q.weights; mo.Yslot = q.Yslot;
  // row tile from the mean rows per expert (M k / E): 128 up to 128, else 256; split-K (down, atomics
  // only) for the grid the ACTIVE row blocks form, except at 128-row tiles (unsplit, below).  A 64-row tile (knob GEMM4_MOE64) drops the
  // padding rows of Mixtral's 64 rows per expert at 256 tokens but halves the MFMAs per stage for
  // the same per-stage overhead: gate/up 499 vs 454 us, 8036 vs 8920 tok/s (profiles/r8ij_engine_ab.txt)
  const int avg = std::max(1, q.M * q.k / std::max(1, q.E));
  const int n_cg = (q.ntiles + 15) / 16;
  auto g4_splits = [&](int wgs, int n_stages) {   // the GEMM3_SPLIT knob forces it (A/B runs)
    return knob(KNOB_GEMM3_SPLIT) > 0 ? knob(KNOB_GEMM3_SPLIT) : mp::g4_splits(wgs, n_stages);
  };
  if constexpr (is16(PT)) {
    const int ns = EPI == EPI_ATOMIC && !q.Yslot ? g4_splits(n_cg * q.E * ((avg + 127) / 128), q.nsb * 4) : 1;
    gemm4_go<PT, EPI, 128, true>(p, ns, st, mo, q.E);
  } else if (avg <= 64 && knob(KNOB_GEMM4_MOE64) == 1) {   // opt-in: measured slower (r8i)
    // (64-row tiles with 64 columns per wave, TW = 4, measured 33 % slower still: twice the Q4_K
    // dequant per live MFMA, VALU-bound; profiles/r10c_moe_tile64x64.txt)
    const int ns = EPI == EPI_ATOMIC && !q.Yslot ? g4_splits(n_cg * q.E, q.nsb * 4) : 1;
    gemm4_go<PT, EPI, 64, true>(p, ns, st, mo, q.E);
  } else if (avg <= 128) {
    // the down projection unsplit: Mixtral at 256 tokens 10225-10246 vs 10091-10093 tok/s with the
    // 2 K splits that fill the 256 CUs (half the float atomics into the residual; r9i)
    const int ns = EPI == EPI_ATOMIC && !q.Yslot && knob(KNOB_GEMM3_SPLIT) > 0 ? knob(KNOB_GEMM3_SPLIT) : 1;
    // GEMM4_MOE64 = 2: 96-row expert tiles (three 32-row fragments) at <= 80 mean rows per expert:
    // Mixtral's ~64 routed rows per expert at 256 tokens fill 2 of 3 fragments instead of 2 of 4,
    // and an expert rarely needs a second row block (which re-streams its weights)
    // and the down projection split 4 ways over K (float atomics into the token rows, which the two
    // slots of a token share anyway): its ~16 column groups x 8 experts are ~128 live workgroups on
    // 256 CUs.  Mixtral mb256 13495 -> 14546 tok/s with GEMM3_SPLIT=4 (r12m); GEMM4_MOE64=3: unsplit
    if (knob(KNOB_GEMM4_MOE64) >= 2 && avg <= 80) {
      const int ns96 = EPI == EPI_ATOMIC && !q.Yslot && knob(KNOB_GEMM3_SPLIT) == 0 && knob(KNOB_GEMM4_MOE64) == 2 ? 4 : ns;
      gemm4_go<PT, EPI, 96, true>(p, ns96, st, mo, q.E);
    }
    else if (knob(KNOB_GEMM4_TW4) == 3) gemm4_go<PT, EPI, 128, true, 4, 4>(p, ns, st, mo, q.E);   // 4 waves x 64 columns
    else if (knob(KNOB_GEMM4_NW) == 7) gemm4_go<PT, EPI, 128, true, 7>(p, ns, st, mo, q.E);   // 224-column tiles
    else gemm4_go<PT, EPI, 128, true>(p, ns, st, mo, q.E);
  } else {
    const int ns = EPI == EPI_ATOMIC && !q.Yslot ? g4_splits(n_cg * q.E * ((avg + 255) / 256), q.nsb * 4) : 1;
    gemm4_go<PT, EPI, 256, true>(p, ns, st, mo, q.E);
  }
}

template <int PT>
static bool moe4_pt(int epi, const MoeGemvParams& q, hipStream_t st) {
  if constexpr (!mpk::g4_supported<PT>()) {
    return false;
  } else {
    if (epi == EPI_SWIGLU) moe4_go<PT, EPI_SWIGLU>(q, st);
    else if (epi == EPI_ATOMIC) moe4_go<PT, EPI_ATOMIC>(q, st);
    else return false;
    return true;
  }
}

bool launch_moe_gemm4(int ptype, int epi, const MoeGemvParams& q, hipStream_t st) {
  switch (ptype) {
    case P_Q4_K: return moe4_pt<P_Q4_K>(epi, q, st);
    case P_Q5_K: return moe4_pt<P_Q5_K>(epi, q, st);
    case P_Q8_0: return moe4_pt<P_Q8_0>(epi, q, st);
    case P_Q6_K: return moe4_pt<P_Q6_K>(epi, q, st);
    case P_F16: return moe4_pt<P_F16>(epi, q, st);
    case P_BF16: return moe4_pt<P_BF16>(epi, q, st);
    default: return false;
  }
}

bool launch_gemm4_splitk(int ptype, GemvParams p, float* scratch, size_t scratch_n, hipStream_t st, bool reduce,
                         int* nsplit_out) {
  if (p.bias) return false;
  float* Y = p.Y;
  const int ldy = p.ldy;
  int ns = 0;
  if (!gemm4_dispatch(ptype, EPI_STORE, p, false, st, scratch, scratch_n, &ns)) return false;
  if (nsplit_out) *nsplit_out = ns;
  const int ldp = p.ntiles * 16;
  if (reduce) launch_splitk_reduce(scratch, ns, (int64_t)p.M * ldp, ldp, p.M, p.n_valid, Y, ldy, st);
  return true;
}

}  // namespace mp
