// LDS-DMA staging machinery shared by the wide dequant GEMMs (gemm3.hip, gemm4.hip): global ->
// LDS DMA with counted vmcnt, inline-asm LDS reads with counted lgkmcnt, and the per-type raw
// weight images of one wave's tiles for one 64-k stage (W3<PT>: issue / load / prep / frag in the
// 16x16x32 lane mapping; gemm4.hip adds the 32x32x16 mapping over the same images).
#pragma once
#include "kcommon.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"

#include <utility>

namespace mpk {
using namespace mp;

typedef __attribute__((address_space(3))) void lds_t;

__device__ __forceinline__ int g3_swz(int row) { return (row >> 1) & 7; }
__device__ __forceinline__ int g3_off(int row, int c) { return row * 128 + ((c ^ g3_swz(row)) << 4); }

// global -> LDS DMA of SZ (16 | 4) bytes per lane (LDS destination: wave-uniform base + lane * SZ;
// the sub-dword forms are not used: they land a dword per lane).  Issued as inline asm on purpose:
// the compiler's own form (__builtin_amdgcn_global_load_lds) makes hipcc wait vmcnt(0) before the
// first ds_read after it (it cannot tell which LDS bytes a DMA writes), which drains the whole
// prefetch pipeline every stage.  These loads are invisible to the compiler's waitcnt pass: every
// wait on them is the kernel's own counted s_waitcnt vmcnt (wait_vmcnt) before a barrier.
// LDS byte address of a generic pointer into a __shared__ array: its low 32 bits (a generic LDS
// address is the shared aperture in the high half and the LDS offset in the low half).  Not an
// address-space cast: that one null-checks the 64-bit pointer (s_cmp_lg_u64 + s_cselect per DMA /
// read address, 14 scalar instructions of gemm4's 2-stage loop)
__device__ __forceinline__ uint32_t lds_off(const void* p) { return (uint32_t)(uintptr_t)p; }

// m0 (the DMA's LDS base) is an input operand bound to the register ("{m0}"), not a clobber: the
// compiler then knows what m0 holds (a clobbered m0 is a reserved register it does not preserve,
// -Winline-asm).  The s_nop covers the m0 write -> LDS-DMA hazard, which the compiler's hazard
// recognizer does not see through the asm.
template <int SZ>
__device__ __forceinline__ void glds(const void* g, char* lds) {
  static_assert(SZ == 16 || SZ == 4, "glds: 16 or 4 bytes per lane");
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds));
  if constexpr (SZ == 16)
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
  else
    asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}
// the same with the non-temporal policy when nt (wave-uniform): streamed weights that one workgroup
// reads once, so they do not evict the x rows every column group re-reads from L2
template <int SZ>
__device__ __forceinline__ void glds(bool nt, const void* g, char* lds) {
  if (!nt) return glds<SZ>(g, lds);
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds));
  if constexpr (SZ == 16)
    asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off nt" ::"v"(g), "{m0}"(m0) : "memory");
  else
    asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off nt" ::"v"(g), "{m0}"(m0) : "memory");
}
// one LDS-DMA wave instruction whose lanes >= n are masked off (every wave issues it: uniform
// vmcnt accounting)
template <int SZ, class F>
__device__ __forceinline__ void glds_n(bool nt, char* lds, int n, int lane, F src) {
  if (lane < n) glds<SZ>(nt, src(lane), lds);
}

// The same DMA with the address split into a wave-uniform 64-bit base (SGPRs) and a per-lane
// 32-bit byte offset (the saddr form): a stage's loads then cost one scalar base per instruction and
// no per-lane 64-bit address arithmetic (v_mad_u64_u32 / v_lshl_add_u64 on the MFMA waves' VALU)
template <int SZ>
__device__ __forceinline__ void glds_s(bool nt, const void* sbase, uint32_t voff, char* lds) {
  static_assert(SZ == 16 || SZ == 4, "glds_s: 16 or 4 bytes per lane");
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds_off(lds));
  if (nt) {
    if constexpr (SZ == 16)
      asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1 nt" ::"v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
    else
      asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, %1 nt" ::"v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
  } else {
    if constexpr (SZ == 16)
      asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" ::"v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
    else
      asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, %1" ::"v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
  }
}
// a wave-uniform pointer in SGPRs
__device__ __forceinline__ const uint8_t* uniform_ptr(const void* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const uint8_t*>((uintptr_t)(((uint64_t)hi << 32) | lo));
}

// Emitters of the per-type DMA schedules (W3<PT>::issue): instruction i moves SZ bytes for lanes
// < n from src(lane) to lds + SZ * lane.
//   EmitDirect: the DMA itself (64-bit per-lane addresses).
//   EmitRecord: records lane offsets src(lane) - base at (sb, q) = (0, 0) and lane 0's, once per
//               kernel: the schedule's addresses are (lane-independent stage delta) + (stage-
//               independent lane offset).
//   EmitSaddr:  the DMA from scalar base src(0)@(sb, q) - lane0 offset and the recorded lane offset.
// A schedule entry of n > 64 lanes (TW = 4: 128 quant pieces) is ceil(n / 64) wave instructions,
// entries 64 k .. 64 k + 63 to lds + 64 k SZ (W3<PT>::NI counts them so).
struct EmitDirect {
  bool nt;
  int lane;
  template <int SZ, class F>
  __device__ __forceinline__ void go(char* lds, int n, F src) {
#pragma unroll
    for (int k = 0; 64 * k < n; ++k)
      glds_n<SZ>(nt, lds + 64 * k * SZ, n - 64 * k, lane, [&](int e) { return src(64 * k + e); });
  }
};
template <int NI>
struct EmitRecord {
  const uint8_t* base;
  int lane;
  uint32_t* off;     // [NI] per-lane
  uint32_t* off0;    // [NI] lane 0's (uniform)
  int i = 0;
  template <int SZ, class F>
  __device__ __forceinline__ void go(char*, int n, F src) {
#pragma unroll
    for (int k = 0; 64 * k < n; ++k) {
      const int nk = min(64, n - 64 * k);
      off[i] = (uint32_t)(reinterpret_cast<const uint8_t*>(src(64 * k + min(lane, nk - 1))) - base);
      off0[i] = __builtin_amdgcn_readfirstlane((uint32_t)(reinterpret_cast<const uint8_t*>(src(64 * k)) - base));
      ++i;
    }
  }
};
template <int NI>
struct EmitSaddr {
  bool nt;
  int lane;
  const uint32_t* off;
  const uint32_t* off0;
  int i = 0;
  template <int SZ, class F>
  __device__ __forceinline__ void go(char* lds, int n, F src) {
#pragma unroll
    for (int k = 0; 64 * k < n; ++k) {
      const uint8_t* sb = uniform_ptr(reinterpret_cast<const uint8_t*>(src(64 * k)) - off0[i]);
      if (lane < n - 64 * k) glds_s<SZ>(nt, sb, off[i], lds + 64 * k * SZ);
      ++i;
    }
  }
};
// wave instructions of a schedule entry of n lanes
constexpr int wi(int n) { return (n + 63) / 64; }

// s_waitcnt vmcnt(N) (expcnt / lgkmcnt left at their maxima), gfx9 encoding
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
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

// 8 nibbles of a dword (T16 order: j = 2i at bit 4i, 2i+1 at bit 16 + 4i) -> 8 f16 = S q + M
__device__ __forceinline__ half8_t nib8(uint32_t w, half2_t S, half2_t M, const Consts& k) {
  const uint32_t t = w >> 8;
  return pack8(as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mlo, k.mag_hi)) - h2c(1024.f), S, M)),
               as_u32(__builtin_elementwise_fma(as_h2(and_or(w, k.mhi, k.mag_lo)) - h2c(64.f), S, M)),
               as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mlo, k.mag_hi)) - h2c(1024.f), S, M)),
               as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mhi, k.mag_lo)) - h2c(64.f), S, M)));
}

// ---------------------------------------------------------------------------------------------
// Per-type raw image of ONE wave for one stage: its TW tiles (u < TW) x quarter q of super-block sb.
// The MFMA B fragment of k-half kk (32 k) for lane l = 16 g + r is column r of the tile, k = 32 kk
// + 8 g + j: in the T16 chunk that is dword g of row r's 16-B piece of half h = kk (dequant.h).
//   issue():  NI(TW) LDS-DMA wave instructions (uniform per wave)
//   prep():   per-stage, per-tile values (scales) of this lane's row
//   frag():   the B fragment (u, kk)
struct W3Src {
  const uint8_t* W;
  int t0, ntiles, nsb, sb, q;   // t0: the wave's first tile
  bool nt = false;              // non-temporal weight DMA
  __device__ __forceinline__ const uint8_t* chunk(int u, int CB) const {
    const int t = min(t0 + u, ntiles - 1);
    return W + ((size_t)t * nsb + sb) * CB;
  }
};

template <int PT> struct W3;

// LDS reads issued as inline asm (the kernel counts lgkmcnt itself, so A fragments can be kept
// in flight AD deep: left to the compiler, each ds_read was followed by lgkmcnt(0) before its two
// MFMAs -- one LDS round trip per 32 MFMA cycles)
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return lds_off(p); }
__device__ __forceinline__ void ds_b32(uint32_t& v, const void* p) {
  asm volatile("ds_read_b32 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
}
__device__ __forceinline__ void ds_u16(uint32_t& v, const void* p) {
  asm volatile("ds_read_u16 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
}
__device__ __forceinline__ void ds_b64(u32x2& v, const void* p) {
  asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
}
__device__ __forceinline__ void ds_b128(u32x4& v, const void* p) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(p)) : "memory");
}
template <int OFF>   // immediate byte offset on an LDS address
__device__ __forceinline__ void ds_b128o(u32x4& v, uint32_t addr) {
  static_assert(OFF >= 0 && OFF < 65536, "ds offset");
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
}
// compile-time loop: f(std::integral_constant<int, J>) for J < N
template <class F, int... J>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, J...>) {
  (f(std::integral_constant<int, J>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) { static_for_impl(f, std::make_integer_sequence<int, N>{}); }

// s_waitcnt lgkmcnt(N) (vmcnt / expcnt at their maxima) + a scheduling fence: the compiler does not
// know the asm reads' results arrive late, so nothing may move above the wait
template <int N>
__device__ __forceinline__ void wait_lgkm() {
  static_assert(N >= 0 && N < 16, "lgkmcnt");
  __builtin_amdgcn_s_waitcnt(0xC07F | (N << 8));
  __builtin_amdgcn_sched_barrier(0);
}

// Q4_K: quants [u][h][r] 16 B, header [u][r] 16 B
template <> struct W3<P_Q4_K> {
  static constexpr int CB = chunk_bytes(P_Q4_K);
  static constexpr int RAW(int TW) { return TW * 768; }
  static constexpr int NI(int TW) { return wi(32 * TW) + wi(16 * TW); }
  static constexpr int NR(int TW) { return 3 * TW; }
  template <int TW> struct Raw { u32x4 hdr[TW]; uint32_t q[TW][2]; };
  struct Prep { half2_t S2, M2; };
  template <int TW, class E>
  __device__ static __forceinline__ void issue(char* R, const W3Src& c, E&& em) {
    em.template go<16>(R, 32 * TW, [&](int e) {
      return c.chunk(e >> 5, CB) + ((e >> 4) & 1) * 1024 + (16 * c.q + (e & 15)) * 16;
    });
    em.template go<16>(R + TW * 512, 16 * TW, [&](int e) { return c.chunk(e >> 4, CB) + 2048 + (e & 15) * 16; });
  }
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, Raw<TW>& w) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      ds_b128(w.hdr[u], R + TW * 512 + (u * 16 + r) * 16);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) ds_b32(w.q[u][kk], R + ((u * 2 + kk) * 16 + r) * 16 + 4 * g);
    }
  }
  template <int TW>
  __device__ static __forceinline__ Prep prep(const Raw<TW>& w, int u, int q, int) {
    Prep p;
    kq_scales(w.hdr[u], (uint32_t)q, p.S2, p.M2);
    return p;
  }
  template <int TW>
  __device__ static __forceinline__ half8_t frag(const Raw<TW>& w, const Prep& p, int u, int kk, int, const Consts& k) {
    return nib8(w.q[u][kk], kk ? h2hi(p.S2) : h2lo(p.S2), kk ? h2hi(p.M2) : h2lo(p.M2), k);
  }
};

// Q5_K: quants [u][h][r] 16 B, high bits [u][h][r] 4 B, header [u][r] 16 B
template <> struct W3<P_Q5_K> {
  static constexpr int CB = chunk_bytes(P_Q5_K);
  static constexpr int RAW(int TW) { return TW * 896; }
  static constexpr int NI(int TW) { return wi(32 * TW) + wi(8 * TW) + wi(16 * TW); }
  static constexpr int NR(int TW) { return 5 * TW; }
  template <int TW> struct Raw { u32x4 hdr[TW]; uint32_t q[TW][2], qh[TW][2]; };
  struct Prep { half2_t S2, M2; };
  template <int TW, class E>
  __device__ static __forceinline__ void issue(char* R, const W3Src& c, E&& em) {
    em.template go<16>(R, 32 * TW, [&](int e) {
      return c.chunk(e >> 5, CB) + ((e >> 4) & 1) * 1024 + (16 * c.q + (e & 15)) * 16;
    });
    // 16-B entries = 4 rows' high-bit words: entry f -> (u, h, rows 4 (f & 3) ..)
    em.template go<16>(R + TW * 512, 8 * TW, [&](int f) {
      return c.chunk(f >> 3, CB) + 2048 + ((f >> 2) & 1) * 256 + (16 * c.q + 4 * (f & 3)) * 4;
    });
    em.template go<16>(R + TW * 640, 16 * TW, [&](int e) { return c.chunk(e >> 4, CB) + 2560 + (e & 15) * 16; });
  }
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, Raw<TW>& w) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      ds_b128(w.hdr[u], R + TW * 640 + (u * 16 + r) * 16);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        ds_b32(w.q[u][kk], R + ((u * 2 + kk) * 16 + r) * 16 + 4 * g);
        ds_b32(w.qh[u][kk], R + TW * 512 + ((u * 2 + kk) * 16 + r) * 4);
      }
    }
  }
  template <int TW>
  __device__ static __forceinline__ Prep prep(const Raw<TW>& w, int u, int q, int) {
    Prep p;
    kq_scales(w.hdr[u], (uint32_t)q, p.S2, p.M2);
    return p;
  }
  template <int TW>
  __device__ static __forceinline__ half8_t frag(const Raw<TW>& w, const Prep& p, int u, int kk, int lane, const Consts& k) {
    const int g = lane >> 4;
    const uint32_t hb = (w.qh[u][kk] >> (8 * g)) & 0xFFu;
    const uint32_t x = hb | (hb << 12);
    const half2_t S = kk ? h2hi(p.S2) : h2lo(p.S2), M = kk ? h2hi(p.M2) : h2lo(p.M2);
    const uint32_t v = w.q[u][kk], t = v >> 8;
    const uint32_t h0 = ((x << 4) & 0x00100010u) | k.mag_hi, h1 = ((x << 7) & 0x01000100u) | k.mag_lo;
    const uint32_t h2 = ((x << 2) & 0x00100010u) | k.mag_hi, h3 = ((x << 5) & 0x01000100u) | k.mag_lo;
    return pack8(as_u32(__builtin_elementwise_fma(as_h2(and_or(v, k.mlo, h0)) - h2c(1024.f), S, M)),
                 as_u32(__builtin_elementwise_fma(as_h2(and_or(v, k.mhi, h1)) - h2c(64.f), S, M)),
                 as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mlo, h2)) - h2c(1024.f), S, M)),
                 as_u32(__builtin_elementwise_fma(as_h2(and_or(t, k.mhi, h3)) - h2c(64.f), S, M)));
  }
};

// Q6_K: quants [u][h][r] 16 B, high bits [u][h][r] 8 B, int8 scales [u][r] 4 B (dword q of the
// row's 16), d [u][r] 2 B (per tile the 32 contiguous bytes, two 16-B entries)
template <> struct W3<P_Q6_K> {
  static constexpr int CB = chunk_bytes(P_Q6_K);
  static constexpr int RAW(int TW) { return TW * 896; }
  static constexpr int NI(int TW) { return wi(32 * TW) + wi(16 * TW) + wi(16 * TW) + wi(2 * TW); }
  static constexpr int NR(int TW) { return 6 * TW; }
  template <int TW> struct Raw { uint32_t sc[TW], d[TW], q[TW][2], qd[TW][2]; };
  struct Prep { uint32_t sc; f16 d; };
  template <int TW, class E>
  __device__ static __forceinline__ void issue(char* R, const W3Src& c, E&& em) {
    em.template go<16>(R, 32 * TW, [&](int e) {
      return c.chunk(e >> 5, CB) + ((e >> 4) & 1) * 1024 + (16 * c.q + (e & 15)) * 16;
    });
    em.template go<16>(R + TW * 512, 16 * TW, [&](int f) {   // (u, h): 16 rows x 8 B contiguous
      return c.chunk(f >> 4, CB) + 2048 + ((f >> 3) & 1) * 512 + 16 * c.q * 8 + (f & 7) * 16;
    });
    em.template go<4>(R + TW * 768, 16 * TW, [&](int e) { return c.chunk(e >> 4, CB) + 3072 + (e & 15) * 16 + 4 * c.q; });
    em.template go<16>(R + TW * 832, 2 * TW, [&](int f) { return c.chunk(f >> 1, CB) + 3328 + (f & 1) * 16; });
  }
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, Raw<TW>& w) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      ds_b32(w.sc[u], R + TW * 768 + (u * 16 + r) * 4);
      ds_u16(w.d[u], R + TW * 832 + (u * 16 + r) * 2);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        ds_b32(w.q[u][kk], R + ((u * 2 + kk) * 16 + r) * 16 + 4 * g);
        ds_b32(w.qd[u][kk], R + TW * 512 + ((u * 2 + kk) * 16 + r) * 8 + 4 * (g >> 1));
      }
    }
  }
  template <int TW>
  __device__ static __forceinline__ Prep prep(const Raw<TW>& w, int u, int, int) {
    return Prep{w.sc[u] ^ 0x80808080u, __builtin_bit_cast(f16, (uint16_t)w.d[u])};
  }
  template <int TW>
  __device__ static __forceinline__ half8_t frag(const Raw<TW>& w, const Prep& p, int u, int kk, int lane, const Consts& k) {
    const int g = lane >> 4;
    const uint32_t h16 = (w.qd[u][kk] >> (16 * (g & 1))) & 0xFFFFu;
    // int8 scale of sub-block 4q + 2kk + (g >> 1): byte 2kk + (g >> 1) of the dword, (sc + 128) by
    // the exponent magic, minus 1152, times d
    const uint32_t sb = (p.sc >> (8 * (2 * kk + (g >> 1)))) & 0xFFu;
    const f16 sf = (as_h2(0x6400u | sb).x - (f16)1152.f) * p.d;
    const half2_t S = half2_t{sf, sf};
    const uint32_t x = h16 | (h16 << 8);
    const uint32_t v = w.q[u][kk], t = v >> 8;
    const uint32_t h0 = ((x << 4) & 0x00300030u) | k.mag_hi, h1 = ((x << 6) & 0x03000300u) | k.mag_lo;
    const uint32_t h2 = (x & 0x00300030u) | k.mag_hi, h3 = ((x << 2) & 0x03000300u) | k.mag_lo;
    return pack8(as_u32((as_h2(and_or(v, k.mlo, h0)) - h2c(1056.f)) * S),
                 as_u32((as_h2(and_or(v, k.mhi, h1)) - h2c(96.f)) * S),
                 as_u32((as_h2(and_or(t, k.mlo, h2)) - h2c(1056.f)) * S),
                 as_u32((as_h2(and_or(t, k.mhi, h3)) - h2c(96.f)) * S));
  }
};

// Q8_0: quants [u][h][r] 32 B (int8 + 128), block scales [u][r] 4 B = (d(2q), d(2q+1))
template <> struct W3<P_Q8_0> {
  static constexpr int CB = chunk_bytes(P_Q8_0);
  static constexpr int RAW(int TW) { return TW * 1088; }
  static constexpr int NI(int TW) { return TW + wi(16 * TW); }
  static constexpr int NR(int TW) { return 3 * TW; }
  template <int TW> struct Raw { uint32_t dd[TW]; u32x2 v[TW][2]; };
  struct Prep { uint32_t dd; };
  template <int TW, class E>
  __device__ static __forceinline__ void issue(char* R, const W3Src& c, E&& em) {
#pragma unroll
    for (int u = 0; u < TW; ++u)   // 64 entries of 16 B per tile: (h, r, half)
      em.template go<16>(R + u * 1024, 64, [&](int l) { return c.chunk(u, CB) + (l >> 5) * 2048 + (16 * c.q + ((l >> 1) & 15)) * 32 + 16 * (l & 1); });
    em.template go<4>(R + TW * 1024, 16 * TW, [&](int e) { return c.chunk(e >> 4, CB) + 4096 + (e & 15) * 16 + 4 * c.q; });
  }
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, Raw<TW>& w) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      ds_b32(w.dd[u], R + TW * 1024 + (u * 16 + r) * 4);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) ds_b64(w.v[u][kk], R + ((u * 2 + kk) * 16 + r) * 32 + 8 * g);
    }
  }
  template <int TW>
  __device__ static __forceinline__ Prep prep(const Raw<TW>& w, int u, int, int) { return Prep{w.dd[u]}; }
  template <int TW>
  __device__ static __forceinline__ half8_t frag(const Raw<TW>& w, const Prep& p, int u, int kk, int, const Consts&) {
    const u32x2 v = w.v[u][kk];
    const half2_t off = h2c(1152.f);
    const half2_t S = kk ? h2hi(as_h2(p.dd)) : h2lo(as_h2(p.dd));
    return pack8(as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, v.x, 0x04010400u)) - off) * S),
                 as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, v.x, 0x04030402u)) - off) * S),
                 as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, v.y, 0x04010400u)) - off) * S),
                 as_u32((as_h2(__builtin_amdgcn_perm(0x64646464u, v.y, 0x04030402u)) - off) * S));
  }
};

// Q4_0: quants [u][h][r] 16 B, block scales [u][r] 4 B = (d(2q), d(2q+1))
template <> struct W3<P_Q4_0> {
  static constexpr int CB = chunk_bytes(P_Q4_0);
  static constexpr int RAW(int TW) { return TW * 576; }
  static constexpr int NI(int TW) { return wi(32 * TW) + wi(16 * TW); }
  static constexpr int NR(int TW) { return 3 * TW; }
  template <int TW> struct Raw { uint32_t dd[TW], q[TW][2]; };
  struct Prep { uint32_t dd; };
  template <int TW, class E>
  __device__ static __forceinline__ void issue(char* R, const W3Src& c, E&& em) {
    em.template go<16>(R, 32 * TW, [&](int e) {
      return c.chunk(e >> 5, CB) + ((e >> 4) & 1) * 1024 + (16 * c.q + (e & 15)) * 16;
    });
    em.template go<4>(R + TW * 512, 16 * TW, [&](int e) { return c.chunk(e >> 4, CB) + 2048 + (e & 15) * 16 + 4 * c.q; });
  }
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, Raw<TW>& w) {
    const int r = lane & 15, g = lane >> 4;
#pragma unroll
    for (int u = 0; u < TW; ++u) {
      ds_b32(w.dd[u], R + TW * 512 + (u * 16 + r) * 4);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) ds_b32(w.q[u][kk], R + ((u * 2 + kk) * 16 + r) * 16 + 4 * g);
    }
  }
  template <int TW>
  __device__ static __forceinline__ Prep prep(const Raw<TW>& w, int u, int, int) { return Prep{w.dd[u]}; }
  template <int TW>
  __device__ static __forceinline__ half8_t frag(const Raw<TW>& w, const Prep& p, int u, int kk, int, const Consts& k) {
    const half2_t S = kk ? h2hi(as_h2(p.dd)) : h2lo(as_h2(p.dd));
    const uint32_t v = w.q[u][kk], t = v >> 8;
    return pack8(as_u32((as_h2(and_or(v, k.mlo, k.mag_hi)) - h2c(1032.f)) * S),
                 as_u32((as_h2(and_or(v, k.mhi, k.mag_lo)) - h2c(72.f)) * S),
                 as_u32((as_h2(and_or(t, k.mlo, k.mag_hi)) - h2c(1032.f)) * S),
                 as_u32((as_h2(and_or(t, k.mhi, k.mag_lo)) - h2c(72.f)) * S));
  }
};

// 16-bit weights (F16, or BF16 for the bf16 MFMA: the A fragments go to bf16): the fragment bytes themselves,
// [u][kk][lane] 16 B = element 4 kk + g of lane (q, r) of the T16 chunk
template <int PT> struct W3_16 {
  static constexpr int CB = chunk_bytes(PT);
  static constexpr int RAW(int TW) { return TW * 2048; }
  static constexpr int NI(int TW) { return 2 * TW; }
  static constexpr int NR(int TW) { return 2 * TW; }
  template <int TW> struct Raw { u32x4 v[TW][2]; };
  struct Prep {};
  template <int TW, class E>
  __device__ static __forceinline__ void issue(char* R, const W3Src& c, E&& em) {
#pragma unroll
    for (int f = 0; f < 2 * TW; ++f)
      em.template go<16>(R + f * 1024, 64, [&](int l) { return c.chunk(f >> 1, CB) + (4 * (f & 1) + (l >> 4)) * 1024 + (16 * c.q + (l & 15)) * 16; });
  }
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, Raw<TW>& w) {
#pragma unroll
    for (int u = 0; u < TW; ++u)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) ds_b128(w.v[u][kk], R + (u * 2 + kk) * 1024 + lane * 16);
  }
  template <int TW>
  __device__ static __forceinline__ Prep prep(const Raw<TW>&, int, int, int) { return Prep{}; }
  template <int TW>
  __device__ static __forceinline__ half8_t frag(const Raw<TW>& w, const Prep&, int u, int kk, int, const Consts&) {
    return __builtin_bit_cast(half8_t, w.v[u][kk]);
  }
};
template <> struct W3<P_F16> : W3_16<P_F16> {};
template <> struct W3<P_BF16> : W3_16<P_BF16> {};

// int8 weights (P_I8, the int8-activation prototype): 16 rows x 256 k int8 per chunk,
// 16-B piece (st, kk, lane) at ((2 st + kk) * 64 + lane) * 16 holding row r = lane & 15,
// k = 128 st + 64 kk + 16 (lane >> 4) + j.  Stages are 128 k (two per super-block): the A image
// keeps its 128-byte rows (128 int8 activations), and one k-half kk is one v_mfma_i32_16x16x64_i8
// (A and B index k the same way inside the 64, which is all a dot product needs).
template <> struct W3<P_I8> {
  static constexpr int CB = chunk_bytes(P_I8);
  static constexpr int RAW(int TW) { return TW * 2048; }
  static constexpr int NI(int TW) { return 2 * TW; }
  static constexpr int NR(int TW) { return 2 * TW; }
  template <int TW> struct Raw { u32x4 v[TW][2]; };
  struct Prep {};
  template <int TW, class E>
  __device__ static __forceinline__ void issue(char* R, const W3Src& c, E&& em) {
#pragma unroll
    for (int f = 0; f < 2 * TW; ++f)
      em.template go<16>(R + f * 1024, 64, [&](int l) { return c.chunk(f >> 1, CB) + ((2 * c.q + (f & 1)) * 64 + l) * 16; });
  }
  template <int TW>
  __device__ static __forceinline__ void load(const char* R, int lane, Raw<TW>& w) {
#pragma unroll
    for (int u = 0; u < TW; ++u)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) ds_b128(w.v[u][kk], R + (u * 2 + kk) * 1024 + lane * 16);
  }
  template <int TW>
  __device__ static __forceinline__ Prep prep(const Raw<TW>&, int, int, int) { return Prep{}; }
  template <int TW>
  __device__ static __forceinline__ half8_t frag(const Raw<TW>& w, const Prep&, int u, int kk, int, const Consts&) {
    return __builtin_bit_cast(half8_t, w.v[u][kk]);
  }
};
// stages per 256-k super-block: 64 k per stage for 16-bit activations, 128 for int8 ones
template <int PT> constexpr int g3_spb() { return PT == P_I8 ? 2 : 4; }

#define G3_AD(BM, TW) 8
template <int PT, int BM, int TW>
struct G3Geom {
  static constexpr int A_BYTES = BM * 128;                    // x rows of one stage
  static constexpr int R_WAVE = W3<PT>::RAW(TW);             // one wave's raw bytes of one stage
  static constexpr int STAGE = A_BYTES + 8 * R_WAVE;
  static constexpr int NB = 3 * STAGE <= 160 * 1024 ? 3 : 2;  // pipeline depth (stages in LDS)
  static constexpr int A_INSTR = BM / 64;                     // 1-KB A pieces per wave per stage
  static constexpr int LOADS = A_INSTR + W3<PT>::NI(TW);      // LDS-DMA instructions per wave per stage
};

}  // namespace mpk
