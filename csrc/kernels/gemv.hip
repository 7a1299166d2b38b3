// Skinny dequant-GEMM for decode micro-batches (M <= 16 rows of activations).
//
//   Y[m][n] (+)= sum_k X[m][k] * W[n][k]      X: f16 [M][ldx], W: T16-packed quantized weights
//
// One wavefront owns one 16-row tile of W and a contiguous range of 256-k super-blocks; four
// waves per workgroup own four adjacent tiles.  Each lane streams its share of the packed tile
// with 16-B non-temporal loads (double-buffered in registers), dequantizes to f16 in registers
// (dequant.h) and feeds v_mfma_f32_16x16x32_f16 with A = X (rows m), B = W^T (cols n).  The MFMA
// is ~14 % busy at HBM speed: the kernel is weight-bandwidth bound for any M <= 16, so a decode
// micro-batch of 16 sequences costs about the same as one.
// Split-K over super-blocks (grid.y) with f32 atomics into the destination gives >= 2k waves on
// the 256 CUs for every Llama shape; residual adds (Wo, Wdown) atomically accumulate straight
// into the f32 residual stream, and the gate/up projection is packed interleaved (rows 0-7 gate,
// 8-15 up of the same 8 outputs) so SwiGLU is fused in the epilogue (K8/K9 fusion).
#include "kcommon.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"

#include <cstdlib>

namespace mpk {

template <int PT, int EPI, int WPB, int TPW, int NSLOT>
__global__ __launch_bounds__(WPB * 64) void gemv_kernel(const mp::GemvParams p) {
  // TPW tiles per wave share every x fragment (x traffic / weight traffic = 3.5 / TPW at M = 16);
  // NSLOT super-blocks per tile are kept in flight in a compile-time indexed register ring.
  using D = Deq<PT>;
  constexpr int CB = D::CB;
  // WPB waves of a workgroup share the same TPW tiles and split the workgroup's K range among
  // themselves (intra-workgroup split-K, reduced through LDS before the epilogue): more waves per
  // SIMD for the same tiles, no extra x traffic and no atomics.
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int tile0 = blockIdx.x * TPW;
  if (tile0 >= p.ntiles) return;
  const int sbA = blockIdx.y * p.sb_per_split;
  const int sbB = min(sbA + p.sb_per_split, p.nsb);
  if (sbA >= sbB) return;
  const int sb0 = sbA + ((sbB - sbA) * wave) / WPB;
  const int sb1 = sbA + ((sbB - sbA) * (wave + 1)) / WPB;
  const int g = lane >> 4, r = lane & 15;
  const uint8_t* wt[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) wt[t] = p.W + (size_t)min(tile0 + t, p.ntiles - 1) * p.nsb * CB;
  // rows m >= M read row M-1 (clamped address, no exec masking); their outputs are never stored
  const f16* xp = p.X + (size_t)min(r, p.M - 1) * p.ldx + t16_xoff(g, 0);

  f32x4 acc[TPW];
#pragma unroll
  for (int t = 0; t < TPW; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int last = sb1 - 1;
  // Register ring of NSLOT super-blocks; x fragments are fetched at use (an x-in-ring variant
  // measured slower: 32 VGPRs per slot)
  typename D::Raw ring[NSLOT][TPW];
  half8_t xr[1][8];
  auto issue = [&](int sl, int sbi) {
#pragma unroll
    for (int t = 0; t < TPW; ++t) D::load(ring[sl][t], wt[t] + (size_t)sbi * CB, lane);
  };
#pragma unroll
  // (a wave with an empty K share still loads a valid super-block of its workgroup's range)
  for (int sl = 0; sl < NSLOT; ++sl) issue(sl, min(max(sb0, min(sb0 + sl, last)), sbB - 1));

  for (int sb = sb0; sb < sb1; sb += NSLOT) {
#pragma unroll
    for (int sl = 0; sl < NSLOT; ++sl) {
      const int cur = sb + sl;
      if (cur < sb1) {
        if constexpr (EPI == 3) {   // bandwidth probe: consume the raw words, no dequant / MFMA
#pragma unroll
          for (int t = 0; t < TPW; ++t) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(&ring[sl][t]);
            uint32_t h = 0;
#pragma unroll
            for (int i = 0; i < (int)(sizeof(typename D::Raw) / 4); ++i) h ^= w[i];
            acc[t][0] += __uint_as_float(h & 0x3FFFFFFFu);
          }
        } else if constexpr (EPI == 4) {   // probe: weight + x loads, no dequant / MFMA
#pragma unroll
          for (int i = 0; i < 8; ++i) xr[0][i] = *reinterpret_cast<const half8_t*>(xp + (size_t)cur * 256 + 8 * i);
#pragma unroll
          for (int t = 0; t < TPW; ++t) {
            const uint32_t* w = reinterpret_cast<const uint32_t*>(&ring[sl][t]);
            uint32_t h = 0;
#pragma unroll
            for (int i = 0; i < (int)(sizeof(typename D::Raw) / 4); ++i) h ^= w[i];
#pragma unroll
            for (int i = 0; i < 8; ++i) h ^= __builtin_bit_cast(u32x4, xr[0][i]).x;
            acc[t][0] += __uint_as_float(h & 0x3FFFFFFFu);
          }
        } else {
          const int xs = 0;
          if constexpr (EPI == 5) {   // probe: dequant + MFMA on a constant x (no x loads)
            if (cur == sb0) {
#pragma unroll
              for (int i = 0; i < 8; ++i) xr[0][i] = *reinterpret_cast<const half8_t*>(xp + 8 * i);
            }
          } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) xr[0][i] = *reinterpret_cast<const half8_t*>(xp + (size_t)cur * 256 + 8 * i);
          }
#pragma unroll
          for (int t = 0; t < TPW; ++t) {
            half8_t b[4];
            D::template dequant<0>(ring[sl][t], b, lane);
#pragma unroll
            for (int s = 0; s < 4; ++s) acc[t] = mfma16x16x32(xr[xs][s], b[s], acc[t]);
            D::template dequant<1>(ring[sl][t], b, lane);
#pragma unroll
            for (int s = 0; s < 4; ++s) acc[t] = mfma16x16x32(xr[xs][4 + s], b[s], acc[t]);
          }
        }
      }
      // unconditional refill (clamped to the last super-block: an L2 hit) keeps the number of loads
      // in flight path-independent, so the compiler emits exact vmcnt(N) waits, not vmcnt(0)
      issue(sl, min(cur + NSLOT, last));
    }
  }
  if constexpr (WPB > 1) {
    __shared__ f32x4 red[WPB - 1][TPW][64];
    if (wave > 0) {
#pragma unroll
      for (int t = 0; t < TPW; ++t) red[wave - 1][t][lane] = acc[t];
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int w = 0; w < WPB - 1; ++w)
#pragma unroll
      for (int t = 0; t < TPW; ++t) acc[t] += red[w][t][lane];
  }

  // lane holds C[m = 4g + i][n = 16*tile + r]
#pragma unroll
  for (int t = 0; t < TPW; ++t) {
    const int tile = tile0 + t;
    if (tile >= p.ntiles) break;
    if constexpr (EPI == mp::EPI_SWIGLU) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float other = __shfl_xor(acc[t][i], 8);
        const int m = 4 * g + i;
        if (r < 8 && m < p.M) {
          const int o = tile * 8 + r;
          if (o < p.n_valid) p.H[(size_t)m * p.ldh + o] = (f16)(silu(acc[t][i]) * other);
        }
      }
    } else {
      const int n = tile * 16 + r;
      if (n < p.n_valid) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = 4 * g + i;
          if (m < p.M) {
            float* dst = p.Y + (size_t)m * p.ldy + n;
            if constexpr (EPI == mp::EPI_ATOMIC) unsafeAtomicAdd(dst, acc[t][i]);
            else *dst = acc[t][i];
          }
        }
      }
    }
  }
}

// Dense dequantization of a T16-packed matrix back to f16 [N_pad][K_pad] (tests, prefill staging).
template <int PT>
__global__ __launch_bounds__(64) void unpack_kernel(const uint8_t* W, int nsb, f16* out, int ldo) {
  using D = Deq<PT>;
  const int lane = threadIdx.x;
  const int tile = blockIdx.x, sb = blockIdx.y;
  const uint8_t* c = W + ((size_t)tile * nsb + sb) * D::CB;
  typename D::Raw raw;
  D::load(raw, c, lane);
  half8_t b[4];
  const int g = lane >> 4, r = lane & 15;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h == 0) D::template dequant<0>(raw, b, lane);
    else D::template dequant<1>(raw, b, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      f16* o = out + (size_t)(tile * 16 + r) * ldo + sb * 256 + t16_xoff(g, 4 * h + s);
      *reinterpret_cast<half8_t*>(o) = b[s];
    }
  }
}

}  // namespace mpk

namespace mp {

static int g_wpb = 1;   // waves per workgroup (tuning knob, MP_GEMV_WPB)
static int g_tpw = 0;   // tiles per wave: 0 = auto (1 for M <= 4, else 2)

template <int PT, int WPB, int TPW, int NSLOT>
static void launch_cfg(int epi, const GemvParams& p, int nsplit, hipStream_t st) {
  dim3 grid((p.ntiles + TPW - 1) / TPW, nsplit);
  dim3 block(WPB * 64);
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((mpk::gemv_kernel<PT, EPI_STORE, WPB, TPW, NSLOT>), grid, block, 0, st, p); break;
    case EPI_ATOMIC: hipLaunchKernelGGL((mpk::gemv_kernel<PT, EPI_ATOMIC, WPB, TPW, NSLOT>), grid, block, 0, st, p); break;
    case EPI_SWIGLU: hipLaunchKernelGGL((mpk::gemv_kernel<PT, EPI_SWIGLU, WPB, TPW, NSLOT>), grid, block, 0, st, p); break;
    case 3: hipLaunchKernelGGL((mpk::gemv_kernel<PT, 3, WPB, TPW, NSLOT>), grid, block, 0, st, p); break;
    case 4: hipLaunchKernelGGL((mpk::gemv_kernel<PT, 4, WPB, TPW, NSLOT>), grid, block, 0, st, p); break;
    case 5: hipLaunchKernelGGL((mpk::gemv_kernel<PT, 5, WPB, TPW, NSLOT>), grid, block, 0, st, p); break;
  }
}

// Tiles per wave: with M > 4 the x fragments (16 rows x 32 k per MFMA) cost more L1/L2 traffic
// than the weights themselves (3.5x at M = 16); sharing them across tiles pays.  Measured on
// MI355X (tools/gemv_bench.py, 70B shapes): M = 16 gate/up 115 -> 67 us with 4 tiles per wave.
void launch_gemv2(int ptype, int epi, const GemvParams& p, int nsplit, int nw, int tw, hipStream_t st);

// kernel version (MIPIPE_GEMV_V: 1 = per-wave x loads, 2 = workgroup-shared x in LDS, default 2)
// and waves per workgroup of v2 (MIPIPE_GEMV_NW: 4 or 8), tiles per wave of v2 at M > 32
// (MIPIPE_GEMV2_TW: 1 or 2; 0 = auto: 2 for the gate/up SwiGLU GEMV only).  Measured on MI355X
// (profiles/r1g_gemv_tiles_per_wave_ab.txt, 70B Q4_K, M = 64): gate/up 115.9 -> 104.3 us with two
// tiles per wave; the split-K projections (qkv, o, down) gain nothing at their best split.
static int g_ver = -1, g_nw = 8, g_tw2 = 0;
static int gemv2_tw(int M, int epi, int ntiles = 1 << 30) {
  if (M <= 32) return 1;
  if (g_tw2) return g_tw2;
  // two tiles per wave halve the workgroups: only where >= 192 remain (70B gate/up: 224;
  // 8B gate/up would drop to 112 of 256 CUs)
  // (split-free epilogues only: the split-K projections gain nothing; the Q6_K LM head at M = 64:
  // 294 -> 266 us)
  return (epi == EPI_SWIGLU || epi == EPI_STORE) && ntiles / (2 * g_nw) >= 192 ? 2 : 1;
}
static int gemv_version() {
  if (g_ver < 0) {
    const char* e = getenv("MIPIPE_GEMV_V");
    g_ver = e ? atoi(e) : 2;
    if (const char* w = getenv("MIPIPE_GEMV_NW")) g_nw = atoi(w) == 4 ? 4 : 8;
    if (const char* w = getenv("MIPIPE_GEMV2_TW")) g_tw2 = atoi(w) == 2 ? 2 : atoi(w) == 1 ? 1 : 0;
  }
  return g_ver;
}

int gemv_tiles_per_wave(int M, int epi) {
  if (gemv_version() == 2) return gemv2_tw(M, epi);   // v2: x shared through LDS
  if (g_tpw) return g_tpw;
  return M <= 4 ? 1 : 4;
}

template <int PT, int TPW, int NSLOT>
static void launch_ks(int epi, const GemvParams& p, int nsplit, hipStream_t st) {
  if (g_wpb == 4) launch_cfg<PT, 4, TPW, NSLOT>(epi, p, nsplit, st);
  else if (g_wpb == 2) launch_cfg<PT, 2, TPW, NSLOT>(epi, p, nsplit, st);
  else launch_cfg<PT, 1, TPW, NSLOT>(epi, p, nsplit, st);
}

template <int PT>
static void launch_pt(int epi, const GemvParams& p, int nsplit, hipStream_t st) {
  static bool env_done = false;
  if (!env_done) {
    env_done = true;
    if (const char* e = getenv("MIPIPE_GEMV_KS")) g_wpb = atoi(e);
  }
  const int tpw = gemv_tiles_per_wave(p.M, epi);
  if (tpw == 1) launch_ks<PT, 1, 4>(epi, p, nsplit, st);
  else if (tpw == 2) launch_ks<PT, 2, 2>(epi, p, nsplit, st);
  else launch_ks<PT, 4, 2>(epi, p, nsplit, st);
}

void set_gemv_wpb(int w) { g_wpb = (w == 1 || w == 2 || w == 4) ? w : 1; }
void set_gemv_tpw(int t) { g_tpw = (t == 1 || t == 2 || t == 4) ? t : 0; }

void launch_gemv(int ptype, int epi, GemvParams p, int nsplit, hipStream_t st) {
  if (nsplit < 1) nsplit = 1;
  p.sb_per_split = (p.nsb + nsplit - 1) / nsplit;
  nsplit = (p.nsb + p.sb_per_split - 1) / p.sb_per_split;
  if (gemv_version() == 2 && epi < 3 && p.M <= 64) return launch_gemv2(ptype, epi, p, nsplit, g_nw, gemv2_tw(p.M, epi, p.ntiles), st);
  switch (ptype) {
    case P_Q4_K: launch_pt<P_Q4_K>(epi, p, nsplit, st); break;
    case P_Q5_K: launch_pt<P_Q5_K>(epi, p, nsplit, st); break;
    case P_Q6_K: launch_pt<P_Q6_K>(epi, p, nsplit, st); break;
    case P_Q8_0: launch_pt<P_Q8_0>(epi, p, nsplit, st); break;
    case P_Q4_0: launch_pt<P_Q4_0>(epi, p, nsplit, st); break;
    case P_F16: launch_pt<P_F16>(epi, p, nsplit, st); break;
  }
}

void launch_unpack(int ptype, const uint8_t* W, int ntiles, int nsb, f16* out, int ldo, hipStream_t st) {
  dim3 grid(ntiles, nsb);
  switch (ptype) {
    case P_Q4_K: hipLaunchKernelGGL(mpk::unpack_kernel<P_Q4_K>, grid, dim3(64), 0, st, W, nsb, out, ldo); break;
    case P_Q5_K: hipLaunchKernelGGL(mpk::unpack_kernel<P_Q5_K>, grid, dim3(64), 0, st, W, nsb, out, ldo); break;
    case P_Q6_K: hipLaunchKernelGGL(mpk::unpack_kernel<P_Q6_K>, grid, dim3(64), 0, st, W, nsb, out, ldo); break;
    case P_Q8_0: hipLaunchKernelGGL(mpk::unpack_kernel<P_Q8_0>, grid, dim3(64), 0, st, W, nsb, out, ldo); break;
    case P_Q4_0: hipLaunchKernelGGL(mpk::unpack_kernel<P_Q4_0>, grid, dim3(64), 0, st, W, nsb, out, ldo); break;
    case P_F16: hipLaunchKernelGGL(mpk::unpack_kernel<P_F16>, grid, dim3(64), 0, st, W, nsb, out, ldo); break;
  }
}

}  // namespace mp
