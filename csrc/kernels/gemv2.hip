// Decode GEMV v2: workgroup-shared activations.
//
// Measured on MI355X (tools/gemv_bench.py probes, 70B gate/up, 264 MB Q4_K): weight loads alone
// stream at 6-6.6 TB/s; dequant + MFMA alone (no x loads) at ~4.9 TB/s with one tile per wave;
// but per-wave x fragment loads (8 x 1 KB wave-instructions per super-block, 16 rows at M = 16)
// tripled the time at one tile per wave: the texture-address path, not HBM, was the limit.
// v2 therefore keeps one 16-row weight tile per wave (best VALU/MFMA issue: several waves per
// SIMD) and stages x ONCE per workgroup of NW waves into LDS (one 16 B load per thread per
// super-block for 16 rows), from which every wave reads its A fragments with ds_read_b128.
//
//   grid (ceil(ntiles / NW), nsplit)   block NW * 64
//   wave w of workgroup b: tile b*NW + w, super-blocks [sbA, sbB) of split blockIdx.y
//
// Ordering: x(sb+1) is issued BEFORE the weight refill of the current step, so waiting for it
// (vmcnt) never drains the weight prefetches issued after it (vmcnt retires in issue order).
#include "kcommon.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"

#include <cstdlib>

namespace mpk {
using namespace mp;

// x tile in LDS: padded f16 rows (528 B) and the quarters of rows 8..15 (mod 16) swapped in pairs
// (k-quarter q of row m stored at quarter q ^ ((m >> 3) & 1)).  The padding alone left every
// ds_read_b128 of an A fragment 2-way bank-conflicted (its lane groups {0-3,12-15,20-27}.. mix
// rows r and r + 8 of two quarters: SQ_LDS_BANK_CONFLICT = 44 % of SQ_LDS_IDX_ACTIVE); with the
// swap the 16 lanes of each group cover the 64 banks exactly once.  The 8-lane groups of the
// ds_write_b128 staging stay within one row and one quarter: conflict-free as before.
constexpr int G2_LDX = 256 + 8;

// MT row groups of 16 activation rows (M <= 16 MT) share every dequantized weight fragment: the
// dequant VALU work, which bounds the kernel near HBM speed at M = 16, is paid once for 16 MT rows.
// TW weight tiles per wave share every A fragment read from LDS (and a workgroup of NW waves then
// stages x once for NW * TW tiles): at M = 64 one tile per wave reads 14x more bytes of x (LDS and
// L2 -> CU) than of weights.
template <int PT, int EPI, int NW, int NSLOT, int MT, int TW>
__global__ __launch_bounds__(NW * 64) void gemv2_kernel(const GemvParams p) {
  using D = Deq<PT>;
  constexpr int CB = D::CB;
  constexpr int NT = NW * 64;
  constexpr int XC = 512 * MT;   // 16 B x chunks per super-block
  __shared__ __attribute__((aligned(16))) f16 xs[2][16 * MT * G2_LDX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int tile0 = (blockIdx.x * NW + wave) * TW;
  const int sbA = blockIdx.y * p.sb_per_split;
  const int sbB = min(sbA + p.sb_per_split, p.nsb);
  if (sbA >= sbB) return;   // uniform over the workgroup
  const uint8_t* wt[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) wt[t] = p.W + (size_t)min(tile0 + t, p.ntiles - 1) * p.nsb * CB;
  const int M = p.M;

  // x staging: 16 MT rows x 256 k per super-block = 512 MT chunks of 16 B; thread t owns chunks t, t+NT..
  // The x chunks of super-block j are loaded TOGETHER with its weights (register rings of NSLOT),
  // NSLOT steps ahead, and copied to LDS one step before use: every vmcnt wait then leaves the
  // loads of the NSLOT-1 later super-blocks in flight.
  constexpr int XCH = (XC + NT - 1) / NT;
  u32x4 xv[NSLOT][XCH];
  typename D::Raw ring[NSLOT][TW];
  const int last = sbB - 1;
  auto issue = [&](const int sl, const int sb) {
#pragma unroll
    for (int t = 0; t < TW; ++t) D::load(ring[sl][t], wt[t] + (size_t)sb * CB, lane);
#pragma unroll
    for (int j = 0; j < XCH; ++j) {
      const int c = tid + NT * j;
      if (c < XC) {
        const int row = c >> 5, col = (c & 31) * 8;
        xv[sl][j] = row < M ? *reinterpret_cast<const u32x4*>(p.X + (size_t)row * p.ldx + (size_t)sb * 256 + col)
                            : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  auto store_x = [&](const int sl, const int buf) {
#pragma unroll
    for (int j = 0; j < XCH; ++j) {
      const int c = tid + NT * j;
      if (c < XC) {
        const int row = c >> 5, col = (c & 31) * 8;
        *reinterpret_cast<u32x4*>(&xs[buf][row * G2_LDX + (col ^ x_qswap(row))]) = xv[sl][j];
      }
    }
  };

  f32x4 acc[TW][MT];
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sl = 0; sl < NSLOT; ++sl) issue(sl, min(sbA + sl, last));
  store_x(0, 0);
  __syncthreads();

  // rows >= M are zero in LDS (their outputs are never stored)
  const f16* xrow0 = &xs[0][r * G2_LDX + (t16_xoff(g, 0) ^ x_qswap(r))];
  const f16* xrow1 = &xs[1][r * G2_LDX + (t16_xoff(g, 0) ^ x_qswap(r))];
  // one super-block; all loads unconditional (clamped to the range): path-independent vmcnt
  auto step = [&](const int sl, const int cur) {
    const int buf = (cur - sbA) & 1;
    const f16* xr = buf ? xrow1 : xrow0;
    half8_t b[TW][4];
#pragma unroll
    for (int t = 0; t < TW; ++t) D::template dequant<0>(ring[sl][t], b[t], lane);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const half8_t a = *reinterpret_cast<const half8_t*>(xr + mt * 16 * G2_LDX + 8 * s);
#pragma unroll
        for (int t = 0; t < TW; ++t) acc[t][mt] = mfma16x16x32(a, b[t][s], acc[t][mt]);
      }
#pragma unroll
    for (int t = 0; t < TW; ++t) D::template dequant<1>(ring[sl][t], b[t], lane);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const half8_t a = *reinterpret_cast<const half8_t*>(xr + mt * 16 * G2_LDX + 32 + 8 * s);
#pragma unroll
        for (int t = 0; t < TW; ++t) acc[t][mt] = mfma16x16x32(a, b[t][s], acc[t][mt]);
      }
    store_x((sl + 1) % NSLOT, buf ^ 1);   // x(cur + 1), loaded NSLOT - 1 steps ago
    issue(sl, min(cur + NSLOT, last));
    __syncthreads();
  };
  int sb = sbA;
  for (; sb + NSLOT <= sbB; sb += NSLOT) {
#pragma unroll
    for (int sl = 0; sl < NSLOT; ++sl) step(sl, sb + sl);
  }
#pragma unroll
  for (int sl = 0; sl < NSLOT - 1; ++sl)   // tail (< NSLOT super-blocks; uniform over the workgroup)
    if (sb + sl < sbB) step(sl, sb + sl);
  // lane holds C[m = 16 mt + 4g + i][n = 16*tile + r]
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int tile = tile0 + t;
    if (tile >= p.ntiles) break;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      if constexpr (EPI == EPI_SWIGLU) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float other = __shfl_xor(acc[t][mt][i], 8);
          const int m = 16 * mt + 4 * g + i;
          const int o = tile * 8 + r;
          if (r < 8 && m < M && o < p.n_valid) p.H[(size_t)m * p.ldh + o] = (f16)(silu(acc[t][mt][i]) * other);
        }
      } else {
        const int n = tile * 16 + r;
        if (n < p.n_valid) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = 16 * mt + 4 * g + i;
            if (m < M) {
              float* dst = p.Y + (size_t)m * p.ldy + n;
              if constexpr (EPI == EPI_ATOMIC) unsafeAtomicAdd(dst, acc[t][mt][i]);
              else *dst = acc[t][mt][i];
            }
          }
        }
      }
    }
  }
}

}  // namespace mpk

namespace mp {

template <int PT, int EPI, int NW, int TW>
static void gemv2_go(const GemvParams& p, int nsplit, hipStream_t st) {
  // super-blocks in flight per wave: 4, fewer for the fat chunks so the kernel stays within
  // 128 VGPRs (4 waves per SIMD = two 8-wave workgroups per CU); two row groups (M <= 32) hold
  // twice the x ring, so one slot less
  constexpr int NS = PT == P_F16 ? 2 : (PT == P_Q6_K || PT == P_Q8_0) ? 3 : 4;
  const dim3 block(NW * 64);
  if constexpr (TW == 1) {
    const dim3 grid((p.ntiles + NW - 1) / NW, nsplit);
    if (p.M <= 16) hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, NS, 1, 1>), grid, block, 0, st, p);
    else if (p.M <= 32) hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, (NS > 2 ? NS - 1 : 2), 2, 1>), grid, block, 0, st, p);
    else if (p.M <= 48) hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, 2, 3, 1>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, 2, 4, 1>), grid, block, 0, st, p);
  } else {
    // wide row groups only (M > 32), where the A-fragment traffic dominates
    const dim3 grid((p.ntiles + NW * TW - 1) / (NW * TW), nsplit);
    if (p.M <= 48) hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, 2, 3, TW>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, 2, 4, TW>), grid, block, 0, st, p);
  }
}

template <int PT, int NW, int TW>
static void gemv2_cfg(int epi, const GemvParams& p, int nsplit, hipStream_t st) {
  switch (epi) {
    case EPI_STORE: return gemv2_go<PT, EPI_STORE, NW, TW>(p, nsplit, st);
    case EPI_ATOMIC: return gemv2_go<PT, EPI_ATOMIC, NW, TW>(p, nsplit, st);
    case EPI_SWIGLU: return gemv2_go<PT, EPI_SWIGLU, NW, TW>(p, nsplit, st);
  }
}

template <int PT>
static void gemv2_pt(int epi, const GemvParams& p, int nsplit, int nw, int tw, hipStream_t st) {
  if (PT != P_F16 && tw == 2 && p.M > 32) {
    if (nw == 8) gemv2_cfg<PT, 8, 2>(epi, p, nsplit, st);
    else gemv2_cfg<PT, 4, 2>(epi, p, nsplit, st);
  } else if (nw == 8) gemv2_cfg<PT, 8, 1>(epi, p, nsplit, st);
  else gemv2_cfg<PT, 4, 1>(epi, p, nsplit, st);
}

// p.sb_per_split must be set by the caller (launch_gemv does)
void launch_gemv2(int ptype, int epi, const GemvParams& p, int nsplit, int nw, int tw, hipStream_t st) {
  switch (ptype) {
    case P_Q4_K: gemv2_pt<P_Q4_K>(epi, p, nsplit, nw, tw, st); break;
    case P_Q5_K: gemv2_pt<P_Q5_K>(epi, p, nsplit, nw, tw, st); break;
    case P_Q6_K: gemv2_pt<P_Q6_K>(epi, p, nsplit, nw, tw, st); break;
    case P_Q8_0: gemv2_pt<P_Q8_0>(epi, p, nsplit, nw, tw, st); break;
    case P_Q4_0: gemv2_pt<P_Q4_0>(epi, p, nsplit, nw, tw, st); break;
    case P_F16: gemv2_pt<P_F16>(epi, p, nsplit, nw, tw, st); break;
  }
}

}  // namespace mp
