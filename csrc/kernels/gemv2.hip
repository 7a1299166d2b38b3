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
#include "../runtime/tuning.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

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
template <int PT, int EPI, int NW, int NSLOT, int MT, int TW, bool NORM>
__global__ __launch_bounds__(NW * 64) void gemv2_kernel(const GemvParams p) {
  using D = Deq<PT>;
  constexpr bool BF = PT == P_BF16;
  constexpr int CB = D::CB;
  constexpr int NT = NW * 64;
  constexpr int XC = 512 * MT;   // 16 B x chunks per super-block
  static_assert(!NORM || (MT == 1 && TW == 1), "fused RMSNorm: one row group, M <= 4");
  __shared__ __attribute__((aligned(16))) f16 xs[2][16 * MT * G2_LDX];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int mblk = 0;   // one row block of <= 64 rows (the 128-row prompt GEMM form, gemm2, is retired: gemm4)
  const int bx = (int)blockIdx.x;
  const int tile0 = (bx * NW + wave) * TW;
  const size_t r_off = (size_t)mblk * 16 * MT;   // first row of this workgroup
  const int sbA = blockIdx.y * p.sb_per_split;
  const int sbB = min(sbA + p.sb_per_split, p.nsb);
  if (sbA >= sbB) return;   // uniform over the workgroup
  // each tile's super-block range [sbA, sbB) as a buffer descriptor: ring slots past the end of
  // the range load zeros without memory traffic (v1 re-loaded the clamped last super-block: up to
  // NSLOT - 1 redundant chunk loads per wave at 2-4 super-blocks per split)
  __amdgpu_buffer_rsrc_t wsrc[TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) {
    const int tl = __builtin_amdgcn_readfirstlane(tile0 + t);
    const int nb = tl < p.ntiles ? sbB - sbA : 0;
    wsrc[t] = make_rsrc(p.W + ((size_t)min(tl, p.ntiles - 1) * p.nsb + sbA) * CB, (uint32_t)(nb * CB));
  }
  const int M = min(p.M - (int)r_off, 16 * MT);
  const f16* const Xg = p.X + r_off * p.ldx;

  // x staging: 16 MT rows x 256 k per super-block = 512 MT chunks of 16 B; thread t owns chunks t, t+NT..
  // The x chunks of super-block j are loaded TOGETHER with its weights (register rings of NSLOT),
  // NSLOT steps ahead, and copied to LDS one step before use: every vmcnt wait then leaves the
  // loads of the NSLOT-1 later super-blocks in flight.
  // NORM (deferred RMSNorm): the chunk is 8 f32 of the residual row plus 8 of gamma; LDS gets
  // f16(x * gamma) and the thread accumulates sum(x^2) of its row while staging, so the per-row
  // factor rsqrt(mean(x^2) + eps) is applied to the accumulators at the end (STORE / SWIGLU: every
  // workgroup staged the whole row) or by the consumer from the published per-split partial sums
  // (ATOMIC: p.ssq, the decode attention).  (gamma staged in LDS instead of the register ring took
  // 199 VGPRs against 164: the compiler kept the per-step LDS gamma reads live across steps.)
  constexpr int XCH = (XC + NT - 1) / NT;
  constexpr int XW = NORM ? 4 : 1;   // NORM: x (2 x 16 B f32) + gamma (2 x 16 B f32)
  u32x4 xv[NSLOT][XCH][XW];
  typename D::Raw ring[NSLOT][TW];
  const int last = sbB - 1;
  auto issue = [&](const int sl, const int sb) {
#pragma unroll
    for (int t = 0; t < TW; ++t) D::load(ring[sl][t], BufSrc{wsrc[t], (sb - sbA) * CB}, lane);
    const int sbx = min(sb, last);
#pragma unroll
    for (int j = 0; j < XCH; ++j) {
      const int c = tid + NT * j;
      if (c < XC) {
        const int row = c >> 5, col = (c & 31) * 8;
        if constexpr (NORM) {
          const int k = sbx * 256 + col;
          const bool in = row < M && k < p.d_norm;
          const float* src = p.Xf + (size_t)row * p.ldxf + k;
          xv[sl][j][0] = in ? *reinterpret_cast<const u32x4*>(src) : u32x4{0u, 0u, 0u, 0u};
          xv[sl][j][1] = in ? *reinterpret_cast<const u32x4*>(src + 4) : u32x4{0u, 0u, 0u, 0u};
          xv[sl][j][2] = in ? *reinterpret_cast<const u32x4*>(p.gamma + k) : u32x4{0u, 0u, 0u, 0u};
          xv[sl][j][3] = in ? *reinterpret_cast<const u32x4*>(p.gamma + k + 4) : u32x4{0u, 0u, 0u, 0u};
        } else {
          xv[sl][j][0] = row < M ? *reinterpret_cast<const u32x4*>(Xg + (size_t)row * p.ldx + (size_t)sbx * 256 + col)
                                 : u32x4{0u, 0u, 0u, 0u};
        }
      }
    }
  };
  float ssn = 0.f;   // NORM: this thread's partial sum(x^2) of its row (c = tid: one row per thread)
  auto store_x = [&](const int sl, const int buf, const bool count) {
#pragma unroll
    for (int j = 0; j < XCH; ++j) {
      const int c = tid + NT * j;
      if (c < XC) {
        const int row = c >> 5, col = (c & 31) * 8;
        u32x4 v;
        if constexpr (NORM) {
          const float4 a = __builtin_bit_cast(float4, xv[sl][j][0]), b = __builtin_bit_cast(float4, xv[sl][j][1]);
          const float4 ga = __builtin_bit_cast(float4, xv[sl][j][2]), gb = __builtin_bit_cast(float4, xv[sl][j][3]);
          if (count) ssn += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w + b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w;
          v = x8_pack<BF>(a.x * ga.x, a.y * ga.y, a.z * ga.z, a.w * ga.w, b.x * gb.x, b.y * gb.y, b.z * gb.z, b.w * gb.w);
        } else {
          v = x8_from_h8<BF>(xv[sl][j][0]);   // bf16 weights: the x tile is staged as bf16
        }
        *reinterpret_cast<u32x4*>(&xs[buf][row * G2_LDX + (col ^ x_qswap(row))]) = v;
      }
    }
  };

  f32x4 acc[TW][MT];
#pragma unroll
  for (int t = 0; t < TW; ++t)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[t][mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sl = 0; sl < NSLOT; ++sl) issue(sl, sbA + sl);
  store_x(0, 0, true);
  __syncthreads();

  // rows >= M are zero in LDS (their outputs are never stored)
  const f16* xrow0 = &xs[0][r * G2_LDX + (t16_xoff(g, 0) ^ x_qswap(r))];
  const f16* xrow1 = &xs[1][r * G2_LDX + (t16_xoff(g, 0) ^ x_qswap(r))];
  // one super-block; all loads unconditional (clamped to the range): path-independent vmcnt
  const Consts kc = make_consts();   // nibble masks / exponent magics, once per kernel
  auto step = [&](const int sl, const int cur) {
    const int buf = (cur - sbA) & 1;
    const f16* xr = buf ? xrow1 : xrow0;
    half8_t b[TW][4];
#pragma unroll
    for (int t = 0; t < TW; ++t) D::template dequant<0>(ring[sl][t], b[t], lane, kc);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const half8_t a = *reinterpret_cast<const half8_t*>(xr + mt * 16 * G2_LDX + 8 * s);
#pragma unroll
        for (int t = 0; t < TW; ++t) acc[t][mt] = mma<BF>(a, b[t][s], acc[t][mt]);
      }
#pragma unroll
    for (int t = 0; t < TW; ++t) D::template dequant<1>(ring[sl][t], b[t], lane, kc);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const half8_t a = *reinterpret_cast<const half8_t*>(xr + mt * 16 * G2_LDX + 32 + 8 * s);
#pragma unroll
        for (int t = 0; t < TW; ++t) acc[t][mt] = mma<BF>(a, b[t][s], acc[t][mt]);
      }
    store_x((sl + 1) % NSLOT, buf ^ 1, cur + 1 < sbB);   // x(cur + 1), loaded NSLOT - 1 steps ago
    issue(sl, cur + NSLOT);
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
  if constexpr (NORM) {
    // rows r < M <= 4 are staged by threads [32 r, 32 r + 32): reduce over those 32 lanes
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) ssn += __shfl_xor(ssn, o);
    if ((tid & 31) == 0 && (tid >> 5) < 4) red[tid >> 5] = ssn;
    __syncthreads();
    if constexpr (EPI == EPI_ATOMIC) {
      // publish this split's partial sum of squares (one tile group per split adds it)
      if (p.ssq && blockIdx.x == 0 && tid < M) atomicAdd(p.ssq + tid, red[tid]);
    } else {
      // the workgroup staged the whole row: scale its rows' accumulators by rsqrt(mean + eps)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = 4 * g + i;
        const float rs = m < M ? rsqrtf(red[m < 4 ? m : 0] / (float)p.d_norm + p.eps) : 0.f;
        acc[0][0][i] *= rs;
      }
    }
  }
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
          if (r < 8 && m < M && o < p.n_valid) p.H[(r_off + m) * p.ldh + o] = sat_f16(silu(acc[t][mt][i]) * other);
        }
      } else {
        const int n = tile * 16 + r;
        if (n < p.n_valid) {
          const float bias = (p.bias && blockIdx.y == 0) ? p.bias[n] : 0.f;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = 16 * mt + 4 * g + i;
            if (m < M) {
              float* dst = p.Y + (size_t)blockIdx.y * p.split_stride + (r_off + m) * p.ldy + n;
              if constexpr (EPI == EPI_ATOMIC) unsafeAtomicAdd(dst, acc[t][mt][i] + bias);
              else *dst = acc[t][mt][i] + bias;
            }
          }
        }
      }
    }
  }
  if (p.zero) {   // side job: clear zero_n floats (e.g. the consumed q|k|v split-K accumulator)
    const int64_t nb = (int64_t)gridDim.x * gridDim.y, b = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    const int64_t per = ((p.zero_n + nb - 1) / nb + 3) & ~(int64_t)3;
    const int64_t z0 = b * per, z1 = min(p.zero_n, z0 + per);
    for (int64_t i = z0 + tid * 4; i < z1; i += NT * 4) {
      if (i + 4 <= z1) *reinterpret_cast<float4*>(p.zero + i) = make_float4(0.f, 0.f, 0.f, 0.f);
      else for (int64_t k = i; k < z1; ++k) p.zero[k] = 0.f;
    }
  }
}

}  // namespace mpk

namespace mp {

template <int PT, int EPI, int NW, int TW>
static void gemv2_go(const GemvParams& p, int nsplit, hipStream_t st) {
  if constexpr (TW == 1) {
    if (p.Xf) {   // fused RMSNorm: M <= 4 (checked by launch_gemv)
      constexpr int NS = is16(PT) ? 2 : (PT == P_Q6_K || PT == P_Q8_0) ? 3 : 4;
      hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, NS, 1, 1, true>), dim3((p.ntiles + NW - 1) / NW, nsplit),
                         dim3(NW * 64), 0, st, p);
      return;
    }
  }
  // super-blocks in flight per wave: 4, fewer for the fat chunks so the kernel stays within
  // 128 VGPRs (4 waves per SIMD = two 8-wave workgroups per CU); two row groups (M <= 32) hold
  // twice the x ring, so one slot less
  constexpr int NS = is16(PT) ? 2 : (PT == P_Q6_K || PT == P_Q8_0) ? 3 : 4;
  const dim3 block(NW * 64);
  if constexpr (TW == 1) {
    const dim3 grid((p.ntiles + NW - 1) / NW, nsplit);
    if (p.M <= 16) hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, NS, 1, 1, false>), grid, block, 0, st, p);
    else if (p.M <= 32) hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, (NS > 2 ? NS - 1 : 2), 2, 1, false>), grid, block, 0, st, p);
    else if (p.M <= 48) hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, 2, 3, 1, false>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, 2, 4, 1, false>), grid, block, 0, st, p);
  } else {
    // wide row groups only (M > 32), where the A-fragment traffic dominates
    const dim3 grid((p.ntiles + NW * TW - 1) / (NW * TW), nsplit);
    if (p.M <= 48) hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, 2, 3, TW, false>), grid, block, 0, st, p);
    else hipLaunchKernelGGL((mpk::gemv2_kernel<PT, EPI, NW, 2, 4, TW, false>), grid, block, 0, st, p);
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
  if (!is16(PT) && tw == 2 && p.M > 32) {
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
    case P_BF16: gemv2_pt<P_BF16>(epi, p, nsplit, nw, tw, st); break;
  }
}

}  // namespace mp
