// Mixture-of-experts FFN (Mixtral): device-side top-k routing and a grouped
// dequant-GEMV over the routed experts.  Everything stays on the GPU (graph-capturable): the
// router writes per-expert token lists, the expert kernels read the counts and exit early for
// idle experts, so a decode step streams only the weights of the experts actually selected.
#include "kcommon.h"
#include "../runtime/tuning.h"
#include <cstdlib>
#include <stdexcept>
#include "dequant.h"
#include "../runtime/kernels_api.h"

namespace mpk {
using namespace mp;

// Router logits [M][ld] = x[M][K] . R[E][K]^T on the dense f16 copy of the router (E <= 64 rows,
// HipStage::build_router_dense).  RB token rows per 256-thread workgroup; each thread takes 8-k
// slices (16-B loads, v_dot2 accumulation), then fixed-order wave and workgroup reductions: the
// result is bitwise repeatable (no atomics), and the launch has M / RB workgroups whatever E is.
// Through the generic GEMM paths this N = E call took 33 us at M = 256 (gemm3: one column group,
// split-K capped at 4: profiles/r8b_prof_mixtral_mb256.txt).
template <int RB>
__global__ __launch_bounds__(256) void router_logits_kernel(const f16* __restrict__ X, int ldx,
                                                            const f16* __restrict__ R, int K, int E, int M,
                                                            float* __restrict__ out, int ld) {
  __shared__ float red[4][RB][8];
  const int m0 = blockIdx.x * RB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int e0 = 0; e0 < E; e0 += 8) {
    float acc[RB][8];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[r][e] = 0.f;
    for (int k = threadIdx.x * 8; k < K; k += 256 * 8) {
      half8_t xv[RB];
#pragma unroll
      for (int r = 0; r < RB; ++r)
        xv[r] = m0 + r < M ? *reinterpret_cast<const half8_t*>(X + (size_t)(m0 + r) * ldx + k) : half8_t{};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (e0 + e >= E) break;
        const half8_t w = *reinterpret_cast<const half8_t*>(R + (size_t)(e0 + e) * K + k);
#pragma unroll
        for (int r = 0; r < RB; ++r)
#pragma unroll
          for (int j = 0; j < 8; j += 2)
            acc[r][e] = __builtin_amdgcn_fdot2(half2_t{xv[r][j], xv[r][j + 1]}, half2_t{w[j], w[j + 1]}, acc[r][e], false);
      }
    }
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = wave_sum(acc[r][e]);
        if (lane == 0) red[wave][r][e] = v;
      }
    __syncthreads();
    if (threadIdx.x < RB * 8) {
      const int r = threadIdx.x >> 3, e = threadIdx.x & 7;
      if (m0 + r < M && e0 + e < E)
        out[(size_t)(m0 + r) * ld + e0 + e] = red[0][r][e] + red[1][r][e] + red[2][r][e] + red[3][r][e];
    }
    __syncthreads();
  }
}

// one block of 1024 threads: softmax over E router logits per token, top-k, renormalise, bucket by
// expert.  The bucket positions come from LDS atomics (a prompt chunk of 2048 tokens places 4096
// slots: as global atomics on 8 addresses they serialised at one L2 channel), then the counts go out
// once.  The order of slots inside an expert's list does not change any slot's result.
__global__ __launch_bounds__(1024) void moe_route_kernel(const MoeRouteParams p) {
  __shared__ int cnt[64];
  for (int e = threadIdx.x; e < p.E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int t = threadIdx.x; t < p.M; t += blockDim.x) {
    const float* lg = p.logits + (size_t)t * p.ld;
    float mx = -INFINITY;
    for (int e = 0; e < p.E; ++e) mx = fmaxf(mx, lg[e]);
    float sum = 0.f;
    for (int e = 0; e < p.E; ++e) sum += __expf(lg[e] - mx);
    unsigned long long taken = 0;
    float wsel[8];
    int esel[8];
    float wsum = 0.f;
    for (int j = 0; j < p.k; ++j) {
      int best = -1;
      float bv = -INFINITY;
      for (int e = 0; e < p.E; ++e)
        if (!((taken >> e) & 1ull) && lg[e] > bv) { bv = lg[e]; best = e; }
      taken |= 1ull << best;
      esel[j] = best;
      wsel[j] = __expf(bv - mx) / sum;
      wsum += wsel[j];
    }
    for (int j = 0; j < p.k; ++j) {
      const int slot = t * p.k + j;
      p.weights[slot] = wsel[j] / wsum;
      const int pos = atomicAdd(&cnt[esel[j]], 1);
      p.lists[(size_t)esel[j] * p.list_cap + pos] = slot;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < p.E; e += blockDim.x) p.counts[e] = cnt[e];
}

// Grouped skinny GEMV: grid (tiles, splits, experts).  Rows = the slots routed to expert e,
// processed 16 at a time (one MFMA row tile); weights of expert e at W + e * estride.
template <int PT, int EPI>
__global__ __launch_bounds__(64) void moe_gemv_kernel(const MoeGemvParams p) {
  using D = Deq<PT>;
  constexpr int CB = D::CB;
  constexpr int NSLOT = 4;
  const int e = blockIdx.z;
  const int count = p.counts[e];
  if (count == 0) return;
  const int lane = threadIdx.x;
  const int tile = blockIdx.x;
  const int sb0 = blockIdx.y * p.sb_per_split;
  const int sb1 = min(sb0 + p.sb_per_split, p.nsb);
  if (sb0 >= sb1) return;
  const int g = lane >> 4, r = lane & 15;
  const uint8_t* wt = p.W + (size_t)e * p.estride + (size_t)tile * p.nsb * CB;
  const int32_t* list = p.lists + (size_t)e * p.list_cap;
  const int last = sb1 - 1;
  for (int r0 = 0; r0 < count; r0 += 16) {
    const int rows = min(16, count - r0);
    const int slot_r = list[r0 + min(r, rows - 1)];
    const int xrow = p.x_per_slot ? slot_r : slot_r / p.k;
    const f16* xp = p.X + (size_t)xrow * p.ldx + t16_xoff(g, 0);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    typename D::Raw ring[NSLOT];
#pragma unroll
    for (int sl = 0; sl < NSLOT; ++sl) D::load(ring[sl], wt + (size_t)min(sb0 + sl, last) * CB, lane);
    for (int sb = sb0; sb < sb1; sb += NSLOT) {
#pragma unroll
      for (int sl = 0; sl < NSLOT; ++sl) {
        const int cur = sb + sl;
        if (cur < sb1) {
          half8_t a[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) a[i] = x_op<PT == P_BF16>(*reinterpret_cast<const half8_t*>(xp + (size_t)cur * 256 + 8 * i));
          half8_t b[4];
          D::template dequant<0>(ring[sl], b, lane);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mma<PT == P_BF16>(a[s], b[s], acc);
          D::template dequant<1>(ring[sl], b, lane);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mma<PT == P_BF16>(a[4 + s], b[s], acc);
          if (cur + NSLOT < sb1) D::load(ring[sl], wt + (size_t)(cur + NSLOT) * CB, lane);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 4 * g + i;
      if (EPI == EPI_SWIGLU) {
        const float other = __shfl_xor(acc[i], 8);
        if (r < 8 && m < rows) {
          const int o = tile * 8 + r;
          const int slot = list[r0 + m];
          if (o < p.n_valid) p.H[(size_t)slot * p.ldh + o] = sat_f16(silu(acc[i]) * other);
        }
      } else if (m < rows) {
        const int n = tile * 16 + r;
        const int slot = list[r0 + m];
        if (n < p.n_valid) {
          if (p.Yslot) p.Yslot[(size_t)slot * p.ldy + n] = p.weights[slot] * acc[i];   // deterministic mode
          else unsafeAtomicAdd(p.Y + (size_t)(slot / p.k) * p.ldy + n, p.weights[slot] * acc[i]);
        }
      }
    }
  }
}

// Grouped GEMV v2 (decode, M <= 64 tokens): the gemv2 design per expert.  Workgroup = NW waves =
// NW weight tiles of expert blockIdx.z; the x rows routed to that expert (gathered through its
// slot list) are staged ONCE per workgroup in LDS per super-block (double-buffered, quarter-swapped
// rows as in gemv2.hip), and every dequantized weight fragment feeds MT MFMA row groups (all of
// the expert's rows in one pass: count <= M <= 16 MT).  v1 above re-streamed the expert's weights
// for every 16 routed rows and loaded x fragments per wave.
constexpr int MOE_LDX = 256 + 8;

template <int PT, int EPI, int NW, int NSLOT, int MT>
__global__ __launch_bounds__(NW * 64) void moe_gemv2_kernel(const MoeGemvParams p) {
  using D = Deq<PT>;
  constexpr int CB = D::CB;
  constexpr bool BF = PT == P_BF16;
  constexpr int NT = NW * 64;
  constexpr int XC = 512 * MT;
  constexpr int XCH = (XC + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) f16 xs[2][16 * MT * MOE_LDX];
  __shared__ int s_xrow[16 * MT];
  const int e = blockIdx.z;
  const int count = p.counts[e];
  if (count == 0) return;   // uniform over the workgroup
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int tile = blockIdx.x * NW + wave;
  const int sbA = blockIdx.y * p.sb_per_split;
  const int sbB = min(sbA + p.sb_per_split, p.nsb);
  if (sbA >= sbB) return;
  const int32_t* list = p.lists + (size_t)e * p.list_cap;
  const int rows = min(count, 16 * MT);
  for (int i = tid; i < 16 * MT; i += NT) s_xrow[i] = i < rows ? (p.x_per_slot ? list[i] : list[i] / p.k) : -1;
  __syncthreads();
  const uint8_t* wt = p.W + (size_t)e * p.estride + (size_t)min(tile, p.ntiles - 1) * p.nsb * CB;

  u32x4 xv[NSLOT][XCH];
  typename D::Raw ring[NSLOT];
  const int last = sbB - 1;
  auto issue = [&](const int sl, const int sb) {
    D::load(ring[sl], wt + (size_t)sb * CB, lane);
#pragma unroll
    for (int j = 0; j < XCH; ++j) {
      const int c = tid + NT * j;
      if (c < XC) {
        const int row = c >> 5, col = (c & 31) * 8;
        const int xr = s_xrow[row];
        xv[sl][j] = xr >= 0 ? *reinterpret_cast<const u32x4*>(p.X + (size_t)xr * p.ldx + (size_t)sb * 256 + col)
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
        *reinterpret_cast<u32x4*>(&xs[buf][row * MOE_LDX + (col ^ x_qswap(row))]) = xv[sl][j];
      }
    }
  };
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int sl = 0; sl < NSLOT; ++sl) issue(sl, min(sbA + sl, last));
  store_x(0, 0);
  __syncthreads();
  const f16* xrow0 = &xs[0][r * MOE_LDX + (t16_xoff(g, 0) ^ x_qswap(r))];
  const f16* xrow1 = &xs[1][r * MOE_LDX + (t16_xoff(g, 0) ^ x_qswap(r))];
  // row groups holding routed rows (uniform over the workgroup): with ~M k / E rows per expert,
  // most experts need 1-2 of the MT groups sized for the worst case
  const int mte = (rows + 15) >> 4;
  auto step = [&](const int sl, const int cur) {
    const int buf = (cur - sbA) & 1;
    const f16* xr = buf ? xrow1 : xrow0;
    half8_t b[4];
    D::template dequant<0>(ring[sl], b, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        if (mt == 0 || mt < mte)
          acc[mt] = mma<BF>(x_op<BF>(*reinterpret_cast<const half8_t*>(xr + mt * 16 * MOE_LDX + 8 * s)), b[s], acc[mt]);
    D::template dequant<1>(ring[sl], b, lane);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        if (mt == 0 || mt < mte)
          acc[mt] = mma<BF>(x_op<BF>(*reinterpret_cast<const half8_t*>(xr + mt * 16 * MOE_LDX + 32 + 8 * s)), b[s], acc[mt]);
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
  for (int sl = 0; sl < NSLOT - 1; ++sl)
    if (sb + sl < sbB) step(sl, sb + sl);
  if (tile >= p.ntiles) return;
  // lane holds C[m = 16 mt + 4g + i][n = 16*tile + r]; row m = the expert's m-th routed slot
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = 16 * mt + 4 * g + i;
      if constexpr (EPI == EPI_SWIGLU) {
        const float other = __shfl_xor(acc[mt][i], 8);
        const int o = tile * 8 + r;
        if (r < 8 && m < rows && o < p.n_valid) p.H[(size_t)list[m] * p.ldh + o] = sat_f16(silu(acc[mt][i]) * other);
      } else {
        const int n = tile * 16 + r;
        if (m < rows && n < p.n_valid) {
          const int slot = list[m];
          if (p.Yslot) p.Yslot[(size_t)slot * p.ldy + n] = p.weights[slot] * acc[mt][i];   // deterministic mode
          else unsafeAtomicAdd(p.Y + (size_t)(slot / p.k) * p.ldy + n, p.weights[slot] * acc[mt][i]);
        }
      }
    }
  }
}

}  // namespace mpk

namespace mp {

void launch_router_logits(const f16* X, int ldx, const f16* R, int K, int E, int M, float* out, int ld, hipStream_t st) {
  if (K % 8 || E < 1 || E > 64 || M < 1) throw std::runtime_error("launch_router_logits: K % 8, 1 <= E <= 64, M >= 1");
  // one row per workgroup up to 1024 rows (M = 256: 256 workgroups; 4 rows each took 10.5 us per
  // Mixtral layer on 64 workgroups, profiles/r8i_*), 4 rows per workgroup for longer prompt chunks
  if (M <= 1024) hipLaunchKernelGGL(mpk::router_logits_kernel<1>, dim3(M), dim3(256), 0, st, X, ldx, R, K, E, M, out, ld);
  else hipLaunchKernelGGL(mpk::router_logits_kernel<4>, dim3((M + 3) / 4), dim3(256), 0, st, X, ldx, R, K, E, M, out, ld);
}

void launch_moe_route(const MoeRouteParams& p, hipStream_t st) {
  hipLaunchKernelGGL(mpk::moe_route_kernel, dim3(1), dim3(1024), 0, st, p);
}

template <int PT, int EPI, int MT>
static void moe2_go(const MoeGemvParams& p, int nsplit, hipStream_t st) {
  constexpr int NW = 8;
  // super-blocks in flight: as gemv2 (<= 128 VGPRs), one less per extra row group
  constexpr int NS = is16(PT) ? 2 : (PT == P_Q6_K || PT == P_Q8_0) ? 3 : 4;
  constexpr int NSL = MT == 1 ? NS : MT == 2 ? (NS > 2 ? NS - 1 : 2) : 2;
  const dim3 grid((p.ntiles + NW - 1) / NW, nsplit, p.E);
  hipLaunchKernelGGL((mpk::moe_gemv2_kernel<PT, EPI, NW, NSL, MT>), grid, dim3(NW * 64), 0, st, p);
}

template <int PT, int EPI>
static void moe2_mt(const MoeGemvParams& p, int nsplit, hipStream_t st) {
  if (p.M <= 16) moe2_go<PT, EPI, 1>(p, nsplit, st);
  else if (p.M <= 32) moe2_go<PT, EPI, 2>(p, nsplit, st);
  else if (p.M <= 48) moe2_go<PT, EPI, 3>(p, nsplit, st);
  else moe2_go<PT, EPI, 4>(p, nsplit, st);
}

template <int PT>
static void moe_launch_pt(int epi, const MoeGemvParams& p, int nsplit, hipStream_t st) {
  const bool v1 = knob(KNOB_MOE_V) == 1;
  if (!v1 && p.M >= 1 && p.M <= 64) {   // every expert's rows fit one pass of <= 4 row groups
    if (epi == EPI_SWIGLU) moe2_mt<PT, EPI_SWIGLU>(p, nsplit, st);
    else moe2_mt<PT, EPI_ATOMIC>(p, nsplit, st);
    return;
  }
  dim3 grid(p.ntiles, nsplit, p.E);
  if (epi == EPI_SWIGLU) hipLaunchKernelGGL((mpk::moe_gemv_kernel<PT, EPI_SWIGLU>), grid, dim3(64), 0, st, p);
  else hipLaunchKernelGGL((mpk::moe_gemv_kernel<PT, EPI_ATOMIC>), grid, dim3(64), 0, st, p);
}

void launch_moe_gemv(int ptype, int epi, MoeGemvParams p, int nsplit, hipStream_t st) {
  if (nsplit < 1 || epi == EPI_SWIGLU || p.Yslot) nsplit = 1;
  p.sb_per_split = (p.nsb + nsplit - 1) / nsplit;
  nsplit = (p.nsb + p.sb_per_split - 1) / p.sb_per_split;
  switch (ptype) {
    case P_Q4_K: moe_launch_pt<P_Q4_K>(epi, p, nsplit, st); break;
    case P_Q5_K: moe_launch_pt<P_Q5_K>(epi, p, nsplit, st); break;
    case P_Q6_K: moe_launch_pt<P_Q6_K>(epi, p, nsplit, st); break;
    case P_Q8_0: moe_launch_pt<P_Q8_0>(epi, p, nsplit, st); break;
    case P_Q4_0: moe_launch_pt<P_Q4_0>(epi, p, nsplit, st); break;
    case P_F16: moe_launch_pt<P_F16>(epi, p, nsplit, st); break;
    case P_BF16: moe_launch_pt<P_BF16>(epi, p, nsplit, st); break;
  }
}

}  // namespace mp
