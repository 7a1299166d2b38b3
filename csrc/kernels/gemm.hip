// Prefill dequant-GEMM: Y[M][N] (+)= X[M][K] W^T for M > 16 prompt tokens,
// W in the T16 packed layout the decode GEMV streams (no second copy of the weights).
//
// Workgroup = 4 waves = a 64 (rows m) x 64 (cols n) output tile.  Per 256-k super-block:
//   - the workgroup stages X[64][256] f16 (32 KB) into LDS (double-buffered, padded rows so the
//     16 rows of an MFMA fragment read hit distinct banks), loaded one super-block ahead;
//   - wave w dequantizes ITS 16-column weight tile once (dequant.h, registers) and reuses the
//     B fragments for all four 16-row m sub-tiles (4 x 8 v_mfma_f32_16x16x32_f16);
// so every weight byte is read and dequantized once per 64 prompt rows, and the kernel is MFMA /
// LDS bound instead of weight-bandwidth bound (the decode GEMV re-streams W per 16 rows).
// Epilogues as the GEMV: STORE, ADD (residual, single owner: plain read-modify-write) and the
// fused SwiGLU of interleaved gate/up tiles.
#include "kcommon.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"

namespace mpk {
using namespace mp;

constexpr int GM_BM = 64;          // rows per workgroup
constexpr int GM_LDX = 256 + 8;    // padded LDS row (f16), quarters swapped per x_qswap (dequant.h)

template <int PT, int EPI>
__global__ __launch_bounds__(256) void gemm_kernel(const GemvParams p) {
  using D = Deq<PT>;
  constexpr int CB = D::CB;
  __shared__ __attribute__((aligned(16))) f16 xs[2][GM_BM * GM_LDX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, r = lane & 15;
  const int tile = blockIdx.x * 4 + wave;
  const bool tile_ok = tile < p.ntiles;
  const int m0 = blockIdx.y * GM_BM;
  const uint8_t* wt = p.W + (size_t)min(tile, p.ntiles - 1) * p.nsb * CB;

  // X staging: 64 rows x 32 chunks of 16 B per super-block = 8 chunks per thread
  u32x4 xv[8];
  auto load_x = [&](int sb) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = tid + 256 * j, row = c >> 5, col = (c & 31) * 8;
      const int m = min(m0 + row, p.M - 1);
      xv[j] = *reinterpret_cast<const u32x4*>(p.X + (size_t)m * p.ldx + (size_t)sb * 256 + col);
    }
  };
  auto store_x = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = tid + 256 * j, row = c >> 5, col = (c & 31) * 8;
      *reinterpret_cast<u32x4*>(&xs[buf][row * GM_LDX + (col ^ x_qswap(row))]) = xv[j];
    }
  };

  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  typename D::Raw raw[2];
  D::load(raw[0], wt, lane);
  load_x(0);
  store_x(0);
  if (p.nsb > 1) D::load(raw[1], wt + CB, lane);
  __syncthreads();

  // one super-block step; `cur` is a literal at both call sites so raw[] stays in registers
  auto step = [&](const int cur, const int sb) {
    if (sb + 1 < p.nsb) load_x(sb + 1);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      half8_t b[4];
      if (h == 0) D::template dequant<0>(raw[cur], b, lane);
      else D::template dequant<1>(raw[cur], b, lane);
#pragma unroll
      for (int ms = 0; ms < 4; ++ms) {
        const f16* xr = &xs[cur][(16 * ms + r) * GM_LDX + (t16_xoff(g, 4 * h) ^ x_qswap(r))];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const half8_t a = x_op<PT == P_BF16>(*reinterpret_cast<const half8_t*>(xr + 8 * s));
          acc[ms] = mma<PT == P_BF16>(a, b[s], acc[ms]);
        }
      }
    }
    if (sb + 2 < p.nsb) D::load(raw[cur], wt + (size_t)(sb + 2) * CB, lane);
    if (sb + 1 < p.nsb) store_x(cur ^ 1);
    __syncthreads();
  };
  for (int sb = 0; sb < p.nsb; sb += 2) {
    step(0, sb);
    if (sb + 1 < p.nsb) step(1, sb + 1);
  }
  if (!tile_ok) return;
  // lane holds C[m = m0 + 16 ms + 4g + i][n = 16 tile + r]
#pragma unroll
  for (int ms = 0; ms < 4; ++ms) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + 16 * ms + 4 * g + i;
      if constexpr (EPI == EPI_SWIGLU) {
        const float other = __shfl_xor(acc[ms][i], 8);
        const int o = tile * 8 + r;
        if (r < 8 && m < p.M && o < p.n_valid) p.H[(size_t)m * p.ldh + o] = sat_f16(silu(acc[ms][i]) * other);
      } else {
        const int n = tile * 16 + r;
        if (m < p.M && n < p.n_valid) {
          float* dst = p.Y + (size_t)m * p.ldy + n;
          if constexpr (EPI == EPI_ATOMIC) *dst += acc[ms][i];
          else *dst = acc[ms][i];
        }
      }
    }
  }
}

}  // namespace mpk

namespace mp {

template <int PT>
static void gemm_pt(int epi, const GemvParams& p, hipStream_t st) {
  dim3 grid((p.ntiles + 3) / 4, (p.M + mpk::GM_BM - 1) / mpk::GM_BM);
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL((mpk::gemm_kernel<PT, EPI_STORE>), grid, dim3(256), 0, st, p); break;
    case EPI_ATOMIC: hipLaunchKernelGGL((mpk::gemm_kernel<PT, EPI_ATOMIC>), grid, dim3(256), 0, st, p); break;
    case EPI_SWIGLU: hipLaunchKernelGGL((mpk::gemm_kernel<PT, EPI_SWIGLU>), grid, dim3(256), 0, st, p); break;
  }
}

void launch_gemm(int ptype, int epi, GemvParams p, hipStream_t st) {
  switch (ptype) {
    case P_Q4_K: gemm_pt<P_Q4_K>(epi, p, st); break;
    case P_Q5_K: gemm_pt<P_Q5_K>(epi, p, st); break;
    case P_Q6_K: gemm_pt<P_Q6_K>(epi, p, st); break;
    case P_Q8_0: gemm_pt<P_Q8_0>(epi, p, st); break;
    case P_Q4_0: gemm_pt<P_Q4_0>(epi, p, st); break;
    case P_F16: gemm_pt<P_F16>(epi, p, st); break;
    case P_BF16: gemm_pt<P_BF16>(epi, p, st); break;
  }
}

}  // namespace mp
