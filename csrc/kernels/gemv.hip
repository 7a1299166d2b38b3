// Decode GEMV dispatch (the kernel itself is gemv2.hip) and the dense T16 unpack kernel.
//
//   Y[m][n] (+)= sum_k X[m][k] * W[n][k]      X: f16 [M][ldx], W: T16-packed quantized weights
//
// Split-K over super-blocks (grid.y) with f32 atomics into the destination gives enough waves on
// the 256 CUs for every Llama shape; residual adds (Wo, Wdown) atomically accumulate straight
// into the f32 residual stream, and the gate/up projection is packed interleaved (rows 0-7 gate,
// 8-15 up of the same 8 outputs) so SwiGLU is fused in the epilogue (K8/K9 fusion).
// (The round-1 per-wave-x v1 kernel and its bandwidth probes were retired: the LDS-shared v2 won
// every shape, profiles/r1b_gemv_*.)
#include "kcommon.h"
#include "../runtime/tuning.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"

#include <cstdlib>
#include <stdexcept>

namespace mpk {

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
      if constexpr (PT == P_BF16) b[s] = bf8_to_h8(__builtin_bit_cast(u32x4, b[s]));   // dense f16 output
      f16* o = out + (size_t)(tile * 16 + r) * ldo + sb * 256 + t16_xoff(g, 4 * h + s);
      *reinterpret_cast<half8_t*>(o) = b[s];
    }
  }
}

}  // namespace mpk

namespace mp {

void launch_gemv2(int ptype, int epi, const GemvParams& p, int nsplit, int nw, int tw, hipStream_t st);

// waves per workgroup (MIPIPE_GEMV_NW: 4 or 8) and tiles per wave at M > 32 (MIPIPE_GEMV2_TW or
// set_gemv_tpw: 1 or 2; 0 = auto: 2 for the split-free SwiGLU / store GEMVs with >= 192
// workgroups left).  Measured on MI355X (profiles/r1g_gemv_tiles_per_wave_ab.txt, 70B Q4_K,
// M = 64): gate/up 115.9 -> 104.3 us with two tiles per wave; the split-K projections (qkv, o,
// down) gain nothing at their best split.
static int g_nw = 8, g_tw2 = 0;
static void read_env() {   // the knobs (tuning.h), re-read per launch: set_gemv_tpw overrides the TW one
  g_nw = knob(KNOB_GEMV_NW);
  g_tw2 = knob(KNOB_GEMV2_TW);
}
static int gemv2_tw(int M, int epi, int ntiles = 1 << 30) {
  read_env();
  if (M <= 32) return 1;
  if (g_tw2) return g_tw2;
  // two tiles per wave halve the workgroups: only where >= 192 remain (70B gate/up: 224;
  // 8B gate/up would drop to 112 of 256 CUs; the Q6_K LM head at M = 64: 294 -> 266 us)
  return (epi == EPI_SWIGLU || epi == EPI_STORE) && ntiles / (2 * g_nw) >= 192 ? 2 : 1;
}

int gemv_tiles_per_wave(int M, int epi) { return gemv2_tw(M, epi); }

int gemv_auto_split(int ntiles, int nsb, int M, int epi) {
  if (epi != EPI_ATOMIC) return 1;
  const int tpw = gemv_tiles_per_wave(M, epi);
  // wide row groups (M > 32) pay more per split (x re-staged per split, M atomics per output):
  // 70B M=64 best at ~2048 tile-waves (qkv 31 -> 29 us, o 25.4 -> 22.1 us; r1g_gemv_tiles_per_wave_ab.txt)
  const int target_waves = (M > 32 ? knob(KNOB_GEMV_SPLIT_WAVES) : 4096) / tpw;
  const int waves = (ntiles + tpw - 1) / tpw;
  int s = (target_waves + waves - 1) / waves;
  // >= GEMV_SPLIT_MINSB (4) super-blocks per split, except for a handful of tiles (MoE router: one
  // tile), where the serial super-block loop of a single workgroup would dominate
  const int minsb = knob(KNOB_GEMV_SPLIT_MINSB);
  const int smax = ntiles <= 4 ? nsb : (nsb / minsb > 1 ? nsb / minsb : 1);
  return s < 1 ? 1 : (s > smax ? smax : s);
}
void set_gemv_tpw(int t) { set_knob("GEMV2_TW", (t == 1 || t == 2) ? t : 0); }

void launch_gemv(int ptype, int epi, GemvParams p, int nsplit, hipStream_t st) {
  read_env();
  if (nsplit < 1) nsplit = 1;
  if (p.M < 1 || p.M > 64) throw std::runtime_error("launch_gemv: M must be 1..64 (longer chunks: launch_gemm)");
  if (p.Xf && p.M > 4) throw std::runtime_error("launch_gemv: the fused RMSNorm takes M <= 4");
  p.sb_per_split = (p.nsb + nsplit - 1) / nsplit;
  nsplit = (p.nsb + p.sb_per_split - 1) / p.sb_per_split;
  launch_gemv2(ptype, epi, p, nsplit, g_nw, gemv2_tw(p.M, epi, p.ntiles), st);
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
    case P_BF16: hipLaunchKernelGGL(mpk::unpack_kernel<P_BF16>, grid, dim3(64), 0, st, W, nsb, out, ldo); break;
  }
}

}  // namespace mp
