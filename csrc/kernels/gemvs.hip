// Small-M decode GEMV ("gemvs", M <= 4: single-stream and tiny micro-batches).
//
// At M = 1 the v2 GEMV (gemv2.hip) is latency-bound, not bandwidth-bound: 7.3 us for a 9.4 MB
// Llama-3-8B o-proj whose bytes need ~1.6 us, unchanged when the weights are MALL-resident
// (profiles/r2u_prof_8b_mb1.txt, r2w_gemv_mall_hot_cold.txt).  Its per-super-block chain (x ring
// -> LDS -> workgroup barrier -> dequant -> MFMA) and the split-K atomics cost round trips that a
// batch of one cannot hide, and every projection needs a separate RMSNorm launch (4.6 us, 65 per
// 8B token).  gemvs removes both:
//
//  * the workgroup stages ITS WHOLE k-range of x into LDS once (a prologue), so the weight loop
//    has no barrier and no x loads: a wave issues its first NS super-blocks of weights before the
//    prologue and then streams its k-slice through a register ring (MI355X guide: "GEMV / M <= 16
//    decode weights ... load straight to VGPRs, deep unroll, late vmcnt");
//  * the RMSNorm is fused into the prologue (NORM): every workgroup reduces sum(x^2) over the full
//    f32 residual row (L2-resident, 16-32 KB) and stages f16(x * rsqrt(mean + eps) * gamma), the
//    same rounding as the standalone rmsnorm kernel (elementwise.hip);
//  * split-K runs INSIDE the workgroup (KSW waves per tile, partials reduced through LDS): the
//    outputs are complete per workgroup, so STORE / SWIGLU need no zero-filled accumulator and
//    ADD (the residual update of o / down) is a plain read-modify-write by the single owner --
//    deterministic -- unless the host also splits K over grid.y (atomics).
//
//   grid (ceil(ntiles / G), nsplit)   block NW * 64 (NW = 8)
//   wave w: tile blockIdx.x * G + w / KSW (KSW = NW / G), k-slice w % KSW of the workgroup's
//   super-blocks [sbA, sbB) (split blockIdx.y)
//
// Layout: T16 chunks (csrc/runtime/qtypes.h, dequant.h): lane (g, r) holds weight column r;
// MFMA i of a super-block covers k = 64 g + 8 i + j.  The A fragment of lane (g, r) is x[r][...]
// for r < M, zero above (LDS holds M rows only).  C: lane (g, r) holds rows 4g + i: the M <= 4
// valid rows are in lanes 0-15 (g = 0), acc[i] = row i, column r.
#include "kcommon.h"
#include "../runtime/tuning.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"

#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <stdexcept>

namespace mpk {
using namespace mp;

constexpr int GS_NW = 8;
constexpr int GS_NT = GS_NW * 64;
constexpr int EPI_QKV = 3;   // STORE with the RoPE + KV-append epilogue (GemvParams::qa)

// bx: this workgroup's tile-group index (blockIdx.x, or its offset inside a segment of gemvs2)
// D1: one activation row on the v_dot2 form (dequant.h dot1): biased magic pairs against x, the bias
// removed through a per-(super-block, lane group) correction table built from the staged x
template <int PT, int EPI, int G, bool NORM, int NSO = 0, bool D1 = false>
__device__ __forceinline__ void gemvs_body(const GemvParams& p, const int nsplit, const int bx) {
  static_assert(!D1 || dot1_supported<PT>(), "gemvs: no single-row dot form for this type");
  using D = Deq<PT>;
  constexpr int CB = D::CB;
  constexpr bool BF = PT == P_BF16;
  constexpr int KSW = GS_NW / G;
  constexpr int NS = NSO ? NSO : is16(PT) ? 2 : 4;   // weight super-blocks in flight per wave
  extern __shared__ __attribute__((aligned(16))) f16 xs[];   // [M][krange] (bf16 bits for BF16 weights)
  __shared__ float red[GS_NW][64];
  __shared__ float red_ss[GS_NW][4];
  __shared__ float rs_s[4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, r = lane & 15;
  const int M = p.M;
  const int split = blockIdx.y;
  const int sbA = split * p.sb_per_split;
  const int sbB = min(sbA + p.sb_per_split, p.nsb);
  if (sbA >= sbB) return;   // uniform over the workgroup
  const int krange = (sbB - sbA) * 256;

  // this wave's tile and contiguous k-slice [wA, wB) of the workgroup's super-blocks
  const int gi = wave / KSW, ks = wave % KSW;
  const int tile = bx * G + gi;
  const int per = (sbB - sbA + KSW - 1) / KSW;
  const int wA = min(sbA + ks * per, sbB), wB = min(wA + per, sbB);
  const bool live = tile < p.ntiles;
  const __amdgpu_buffer_rsrc_t wsrc =
      make_rsrc(p.W + ((size_t)min(tile, p.ntiles - 1) * p.nsb + wA) * CB, (uint32_t)(live ? (wB - wA) * CB : 0));
#ifdef MIPIPE_TIMING_PROBES
  const int probe = p.probe;
#else
  constexpr int probe = 0;
#endif
  // the single owner's residual (ATOMIC, one split): loaded first, so the epilogue is a plain store
  // instead of a read-modify-write round trip after the reduction.  Epilogue wave e < G owns tile
  // bx * G + e; lane (m = lane >> 4, column r)
  float resid = 0.f;
  if constexpr (EPI == EPI_ATOMIC) {
    const int et0 = bx * G + wave, nc0 = et0 * 16 + r;
    if (nsplit == 1 && p.rpf && wave < G && et0 < p.ntiles && (lane >> 4) < M && nc0 < p.n_valid)
      resid = p.Y[(size_t)(lane >> 4) * p.ldy + nc0];
  }
  // Load order.  The vector memory counter retires in issue order, so a wave that waits for a load
  // issued AFTER the weight ring waits for the ring too: the prologue's x (and the QKV epilogue's
  // position) used to sit behind the first NS super-blocks of weights, and the pos -> page -> (cos,
  // sin) chain behind them again -- the qkv GEMV ran ~2x its weight-stream floor.  Now the loads the
  // prologue needs go FIRST (one-row fast paths: every load of the row in flight at once), the ring
  // next, and the dependent epilogue loads after the prologue, all under the weight stream.
  const int k0 = sbA * 256;
  const bool fast_norm = NORM && !(probe & 2) && M == 1 && (p.d_norm >> 2) <= 4 * GS_NT;
  const bool fast_x = !NORM && !(probe & 2) && M == 1 && (krange >> 3) <= 4 * GS_NT;
  // fast_norm: the first 2 float4 per thread of the f32 row and gamma (rows up to 4096; a wider
  // row's other half follows the ring: 4 early slots took the fused-norm kernels past their register
  // budget -- gemvs2 130 VGPRs, one workgroup per CU instead of two, 10.6 -> 13.2 us)
  float4 xv[2], xg[2];
  u32x4 xh[4];           // fast_x: the f16 row's k-range, 8 per thread-chunk
  if (fast_norm) {
    const int d4 = p.d_norm >> 2, k1 = min(sbB * 256, p.d_norm);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = tid + u * GS_NT;
      const bool in = c < d4, mine = in && 4 * c >= k0 && 4 * c < k1;
      xv[u] = in ? *reinterpret_cast<const float4*>(p.Xf + 4 * c) : make_float4(0.f, 0.f, 0.f, 0.f);
      xg[u] = mine ? reinterpret_cast<const float4*>(p.gamma)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  if (fast_x) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + u * GS_NT;
      xh[u] = c < (krange >> 3) ? *reinterpret_cast<const u32x4*>(p.X + (size_t)k0 + 8 * c) : u32x4{0u, 0u, 0u, 0u};
    }
  }
  // QKV epilogue: the position first (its page and (cos, sin) follow the prologue)
  int qa_pos = 0, qa_page = 0;
  float2 qa_cs = make_float2(1.f, 0.f);
  const int qa_m = lane >> 4, qa_c = p.qa.col0 + (bx * G + wave) * 16 + r;
  const bool qa_live = EPI == EPI_QKV && wave < G && qa_m < M;
  if constexpr (EPI == EPI_QKV) {
    if (qa_live) qa_pos = p.qa.pos[qa_m];
  }
  __builtin_amdgcn_sched_barrier(0);   // keep the early loads ahead of the ring
  typename D::Raw ring[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) D::load(ring[s], BufSrc{wsrc, s * CB}, lane);   // past the range: zeros, no traffic
  __builtin_amdgcn_sched_barrier(0);

  // ---- prologue: x of rows [0, M), k in [sbA*256, sbB*256) -> LDS as f16
  if (probe & 2) {
  } else if constexpr (NORM) {
    const int d4 = p.d_norm >> 2;
    const int k1 = min(sbB * 256, p.d_norm);   // this workgroup's k-range (valid part)
    if (fast_norm) {
      // one row of <= 8192: every float4 of the row loaded once, in one batch ahead of the weight
      // ring, and kept: the thread that reduced a chunk also stages it (no second pass over x)
      float4 v[4] = {xv[0], xv[1], make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
      float4 gm[4] = {xg[0], xg[1], make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
      if (d4 > 2 * GS_NT) {   // uniform: only rows wider than 4096 issue (and wait for) the second half
#pragma unroll
        for (int u = 2; u < 4; ++u) {
          const int c = tid + u * GS_NT;
          const bool in = c < d4, mine = in && 4 * c >= k0 && 4 * c < k1;
          v[u] = in ? *reinterpret_cast<const float4*>(p.Xf + 4 * c) : make_float4(0.f, 0.f, 0.f, 0.f);
          gm[u] = mine ? reinterpret_cast<const float4*>(p.gamma)[c] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      float ss = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) ss += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
      ss = wave_sum(ss);
      if (lane == 0) red_ss[wave][0] = ss;
      // the k-range's zero tail (k >= d_norm, up to sbB * 256)
      for (int c = k1 / 4 + tid; c < sbB * 64; c += GS_NT) *reinterpret_cast<u32x2*>(xs + 4 * c - k0) = u32x2{0u, 0u};
      __syncthreads();
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < GS_NW; ++w) t += red_ss[w][0];
      const float sc = rsqrtf(t / (float)p.d_norm + p.eps);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = tid + u * GS_NT;
        if (c < d4 && 4 * c >= k0 && 4 * c < k1) {
          *reinterpret_cast<u32x2*>(xs + 4 * c - k0) =
              x4_pack<BF>(v[u].x * sc * gm[u].x, v[u].y * sc * gm[u].y, v[u].z * sc * gm[u].z, v[u].w * sc * gm[u].w);
        }
      }
    } else {
      // pass 1: sum(x^2) over the full rows (d_norm f32, a multiple of 4), loads batched by 4
      float ss[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        if (m < M) {
          const float4* xr = reinterpret_cast<const float4*>(p.Xf + (size_t)m * p.ldxf);
          for (int c0 = 0; c0 < d4; c0 += 4 * GS_NT) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int c = c0 + tid + u * GS_NT;
              v[u] = c < d4 ? xr[c] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) ss[m] += v[u].x * v[u].x + v[u].y * v[u].y + v[u].z * v[u].z + v[u].w * v[u].w;
          }
        }
      }
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        ss[m] = wave_sum(ss[m]);
        if (lane == 0) red_ss[wave][m] = ss[m];
      }
      __syncthreads();
      if (tid < 4) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < GS_NW; ++w) t += red_ss[w][tid];
        rs_s[tid] = rsqrtf(t / (float)p.d_norm + p.eps);
      }
      __syncthreads();
      // pass 2: this workgroup's k-range, f16(x * rs * gamma) (the rmsnorm kernel's rounding)
      const int k8 = krange >> 3;
      for (int c = tid; c < M * k8; c += GS_NT) {
        const int m = c / k8, kl = (c - m * k8) * 8, kg = k0 + kl;
        u32x4 o = {0u, 0u, 0u, 0u};
        if (kg < p.d_norm) {
          const float* xr = p.Xf + (size_t)m * p.ldxf + kg;
          const float4 a = *reinterpret_cast<const float4*>(xr), b = *reinterpret_cast<const float4*>(xr + 4);
          const float4 ga = *reinterpret_cast<const float4*>(p.gamma + kg), gb = *reinterpret_cast<const float4*>(p.gamma + kg + 4);
          const float sc = rs_s[m];
          o = x8_pack<BF>(a.x * sc * ga.x, a.y * sc * ga.y, a.z * sc * ga.z, a.w * sc * ga.w, b.x * sc * gb.x,
                          b.y * sc * gb.y, b.z * sc * gb.z, b.w * sc * gb.w);
        }
        *reinterpret_cast<u32x4*>(xs + (size_t)m * krange + kl) = o;
      }
    }
  } else if (fast_x) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + u * GS_NT;
      if (c < (krange >> 3)) *reinterpret_cast<u32x4*>(xs + 8 * c) = x8_from_h8<BF>(xh[u]);
    }
  } else {
    // f16 activations [M][ldx] with a zero tail up to nsb * 256; loads batched by 4
    const int k8 = krange >> 3, tot = M * k8;
    for (int c0 = 0; c0 < tot; c0 += 4 * GS_NT) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + tid + u * GS_NT;
        const int m = c / k8, kl = (c - m * k8) * 8;
        if (c < tot) v[u] = *reinterpret_cast<const u32x4*>(p.X + (size_t)m * p.ldx + (size_t)sbA * 256 + kl);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = c0 + tid + u * GS_NT;
        const int m = c / k8, kl = (c - m * k8) * 8;
        if (c < tot) *reinterpret_cast<u32x4*>(xs + (size_t)m * krange + kl) = x8_from_h8<BF>(v[u]);
      }
    }
  }
  __syncthreads();
  if constexpr (EPI == EPI_QKV) {   // the position has arrived with x: page and (cos, sin), consumed in the epilogue
    const QkvAppend& q = p.qa;
    if (qa_live) {
      qa_page = q.block_table[(size_t)(q.slot0 + qa_m) * q.max_pages + (qa_pos >> 6)];
      if (qa_c < (q.Hq + q.Hkv) * q.hd) qa_cs = q.rope_cs[(size_t)qa_pos * (q.hd >> 1) + ((qa_c % q.hd) >> 1)];
    }
  }
  // D1: the bias-correction table, 4 floats per (super-block, lane group) of the workgroup's range
  float4* corr = reinterpret_cast<float4*>(xs + (size_t)M * krange);
  if constexpr (D1) {
    for (int e = tid; e < (sbB - sbA) * 4; e += GS_NT) {
      const f16* q = xs + (e >> 2) * 256 + 64 * (e & 3);
      float a[8], b[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const half8_t v = *reinterpret_cast<const half8_t*>(q + 8 * i);
        a[i] = ((float)v[0] + (float)v[1]) + ((float)v[4] + (float)v[5]);
        b[i] = ((float)v[2] + (float)v[3]) + ((float)v[6] + (float)v[7]);
      }
      corr[e] = DotCorr<PT>::make(a, b);
    }
    __syncthreads();
  }

  // ---- weight stream: no barriers; slot s holds super-block wA + j + s
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float acc1 = 0.f;   // D1
  const Consts kc = make_consts();
  const f16* xrow = xs + (size_t)r * krange + t16_xoff(g, 0);   // valid for r < M only
  const bool xr_ok = r < M;
  auto step = [&](const int s, const int sbl) {   // sbl: super-block index relative to sbA
    if (probe & 1) {   // timing probe: consume the loads, no dequant / MFMA
      acc[0] += __uint_as_float(*reinterpret_cast<const uint32_t*>(&ring[s]) & 1u);
      return;
    }
    if constexpr (D1) {
      acc1 += dot1<PT>(ring[s], xs + sbl * 256 + t16_xoff(g, 0), corr[sbl * 4 + g], lane, kc);
      return;
    }
    half8_t b[4];
    D::template dequant<0>(ring[s], b, lane, kc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      half8_t a = {};
      if (xr_ok) a = *reinterpret_cast<const half8_t*>(xrow + sbl * 256 + 8 * i);   // bf16 already for BF
      acc = mma<BF>(a, b[i], acc);
    }
    D::template dequant<1>(ring[s], b, lane, kc);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      half8_t a = {};
      if (xr_ok) a = *reinterpret_cast<const half8_t*>(xrow + sbl * 256 + 32 + 8 * i);
      acc = mma<BF>(a, b[i], acc);
    }
  };
  const int n = wB - wA;
  int j = 0;
  for (; j + NS <= n; j += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      step(s, wA - sbA + j + s);
      D::load(ring[s], BufSrc{wsrc, (j + s + NS) * CB}, lane);
    }
  }
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (j + s < n) step(s, wA - sbA + j + s);

  // ---- reduce the KSW k-slices of each tile, then the epilogue (one wave per tile)
  float v[4];
  if constexpr (D1) {   // the 4 lane groups' k-quarters of column r, then row 0 of the MFMA layout
    acc1 += __shfl_xor(acc1, 16);
    acc1 += __shfl_xor(acc1, 32);
    v[0] = acc1;
    v[1] = v[2] = v[3] = 0.f;
  }
  if constexpr (KSW == 1) {
    if constexpr (!D1) {
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = acc[i];
    }
  } else {
    if (g == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wave][i * 16 + r] = D1 ? v[i] : acc[i];
    }
    __syncthreads();
    if (wave >= G) return;
  }
  // epilogue wave e = gi' handles tile blockIdx.x * G + e; lane -> (row i = lane >> 4, column r)
  const int et = KSW == 1 ? tile : bx * G + wave;
  float val;
  if constexpr (KSW == 1 && D1) {
    val = lane < 16 ? v[0] : 0.f;   // lane r of group 0: row 0, column r
  } else if constexpr (KSW == 1) {
    // lane (g, r): rows 4g + i; only g = 0 is valid (M <= 4): move row i to lane 16 i + r
    const int i = lane >> 4;
    const float a0 = __shfl(v[0], r), a1 = __shfl(v[1], r), a2 = __shfl(v[2], r), a3 = __shfl(v[3], r);
    val = i == 0 ? a0 : i == 1 ? a1 : i == 2 ? a2 : a3;
  } else {
    val = 0.f;
#pragma unroll
    for (int k = 0; k < KSW; ++k) val += red[wave * KSW + k][lane];
  }
  const int m = lane >> 4;
  if (et >= p.ntiles) return;
  if constexpr (EPI == EPI_SWIGLU) {
    const float up = __shfl_xor(val, 8);
    const int o = et * 8 + r;
    if (r < 8 && m < M && o < p.n_valid) p.H[(size_t)m * p.ldh + o] = sat_f16(silu(val) * up);
  } else if constexpr (EPI == EPI_QKV) {
    // q / k: rotate the adjacent pair (c, c ^ 1) (lanes r, r ^ 1); q -> Y (f32), k and v -> the cache
    const QkvAppend& q = p.qa;
    const int nc = et * 16 + r;
    const float out = val + (p.bias ? p.bias[nc] : 0.f);
    const float oth = __shfl_xor(out, 1);
    const int c = q.col0 + nc;
    const int qn = q.Hq * q.hd, kn = q.Hkv * q.hd;
    const bool odd = r & 1;
    const float x0 = odd ? oth : out, x1 = odd ? out : oth;
    const float rot = odd ? x0 * qa_cs.y + x1 * qa_cs.x : x0 * qa_cs.x - x1 * qa_cs.y;
    const float rp = __shfl_xor(rot, 1);   // the pair's other rotated value
    if (m < M && nc < p.n_valid) {
      const int idx = qa_pos & 63;
      if (c < qn) {
        p.Y[(size_t)m * p.ldy + nc] = rot;
      } else if (c < qn + kn) {
        const int h = (c - qn) / q.hd, d = (c - qn) % q.hd;
        const size_t ko = (((size_t)qa_page * q.Hkv + h) * 64 + idx) * q.Dp + d;
        if (!odd) {
          if (q.kv_fp8) *reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(q.k_cache) + ko) = (uint16_t)f8x2_pack(rot, rp);
          else *reinterpret_cast<half2_t*>(q.k_cache + ko) = half2_t{(f16)rot, (f16)rp};
        }
      } else {
        const int h = (c - qn - kn) / q.hd, d = (c - qn - kn) % q.hd;
        const size_t vo = (((size_t)qa_page * q.Hkv + h) * q.Dp + d) * 64 + idx;
        if (q.kv_fp8) reinterpret_cast<uint8_t*>(q.v_cache)[vo] = (uint8_t)f8x2_pack(out, 0.f);
        else q.v_cache[vo] = (f16)out;
      }
    }
  } else {
    const int nc = et * 16 + r;
    if (m < M && nc < p.n_valid) {
      const float out = val + ((p.bias && split == 0) ? p.bias[nc] : 0.f);
      float* dst = p.Y + (size_t)m * p.ldy + nc;
      if constexpr (EPI == EPI_ATOMIC) {
        if (nsplit == 1) {   // single owner: deterministic
          if (p.rpf != 0 || (probe & 4) != 0) *dst = resid + out;
          else *dst += out;
        }
        else unsafeAtomicAdd(dst, out);
      } else {
        *dst = out;
      }
    }
  }
}

template <int PT, int EPI, int G, bool NORM, int NSO = 0, bool D1 = false>
__global__ __launch_bounds__(GS_NT) void gemvs_kernel(const GemvParams p, const int nsplit) {
  gemvs_body<PT, EPI, G, NORM, NSO, D1>(p, nsplit, blockIdx.x);
}

// two weight segments with different quant types over the same normed input in ONE launch (the
// q+k and v projections of a mixed-type layer, e.g. Q4_K_M's Q6_K attn_v): workgroups [0, nwg1)
// take segment 1, the rest segment 2.  STORE epilogue, RMSNorm fused, no k-split.
template <int PT, int PT2, int G, int EPI = EPI_STORE, bool D1 = false>
__global__ __launch_bounds__(GS_NT) void gemvs2_kernel(const GemvParams p, const GemvParams p2, const int nwg1) {
  if ((int)blockIdx.x < nwg1) gemvs_body<PT, EPI, G, true, 0, D1>(p, 1, blockIdx.x);
  else gemvs_body<PT2, EPI, G, true, 0, D1>(p2, 1, blockIdx.x - nwg1);
}

}  // namespace mpk

namespace mp {

// Work split: G tiles per workgroup (KSW = 8 / G waves share each tile's k-range) and nsplit
// k-splits over grid.y (ATOMIC only).  Aim: ~S_target super-blocks per wave, >= 512 workgroups
// (two per CU), x k-range in LDS <= 96 KB.
GemvsPlan plan_gemvs(int ntiles, int nsb, int M, int epi, bool norm, bool deterministic) {
  GemvsPlan pl;
  // super-blocks per wave target.  8B mb1 sweep (r4c): S 4 / 8 / 16 -> 468 / 499 / 502 tok/s, flat above;
  // 70B mb1 (r5g/r5h): S 8 / 16 / 32 / 64 / 128 -> 97.9 / 101.2 / 103.6-104.8 / 105.1 / 105.3
  const int s_target = knob(KNOB_GEMVS_S);
  const int ks_needed = std::max(1, (nsb + s_target - 1) / s_target);
  int G = ks_needed >= 8 ? 1 : ks_needed >= 5 ? 1 : ks_needed >= 3 ? 2 : ks_needed == 2 ? 4 : 8;
  const int min_wg = knob(KNOB_GEMVS_MINWG);
  while (G > 1 && (ntiles + G - 1) / G < min_wg) G >>= 1;
  if (const int eg = knob(KNOB_GEMVS_G)) G = eg;
  int nsplit = 1;
  const bool can_split = epi == EPI_ATOMIC && !deterministic;
  if (can_split && G == 1) {
    while ((nsb + 8 * nsplit - 1) / (8 * nsplit) > s_target && (ntiles * nsplit) < 1024 && nsb / (2 * nsplit) >= 8)
      nsplit *= 2;
    if (const int es = knob(KNOB_GEMVS_SPLIT)) nsplit = es;
  }
  // LDS: M rows x the split's k-range of f16 x
  auto lds_of = [&](int ns) { return (size_t)M * ((nsb + ns - 1) / ns) * 256 * 2; };
  while (lds_of(nsplit) > 96 * 1024 && can_split) nsplit *= 2;
  pl.G = G;
  pl.sb_per_split = (nsb + nsplit - 1) / nsplit;
  pl.nsplit = (nsb + pl.sb_per_split - 1) / pl.sb_per_split;
  pl.lds = (size_t)M * pl.sb_per_split * 256 * 2;
  return pl;
}

// dynamic LDS of the single-row dot form: the staged x plus its correction table (16 B per
// super-block and lane group)
static size_t d1_lds(const GemvsPlan& pl) { return pl.lds + (size_t)pl.sb_per_split * 64; }

template <int PT, int EPI, int G, bool NORM, int NSO = 0, bool D1 = false>
static void gemvs_go(const GemvParams& p, const GemvsPlan& pl, hipStream_t st) {
  static const bool attr = [] {   // dynamic LDS past the 64 KB default (gfx950: 160 KB per workgroup)
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&mpk::gemvs_kernel<PT, EPI, G, NORM, NSO, D1>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024) == hipSuccess;
  }();
  const size_t lds = D1 ? d1_lds(pl) : pl.lds;
  if (!attr && lds > 60 * 1024) throw std::runtime_error("gemvs: cannot raise the dynamic LDS limit");
  hipLaunchKernelGGL((mpk::gemvs_kernel<PT, EPI, G, NORM, NSO, D1>), dim3((p.ntiles + G - 1) / G, pl.nsplit),
                     dim3(mpk::GS_NT), lds, st, p, pl.nsplit);
}

template <int PT, int EPI, bool NORM, int NSO, bool D1 = false>
static void gemvs_gn(const GemvParams& p, const GemvsPlan& pl, hipStream_t st) {
  switch (pl.G) {
    case 1: return gemvs_go<PT, EPI, 1, NORM, NSO, D1>(p, pl, st);
    case 2: return gemvs_go<PT, EPI, 2, NORM, NSO, D1>(p, pl, st);
    case 4: return gemvs_go<PT, EPI, 4, NORM, NSO, D1>(p, pl, st);
    case 8: return gemvs_go<PT, EPI, 8, NORM, NSO, D1>(p, pl, st);
    default: throw std::runtime_error("gemvs: G must be 1, 2, 4 or 8");
  }
}

// one row on the dot form (knob GEMVS_DOT): the quantized types that have one, default ring depth.
// Q6_K only behind the fused norm (qkv, gate/up, LM head): its unnormed down projection measured
// slower on the dot form (8B: 14.20 vs 13.59 us, 6 vs 7 waves per SIMD; profiles/r11f_*)
static bool use_d1(int pt, const GemvParams& p) {
  return p.M == 1 && knob(KNOB_GEMVS_DOT) != 0 &&
         (pt == P_Q4_K || pt == P_Q5_K || pt == P_Q8_0 || (pt == P_Q6_K && p.Xf != nullptr));
}

template <int PT, int EPI, bool NORM>
static void gemvs_g(const GemvParams& p, const GemvsPlan& pl, hipStream_t st) {
  // weight super-blocks in flight per wave: 2 by default -- residency beats per-wave depth here
  // (NS 2: 80 VGPRs, 3 workgroups per CU; NS 4: 104 VGPRs, 2; NS 8: 3 waves/SIMD).  r5o / r5p:
  // 8B Q4_K_M mb1 NS 2 / 3 / 4 / 8 -> 548 / 541 / 524 / 441 tok/s, 70B Q4_K 105.4 / 106.6 / 104.4 / 91.1
  // (the knob only admits 2, 3 and 4; 16-bit weights always run the default depth)
  // (4 super-blocks in flight for the one-round residual GEMVs -- down, o: one workgroup per CU, so
  // residency is not what limits them -- measured slower: Q6_K down 12.81 -> 14.96 us, Q4_K down
  // 9.41 -> 9.58; profiles/r12g_prof_8b_mb1.txt)
  const int ns = knob(KNOB_GEMVS_NS);
  if constexpr (mpk::dot1_supported<PT>()) {
    if (use_d1(PT, p)) return gemvs_gn<PT, EPI, NORM, 2, true>(p, pl, st);
  }
  if constexpr (!is16(PT)) {
    if (ns == 2) return gemvs_gn<PT, EPI, NORM, 2>(p, pl, st);
    if (ns == 3) return gemvs_gn<PT, EPI, NORM, 3>(p, pl, st);
  }
  gemvs_gn<PT, EPI, NORM, 0>(p, pl, st);   // NS 4
}

template <int PT>
static void gemvs_pt(int epi, const GemvParams& p, const GemvsPlan& pl, hipStream_t st) {
  const bool norm = p.Xf != nullptr;
  switch (epi) {
    case EPI_STORE:
      if (p.qa.pos) return gemvs_g<PT, mpk::EPI_QKV, true>(p, pl, st);   // norm required (launch_gemvs checks)
      return norm ? gemvs_g<PT, EPI_STORE, true>(p, pl, st) : gemvs_g<PT, EPI_STORE, false>(p, pl, st);
    case EPI_ATOMIC: return norm ? gemvs_g<PT, EPI_ATOMIC, true>(p, pl, st) : gemvs_g<PT, EPI_ATOMIC, false>(p, pl, st);
    case EPI_SWIGLU: return norm ? gemvs_g<PT, EPI_SWIGLU, true>(p, pl, st) : gemvs_g<PT, EPI_SWIGLU, false>(p, pl, st);
  }
}

template <int PT, int PT2, int G, int EPI, bool D1>
static void gemvs2_go_e(const GemvParams& p, const GemvParams& p2, size_t lds, hipStream_t st) {
  static const bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&mpk::gemvs2_kernel<PT, PT2, G, EPI, D1>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, 152 * 1024) == hipSuccess;
  }();
  if (D1) lds += (size_t)p.sb_per_split * 64;   // the correction table
  if (!attr && lds > 60 * 1024) throw std::runtime_error("gemvs2: cannot raise the dynamic LDS limit");
  const int nwg1 = (p.ntiles + G - 1) / G, nwg2 = (p2.ntiles + G - 1) / G;
  hipLaunchKernelGGL((mpk::gemvs2_kernel<PT, PT2, G, EPI, D1>), dim3(nwg1 + nwg2), dim3(mpk::GS_NT), lds, st, p, p2, nwg1);
}
template <int PT, int PT2, int G>
static void gemvs2_go(const GemvParams& p, const GemvParams& p2, size_t lds, hipStream_t st) {
  const bool d1 = use_d1(PT, p) && use_d1(PT2, p2);
  if (p.qa.pos) {
    if (d1) gemvs2_go_e<PT, PT2, G, mpk::EPI_QKV, true>(p, p2, lds, st);
    else gemvs2_go_e<PT, PT2, G, mpk::EPI_QKV, false>(p, p2, lds, st);
  } else {
    if (d1) gemvs2_go_e<PT, PT2, G, EPI_STORE, true>(p, p2, lds, st);
    else gemvs2_go_e<PT, PT2, G, EPI_STORE, false>(p, p2, lds, st);
  }
}

template <int PT, int PT2>
static void gemvs2_g(int G, const GemvParams& p, const GemvParams& p2, size_t lds, hipStream_t st) {
  switch (G) {
    case 1: return gemvs2_go<PT, PT2, 1>(p, p2, lds, st);
    case 2: return gemvs2_go<PT, PT2, 2>(p, p2, lds, st);
    case 4: return gemvs2_go<PT, PT2, 4>(p, p2, lds, st);
    case 8: return gemvs2_go<PT, PT2, 8>(p, p2, lds, st);
    default: throw std::runtime_error("gemvs2: G must be 1, 2, 4 or 8");
  }
}

bool gemvs2_supported(int pt, int pt2) {
  return (pt == P_Q4_K || pt == P_Q5_K) && (pt2 == P_Q6_K || pt2 == P_Q8_0);
}

void launch_gemvs2(int pt, int pt2, GemvParams p, GemvParams p2, hipStream_t st) {
  if (!gemvs2_supported(pt, pt2)) throw std::runtime_error("launch_gemvs2: unsupported type pair");
  if (p.M < 1 || p.M > 4 || p2.M != p.M) throw std::runtime_error("launch_gemvs2: M must be 1..4 and equal");
  if ((p.qa.pos != nullptr) != (p2.qa.pos != nullptr) || (p.qa.pos && (p.qa.hd % 16 || p.qa.col0 % 16 || p2.qa.col0 % 16)))
    throw std::runtime_error("launch_gemvs2: both segments take the q|k|v append epilogue or neither");
  if (!p.Xf || !p2.Xf || p.nsb != p2.nsb || p.d_norm != p2.d_norm || (p.d_norm & 7) || p.d_norm > p.nsb * 256)
    throw std::runtime_error("launch_gemvs2: both segments need the same fused-norm input and K");
  // one plan for the union of the tiles (the shared G sizes both segments' workgroups)
  const GemvsPlan pl = plan_gemvs(p.ntiles + p2.ntiles, p.nsb, p.M, EPI_STORE, true, true);
  if (pl.nsplit != 1 || pl.lds + (size_t)pl.sb_per_split * 64 > 150 * 1024)
    throw std::runtime_error("launch_gemvs2: x k-range does not fit LDS");
  p.sb_per_split = p2.sb_per_split = pl.sb_per_split;
#ifdef MIPIPE_TIMING_PROBES
  p.probe = p2.probe = knob(KNOB_GEMVS_PROBE);
#endif
  if (pt == P_Q4_K) {
    if (pt2 == P_Q6_K) gemvs2_g<P_Q4_K, P_Q6_K>(pl.G, p, p2, pl.lds, st);
    else gemvs2_g<P_Q4_K, P_Q8_0>(pl.G, p, p2, pl.lds, st);
  } else {
    if (pt2 == P_Q6_K) gemvs2_g<P_Q5_K, P_Q6_K>(pl.G, p, p2, pl.lds, st);
    else gemvs2_g<P_Q5_K, P_Q8_0>(pl.G, p, p2, pl.lds, st);
  }
}

void launch_gemvs(int ptype, int epi, GemvParams p, bool deterministic, hipStream_t st, int force_G, int force_split) {
  if (p.M < 1 || p.M > 4) throw std::runtime_error("launch_gemvs: M must be 1..4");
  if (p.Xf && (p.d_norm <= 0 || (p.d_norm & 7) || p.d_norm > p.nsb * 256))
    throw std::runtime_error("launch_gemvs: fused RMSNorm needs d_norm a multiple of 8 within the padded K");
  if (!p.Xf && !p.X) throw std::runtime_error("launch_gemvs: no input");
  if (p.qa.pos && (epi != EPI_STORE || !p.Xf || p.qa.hd % 16 || p.qa.col0 % 16 || p.qa.hd > p.qa.Dp))
    throw std::runtime_error("launch_gemvs: the q|k|v append epilogue needs STORE, the fused norm and 16-aligned heads");
  GemvsPlan pl = plan_gemvs(p.ntiles, p.nsb, p.M, epi, p.Xf != nullptr, deterministic);
  if (force_G) pl.G = force_G;
  if (force_split) {   // tests: an explicit k-split over grid.y
    pl.sb_per_split = (p.nsb + force_split - 1) / force_split;
    pl.nsplit = (p.nsb + pl.sb_per_split - 1) / pl.sb_per_split;
    pl.lds = (size_t)p.M * pl.sb_per_split * 256 * 2;
  }
  if (pl.lds + (size_t)pl.sb_per_split * 64 > 150 * 1024) throw std::runtime_error("launch_gemvs: x k-range does not fit LDS");
  if (epi != EPI_ATOMIC && pl.nsplit != 1) throw std::runtime_error("launch_gemvs: only ATOMIC splits K");
  p.sb_per_split = pl.sb_per_split;
  p.rpf = knob(KNOB_GEMVS_RPF);
#ifdef MIPIPE_TIMING_PROBES
  p.probe = knob(KNOB_GEMVS_PROBE);
#endif
  switch (ptype) {
    case P_Q4_K: gemvs_pt<P_Q4_K>(epi, p, pl, st); break;
    case P_Q5_K: gemvs_pt<P_Q5_K>(epi, p, pl, st); break;
    case P_Q6_K: gemvs_pt<P_Q6_K>(epi, p, pl, st); break;
    case P_Q8_0: gemvs_pt<P_Q8_0>(epi, p, pl, st); break;
    case P_Q4_0: gemvs_pt<P_Q4_0>(epi, p, pl, st); break;
    case P_F16: gemvs_pt<P_F16>(epi, p, pl, st); break;
    case P_BF16: gemvs_pt<P_BF16>(epi, p, pl, st); break;
    default: throw std::runtime_error("launch_gemvs: unknown packed type");
  }
}

}  // namespace mp
