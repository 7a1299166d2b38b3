// Prefill flash attention on MFMA (K7, prompt chunks): many query rows per workgroup, K/V tiles
// staged once per workgroup in LDS, causal tile skipping, one launch per packed chunk.
//
// The decode-shaped attn_kernel (attention.hip) gave every row group of 16 MFMA rows (2-4 tokens x
// the G heads of one kv head) its own pass over the whole K/V of the sequence: at a 32K prompt each
// layer-chunk re-streamed ~16 GB of K/V and attention was 64 % of prefill time
// (profiles/r1g_prof_8b_ctx32k_mb1.txt).  Here one 512-thread workgroup owns 128 MFMA rows
// rho = t * G + g (BT = 128 / G consecutive tokens of ONE sequence x the G query heads of kv head
// `kvh`), 16 rows per wave, and walks the 64-key pages up to its last token's position:
//   * the page's K [64][Dp] and V^T [Dp][64] are loaded once per workgroup (register prefetch of
//     page j+1 while page j is consumed) into padded, double-buffered LDS tiles shared by 8 waves;
//   * per 32-key chunk a wave computes S^T = K Q^T (A = K rows in the permuted order
//     pi(c, R) = 8(R>>2) + 4c + (R&3), B = Q^T in registers) so the exponentiated scores already
//     form the B operand of O^T += V^T P^T (A = V^T rows from LDS) -- as in the decode kernel;
//   * online softmax in f32 registers; keys past a row's own position are masked; pages past the
//     workgroup's last token are never touched (causal tile skip).
// Work list: the host splits every prefill segment (rows of one sequence, consecutive positions)
// into tiles of <= BT rows and passes them as kernel arguments (m0 | n << 16), so a chunk packing
// many sequences is one launch.
#include "kcommon.h"
#include "../runtime/kernels_api.h"

#include <algorithm>
#include <type_traits>
#include <stdexcept>

namespace mpk {
using namespace mp;

// NW waves x RG row groups of 16 MFMA rows = 128 rows per workgroup.  RG = 2 (every K / V^T
// fragment read from LDS feeding two MFMAs, 4 waves) took 260 us per 8B 32K-prompt layer chunk
// against 184 us for RG = 1 with 8 waves (190 vs 119 VGPRs: half the waves per SIMD;
// profiles/r2n_prof_8b_32k_rg*.txt), so the launcher instantiates RG = 1.
// F8: e4m3 KV pages (kv_dtype "fp8"), converted to f16 while staging into LDS
template <int DP, int NW, int RG, bool F8>
__global__ __launch_bounds__(NW * 64) void attn_prefill_kernel(const PrefillAttnParams p) {
  using KR = std::conditional_t<F8, u32x2, u32x4>;   // raw 8-element chunk
  constexpr int KK = DP / 32;    // k-steps of S^T over d
  constexpr int DT = DP / 16;    // 16-row d tiles of O^T
  constexpr int KLD = DP + 8;    // K tile row stride (f16): 16 key rows of a fragment hit distinct banks
  constexpr int VLD = 64 + 8;    // V^T tile row stride (f16)
  constexpr int NT = NW * 64;
  constexpr int KCH = 64 * DP / 8 / NT;   // 16 B K chunks per thread per page (= V chunks)
  static_assert(NW * RG * 16 == 128, "128 MFMA rows per workgroup");
  __shared__ __attribute__((aligned(16))) f16 ks[2][64 * KLD];
  __shared__ __attribute__((aligned(16))) f16 vs[2][DP * VLD];

  const int tile = blockIdx.x, kvh = blockIdx.y, z = blockIdx.z;
  if (tile >= p.n_tiles) return;
  const int m0 = (int)(p.tiles[tile] & 0xFFFFu), n = (int)(p.tiles[tile] >> 16);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q4 = lane >> 4, col = lane & 15;
  const int G = p.Hq / p.Hkv;
  bool rvalid[RG];
  int m[RG], h[RG], my_pos[RG];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg) {
    const int R = 16 * (RG * wave + rg) + col;   // MFMA row of this lane's column
    const int t = R / G, g = R - t * G;
    rvalid[rg] = t < n && R < (128 / G) * G;
    m[rg] = m0 + (rvalid[rg] ? t : 0);
    h[rg] = kvh * G + g;
    my_pos[rg] = rvalid[rg] ? p.pos[m[rg]] : -1;
  }
  const int pmax = p.pos[m0 + n - 1];       // rows of a tile: consecutive positions of one slot
  const int32_t* bt = p.block_table + (size_t)p.slot[m0] * p.max_pages;
  const int n_kt_all = pmax / 64 + 1;       // causal: pages past the last row are skipped
  // KV split z (grid.z) takes pages [kt0, kt1); its (m, l, O) partials are merged by attn_combine
  const int sp = p.n_split > 1 ? p.split_pages : n_kt_all;
  const int kt0 = min(z * sp, n_kt_all), kt1 = min(kt0 + sp, n_kt_all);
  const int n_kt = kt1 - kt0;

  // Q^T fragments: lane holds q[m][h][d = 32kk + 8q4 + j] (q_scale already applied), times log2(e)
  // so the softmax runs on v_exp_f32 (2^x) directly; m is kept in that base-2 domain
  half8_t qf[RG][KK];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      half8_t v = rvalid[rg] ? *reinterpret_cast<const half8_t*>(p.q + ((size_t)m[rg] * p.Hq + h[rg]) * DP + 32 * kk + 8 * q4)
                             : half8_t{};
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (f16)((float)v[j] * 1.4426950408889634f);
      qf[rg][kk] = v;
    }

  // page staging: thread owns K chunks (key = c / (DP/8), d8 = c % (DP/8)) and V^T chunks
  // (d = c / 8, k8 = c % 8), c = tid + NT j
  KR kr[KCH], vr[KCH];
  constexpr int EB = F8 ? 1 : 2;   // bytes per cached element
  auto load_page = [&](int kt) {
    const int page = bt[kt];
    const uint8_t* kb = reinterpret_cast<const uint8_t*>(p.k_cache) + ((size_t)page * p.Hkv + kvh) * 64 * DP * EB;
    const uint8_t* vb = reinterpret_cast<const uint8_t*>(p.v_cache) + ((size_t)page * p.Hkv + kvh) * DP * 64 * EB;
#pragma unroll
    for (int j = 0; j < KCH; ++j) {
      const int c = tid + NT * j;
      kr[j] = *reinterpret_cast<const KR*>(kb + (size_t)c * 8 * EB);
      vr[j] = *reinterpret_cast<const KR*>(vb + (size_t)c * 8 * EB);
    }
  };
  auto as16 = [](const KR& r) -> u32x4 {
    if constexpr (F8) return __builtin_bit_cast(u32x4, f8x8_to_h8(r));
    else return r;
  };
  auto store_page = [&](int buf) {
#pragma unroll
    for (int j = 0; j < KCH; ++j) {
      const int c = tid + NT * j;
      *reinterpret_cast<u32x4*>(&ks[buf][(c / (DP / 8)) * KLD + (c % (DP / 8)) * 8]) = as16(kr[j]);
      *reinterpret_cast<u32x4*>(&vs[buf][(c / 8) * VLD + (c % 8) * 8]) = as16(vr[j]);
    }
  };

  f32x4 o[RG][DT];
  float m_run[RG], l_run[RG];
#pragma unroll
  for (int rg = 0; rg < RG; ++rg) {
#pragma unroll
    for (int i = 0; i < DT; ++i) o[rg][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    m_run[rg] = -INFINITY;
    l_run[rg] = 0.f;
  }
  const int krow0 = 8 * (col >> 2) + (col & 3);   // pi(c, R) - 4c

  if (n_kt > 0) {
    load_page(kt0);
    store_page(0);
    __syncthreads();
    if (n_kt > 1) load_page(kt0 + 1);
  }
  const int pmin = p.pos[m0];               // the tile's first (smallest) position
  for (int kt = 0; kt < n_kt; ++kt) {
    const int buf = kt & 1;
    const f16* kt_s = ks[buf];
    const f16* vt_s = vs[buf];
    const bool full = (kt0 + kt) * 64 + 63 <= pmin;   // every key of the page is visible to every row
#pragma unroll
    for (int kc = 0; kc < 2; ++kc) {
      const int P0 = (kt0 + kt) * 64 + kc * 32;
      f32x4 s[RG][2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) s[rg][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          const half8_t kf = *reinterpret_cast<const half8_t*>(kt_s + (32 * kc + krow0 + 4 * c) * KLD + 32 * kk + 8 * q4);
#pragma unroll
          for (int rg = 0; rg < RG; ++rg) s[rg][c] = mfma16x16x32(kf, qf[rg][kk], s[rg][c]);
        }
      }
      half8_t pf[RG];
#pragma unroll
      for (int rg = 0; rg < RG; ++rg) {
        // lane holds scores of row `col` (row group rg) for keys P0 + 8 q4 + 4c + i
        float mx = -INFINITY;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float v = full || P0 + 8 * q4 + 4 * c + i <= my_pos[rg] ? s[rg][c][i] : -INFINITY;
            s[rg][c][i] = v;
            mx = fmaxf(mx, v);
          }
        mx = fmaxf(mx, __shfl_xor(mx, 16));
        mx = fmaxf(mx, __shfl_xor(mx, 32));
        // lazy rescale: the running max only moves when a score exceeds it by > 8 (2^8: P stays
        // far inside f16 range), so the O^T rescale (DT x 4 multiplies) is skipped on most chunks
        const bool resc = mx > m_run[rg] + 8.f;
        if (__any(resc)) {
          const float m_new = resc ? mx : m_run[rg];
          const float alpha = m_run[rg] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run[rg] - m_new);
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[rg][dt] *= alpha;
          l_run[rg] *= alpha;
          m_run[rg] = m_new;
        }
        float psum = 0.f;
        const float mb = m_run[rg] == -INFINITY ? 0.f : m_run[rg];   // all scores -inf then: 2^-inf = 0
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float e = __builtin_amdgcn_exp2f(s[rg][c][i] - mb);
            psum += e;
            pf[rg][4 * c + i] = (f16)e;
          }
        l_run[rg] += psum;
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const half8_t vf = *reinterpret_cast<const half8_t*>(vt_s + (16 * dt + col) * VLD + 32 * kc + 8 * q4);
#pragma unroll
        for (int rg = 0; rg < RG; ++rg) o[rg][dt] = mfma16x16x32(vf, pf[rg], o[rg][dt]);
      }
    }
    if (kt + 1 < n_kt) {
      store_page(buf ^ 1);        // page kt+1 (loaded one page ago); buf^1 was released by the last barrier
      __syncthreads();
      if (kt + 2 < n_kt) load_page(kt0 + kt + 2);
    }
  }
#pragma unroll
  for (int rg = 0; rg < RG; ++rg) {
    float l = l_run[rg];
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    if (!rvalid[rg]) continue;
    if (p.n_split > 1) {   // unnormalised partials, the attn_combine layout [z][m * Hq + h][Dp]
      const size_t rid = (size_t)m[rg] * p.Hq + h[rg], stride = (size_t)p.M * p.Hq;
      float* op = p.o_part + ((size_t)z * stride + rid) * DP;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
        *reinterpret_cast<float4*>(op + 16 * dt + 4 * q4) =
            make_float4(o[rg][dt][0], o[rg][dt][1], o[rg][dt][2], o[rg][dt][3]);
      if (q4 == 0) {
        float* ml = p.ml_part + ((size_t)z * stride + rid) * 2;
        ml[0] = n_kt > 0 && m_run[rg] != -INFINITY ? m_run[rg] * 0.6931471805599453f : -INFINITY;   // natural log
        ml[1] = n_kt > 0 ? l : 0.f;
      }
      continue;
    }
    const float inv = l > 0.f ? 1.f / l : 0.f;
    f16* orow = p.out + (size_t)m[rg] * p.ldo + (size_t)h[rg] * p.hd;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      const int d0 = 16 * dt + 4 * q4;   // lane holds O^T[d0 + i][row]
      if (d0 + 4 <= p.hd) {
        typedef _Float16 h4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<h4*>(orow + d0) = h4{(f16)(o[rg][dt][0] * inv), (f16)(o[rg][dt][1] * inv),
                                               (f16)(o[rg][dt][2] * inv), (f16)(o[rg][dt][3] * inv)};
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (d0 + i < p.hd) orow[d0 + i] = (f16)(o[rg][dt][i] * inv);
      }
    }
  }
}

}  // namespace mpk

namespace mp {

int prefill_attn_rows_per_tile(int G) { return 128 / G; }

void launch_attn_combine(const AttnParams& p, hipStream_t st);

void launch_attn_prefill(const PrefillAttnParams& p, hipStream_t st) {
  if (p.n_tiles <= 0) return;
  if (p.n_tiles > kPrefillAttnMaxTiles) throw std::runtime_error("launch_attn_prefill: too many tiles");
  if (p.Hq % p.Hkv || p.Hq / p.Hkv > 128) throw std::runtime_error("launch_attn_prefill: bad GQA group");
  if (p.n_split > 1 && (!p.o_part || !p.ml_part || p.split_pages < 1))
    throw std::runtime_error("launch_attn_prefill: split without partial buffers");
  const dim3 grid(p.n_tiles, p.Hkv, std::max(1, p.n_split));
  if (p.kv_fp8) {
    if (p.Dp == 128) hipLaunchKernelGGL((mpk::attn_prefill_kernel<128, 8, 1, true>), grid, dim3(512), 0, st, p);
    else if (p.Dp == 64) hipLaunchKernelGGL((mpk::attn_prefill_kernel<64, 8, 1, true>), grid, dim3(512), 0, st, p);
  } else if (p.Dp == 128) hipLaunchKernelGGL((mpk::attn_prefill_kernel<128, 8, 1, false>), grid, dim3(512), 0, st, p);
  else if (p.Dp == 64) hipLaunchKernelGGL((mpk::attn_prefill_kernel<64, 8, 1, false>), grid, dim3(512), 0, st, p);
  else throw std::runtime_error("launch_attn_prefill: Dp must be 64 or 128");
  if (p.n_split > 1) {   // LSE merge of the splits into out (attention.hip)
    AttnParams a{};
    a.M = p.M; a.Hq = p.Hq; a.hd = p.hd; a.Dp = p.Dp; a.n_split = p.n_split;
    a.o_part = p.o_part; a.ml_part = p.ml_part; a.out = p.out; a.ldo = p.ldo;
    launch_attn_combine(a, st);
  }
}

// KV splits for a chunk: enough (tile, kv head, split) workgroups to cover the CUs twice, >= 4 pages
// per split, at most max_split (the partial buffers)
int prefill_attn_splits(int n_tiles, int Hkv, int max_pages_needed, int max_split, int* split_pages) {
  const int wgs = std::max(1, n_tiles * Hkv);
  int ns = std::min(max_split, std::max(1, (512 + wgs - 1) / wgs));
  ns = std::max(1, std::min(ns, max_pages_needed / 4));
  *split_pages = (max_pages_needed + ns - 1) / ns;
  return (max_pages_needed + *split_pages - 1) / *split_pages;
}

}  // namespace mp
