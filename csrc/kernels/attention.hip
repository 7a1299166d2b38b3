// Paged GQA attention on MFMA (K7): flash-decoding split-K for decode, the same kernel with
// several query tokens per row group for (chunked) prefill.
//
// One workgroup = (row group, kv head, kv split).  A row group is up to 16 MFMA rows
// rho = tq_i * G + g (tq tokens of ONE sequence x the G query heads sharing kv head `kvh`).
// Per 32-key chunk a wave computes S^T = K * Q^T with two chains of v_mfma_f32_16x16x32_f16
// (A = K rows, B = Q^T), with key rows permuted pi(c, R) = 8(R>>2) + 4c + (R&3) so that the
// exponentiated scores already sit in the lanes/registers of the B operand of the P.V product
// (O^T = V^T P^T, A = V^T read from the transposed V page) -- no LDS round trip, no shuffles for P.
// Online softmax in registers; 4 waves interleave chunks and are merged through LDS; splits are
// merged by attn_combine (LSE merge).  KV pages hold 64 tokens: K [64][Dp], V^T [Dp][64].
#include <stdexcept>
#include <type_traits>
#include "../runtime/tuning.h"

#include "kcommon.h"
#include "dequant.h"
#include "../runtime/kernels_api.h"

namespace mpk {
using namespace mp;

template <int DP>
__global__ __launch_bounds__(256) void attn_kernel(const AttnParams p) {
  constexpr int KK = DP / 32;   // k-steps of QK^T
  constexpr int DT = DP / 16;   // 16-row d tiles of O^T
  __shared__ float sm_m[4][16], sm_l[4][16];
  __shared__ float sm_o[4][16][DP];

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q4 = lane >> 4, col = lane & 15;
  const int grp = blockIdx.x, kvh = blockIdx.y, z = blockIdx.z;
  const int G = p.Hq / p.Hkv;
  const int t0 = grp * p.tq;
  const int tq_i = col / G, g = col % G;
  const int t = t0 + tq_i;
  const bool rvalid = (tq_i < p.tq) && (t < p.M) && (col < G * p.tq);
  const int tl = min(t0 + p.tq, p.M) - 1;           // last token of the group
  const int slot = p.slot[t0];
  const int maxlen = p.kvlen[tl];
  const int my_len = rvalid ? p.kvlen[t] : 0;
  const int h = kvh * G + g;

  const int start = z * p.split_len;
  const int end = min(start + p.split_len, maxlen);
  const size_t row_id = (size_t)t * p.Hq + h;

  if (start >= end) {
    // empty split: publish (m=-inf, l=0); combine skips it
    if (wave == 0 && q4 == 0 && rvalid && p.n_split > 1) {
      float* ml = p.ml_part + ((size_t)z * p.M * p.Hq + row_id) * 2;
      ml[0] = -INFINITY; ml[1] = 0.f;
    }
    return;
  }

  // Q^T fragments: lane holds q[t][h][d = 32kk + 8q4 + j]
  half8_t qf[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    half8_t zf = {};
    qf[kk] = rvalid ? *reinterpret_cast<const half8_t*>(p.q + row_id * DP + 32 * kk + 8 * q4) : zf;
  }

  f32x4 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run = -INFINITY, l_run = 0.f;

  const int32_t* bt = p.block_table + (size_t)slot * p.max_pages;
  const int nch = (end - start + 31) / 32;
  const int R = col;
  const int krow0 = 8 * (R >> 2) + (R & 3);      // pi(c, R) - 4c

  for (int ci = wave; ci < nch; ci += 4) {
    const int P0 = start + ci * 32;
    const int page = bt[P0 >> 6];
    const int in_page = P0 & 63;
    const f16* kbase = p.k_cache + ((size_t)page * p.Hkv + kvh) * 64 * DP;
    const f16* vbase = p.v_cache + ((size_t)page * p.Hkv + kvh) * DP * 64;
    half8_t kf[2][KK];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        kf[c][kk] = *reinterpret_cast<const half8_t*>(kbase + (size_t)(in_page + krow0 + 4 * c) * DP + 32 * kk + 8 * q4);
    half8_t vf[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      vf[dt] = *reinterpret_cast<const half8_t*>(vbase + (size_t)(16 * dt + col) * 64 + in_page + 8 * q4);

    f32x4 s[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) a = mfma16x16x32(kf[c][kk], qf[kk], a);
      s[c] = a;
    }
    // lane holds scores for row `col`, keys P0 + 8*q4 + 4c + i
    float mx = -INFINITY;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kpos = P0 + 8 * q4 + 4 * c + i;
        const float v = kpos < my_len ? s[c][i] : -INFINITY;
        s[c][i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    const float m_new = fmaxf(m_run, mx);
    const float alpha = (m_new == -INFINITY) ? 1.f : __expf(m_run - m_new);
    float pv[2][4];
    float psum = 0.f;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float e = (m_new == -INFINITY) ? 0.f : __expf(s[c][i] - m_new);
        pv[c][i] = e;
        psum += e;
      }
    l_run = l_run * alpha + psum;
    m_run = m_new;
    half8_t pf = {(f16)pv[0][0], (f16)pv[0][1], (f16)pv[0][2], (f16)pv[0][3],
                  (f16)pv[1][0], (f16)pv[1][1], (f16)pv[1][2], (f16)pv[1][3]};
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      f32x4 acc = o[dt] * alpha;
      o[dt] = mfma16x16x32(vf[dt], pf, acc);
    }
  }
  // per-row totals across the 4 lane groups
  l_run += __shfl_xor(l_run, 16);
  l_run += __shfl_xor(l_run, 32);
  if (q4 == 0) { sm_m[wave][col] = m_run; sm_l[wave][col] = l_run; }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) sm_o[wave][col][16 * dt + 4 * q4 + i] = o[dt][i];
  __syncthreads();

  // merge the 4 waves: thread handles (row, d) pairs
  for (int e = threadIdx.x; e < 16 * DP; e += 256) {
    const int row = e / DP, d = e % DP;
    const int rt = t0 + row / G;
    const bool ok = (row / G < p.tq) && (rt < p.M) && (row < G * p.tq);
    if (!ok) continue;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < 4; ++w) M = fmaxf(M, sm_m[w][row]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      if (sm_m[w][row] == -INFINITY) continue;
      const float f = __expf(sm_m[w][row] - M);
      L += sm_l[w][row] * f;
      O += sm_o[w][row][d] * f;
    }
    const int hh = kvh * G + row % G;
    const size_t rid = (size_t)rt * p.Hq + hh;
    if (p.n_split == 1) {
      if (d < p.hd) p.out[(size_t)rt * p.ldo + hh * p.hd + d] = (f16)(L > 0.f ? O / L : 0.f);
    } else {
      p.o_part[((size_t)z * p.M * p.Hq + rid) * DP + d] = O;
      if (d == 0) {
        float* ml = p.ml_part + ((size_t)z * p.M * p.Hq + rid) * 2;
        ml[0] = M; ml[1] = L;
      }
    }
  }
}

template <int DP>
__global__ __launch_bounds__(DP) void attn_combine_kernel(const AttnParams p) {
  const int rid = blockIdx.x;                // t*Hq + h
  const int t = rid / p.Hq, h = rid % p.Hq;
  const int d = threadIdx.x;
  const size_t stride = (size_t)p.M * p.Hq;
  float M = -INFINITY;
  for (int z = 0; z < p.n_split; ++z) M = fmaxf(M, p.ml_part[(z * stride + rid) * 2]);
  float L = 0.f, O = 0.f;
  for (int z = 0; z < p.n_split; ++z) {
    const float mz = p.ml_part[(z * stride + rid) * 2], lz = p.ml_part[(z * stride + rid) * 2 + 1];
    if (lz == 0.f || mz == -INFINITY) continue;
    const float f = __expf(mz - M);
    L += lz * f;
    O += p.o_part[(z * stride + rid) * DP + d] * f;
  }
  if (d < p.hd) p.out[(size_t)t * p.ldo + h * p.hd + d] = (f16)(L > 0.f ? O / L : 0.f);
}


// ---------------------------------------------------------------- fused decode attention
// One launch per layer for decode (tq = 1): RoPE of q (in registers) and of the new k, the KV-cache
// append (done by the split that owns the new position, before it reads its keys), flash-decoding
// over the split, and the split merge by the LAST-arriving split of each (token, kv head)
// (partials published with sc1 write-through stores, an agent-scope counter, sc1 loads): replaces
// rope_kv + attn + attn_combine (three launches, ~16 us per layer at 16 sequences).
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int ATTN_MAX_SPLITS = 128;   // host clamps n_split (hip_stage.cpp)

// F8: the KV pages hold e4m3 bytes (kv_dtype "fp8"): half the KV bytes per step; fragments are
// loaded raw (8 bytes per 8 keys / dims), kept raw through the prefetch, converted to f16 at use
// PF: each wave loads its next chunk before the current chunk's math (short contexts: one split,
// latency-bound); without it the kernel needs ~40 % fewer VGPRs (occupancy 3 instead of 2), which
// the many-split long contexts need more (8B 32K mb8: 1019 vs 960 tok/s)
// (t, kvh, z): token, kv head, KV split.  xo (LDS, one split only): the G heads' outputs of token
// t land there, [r * hd + d], instead of p.out (the fused attention + o-projection kernel)
// q fragments of the G query heads of kv head kvh for token t with RoPE applied in registers:
// lane (q4, col) holds q[h = kvh G + col][d = 32kk + 8q4 + j] (zero for col >= G).  Used by the
// fused decode attention bodies (workgroup- and wave-level).
// A block-table entry through the scalar cache: the table is read-only for the whole launch, but
// with K / V stores in the same kernel the compiler cannot prove that and loads it with a VECTOR
// load -- whose use then waits vmcnt(0), draining every K / V chunk still in flight (in the wave
// kernel that serialised the two-chunks-in-flight loop to one chunk; r8o ISA).  The constant
// address space lets it use s_load (lgkm counter only).
__device__ __forceinline__ int ld_bt(const int32_t* p) {
  typedef const __attribute__((address_space(4))) int32_t cint;
  return *(cint*)(uintptr_t)p;
}

// One 32-key chunk's online softmax for the decode attention, in the exp2 domain (the q fragments
// carry log2(e) in their scale, decode_q_frags) with a lazy rescale: the running reference m_run
// moves only when some lane's chunk maximum exceeds it by more than 8 (p = 2^(s - m_run) <= 256,
// exact enough in f16 for the PV MFMA; l and O stay relative to the same reference), so most
// chunks skip the exp of alpha and the 4 DT multiplies of O * alpha; the key mask only in the
// chunk that crosses the context end.  (Per 32-key chunk the old form spent ~240 VALU; the decode
// attention is bound by this per-chunk work, not by its loads: profiles/r8n_attn_variants.txt.)
template <int DT>
__device__ __forceinline__ half8_t softmax_chunk(f32x4 (&sc)[2], bool mask, int P0, int q4, int end, float& m_run,
                                                 float& l_run, f32x4 (&o)[DT]) {
  if (mask) {   // wave-uniform
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (P0 + 8 * q4 + 4 * c + i >= end) sc[c][i] = -INFINITY;
  }
  float mx = fmaxf(fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3])),
                   fmaxf(fmaxf(sc[1][0], sc[1][1]), fmaxf(sc[1][2], sc[1][3])));
  mx = fmaxf(mx, __shfl_xor(mx, 16));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  if (__builtin_amdgcn_ballot_w64(mx > m_run + 8.f) != 0) {   // wave-uniform rescale
    const float m_new = fmaxf(m_run, mx);
    const float alpha = m_run == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m_run - m_new);
    l_run *= alpha;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    m_run = m_new;
  }
  const float mr = m_run == -INFINITY ? 0.f : m_run;   // (a lane with no finite score yet: p = 0)
  float pv[2][4];
  float psum = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float e = __builtin_amdgcn_exp2f(sc[c][i] - mr);
      pv[c][i] = e;
      psum += e;
    }
  l_run += psum;
  return half8_t{(f16)pv[0][0], (f16)pv[0][1], (f16)pv[0][2], (f16)pv[0][3],
                 (f16)pv[1][0], (f16)pv[1][1], (f16)pv[1][2], (f16)pv[1][3]};
}

// ROT = false: q is already rotated (the qkv GEMV's append epilogue, DecodeAttnParams::pre)
template <int KK, bool ROT = true>
__device__ __forceinline__ void decode_q_frags(const DecodeAttnParams& p, const float* row, const float2* cs, float nrs,
                                               int kvh, int G, int q4, int col, half8_t (&qf)[KK]) {
  const int g = col;
  const bool rvalid = col < G;
  const int h = kvh * G + g;
  const float qsc = p.q_scale * 1.4426950408889634f;   // exp2-domain scores (softmax_chunk)
  auto qkv_at = [&](int i) { return p.bias ? fmaf(nrs, row[i], p.bias[i]) : nrs * row[i]; };
  // q fragments with RoPE applied in registers: lane holds q[h][d = 32kk + 8q4 + j].  Built
  // before the append so its loads overlap the append's, and (head_dim % 8 == 0) from
  // unconditional 16-byte loads issued together: written as guarded scalar reads (qkv_at per
  // element) the compiler serialised ~32 dependent load round trips here, ~10 us of fixed cost per
  // call whatever the context (measured: 12.7 us at 20 keys, mb64).
  if ((p.hd & 7) == 0) {
    const int hs = rvalid ? h : kvh * G;          // idle MFMA columns read a valid head, then zero
    // bias / no-bias as two straight-line bodies: a bias branch inside the loop split the loads
    // into per-kk groups, each waited for before the next was issued
    // two k-slices per batch of loads: all KK at once peaked at ~180 VGPRs for DP=128 (occupancy 2)
    constexpr int KH = KK < 2 ? KK : 2;
    auto build = [&](auto with_bias) {
      constexpr bool HB = decltype(with_bias)::value;
#pragma unroll
      for (int k0 = 0; k0 < KK; k0 += KH) {
      float4 xa[KH][2], ca[KH][2], ba[KH][2];
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) {
        const int kk = k0 + kh;
        const int d0 = 32 * kk + 8 * q4;
        const int dl = d0 < p.hd ? d0 : 0;
        const float4* xs = reinterpret_cast<const float4*>(row + hs * p.hd + dl);
        const float4* cp = reinterpret_cast<const float4*>(cs + dl / 2);
        xa[kh][0] = xs[0]; xa[kh][1] = xs[1];
        if constexpr (ROT) { ca[kh][0] = cp[0]; ca[kh][1] = cp[1]; }
        if constexpr (HB) {
          const float4* bs = reinterpret_cast<const float4*>(p.bias + hs * p.hd + dl);
          ba[kh][0] = bs[0]; ba[kh][1] = bs[1];
        }
      }
#pragma unroll
      for (int kh = 0; kh < KH; ++kh) {
        const int kk = k0 + kh;
        const int d0 = 32 * kk + 8 * q4;
        const bool ok = rvalid && d0 < p.hd;
        float x[8] = {xa[kh][0].x, xa[kh][0].y, xa[kh][0].z, xa[kh][0].w, xa[kh][1].x, xa[kh][1].y, xa[kh][1].z, xa[kh][1].w};
        float c[8] = {};
        if constexpr (ROT) {
          const float cc[8] = {ca[kh][0].x, ca[kh][0].y, ca[kh][0].z, ca[kh][0].w, ca[kh][1].x, ca[kh][1].y, ca[kh][1].z, ca[kh][1].w};
#pragma unroll
          for (int j = 0; j < 8; ++j) c[j] = cc[j];
        }
        if constexpr (HB) {
          const float b[8] = {ba[kh][0].x, ba[kh][0].y, ba[kh][0].z, ba[kh][0].w, ba[kh][1].x, ba[kh][1].y, ba[kh][1].z, ba[kh][1].w};
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] = fmaf(nrs, x[j], b[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) x[j] *= nrs;
        }
        half8_t v = {};
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          if constexpr (ROT) {
            v[j] = ok ? (f16)((x[j] * c[j] - x[j + 1] * c[j + 1]) * qsc) : (f16)0.f;
            v[j + 1] = ok ? (f16)((x[j] * c[j + 1] + x[j + 1] * c[j]) * qsc) : (f16)0.f;
          } else {
            v[j] = ok ? (f16)(x[j] * qsc) : (f16)0.f;
            v[j + 1] = ok ? (f16)(x[j + 1] * qsc) : (f16)0.f;
          }
        }
        qf[kk] = v;
      }
      }
    };
    if (p.bias) build(std::true_type{});
    else build(std::false_type{});
  } else {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      half8_t v = {};
      if (rvalid) {
        const int d0 = 32 * kk + 8 * q4;
        const int qr = h * p.hd;
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
          const int d = d0 + j;
          if (d < p.hd) {
            const float x0 = qkv_at(qr + d), x1 = qkv_at(qr + d + 1);
            const float2 c = ROT ? cs[d >> 1] : make_float2(1.f, 0.f);
            v[j] = (f16)((x0 * c.x - x1 * c.y) * qsc);
            v[j + 1] = (f16)((x0 * c.y + x1 * c.x) * qsc);
          }
        }
      }
      qf[kk] = v;
    }
  }

}

#ifdef MIPIPE_TIMING_PROBES
__device__ int g_attn_probe_calls = 0;
#endif

// PRE: q arrives rotated and the new token's K / V are already in the cache (the qkv GEMV's append
// epilogue, DecodeAttnParams::pre): no append, no RoPE, and no dependent position -> page chain
template <int DP, bool F8, bool PF, int NW = 4, bool PRE = false>
__device__ __forceinline__ void attn_decode_body(const DecodeAttnParams& p, const int t, const int kvh, const int z,
                                                 f16* xo = nullptr) {
  using KR = std::conditional_t<F8, u32x2, half8_t>;   // raw fragment: 8 elements
  auto cvt = [](const KR& r) -> half8_t {
    if constexpr (F8) return f8x8_to_h8(r);
    else return r;
  };
  constexpr int KK = DP / 32;
  constexpr int DT = DP / 16;
  __shared__ float sm_m[NW][16], sm_l[NW][16];
  __shared__ float sm_o[NW][16][DP];
  __shared__ float sm_mz[16][ATTN_MAX_SPLITS], sm_lz[16][ATTN_MAX_SPLITS];   // split merge
  __shared__ int sm_last;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#ifdef MIPIPE_TIMING_PROBES
  // bit 2 of the probe: per-phase timestamps of wave 0 (100 MHz s_memrealtime), printed for the
  // first calls by block (0, 0, 0): where a short context's fixed cost goes
  uint64_t ts[8] = {};
  const bool stamp = (p.probe & 4) && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0;
#define ATT_STAMP(i) do { if (stamp) ts[i] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define ATT_STAMP(i) do {} while (0)
#endif
  ATT_STAMP(0);
  const int q4 = lane >> 4, col = lane & 15;
  const int G = p.Hq / p.Hkv;
  const int g = col;
  const bool rvalid = col < G;
  const int pos = p.pos[t];
  const int kvlen = pos + 1;
  // decode rows map to slots slot0 + t (HipStage::slot_of): no dependent load before the block table
  const int slot = __builtin_amdgcn_readfirstlane(p.slot0 >= 0 ? p.slot0 + t : p.slot[t]);
  const int h = kvh * G + g;
  const int hd2 = p.hd / 2;
  const float* row = p.qkv + (size_t)t * p.ldqkv;
  const float2* cs = p.rope_cs + (size_t)pos * hd2;
  const int32_t* bt = p.block_table + (size_t)slot * p.max_pages;
  // deferred RMSNorm of the projection GEMV: value i of q|k|v = nrs * row[i] + bias[i]
  const float nrs = p.ssq ? rsqrtf(p.ssq[t] / (float)p.d_model + p.eps) : 1.f;

  const int start = z * p.split_len;
  const int krow0 = 8 * (col >> 2) + (col & 3);
  const int wv = __builtin_amdgcn_readfirstlane(wave);
  constexpr int EB = F8 ? 1 : 2;   // bytes per cached element
  auto load = [&](int ci, KR (&kf)[2][KK], KR (&vf)[DT]) {
    const int P0 = start + ci * 32;
    const int page = ld_bt(bt + (P0 >> 6));
    const int in_page = P0 & 63;
    const uint8_t* kbase = reinterpret_cast<const uint8_t*>(p.k_cache) + ((size_t)page * p.Hkv + kvh) * 64 * DP * EB;
    const uint8_t* vbase = reinterpret_cast<const uint8_t*>(p.v_cache) + ((size_t)page * p.Hkv + kvh) * DP * 64 * EB;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        kf[c][kk] = *reinterpret_cast<const KR*>(kbase + ((size_t)(in_page + krow0 + 4 * c) * DP + 32 * kk + 8 * q4) * EB);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      vf[dt] = *reinterpret_cast<const KR*>(vbase + ((size_t)(16 * dt + col) * 64 + in_page + 8 * q4) * EB);
  };
  KR kA[2][KK], vA[DT], kB[2][KK], vB[DT];
  // one split (short contexts): each wave's first chunk is loaded before the position arrives
  // (chunks past the sequence read the pool's trash page and are never used; never past the
  // slot's block-table row: split_len may exceed max_pages * 64)
  const bool pre = PF && p.n_split == 1 && 32 * wv < min(p.split_len, p.max_pages * 64 - start);
  if (pre) load(wv, kA, vA);
  // and its second chunk (keys 128-255 of the split): with it loaded only inside the chunk loop,
  // after the q build, wave 0 waited one more dependent round trip at 129-256 keys (the 8B single
  // stream's ~2.8 us chunk phase, r8i attention stamps)
  const bool pre2 = pre && 32 * (wv + NW) < min(p.split_len, p.max_pages * 64 - start);
  if (pre2) load(wv + NW, kB, vB);

  const int end = min(start + p.split_len, kvlen);
  // splits past the sequence's length take no part (no partials, no counter): with n_act == 1 the
  // single active split writes the output directly, so short contexts pay no merge round trip
  const int n_act = (kvlen + p.split_len - 1) / p.split_len;
  if (z >= n_act) return;
  ATT_STAMP(1);

  // 1. the new token's K / V inputs (the split that owns the position) and, without the pre-load,
  // this wave's first chunk: issued BEFORE the q fragments' loads, so the one wait the q build
  // ends with covers them too (issued after it, the append's loads had cost a third dependent
  // global round trip per call: the single-stream fixed cost, profiles/r8d_attn_ctx_sweep.txt)
  __shared__ __attribute__((aligned(16))) f16 sm_kn[DP];
  __shared__ f16 sm_vn[DP];
  const bool owns = !PRE && start <= pos && pos < end;
  const int nch = (end - start + 31) / 32;
  if (PF && !pre && wv < nch) load(wv, kA, vA);   // in flight during the q build and the append
  const int j = threadIdx.x;   // the append: one K pair and one V element per thread (DP <= 256 threads)
  float2 kx = {0.f, 0.f}, kb = {0.f, 0.f}, c = {1.f, 0.f};
  float vx = 0.f, vb = 0.f;
  const bool kin = j < hd2, vin = j < p.hd;
  int a_page = 0;
  if (owns) {
    a_page = bt[pos >> 6];
    const int kr = p.Hq * p.hd + kvh * p.hd;
    const int vr = (p.Hq + p.Hkv) * p.hd + kvh * p.hd;
    if (kin) {
      kx = *reinterpret_cast<const float2*>(row + kr + 2 * j);
      c = cs[j];
      if (p.bias) kb = *reinterpret_cast<const float2*>(p.bias + kr + 2 * j);
    }
    if (vin) {
      vx = row[vr + j];
      if (p.bias) vb = p.bias[vr + j];
    }
  }

  // 2. q fragments with RoPE applied in registers (decode_q_frags)
  half8_t qf[KK];
  decode_q_frags<KK, !PRE>(p, row, cs, nrs, kvh, G, q4, col, qf);
  ATT_STAMP(2);

  // 3. append the new token's K (rotated) and V to the cache.  The split that reads the new token
  // also keeps them in LDS and patches them into the registers of the chunk that holds it, so no
  // wave waits for its own global append to land (no store -> barrier -> load round trip).
  if (owns) {
    const int page = a_page, idx = pos & 63;
    const size_t koff = (((size_t)page * p.Hkv + kvh) * 64 + idx) * DP;     // element offsets
    const size_t voff = ((size_t)page * p.Hkv + kvh) * DP * 64 + idx;
    if (j < DP / 2) {
      const float x0 = fmaf(nrs, kx.x, kb.x), x1 = fmaf(nrs, kx.y, kb.y);
      const float r0 = kin ? x0 * c.x - x1 * c.y : 0.f, r1 = kin ? x0 * c.y + x1 * c.x : 0.f;
      half2_t o;
      if constexpr (F8) {   // the patch sees exactly what later steps read back from the cache
        const uint32_t q = f8x2_pack(r0, r1);
        *reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(p.k_cache) + koff + 2 * j) = (uint16_t)q;
        o = f8x2_lo(q);
      } else {
        o = half2_t{(f16)r0, (f16)r1};
        if (!(p.probe & 2)) *reinterpret_cast<half2_t*>(p.k_cache + koff + 2 * j) = o;
      }
      *reinterpret_cast<half2_t*>(sm_kn + 2 * j) = o;
    }
    if (j < DP) {
      const float vv = vin ? fmaf(nrs, vx, vb) : 0.f;
      f16 v;
      if constexpr (F8) {
        const uint32_t q = f8x2_pack(vv, 0.f);
        reinterpret_cast<uint8_t*>(p.v_cache)[voff + (size_t)j * 64] = (uint8_t)q;
        v = f8x2_lo(q).x;
      } else {
        v = (f16)vv;
        if (!(p.probe & 1)) p.v_cache[voff + (size_t)j * 64] = v;
      }
      sm_vn[j] = v;
    }
    // LDS-only release/acquire around the barrier: the global append needs no wait here
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  }
  ATT_STAMP(3);

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one 32-key chunk: patch the new token in (if this chunk holds it), S^T = K Q^T, online
  // softmax, O^T += V^T P^T
  auto step_h = [&](int ci, half8_t (&kf)[2][KK], half8_t (&vf)[DT]) {
    const int P0 = start + ci * 32;
    if (owns && pos >= P0 && pos < P0 + 32) {   // wave-uniform
      const int r = pos - P0;
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (krow0 + 4 * c == r) {
#pragma unroll
          for (int kk = 0; kk < KK; ++kk) kf[c][kk] = *reinterpret_cast<const half8_t*>(sm_kn + 32 * kk + 8 * q4);
        }
      if ((r >> 3) == q4) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const f16 v = sm_vn[16 * dt + col];
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (e == (r & 7)) vf[dt][e] = v;
        }
      }
    }
    f32x4 sc[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) a = mfma16x16x32(kf[c][kk], qf[kk], a);
      sc[c] = a;
    }
    const half8_t pf = softmax_chunk<DT>(sc, P0 + 32 > end, P0, q4, end, m_run, l_run, o);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = mfma16x16x32(vf[dt], pf, o[dt]);
  };
  auto step = [&](int ci, KR (&kraw)[2][KK], KR (&vraw)[DT]) {
    if constexpr (F8) {   // convert the raw e4m3 fragments at use (the prefetch holds raw bytes)
      half8_t kf[2][KK], vf[DT];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) kf[c][kk] = cvt(kraw[c][kk]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) vf[dt] = cvt(vraw[dt]);
      step_h(ci, kf, vf);
    } else {
      step_h(ci, kraw, vraw);
    }
  };
  // waves take chunks wv, wv + NW, ...; the next chunk's loads are issued before this one's math
  if constexpr (PF) {
    for (int ci = wv; ci < nch;) {
      if (ci + NW < nch && !(pre2 && ci == wv)) load(ci + NW, kB, vB);
      step(ci, kA, vA);
      ci += NW;
      if (ci >= nch) break;
      if (ci + NW < nch) load(ci + NW, kA, vA);
      step(ci, kB, vB);
      ci += NW;
    }
  } else {
    for (int ci = wv; ci < nch; ci += NW) {
      load(ci, kA, vA);
      step(ci, kA, vA);
    }
  }
  l_run += __shfl_xor(l_run, 16);
  l_run += __shfl_xor(l_run, 32);
  ATT_STAMP(4);
  if (q4 == 0) { sm_m[wave][col] = m_run; sm_l[wave][col] = l_run; }
#pragma unroll
  for (int dt = 0; dt < DT; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) sm_o[wave][col][16 * dt + 4 * q4 + i] = o[dt][i];
  __syncthreads();

  // 3. merge the 4 waves; publish (n_split > 1) or write the output
  const size_t stride = (size_t)p.M * p.Hq;
  for (int e = threadIdx.x; e < G * DP; e += NW * 64) {
    const int r = e / DP, d = e % DP;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) M = fmaxf(M, sm_m[w][r]);
    float L = 0.f, O = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      if (sm_m[w][r] == -INFINITY) continue;
      const float f = __builtin_amdgcn_exp2f(sm_m[w][r] - M);
      L += sm_l[w][r] * f;
      O += sm_o[w][r][d] * f;
    }
    const int hh = kvh * G + r;
    const size_t rid = (size_t)t * p.Hq + hh;
    if (n_act == 1) {
      if (d < p.hd) {
        const f16 v = (f16)(L > 0.f ? O / L : 0.f);
        if (xo) xo[r * p.hd + d] = v;
        else p.out[(size_t)t * p.ldo + hh * p.hd + d] = v;
      }
    } else {
      st_sc1(p.o_part + ((size_t)z * stride + rid) * DP + d, O);
      if (d == 0) {
        st_sc1(p.ml_part + ((size_t)z * stride + rid) * 2, M);
        st_sc1(p.ml_part + ((size_t)z * stride + rid) * 2 + 1, L);
      }
    }
  }
#ifdef MIPIPE_TIMING_PROBES
  if (stamp) {
    __builtin_amdgcn_s_waitcnt(0);
    ts[5] = __builtin_amdgcn_s_memrealtime();
    if (atomicAdd(&g_attn_probe_calls, 1) < 6)
      printf("attn stamps (x10 ns from entry): pos %d  pos/bt %d  q+loads %d  append %d  chunks %d  merge+store %d\n", pos,
             (int)(ts[1] - ts[0]), (int)(ts[2] - ts[0]), (int)(ts[3] - ts[0]), (int)(ts[4] - ts[0]), (int)(ts[5] - ts[0]));
  }
#endif
  if (n_act == 1) return;
  // 4. last arriver of this (token, kv head) merges the splits.
  // Hand-off invariant (MI355X_MICROARCH.md 'Valid forms', first row of the sc1 table, measured on
  // gfx950 / ROCm 7.2 rather than guaranteed by the memory model): EVERY store of the partials is an
  // agent-scope relaxed (sc1, write-through) store, every storing wave drains them (vmcnt(0)) before
  // the workgroup barrier, ONE lane then adds to ONE unsharded counter, the workgroup whose add
  // returned n_act - 1 is the last arriver, and EVERY load of the partials below is an sc1 load
  // (ld_sc1), issued after the barrier that the adding wave joins.  Changing any of these (plain
  // stores or loads, a flag store instead of the counter, a read before the barrier) needs the
  // agent release/acquire fences instead.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int old = __hip_atomic_fetch_add(p.counters + (size_t)t * p.Hkv + kvh, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
    sm_last = old == n_act - 1;
  }
  __syncthreads();
  if (!sm_last) return;
  // merge: the (m, l) pairs of every (head row, split) are read once, in parallel, into LDS; each
  // head's max, weights and sum are formed there by one wave; then every output element sums its
  // n_act partials with independent loads.  (Reading the pairs per element in a serial loop made
  // the merge the long-context bottleneck: 8B single stream at 32K context spent ~60 us/layer.)
  for (int i = threadIdx.x; i < G * n_act; i += NW * 64) {
    const int r = i / n_act, zz = i - r * n_act;
    const size_t rid = (size_t)t * p.Hq + kvh * G + r;
    sm_mz[r][zz] = ld_sc1(p.ml_part + (zz * stride + rid) * 2);
    sm_lz[r][zz] = ld_sc1(p.ml_part + (zz * stride + rid) * 2 + 1);
  }
  __syncthreads();
  for (int r = wave; r < G; r += NW) {
    float M = -INFINITY;
    for (int zz = lane; zz < n_act; zz += 64) M = fmaxf(M, sm_mz[r][zz]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) M = fmaxf(M, __shfl_xor(M, o));
    float L = 0.f;
    for (int zz = lane; zz < n_act; zz += 64) {
      const float mz = sm_mz[r][zz];
      const float f = mz == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mz - M);
      sm_mz[r][zz] = f;   // becomes the split's weight
      L += sm_lz[r][zz] * f;
    }
    L = wave_sum(L);
    if (lane == 0) sm_m[0][r] = L;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < G * DP; e += NW * 64) {
    const int r = e / DP, d = e % DP;
    const int hh = kvh * G + r;
    const size_t rid = (size_t)t * p.Hq + hh;
    float O = 0.f;
#pragma unroll 8
    for (int zz = 0; zz < n_act; ++zz) O += sm_mz[r][zz] * ld_sc1(p.o_part + (zz * stride + rid) * DP + d);
    const float L = sm_m[0][r];
    if (d < p.hd) p.out[(size_t)t * p.ldo + hh * p.hd + d] = (f16)(L > 0.f ? O / L : 0.f);
  }
  if (threadIdx.x == 0)
    __hip_atomic_store(p.counters + (size_t)t * p.Hkv + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int DP, bool F8, bool PRE = false>
__global__ __launch_bounds__(256) void attn_decode_kernel(const DecodeAttnParams p) {
  attn_decode_body<DP, F8, true, 4, PRE>(p, blockIdx.x, blockIdx.y, blockIdx.z);
}
// single stream / tiny micro-batches (few (token, kv head) workgroups, short contexts): 8 waves, so
// every 32-key chunk of a context up to 256 keys has its own wave (with 4, wave 0 computed chunks 0
// and 4 one after the other: the ~2.8 us chunk phase of profiles/r8j_attn_stamps.txt)
template <int DP, bool F8, bool PRE = false>
__global__ __launch_bounds__(512) void attn_decode_kernel8(const DecodeAttnParams p) {
  attn_decode_body<DP, F8, true, 8, PRE>(p, blockIdx.x, blockIdx.y, blockIdx.z);
}
// many-split long contexts: 3 workgroups per CU (occupancy, not per-wave latency, is what they need)
template <int DP, bool F8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void attn_decode_kernel_np(
    const DecodeAttnParams p) {
  attn_decode_body<DP, F8, false>(p, blockIdx.x, blockIdx.y, blockIdx.z);
}

// ---------------------------------------------------------------- wave-level decode attention
// Wide micro-batches (many (token, kv head) pairs): ONE WAVE per (token, kv head, split) streams its
// keys chunk after chunk with the next chunk's K / V in flight, and owns the whole softmax state, so
// there is no cross-wave LDS merge and no workgroup barrier; the 4 waves of a workgroup are 4
// independent items (consecutive kv heads of a token: they share the position, block-table and q
// row loads in L2).  The workgroup kernel above spends most of a 128-key context on fixed costs
// (profiles/r7u: 2048 workgroups, waves 55 % of their life waiting on memory, the 4-wave merge);
// here every wave has 32 KB of K / V in flight from its first chunk on.
// Splits (few pairs, long contexts): partials + the last-arriving wave of the (token, kv head)
// merges, with the same sc1 publish / counter / sc1 load hand-off as attn_decode_body.
template <int DP, bool F8>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void attn_decode_wave_kernel(const DecodeAttnParams p) {
  using KR = std::conditional_t<F8, u32x2, half8_t>;
  constexpr int KK = DP / 32, DT = DP / 16, EB = F8 ? 1 : 2;
  __shared__ __attribute__((aligned(16))) f16 sm_kn[4][DP];
  __shared__ f16 sm_vn[4][DP];
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q4 = lane >> 4, col = lane & 15;
  const int item = blockIdx.x * 4 + wv;
  const int per_t = p.Hkv * p.n_split;
  const int t = item / per_t;
  if (t >= p.M) return;   // wave-uniform; no workgroup barrier anywhere below
  const int kvh = (item - t * per_t) / p.n_split, z = item % p.n_split;
  const int G = p.Hq / p.Hkv;
  const int pos = p.pos[t];
  const int kvlen = pos + 1;
  const int start = z * p.split_len;
  const int end = min(start + p.split_len, kvlen);
  const int n_act = (kvlen + p.split_len - 1) / p.split_len;
  if (z >= n_act) return;
  const int hd2 = p.hd / 2;
  const float* row = p.qkv + (size_t)t * p.ldqkv;
  const float2* cs = p.rope_cs + (size_t)pos * hd2;
  const int32_t* bt = p.block_table + (size_t)__builtin_amdgcn_readfirstlane(p.slot0 >= 0 ? p.slot0 + t : p.slot[t]) * p.max_pages;
  const float nrs = p.ssq ? rsqrtf(p.ssq[t] / (float)p.d_model + p.eps) : 1.f;
  const int nch = (end - start + 31) / 32;
  const int krow0 = 8 * (col >> 2) + (col & 3);

  auto load = [&](int ci, KR (&kf)[2][KK], KR (&vf)[DT]) {
    const int P0 = start + ci * 32;
    const int page = ld_bt(bt + (P0 >> 6));
    const int in_page = P0 & 63;
    const uint8_t* kbase = reinterpret_cast<const uint8_t*>(p.k_cache) + ((size_t)page * p.Hkv + kvh) * 64 * DP * EB;
    const uint8_t* vbase = reinterpret_cast<const uint8_t*>(p.v_cache) + ((size_t)page * p.Hkv + kvh) * DP * 64 * EB;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        kf[c][kk] = *reinterpret_cast<const KR*>(kbase + ((size_t)(in_page + krow0 + 4 * c) * DP + 32 * kk + 8 * q4) * EB);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
      vf[dt] = *reinterpret_cast<const KR*>(vbase + ((size_t)(16 * dt + col) * 64 + in_page + 8 * q4) * EB);
  };
  KR kA[2][KK], vA[DT], kB[2][KK], vB[DT];
  load(0, kA, vA);   // in flight during the q build and the append
  if (nch > 1) load(1, kB, vB);

  // the split holding the new position appends its K (rotated) / V and keeps them in this wave's
  // LDS slice to patch the chunk that holds it (the chunk's loads may predate the append).  Its
  // inputs are loaded before the q build, so the q build's wait covers them (no third round trip)
  const bool owns = start <= pos && pos < end;
  f16* kn = sm_kn[wv];
  f16* vn = sm_vn[wv];
  constexpr int KJ = (DP / 2 + 63) / 64, VJ = DP / 64;
  float2 kx[KJ], kb[KJ], cc[KJ];
  float vx[VJ], vb[VJ];
  int a_page = 0;
  const int kr = p.Hq * p.hd + kvh * p.hd;
  const int vr = (p.Hq + p.Hkv) * p.hd + kvh * p.hd;
  if (owns) {
    a_page = bt[pos >> 6];
#pragma unroll
    for (int jj = 0; jj < KJ; ++jj) {   // K: one pair per lane per 128 dims
      const int j = lane + 64 * jj;
      kx[jj] = kb[jj] = float2{0.f, 0.f};
      cc[jj] = float2{1.f, 0.f};
      if (j < DP / 2 && j < hd2) {
        kx[jj] = *reinterpret_cast<const float2*>(row + kr + 2 * j);
        cc[jj] = cs[j];
        if (p.bias) kb[jj] = *reinterpret_cast<const float2*>(p.bias + kr + 2 * j);
      }
    }
#pragma unroll
    for (int jj = 0; jj < VJ; ++jj) {    // V: one element per lane per 64 dims
      const int j = lane + 64 * jj;
      vx[jj] = vb[jj] = 0.f;
      if (j < p.hd) {
        vx[jj] = row[vr + j];
        if (p.bias) vb[jj] = p.bias[vr + j];
      }
    }
  }

  half8_t qf[KK];
  decode_q_frags<KK>(p, row, cs, nrs, kvh, G, q4, col, qf);

  if (owns) {
    const int page = a_page, idx = pos & 63;
    const size_t koff = (((size_t)page * p.Hkv + kvh) * 64 + idx) * DP;
    const size_t voff = ((size_t)page * p.Hkv + kvh) * DP * 64 + idx;
#pragma unroll
    for (int jj = 0; jj < KJ; ++jj) {
      const int j = lane + 64 * jj;
      if (j >= DP / 2) break;
      const bool kin = j < hd2;
      const float x0 = fmaf(nrs, kx[jj].x, kb[jj].x), x1 = fmaf(nrs, kx[jj].y, kb[jj].y);
      const float2 c = cc[jj];
      const float r0 = kin ? x0 * c.x - x1 * c.y : 0.f, r1 = kin ? x0 * c.y + x1 * c.x : 0.f;
      half2_t o;
      if constexpr (F8) {
        const uint32_t q = f8x2_pack(r0, r1);
        *reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(p.k_cache) + koff + 2 * j) = (uint16_t)q;
        o = f8x2_lo(q);
      } else {
        o = half2_t{(f16)r0, (f16)r1};
        *reinterpret_cast<half2_t*>(p.k_cache + koff + 2 * j) = o;
      }
      *reinterpret_cast<half2_t*>(kn + 2 * j) = o;
    }
#pragma unroll
    for (int jj = 0; jj < VJ; ++jj) {
      const int j = lane + 64 * jj;
      const bool vin = j < p.hd;
      const float vv = vin ? fmaf(nrs, vx[jj], vb[jj]) : 0.f;
      f16 v;
      if constexpr (F8) {
        const uint32_t q = f8x2_pack(vv, 0.f);
        reinterpret_cast<uint8_t*>(p.v_cache)[voff + (size_t)j * 64] = (uint8_t)q;
        v = f8x2_lo(q).x;
      } else {
        v = (f16)vv;
        p.v_cache[voff + (size_t)j * 64] = v;
      }
      vn[j] = v;
    }
  }

  float m_run = -INFINITY, l_run = 0.f;
  f32x4 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto step_h = [&](int ci, half8_t (&kf)[2][KK], half8_t (&vf)[DT]) {
    const int P0 = start + ci * 32;
    if (owns && pos >= P0 && pos < P0 + 32) {   // wave-uniform
      const int r = pos - P0;
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (krow0 + 4 * c == r) {
#pragma unroll
          for (int kk = 0; kk < KK; ++kk) kf[c][kk] = *reinterpret_cast<const half8_t*>(kn + 32 * kk + 8 * q4);
        }
      if ((r >> 3) == q4) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          const f16 v = vn[16 * dt + col];
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (e == (r & 7)) vf[dt][e] = v;
        }
      }
    }
    f32x4 sc[2];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f32x4 a = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) a = mfma16x16x32(kf[c][kk], qf[kk], a);
      sc[c] = a;
    }
    const half8_t pf = softmax_chunk<DT>(sc, P0 + 32 > end, P0, q4, end, m_run, l_run, o);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) o[dt] = mfma16x16x32(vf[dt], pf, o[dt]);
  };
  // f16 pages: the loaded registers are used (and patched) in place; e4m3: converted at use
  auto step = [&](int ci, KR (&kraw)[2][KK], KR (&vraw)[DT]) {
    if constexpr (F8) {
      half8_t kf[2][KK], vf[DT];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) kf[c][kk] = f8x8_to_h8(kraw[c][kk]);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) vf[dt] = f8x8_to_h8(vraw[dt]);
      step_h(ci, kf, vf);
    } else {
      step_h(ci, kraw, vraw);
    }
  };
  // two chunks in flight: chunk ci + 2 is loaded into the registers chunk ci frees
  for (int ci = 0; ci < nch;) {
    step(ci, kA, vA);
    if (ci + 2 < nch) load(ci + 2, kA, vA);
    if (++ci >= nch) break;
    step(ci, kB, vB);
    if (ci + 2 < nch) load(ci + 2, kB, vB);
    ++ci;
  }
  l_run += __shfl_xor(l_run, 16);
  l_run += __shfl_xor(l_run, 32);
  // lane (q4, col) holds O^T[d = 16 dt + 4 q4 + i][head col]
  const int h = kvh * G + col;
  const size_t rid = (size_t)t * p.Hq + h;
  if (n_act == 1) {
    if (col < G) {
      const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        const int d = 16 * dt + 4 * q4;
        if (d < p.hd) {
          typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
          const half4_t v = {(f16)(o[dt][0] * inv), (f16)(o[dt][1] * inv), (f16)(o[dt][2] * inv), (f16)(o[dt][3] * inv)};
          *reinterpret_cast<half4_t*>(p.out + (size_t)t * p.ldo + h * p.hd + d) = v;
        }
      }
    }
    return;
  }
  // publish this split's partials (sc1 write-through), then one counter add per wave
  const size_t stride = (size_t)p.M * p.Hq;
  if (col < G) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) st_sc1(p.o_part + ((size_t)z * stride + rid) * DP + 16 * dt + 4 * q4 + i, o[dt][i]);
    if (q4 == 0) {
      st_sc1(p.ml_part + ((size_t)z * stride + rid) * 2, m_run);
      st_sc1(p.ml_part + ((size_t)z * stride + rid) * 2 + 1, l_run);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0)
    old = __hip_atomic_fetch_add(p.counters + (size_t)t * p.Hkv + kvh, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0);
  if (old != n_act - 1) return;
  // last arriver: lane (q4, col) merges head col's dims 16 dt + 4 q4 + i over the splits
  if (col < G) {
    float M = -INFINITY;
    for (int zz = 0; zz < n_act; ++zz) M = fmaxf(M, ld_sc1(p.ml_part + (zz * stride + rid) * 2));
    float L = 0.f;
    f32x4 acc[DT];
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int zz = 0; zz < n_act; ++zz) {
      const float mz = ld_sc1(p.ml_part + (zz * stride + rid) * 2);
      const float f = mz == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(mz - M);
      L += ld_sc1(p.ml_part + (zz * stride + rid) * 2 + 1) * f;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[dt][i] += f * ld_sc1(p.o_part + (zz * stride + rid) * DP + 16 * dt + 4 * q4 + i);
    }
    const float inv = L > 0.f ? 1.f / L : 0.f;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = 16 * dt + 4 * q4 + i;
        if (d < p.hd) p.out[(size_t)t * p.ldo + h * p.hd + d] = (f16)(acc[dt][i] * inv);
      }
  }
  if (lane == 0)
    __hip_atomic_store(p.counters + (size_t)t * p.Hkv + kvh, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// global -> LDS DMA, 16 B per active lane to (wave-uniform LDS base) + lane * 16 (gemm3.hip glds;
// inline asm so the compiler's waitcnt pass does not drain it at the next ds_read)
__device__ __forceinline__ void glds16(const void* g, void* lds) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds);
  // m0 bound as an input operand (a clobbered m0 is a reserved register: -Winline-asm, gemm_lds.h glds)
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "{m0}"(m0) : "memory");
}

// Fused single-stream decode attention + output projection (one launch instead of two: the o GEMV
// of one token is bound by its launch and ramp, ~5.6 us for 9 MB at 8B, not by its bytes).
//   workgroup (r, kvh), grid (ntiles / TPW, Hkv):
//   1. LDS-DMA of its W_o slice: output tiles [r TPW, r TPW + TPW) x the KS super-blocks of k that
//      kv head kvh's G query heads feed (k in [kvh G hd, (kvh + 1) G hd)); in flight during 2.
//   2. the attention of kv head kvh for every token (one split; the R = ntiles / TPW workgroups of
//      a head each compute it: short contexts only, the host gates on max_ctx), outputs to LDS.
//   3. split-K GEMV of the slice on MFMA (the decode GEMV's dequant), atomics into the residual:
//      Hkv partial sums per output (not bitwise reproducible: the deterministic mode keeps the
//      two-kernel path).
//   Waves 0-3 run the attention, waves 4-7 issue the W_o DMA: the vector memory counter retires in
//   issue order per wave, so when the attention waves issued the DMA too, their first K / V wait
//   waited for the whole W_o slice (~37 KB per CU) behind it.  All 8 waves then take one output tile
//   each.  The DMA waves match the attention body's barriers (PRE: one per token, else two) and the
//   one after each token.
template <int DP, bool F8, int PT, int TPW, int KS, bool PRE>
__global__ __launch_bounds__(512) void attn_o_kernel(const DecodeAttnParams p, const AttnOParams o) {
  using D = Deq<PT>;
  constexpr int CB = D::CB, TB = KS * CB, WB = TPW * TB;
  static_assert(TB % 16 == 0, "attn_o: 16-B DMA pieces");
  static_assert(TPW <= 8, "attn_o: one output tile per wave");
  __shared__ __attribute__((aligned(16))) uint8_t wl[WB];
  __shared__ __attribute__((aligned(16))) f16 xo[4][KS * 256];
  const int r = blockIdx.x, kvh = blockIdx.y;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile0 = r * TPW, sb0 = kvh * KS;
  constexpr int NI = (WB + 1023) / 1024;
  const int M = p.M;
  if (wave >= 4) {
    for (int i = wave - 4; i < NI; i += 4) {
      const int off = i * 1024 + lane * 16;
      if (off < WB) {
        const int u = off / TB, rem = off - u * TB;
        const int tile = min(tile0 + u, o.ntiles - 1);
        glds16(o.W + ((size_t)tile * o.nsb + sb0) * CB + rem, wl + i * 1024);
      }
    }
    for (int t = 0; t < M; ++t) {
      if constexpr (!PRE) __syncthreads();   // the body's append barrier (one split: it owns the position)
      __syncthreads();                       // the body's wave merge
      __syncthreads();                       // after the token
    }
  } else {
    for (int t = 0; t < M; ++t) {
      attn_decode_body<DP, F8, true, 4, PRE>(p, t, kvh, 0, &xo[t][0]);
      __syncthreads();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const Consts kc = make_consts();
  const int g = lane >> 4, m = lane & 15;
  for (int u = wave; u < TPW; u += 8) {
    const int tile = tile0 + u;
    if (tile >= o.ntiles) break;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      typename D::Raw raw;
      D::load(raw, LdsSrc{wl + (u * KS + s) * CB}, lane);
      half8_t b[4];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 0) D::template dequant<0>(raw, b, lane, kc);
        else D::template dequant<1>(raw, b, lane, kc);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          half8_t a = {};
          if (m < M) a = *reinterpret_cast<const half8_t*>(&xo[m][s * 256 + t16_xoff(g, 4 * h + i)]);
          acc = mma<false>(a, b[i], acc);
        }
      }
    }
    // lane holds C[token 4g + v][output 16 tile + m]
    const int n = tile * 16 + m;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int t = 4 * g + v;
      if (t < M && n < o.n_valid) unsafeAtomicAdd(o.Y + (size_t)t * o.ldy + n, acc[v]);
    }
  }
}

}  // namespace mpk

namespace mp {

void launch_attention(const AttnParams& p, hipStream_t st) {
  const int ng = (p.M + p.tq - 1) / p.tq;
  dim3 grid(ng, p.Hkv, p.n_split);
  if (p.Dp == 128) {
    hipLaunchKernelGGL(mpk::attn_kernel<128>, grid, dim3(256), 0, st, p);
    if (p.n_split > 1) hipLaunchKernelGGL(mpk::attn_combine_kernel<128>, dim3(p.M * p.Hq), dim3(128), 0, st, p);
  } else {
    hipLaunchKernelGGL(mpk::attn_kernel<64>, grid, dim3(256), 0, st, p);
    if (p.n_split > 1) hipLaunchKernelGGL(mpk::attn_combine_kernel<64>, dim3(p.M * p.Hq), dim3(64), 0, st, p);
  }
}

// LSE merge of n_split partials (o_part / ml_part, [z][m * Hq + h]) into out
void launch_attn_combine(const AttnParams& p, hipStream_t st) {
  if (p.Dp == 128) hipLaunchKernelGGL(mpk::attn_combine_kernel<128>, dim3(p.M * p.Hq), dim3(128), 0, st, p);
  else hipLaunchKernelGGL(mpk::attn_combine_kernel<64>, dim3(p.M * p.Hq), dim3(64), 0, st, p);
}

// many splits / many workgroups: the 3-per-CU variant without the next-chunk prefetch
template <bool F8>
static void attn_decode_go(const DecodeAttnParams& p, hipStream_t st) {
  dim3 grid(p.M, p.Hkv, p.n_split);
  if (p.Dp == 128) hipLaunchKernelGGL((mpk::attn_decode_kernel_np<128, F8>), grid, dim3(256), 0, st, p);
  else hipLaunchKernelGGL((mpk::attn_decode_kernel_np<64, F8>), grid, dim3(256), 0, st, p);
}

constexpr int kAttnOTpw = 8;   // output tiles per workgroup: 8B's W_o -> 32 x 8 = 256 workgroups

static int attn_o_ks(const DecodeAttnParams& p) { return (p.Hq / p.Hkv) * p.hd / 256; }

bool attn_o_supported(const DecodeAttnParams& p, const AttnOParams& o) {
  const int G = p.Hq / p.Hkv;
  if (p.M < 1 || p.M > 4 || p.Dp != 128 || p.hd != 128 || p.ssq || p.n_split != 1) return false;
  if (G * p.hd % 256 || attn_o_ks(p) != 2 || o.ntiles % kAttnOTpw) return false;
  if (o.ptype != P_Q4_K && o.ptype != P_Q6_K && o.ptype != P_Q8_0) return false;
  // one round of workgroups (LDS ~100 KB: one per CU)
  return o.ntiles / kAttnOTpw * p.Hkv <= 256;
}

template <bool F8, int PT>
static void attn_o_go(const DecodeAttnParams& p, const AttnOParams& o, hipStream_t st) {
  const dim3 grid(o.ntiles / kAttnOTpw, p.Hkv);
  if (p.pre) hipLaunchKernelGGL((mpk::attn_o_kernel<128, F8, PT, kAttnOTpw, 2, true>), grid, dim3(512), 0, st, p, o);
  else hipLaunchKernelGGL((mpk::attn_o_kernel<128, F8, PT, kAttnOTpw, 2, false>), grid, dim3(512), 0, st, p, o);
}

void launch_attn_o(const DecodeAttnParams& p, const AttnOParams& o, hipStream_t st) {
  if (!attn_o_supported(p, o)) throw std::runtime_error("launch_attn_o: unsupported shape");
  switch (o.ptype) {
    case P_Q4_K: return p.kv_fp8 ? attn_o_go<true, P_Q4_K>(p, o, st) : attn_o_go<false, P_Q4_K>(p, o, st);
    case P_Q6_K: return p.kv_fp8 ? attn_o_go<true, P_Q6_K>(p, o, st) : attn_o_go<false, P_Q6_K>(p, o, st);
    case P_Q8_0: return p.kv_fp8 ? attn_o_go<true, P_Q8_0>(p, o, st) : attn_o_go<false, P_Q8_0>(p, o, st);
  }
}

bool attn_decode_wave_selected(const DecodeAttnParams& p) {
  const int mode = knob(KNOB_ATTN_WAVE);   // 0 off, 1 on, 2 auto
  if (mode == 0) return false;
  if (mode == 1) return true;
  return (int64_t)p.M * p.Hkv * p.n_split >= knob(KNOB_ATTN_WAVE_MIN);
}

bool attn_decode_pre_ok(const DecodeAttnParams& p) {
  return !attn_decode_wave_selected(p) && p.n_split == 1 && p.M * p.Hkv <= knob(KNOB_ATTN_PF_MAXWG) && !p.ssq &&
         (p.Dp == 128 || p.Dp == 64);
}

template <bool F8, bool PRE>
static void attn_decode_pf(const DecodeAttnParams& p, hipStream_t st) {
  const dim3 grid(p.M, p.Hkv, 1);
  if (p.M * p.Hkv <= knob(KNOB_ATTN_NW8_MAXWG)) {
    if (p.Dp == 128) hipLaunchKernelGGL((mpk::attn_decode_kernel8<128, F8, PRE>), grid, dim3(512), 0, st, p);
    else hipLaunchKernelGGL((mpk::attn_decode_kernel8<64, F8, PRE>), grid, dim3(512), 0, st, p);
  } else {
    if (p.Dp == 128) hipLaunchKernelGGL((mpk::attn_decode_kernel<128, F8, PRE>), grid, dim3(256), 0, st, p);
    else hipLaunchKernelGGL((mpk::attn_decode_kernel<64, F8, PRE>), grid, dim3(256), 0, st, p);
  }
}

void launch_attn_decode(const DecodeAttnParams& p, hipStream_t st) {
  if (p.pre) {   // q rotated and K / V appended by the qkv GEMV (gemvs QkvAppend)
    if (!attn_decode_pre_ok(p)) throw std::runtime_error("launch_attn_decode: pre-appended inputs need the one-split kernel");
    return p.kv_fp8 ? attn_decode_pf<true, true>(p, st) : attn_decode_pf<false, true>(p, st);
  }
  if (attn_decode_wave_selected(p)) {
    const int items = p.M * p.Hkv * p.n_split;
    const dim3 grid((items + 3) / 4);
    if (p.Dp == 128) {
      if (p.kv_fp8) hipLaunchKernelGGL((mpk::attn_decode_wave_kernel<128, true>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((mpk::attn_decode_wave_kernel<128, false>), grid, dim3(256), 0, st, p);
    } else {
      if (p.kv_fp8) hipLaunchKernelGGL((mpk::attn_decode_wave_kernel<64, true>), grid, dim3(256), 0, st, p);
      else hipLaunchKernelGGL((mpk::attn_decode_wave_kernel<64, false>), grid, dim3(256), 0, st, p);
    }
    return;
  }
  // the next-chunk prefetch variant (2 workgroups per CU) for a single split per (token, kv head)
  // while the grid is small; many workgroups (long contexts, or wide micro-batches: M * Hkv above
  // MIPIPE_ATTN_PF_MAXWG) need occupancy more than per-wave latency: the 3-per-CU variant
  const int pf_max = knob(KNOB_ATTN_PF_MAXWG);
  const bool pf = p.n_split == 1 && p.M * p.Hkv <= pf_max;
  if (pf) return p.kv_fp8 ? attn_decode_pf<true, false>(p, st) : attn_decode_pf<false, false>(p, st);
  p.kv_fp8 ? attn_decode_go<true>(p, st) : attn_decode_go<false>(p, st);
}

}  // namespace mp
