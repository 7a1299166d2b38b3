// Memory-bound row kernels: RMSNorm (K2), embedding gather+dequant (K1), RoPE + paged KV append
// (K5+K6 fused), argmax (K12 greedy), decode-step advance, SwiGLU (K8, unfused fallback).
// All loads/stores of bf16/f16/f32 rows are vectorised (guide Guideline 13).
#include "kcommon.h"
#include <stdexcept>
#include "../runtime/kernels_api.h"
#include "../runtime/qtypes.h"

namespace mpk {
using namespace mp;

__device__ __forceinline__ float block_sum_256(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) t += red[i];
  __syncthreads();
  return t;
}

// One 1024-thread workgroup per row: each thread holds 8 floats of x (d <= 8192) and its 8 norm
// weights, both loaded before anything else so the two reads overlap; the split-K accumulator the
// next GEMV adds into is cleared by the same launch (16K floats per workgroup) after the loads are
// in flight.
// part (optional, d <= 8192 and d % 4 == 0): the residual first absorbs nsplit split-K GEMM partials
// (part + s * pstride + row * ldp, fixed order) and is written back before the norm (gemm_splitk_store)
__global__ __launch_bounds__(1024) void rmsnorm_kernel(const float* x, int ldx, const float* w, int d,
                                                       float eps, f16* out, int ldo, float* zero,
                                                       int64_t zero_n, int M, const float* bias, int bias_n,
                                                       const float* part, int nsplit, int64_t pstride, int ldp,
                                                       int8_t* q8, int ldq8, float* q8s) {
  __shared__ float red[16], red2[16];
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const bool fast = (d & 3) == 0 && d <= 8192;
  const float* xr = x + (size_t)row * ldx;
  float4 v[2], ww[2];
  if (row < M && fast) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = (tid + 1024 * k) * 4;
      v[k] = i < d ? *reinterpret_cast<const float4*>(xr + i) : make_float4(0.f, 0.f, 0.f, 0.f);
      ww[k] = i < d ? *reinterpret_cast<const float4*>(w + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (part) {
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = (tid + 1024 * k) * 4;
        if (i < d) {
          for (int sp = 0; sp < nsplit; ++sp) {
            const float4 a = *reinterpret_cast<const float4*>(part + (size_t)sp * pstride + (size_t)row * ldp + i);
            v[k].x += a.x; v[k].y += a.y; v[k].z += a.z; v[k].w += a.w;
          }
          *reinterpret_cast<float4*>(const_cast<float*>(xr) + i) = v[k];
        }
      }
    }
  }
  if (zero && bias) {
    const int64_t z0 = (int64_t)blockIdx.x * 16384, z1 = min(zero_n, z0 + 16384);
    for (int64_t i = z0 + tid; i < z1; i += 1024) zero[i] = bias[i % bias_n];
  } else if (zero) {
    const int64_t z0 = (int64_t)blockIdx.x * 16384, z1 = min(zero_n, z0 + 16384);
    for (int64_t i = z0 + tid * 4; i < z1; i += 4096) {
      if (i + 4 <= z1) *reinterpret_cast<float4*>(zero + i) = make_float4(0.f, 0.f, 0.f, 0.f);
      else for (int64_t k = i; k < z1; ++k) zero[k] = 0.f;
    }
  }
  if (row >= M) return;
  f16* o = out + (size_t)row * ldo;
  float ss = 0.f;
  if (fast) {
#pragma unroll
    for (int k = 0; k < 2; ++k) ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
  } else {
    for (int i = tid; i < d; i += 1024) ss += xr[i] * xr[i];
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) tot += red[i];
  const float sc = rsqrtf(tot / (float)d + eps);
  if (fast) {
    float qm = 0.f;
    half2_t hv[2][2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = (tid + 1024 * k) * 4;
      hv[k][0] = half2_t{(f16)(v[k].x * sc * ww[k].x), (f16)(v[k].y * sc * ww[k].y)};
      hv[k][1] = half2_t{(f16)(v[k].z * sc * ww[k].z), (f16)(v[k].w * sc * ww[k].w)};
      if (i < d) {
        u32x2 pk = {as_u32(hv[k][0]), as_u32(hv[k][1])};
        *reinterpret_cast<u32x2*>(o + i) = pk;
        qm = fmaxf(qm, fmaxf(fmaxf(fabsf((float)hv[k][0].x), fabsf((float)hv[k][0].y)),
                             fmaxf(fabsf((float)hv[k][1].x), fabsf((float)hv[k][1].y))));
      }
    }
    if (q8) {   // int8_gemm: the same f16 row quantized per row (quant_rows_i8_kernel's rounding)
      qm = wave_max(qm);
      if ((tid & 63) == 0) red2[tid >> 6] = qm;
      __syncthreads();
      qm = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) qm = fmaxf(qm, red2[i]);
      const float s = qm > 0.f ? qm / 127.f : 1.f, inv = 1.f / s;
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int i = (tid + 1024 * k) * 4;
        if (i < d) {
          const float e[4] = {(float)hv[k][0].x, (float)hv[k][0].y, (float)hv[k][1].x, (float)hv[k][1].y};
          uint32_t w = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) w |= ((uint32_t)(uint8_t)(int8_t)__float2int_rn(e[j] * inv)) << (8 * j);
          *reinterpret_cast<uint32_t*>(q8 + (size_t)row * ldq8 + i) = w;
        }
      }
      if (tid == 0) q8s[row] = s;
    }
  } else {
    for (int i = tid; i < d; i += 1024) o[i] = (f16)(xr[i] * sc * w[i]);
  }
}

// ---------------------------------------------------------------- embedding (raw GGUF rows)
__device__ float deq_elem(int t, const uint8_t* row, int e) {
  switch (t) {
    case T_F32: return reinterpret_cast<const float*>(row)[e];
    case T_F16: return h2f(reinterpret_cast<const uint16_t*>(row)[e]);
    case T_BF16: return bf16_to_f32(reinterpret_cast<const uint16_t*>(row)[e]);
    case T_Q8_0: {
      const uint8_t* b = row + (e / 32) * 34;
      return h2f(*reinterpret_cast<const uint16_t*>(b)) * (float)(int8_t)b[2 + e % 32];
    }
    case T_Q4_0: {
      const uint8_t* b = row + (e / 32) * 18;
      const int l = e % 32;
      const int q = l < 16 ? (b[2 + l] & 15) : (b[2 + l - 16] >> 4);
      return h2f(*reinterpret_cast<const uint16_t*>(b)) * (float)(q - 8);
    }
    case T_Q4_K: case T_Q5_K: {
      const int bb = t == T_Q4_K ? 144 : 176;
      const uint8_t* b = row + (e / 256) * bb;
      const int w = e % 256, c = w / 64, l = w % 64;
      const float d = h2f(*reinterpret_cast<const uint16_t*>(b));
      const float dmin = h2f(*reinterpret_cast<const uint16_t*>(b + 2));
      int sc, m;
      scale_min_k4(2 * c + (l >= 32), b + 4, sc, m);
      const uint8_t* qs = b + (t == T_Q4_K ? 16 : 48);
      int q = l < 32 ? (qs[32 * c + l] & 15) : (qs[32 * c + l - 32] >> 4);
      if (t == T_Q5_K) q += ((b[16 + (l & 31)] >> (2 * c + (l >= 32))) & 1) << 4;
      return d * sc * q - dmin * m;
    }
    case T_Q6_K: {
      const uint8_t* b = row + (e / 256) * 210;
      const int w = e % 256, n = w / 128, r = w % 128, k = r / 32, l = r % 32;
      const uint8_t* ql = b + 64 * n;
      const uint8_t* qh = b + 128 + 32 * n;
      const int8_t* sc = reinterpret_cast<const int8_t*>(b + 192) + 8 * n;
      const int lo = (k == 0) ? (ql[l] & 15) : (k == 1) ? (ql[l + 32] & 15) : (k == 2) ? (ql[l] >> 4) : (ql[l + 32] >> 4);
      const int hi = (qh[l] >> (2 * k)) & 3;
      const float d = h2f(*reinterpret_cast<const uint16_t*>(b + 208));
      return d * sc[l / 16 + 2 * k] * (float)((lo | (hi << 4)) - 32);
    }
  }
  return 0.f;
}

__global__ __launch_bounds__(256) void embed_kernel(int t, const uint8_t* table, int64_t rb, int d,
                                                    const int32_t* tokens, float* x, int ldx) {
  // one element per thread, d / 256 workgroups per token: each element is a short chain of
  // dependent block-header loads, so the row's latency is one chain, not d / 256 of them in a row
  // (one workgroup per token took 12.8 us for the 8B row, r5c_prof_8b_mb1.txt)
  const int m = blockIdx.x;
  const int e = blockIdx.y * 256 + threadIdx.x;
  if (e >= d) return;
  const uint8_t* row = table + (int64_t)tokens[m] * rb;
  x[(size_t)m * ldx + e] = deq_elem(t, row, e);
}

// ---------------------------------------------------------------- int8 activation rows (K15 prototype)
// per-row int8 activations: 16-byte loads of 8 f16, a max pass and a quantize pass over the row
// (the second from L2), 8-byte stores (the first version's per-element loads and byte stores took
// 39 us for 256 x 8192)
__global__ __launch_bounds__(256) void quant_rows_i8_kernel(const f16* X, int ldx, int K, int8_t* Q, int ldq, float* xs) {
  __shared__ float red[4];
  const int m = blockIdx.x, tid = threadIdx.x;
  const f16* x = X + (size_t)m * ldx;
  int8_t* q = Q + (size_t)m * ldq;
  const bool vec = (K & 7) == 0 && (ldx & 7) == 0 && (ldq & 7) == 0;
  float mx = 0.f;
  if (vec) {
    for (int k = tid * 8; k < K; k += 2048) {
      const half8_t v = *reinterpret_cast<const half8_t*>(x + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf((float)v[j]));
    }
  } else {
    for (int k = tid; k < K; k += 256) mx = fmaxf(mx, fabsf((float)x[k]));
  }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = mx > 0.f ? mx / 127.f : 1.f, inv = 1.f / s;
  if (vec) {
    for (int k = tid * 8; k < K; k += 2048) {
      const half8_t v = *reinterpret_cast<const half8_t*>(x + k);
      uint32_t w[2] = {0u, 0u};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        w[j >> 2] |= ((uint32_t)(uint8_t)(int8_t)__float2int_rn((float)v[j] * inv)) << (8 * (j & 3));
      *reinterpret_cast<u32x2*>(q + k) = u32x2{w[0], w[1]};
    }
  } else {
    for (int k = tid; k < K; k += 256) q[k] = (int8_t)__float2int_rn((float)x[k] * inv);
  }
  if (tid == 0) xs[m] = s;
}

// per-row int8 re-quantization of a dense f16 weight [n_pad][k_pad] into the P_I8 chunk layout of
// gemm3.hip (byte ((2 st + kk) * 64 + 16 g + r) * 16 + j of chunk (tile t, super-block sb) holds row
// 16 t + r, k = 256 sb + 128 st + 64 kk + 16 g + j): one workgroup per row, one 16-k group per
// thread step (two 16-byte loads, one 16-byte store); rows >= n get zeros and scale 1
__global__ __launch_bounds__(256) void requant_i8_kernel(const f16* W, int ldw, int n, int nsb, uint8_t* out, float* ws) {
  __shared__ float red[4];
  const int row = blockIdx.x, tid = threadIdx.x;
  const int K = nsb * 256;
  const f16* w = W + (size_t)row * ldw;
  float mx = 0.f;
  if (row < n)
    for (int k = tid * 8; k < K; k += 2048) {
      const half8_t v = *reinterpret_cast<const half8_t*>(w + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) mx = fmaxf(mx, fabsf((float)v[j]));
    }
  mx = wave_max(mx);
  if ((tid & 63) == 0) red[tid >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = mx > 0.f ? mx / 127.f : 1.f, inv = 1.f / s;
  const int t = row >> 4, r = row & 15;
  for (int k0 = tid * 16; k0 < K; k0 += 4096) {
    const int sb = k0 >> 8, st = (k0 >> 7) & 1, kk = (k0 >> 6) & 1, g = (k0 >> 4) & 3;
    uint32_t q[4] = {0u, 0u, 0u, 0u};
    if (row < n) {
      const half8_t a = *reinterpret_cast<const half8_t*>(w + k0), b = *reinterpret_cast<const half8_t*>(w + k0 + 8);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const float v = j < 8 ? (float)a[j] : (float)b[j - 8];
        const int qi = max(-127, min(127, __float2int_rn(v * inv)));
        q[j >> 2] |= ((uint32_t)(uint8_t)(int8_t)qi) << (8 * (j & 3));
      }
    }
    uint8_t* dst = out + ((size_t)t * nsb + sb) * 4096 + (size_t)(((2 * st + kk) * 64 + 16 * g + r) * 16);
    *reinterpret_cast<u32x4*>(dst) = u32x4{q[0], q[1], q[2], q[3]};
  }
  if (tid == 0) ws[row] = row < n ? s : 1.f;
}

// ---------------------------------------------------------------- RoPE (NORM, adjacent pairs) + KV append
__global__ __launch_bounds__(256) void rope_kv_kernel(const RopeKvParams p) {
  // grid (M tokens, head groups of 4 over [q heads | k heads | v heads]); one thread per pair
  const int m = blockIdx.x;
  const int pos = p.pos[m];
  const int hd2 = p.hd / 2, Dp2 = p.Dp / 2;
  const float* row = p.qkv + (size_t)m * p.ldqkv;
  const float2* cs = p.rope_cs + (size_t)pos * hd2;
  const int page = p.block_table[(size_t)p.slot[m] * p.max_pages + pos / 64];
  const int idx = pos % 64;
  const int nh = p.Hq + 2 * p.Hkv;
  for (int e = threadIdx.x; e < 4 * Dp2; e += 256) {
    const int hg = blockIdx.y * 4 + e / Dp2, j = e % Dp2;
    if (hg >= nh) break;
    if (hg < p.Hq + p.Hkv) {                       // q or k head: rotate adjacent pair j
      const bool isq = hg < p.Hq;
      const int h = isq ? hg : hg - p.Hq;
      float r0 = 0.f, r1 = 0.f;
      if (j < hd2) {
        const float* src = row + (isq ? 0 : p.Hq * p.hd) + h * p.hd + 2 * j;
        const float x0 = src[0], x1 = src[1];
        const float2 c = cs[j];
        const float sc = isq ? p.q_scale : 1.f;
        r0 = (x0 * c.x - x1 * c.y) * sc;
        r1 = (x0 * c.y + x1 * c.x) * sc;
      }
      const half2_t o = {(f16)r0, (f16)r1};
      const size_t ko = (((size_t)page * p.Hkv + h) * 64 + idx) * p.Dp + 2 * j;
      if (isq) *reinterpret_cast<half2_t*>(p.q_out + ((size_t)m * p.Hq + h) * p.Dp + 2 * j) = o;
      else if (p.kv_fp8) *reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(p.k_cache) + ko) = (uint16_t)f8x2_pack(r0, r1);
      else *reinterpret_cast<half2_t*>(p.k_cache + ko) = o;
    } else {                                        // v head: transposed page layout [Dp][64]
      const int h = hg - p.Hq - p.Hkv;
      const float* vr = row + (p.Hq + p.Hkv) * p.hd + h * p.hd;
      const size_t vo = (((size_t)page * p.Hkv + h) * p.Dp) * 64 + idx;
      const int d0 = 2 * j;
      const float v0 = d0 < p.hd ? vr[d0] : 0.f, v1 = d0 + 1 < p.hd ? vr[d0 + 1] : 0.f;
      if (p.kv_fp8) {
        uint8_t* vd = reinterpret_cast<uint8_t*>(p.v_cache) + vo;
        const uint32_t q = f8x2_pack(v0, v1);
        vd[(size_t)d0 * 64] = (uint8_t)q;
        vd[(size_t)(d0 + 1) * 64] = (uint8_t)(q >> 8);
      } else {
        f16* vd = p.v_cache + vo;
        vd[(size_t)d0 * 64] = (f16)v0;
        vd[(size_t)(d0 + 1) * 64] = (f16)v1;
      }
    }
  }
}

// ---------------------------------------------------------------- argmax
__global__ __launch_bounds__(1024) void argmax_kernel(const float* logits, int ld, int n, int32_t* tok) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const float* r = logits + (size_t)blockIdx.x * ld;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const float v = r[i];
    if (v > bv) { bv = v; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sv[w] = bv; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < 16; ++i)
      if (sv[i] > bv || (sv[i] == bv && si[i] < bi)) { bv = sv[i]; bi = si[i]; }
    tok[blockIdx.x] = bi;
  }
}

// Two-level argmax: grid (nchunk, M) workgroups each reduce one chunk of a row, publish a
// (value, index) partial and count in; the last arriver of the row reduces the nchunk partials.
// (One 1024-thread workgroup per row read 513 KB of Llama-3 logits in 38 us at M = 1.)
// Hand-off per MI355X_MICROARCH.md 'Valid forms', first row of the sc1 table: the partial is ONE
// 8-byte sc1 (agent-scope relaxed) store by the lane that then drains it (vmcnt(0)) and adds to the
// row's counter; the last arriver (told by the value its add returned) reads every partial with
// sc1 loads from the same wave.  (An agent release fence per workgroup wrote back the XCD L2 behind
// every arrival: 66 us at M = 64 with the LM head's 33 MB of fresh logits dirty in L2.)
// Ties -> lowest index.
__device__ __forceinline__ bool am_better(float v, int i, float bv, int bi) { return v > bv || (v == bv && i < bi); }

__global__ __launch_bounds__(256) void argmax2_kernel(const float* logits, int ld, int n, int chunk,
                                                      float2* part, int32_t* counters, int32_t* tok) {
  __shared__ float sv[4];
  __shared__ int si[4];
  __shared__ int last;
  const int m = blockIdx.y, c = blockIdx.x, nchunk = gridDim.x;
  const float* r = logits + (size_t)m * ld;
  const int i0 = c * chunk, i1 = min(n, i0 + chunk);
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = i0 + threadIdx.x * 4; i < i1; i += 1024) {
    if (i + 4 <= i1 && ((ld | i0) & 3) == 0) {
      const float4 v = *reinterpret_cast<const float4*>(r + i);
      if (am_better(v.x, i, bv, bi)) { bv = v.x; bi = i; }
      if (am_better(v.y, i + 1, bv, bi)) { bv = v.y; bi = i + 1; }
      if (am_better(v.z, i + 2, bv, bi)) { bv = v.z; bi = i + 2; }
      if (am_better(v.w, i + 3, bv, bi)) { bv = v.w; bi = i + 3; }
    } else {
      for (int k = i; k < i + 4 && k < i1; ++k)
        if (am_better(r[k], k, bv, bi)) { bv = r[k]; bi = k; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (am_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sv[w] = bv; si[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < 4; ++k)
      if (am_better(sv[k], si[k], bv, bi)) { bv = sv[k]; bi = si[k]; }
    const uint64_t pk = (uint64_t)__float_as_uint(bv) | ((uint64_t)(uint32_t)bi << 32);
    __hip_atomic_store(reinterpret_cast<uint64_t*>(part) + (size_t)m * nchunk + c, pk, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int old = __hip_atomic_fetch_add(counters + m, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == nchunk - 1;
  }
  __syncthreads();
  if (!last || threadIdx.x >= 64) return;
  bv = -INFINITY;
  bi = 0x7fffffff;
  for (int k = threadIdx.x; k < nchunk; k += 64) {
    const uint64_t pk = __hip_atomic_load(reinterpret_cast<uint64_t*>(part) + (size_t)m * nchunk + k, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    const float v = __uint_as_float((uint32_t)pk);
    const int i = (int)(uint32_t)(pk >> 32);
    if (am_better(v, i, bv, bi)) { bv = v; bi = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o);
    const int oi = __shfl_xor(bi, o);
    if (am_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
  }
  if (threadIdx.x == 0) {
    tok[m] = bi == 0x7fffffff ? 0 : bi;
    __hip_atomic_store(counters + m, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// deterministic reductions: a fixed summation order per element, no atomics
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int nsplit, int64_t ss, int ldp,
                                                            int n, float* __restrict__ Y, int ldy) {
  const int m = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  float acc = Y[(size_t)m * ldy + j];
  for (int s = 0; s < nsplit; ++s) acc += part[(size_t)s * ss + (size_t)m * ldp + j];
  Y[(size_t)m * ldy + j] = acc;
}

// 4 consecutive columns per thread (n, ldp, ldy multiples of 4)
__global__ __launch_bounds__(256) void splitk_reduce4_kernel(const float* __restrict__ part, int nsplit, int64_t ss, int ldp,
                                                             int n, float* __restrict__ Y, int ldy) {
  const int m = blockIdx.y, j = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (j >= n) return;
  float4 acc = *reinterpret_cast<const float4*>(Y + (size_t)m * ldy + j);
  for (int s = 0; s < nsplit; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(part + (size_t)s * ss + (size_t)m * ldp + j);
    acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
  }
  *reinterpret_cast<float4*>(Y + (size_t)m * ldy + j) = acc;
}

__global__ __launch_bounds__(256) void moe_combine_kernel(const float* __restrict__ ys, int lds, int k, int n,
                                                          float* __restrict__ Y, int ldy) {
  const int t = blockIdx.y, j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  float acc = Y[(size_t)t * ldy + j];
  for (int e = 0; e < k; ++e) acc += ys[((size_t)t * k + e) * lds + j];
  Y[(size_t)t * ldy + j] = acc;
}

// device probe (probe.cpp): stream a buffer with 16 B loads, one partial sum per workgroup
__global__ __launch_bounds__(256) void stream_read_kernel(const u32x4* __restrict__ buf, size_t n16, float* out) {
  uint32_t acc = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) {
    const u32x4 v = __builtin_nontemporal_load(buf + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[blockIdx.x] = (float)acc;   // keeps the loads; practically never stores
}

// one thread per row of the micro-batch (mb_size up to 1024: a 64-thread single block advanced only
// rows 0-63, so wide micro-batches decoded rows >= 64 at a frozen position)
__global__ __launch_bounds__(256) void advance_kernel(int32_t* pos, int32_t* kvlen, int M, int32_t* step) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < M) { const int p = pos[i] + 1; pos[i] = p; kvlen[i] = p + 1; }
  if (i == 0 && step) step[0] += 1;
}

__global__ __launch_bounds__(256) void swiglu_kernel(const float* gu, int ld, int F, f16* h, int ldh) {
  const int m = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < F) {
    const float g = gu[(size_t)m * ld + j], u = gu[(size_t)m * ld + F + j];
    h[(size_t)m * ldh + j] = sat_f16(silu(g) * u);
  }
}

__global__ __launch_bounds__(256) void f32_to_f16_kernel(const float* x, int ldx, int n, f16* y, int ldy) {
  const int m = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j < n) y[(size_t)m * ldy + j] = (f16)x[(size_t)m * ldx + j];
}

// stage-boundary activation wire format (engine "act_dtype"): f32 residual rows <-> f16 / bf16
// (2 bytes per element on xGMI).  4 elements per thread, round-to-nearest-even by
// the hardware convert (a NaN stays a NaN).
template <int OUT>
__global__ __launch_bounds__(256) void act_pack_kernel(const float* __restrict__ x, void* __restrict__ y, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 4 <= n) {
    const float4 v = *reinterpret_cast<const float4*>(x + i);
    if constexpr (OUT == 1) {
      typedef _Float16 h4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<h4*>(reinterpret_cast<f16*>(y) + i) = h4{(f16)v.x, (f16)v.y, (f16)v.z, (f16)v.w};
    } else {
      typedef __bf16 b4 __attribute__((ext_vector_type(4)));
      *reinterpret_cast<b4*>(reinterpret_cast<__bf16*>(y) + i) = b4{(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    }
  } else {
    for (int64_t k = i; k < n; ++k) {
      if constexpr (OUT == 1) reinterpret_cast<f16*>(y)[k] = (f16)x[k];
      else reinterpret_cast<__bf16*>(y)[k] = (__bf16)x[k];
    }
  }
}
template <int IN>
__global__ __launch_bounds__(256) void act_unpack_kernel(const void* __restrict__ y, float* __restrict__ x, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  for (int64_t k = i; k < i + 4 && k < n; ++k)
    x[k] = IN == 1 ? (float)reinterpret_cast<const f16*>(y)[k] : (float)reinterpret_cast<const __bf16*>(y)[k];
}

__global__ void prefill_meta_kernel(int32_t* pos, int32_t* kvlen, int32_t* slot, int p0, int T, int s) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < T) { pos[i] = p0 + i; kvlen[i] = p0 + i + 1; slot[i] = s; }
}

}  // namespace mpk

namespace mp {

void launch_prefill_meta(int32_t* pos, int32_t* kvlen, int32_t* slot, int p0, int T, int s, hipStream_t st) {
  hipLaunchKernelGGL(mpk::prefill_meta_kernel, dim3((T + 255) / 256), dim3(256), 0, st, pos, kvlen, slot, p0, T, s);
}

void launch_rmsnorm(const float* x, int ldx, const float* w, int d, float eps, f16* out, int ldo, int M,
                    float* zero, int64_t zero_n, hipStream_t st, const float* bias, int bias_n) {
  const int zb = zero ? (int)((zero_n + 16383) / 16384) : 0;
  hipLaunchKernelGGL(mpk::rmsnorm_kernel, dim3(M > zb ? M : zb), dim3(1024), 0, st, x, ldx, w, d, eps, out, ldo, zero,
                     zero_n, M, bias, bias_n, nullptr, 0, 0, 0, nullptr, 0, nullptr);
}

void launch_rmsnorm_acc(float* x, int ldx, const float* w, int d, float eps, f16* out, int ldo, int M,
                        float* zero, int64_t zero_n, const float* part, int nsplit, int64_t ss, int ldp, hipStream_t st,
                        const float* bias, int bias_n, int8_t* q8, int ldq8, float* q8s) {
  if ((d & 3) || d > 8192 || (ldx & 3) || (part && ((ldp & 3) || (ss & 3))) || (q8 && (ldq8 & 3)))
    throw std::runtime_error("launch_rmsnorm_acc: needs d <= 8192 and 4-aligned rows");
  const int zb = zero ? (int)((zero_n + 16383) / 16384) : 0;
  hipLaunchKernelGGL(mpk::rmsnorm_kernel, dim3(M > zb ? M : zb), dim3(1024), 0, st, x, ldx, w, d, eps, out, ldo, zero,
                     zero_n, M, bias, bias_n, part, part ? nsplit : 0, ss, ldp, q8, ldq8, q8s);
}

void launch_embed(int t, const uint8_t* table, int64_t rb, int d, const int32_t* tokens, int M, float* x,
                  int ldx, hipStream_t st) {
  hipLaunchKernelGGL(mpk::embed_kernel, dim3(M, (d + 255) / 256), dim3(256), 0, st, t, table, rb, d, tokens, x, ldx);
}

void launch_quant_rows_i8(const f16* X, int ldx, int M, int K, int8_t* Q, int ldq, float* xs, hipStream_t st) {
  hipLaunchKernelGGL(mpk::quant_rows_i8_kernel, dim3(M), dim3(256), 0, st, X, ldx, K, Q, ldq, xs);
}

void launch_requant_i8(const f16* W, int ldw, int n, int n_pad, int nsb, uint8_t* out, float* ws, hipStream_t st) {
  hipLaunchKernelGGL(mpk::requant_i8_kernel, dim3(n_pad), dim3(256), 0, st, W, ldw, n, nsb, out, ws);
}

void launch_rope_kv(const RopeKvParams& p, hipStream_t st) {
  hipLaunchKernelGGL(mpk::rope_kv_kernel, dim3(p.M, (p.Hq + 2 * p.Hkv + 3) / 4), dim3(256), 0, st, p);
}

void launch_argmax(const float* logits, int ld, int n, int M, int32_t* tokens, hipStream_t st, const ArgmaxScratch* sc) {
  if (!sc || M > sc->rows) {
    hipLaunchKernelGGL(mpk::argmax_kernel, dim3(M), dim3(1024), 0, st, logits, ld, n, tokens);
    return;
  }
  // ~2K logits per 256-thread workgroup, at most kArgmaxChunks per row
  int nchunk = (n + 2047) / 2048;
  nchunk = nchunk < 1 ? 1 : nchunk > kArgmaxChunks ? kArgmaxChunks : nchunk;
  const int chunk = (((n + nchunk - 1) / nchunk) + 3) & ~3;
  nchunk = (n + chunk - 1) / chunk;
  hipLaunchKernelGGL(mpk::argmax2_kernel, dim3(nchunk, M), dim3(256), 0, st, logits, ld, n, chunk,
                     reinterpret_cast<float2*>(sc->part), sc->counters, tokens);
}

void launch_splitk_reduce(const float* part, int nsplit, int64_t split_stride, int ldp, int M, int n, float* Y, int ldy,
                          hipStream_t st) {
  if ((n & 3) == 0 && (ldp & 3) == 0 && (ldy & 3) == 0 && (split_stride & 3) == 0)
    hipLaunchKernelGGL(mpk::splitk_reduce4_kernel, dim3((n / 4 + 255) / 256, M), dim3(256), 0, st, part, nsplit,
                       split_stride, ldp, n, Y, ldy);
  else
    hipLaunchKernelGGL(mpk::splitk_reduce_kernel, dim3((n + 255) / 256, M), dim3(256), 0, st, part, nsplit, split_stride,
                       ldp, n, Y, ldy);
}

void launch_moe_combine(const float* Yslot, int ld_slot, int k, int M, int n, float* Y, int ldy, hipStream_t st) {
  hipLaunchKernelGGL(mpk::moe_combine_kernel, dim3((n + 255) / 256, M), dim3(256), 0, st, Yslot, ld_slot, k, n, Y, ldy);
}

void launch_stream_read(const void* buf, size_t bytes, float* out, hipStream_t st) {
  hipLaunchKernelGGL(mpk::stream_read_kernel, dim3(4096), dim3(256), 0, st, reinterpret_cast<const u32x4*>(buf),
                     bytes / 16, out);
}

void launch_advance(int32_t* pos, int32_t* kvlen, int M, int32_t* step, hipStream_t st) {
  hipLaunchKernelGGL(mpk::advance_kernel, dim3((M + 255) / 256), dim3(256), 0, st, pos, kvlen, M, step);
}

void launch_swiglu(const float* gu, int ld, int F, int M, f16* h, int ldh, hipStream_t st) {
  hipLaunchKernelGGL(mpk::swiglu_kernel, dim3((F + 255) / 256, M), dim3(256), 0, st, gu, ld, F, h, ldh);
}

void launch_act_pack(const float* x, void* y, int64_t n, int dtype, hipStream_t st) {
  const dim3 grid((unsigned)((n + 1023) / 1024));
  if (dtype == ACT_F16) hipLaunchKernelGGL(mpk::act_pack_kernel<1>, grid, dim3(256), 0, st, x, y, n);
  else if (dtype == ACT_BF16) hipLaunchKernelGGL(mpk::act_pack_kernel<2>, grid, dim3(256), 0, st, x, y, n);
}

void launch_act_unpack(const void* y, float* x, int64_t n, int dtype, hipStream_t st) {
  const dim3 grid((unsigned)((n + 1023) / 1024));
  if (dtype == ACT_F16) hipLaunchKernelGGL(mpk::act_unpack_kernel<1>, grid, dim3(256), 0, st, y, x, n);
  else if (dtype == ACT_BF16) hipLaunchKernelGGL(mpk::act_unpack_kernel<2>, grid, dim3(256), 0, st, y, x, n);
}

void launch_f32_to_f16(const float* x, int ldx, int n, int M, f16* y, int ldy, hipStream_t st) {
  hipLaunchKernelGGL(mpk::f32_to_f16_kernel, dim3((n + 255) / 256, M), dim3(256), 0, st, x, ldx, n, y, ldy);
}

}  // namespace mp
