// On-GPU sampler for the last stage (K12): temperature, top-k, min-p, top-p, then inverse-CDF
// draw with a counter-based RNG.  Only int32 token ids leave the GPU (the reference copies the
// 501 KiB logit row of Llama-3 to the host every token and samples on the CPU).
// One 1024-thread workgroup per row; thresholds by bisection (no sort), so the kernel is a few
// streaming passes over the row (L2-resident after the first).
#include "kcommon.h"
#include "../runtime/kernels_api.h"

namespace mpk {
using namespace mp;

constexpr int ST = 1024;

__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float x = __shfl_xor(v, o);
    v = is_max ? fmaxf(v, x) : v + x;
  }
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) sh[w] = v;
  __syncthreads();
  float r = is_max ? -INFINITY : 0.f;
  for (int i = 0; i < ST / 64; ++i) r = is_max ? fmaxf(r, sh[i]) : r + sh[i];
  return r;
}

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL; x ^= x >> 27; x *= 0x94d049bb133111ebULL; x ^= x >> 31;
  return x;
}

__global__ __launch_bounds__(ST) void sample_kernel(const SampleParams p) {
  __shared__ float sh[ST / 64];
  __shared__ float scan[ST];
  const int row = blockIdx.x;
  const float* lg = p.logits + (size_t)row * p.ld;
  const int n = p.n;
  // chunk of contiguous indices per thread (for the ordered CDF walk)
  const int per = (n + ST - 1) / ST;
  const int i0 = threadIdx.x * per, i1 = min(n, i0 + per);

  float mx = -INFINITY;
  int am = 0x7fffffff;
  for (int i = i0; i < i1; ++i) if (lg[i] > mx) { mx = lg[i]; am = i; }
  // argmax (also the temp <= 0 path)
  float gmx = block_reduce(mx, sh, true);
  if (p.temp <= 0.f) {
    __shared__ int best;
    if (threadIdx.x == 0) best = 0x7fffffff;
    __syncthreads();
    if (mx == gmx) atomicMin(&best, am);
    __syncthreads();
    if (threadIdx.x == 0) p.tokens[row] = best;
    return;
  }
  const float invT = 1.f / p.temp;
  // llama.cpp sampler-chain semantics (common_sampler defaults: top-k -> top-p -> min-p -> temp ->
  // dist): the three cuts are taken on the T = 1 distribution, the draw uses temperature T.
  // top-k threshold on logits: largest thr with count(l >= thr) >= k
  float thr = -INFINITY;
  if (p.top_k > 0 && p.top_k < n) {
    float lo = gmx - 60.f, hi = gmx;
    for (int it = 0; it < 28; ++it) {
      const float mid = 0.5f * (lo + hi);
      float c = 0.f;
      for (int i = i0; i < i1; ++i) c += lg[i] >= mid ? 1.f : 0.f;
      c = block_reduce(c, sh, false);
      if (c >= (float)p.top_k) lo = mid; else hi = mid;
    }
    thr = lo;
  }
  // T = 1 probabilities (relative to the max) of the top-k survivors
  auto p1 = [&](float l) { return l >= thr ? __expf(l - gmx) : 0.f; };
  // top-p: largest q with sum_{p1 >= q} p1 >= top_p * sum p1
  float pthr = 0.f;
  if (p.top_p > 0.f && p.top_p < 1.f) {
    float tot = 0.f;
    for (int i = i0; i < i1; ++i) tot += p1(lg[i]);
    tot = block_reduce(tot, sh, false);
    float lo = 0.f, hi = 1.f;
    for (int it = 0; it < 24; ++it) {
      const float mid = 0.5f * (lo + hi);
      float s = 0.f;
      for (int i = i0; i < i1; ++i) { const float q = p1(lg[i]); s += q >= mid ? q : 0.f; }
      s = block_reduce(s, sh, false);
      if (s >= p.top_p * tot) lo = mid; else hi = mid;
    }
    pthr = lo;
  }
  // min-p: p1 >= min_p (the max has p1 = 1)
  pthr = fmaxf(pthr, p.min_p);
  auto keep = [&](float l) { return l >= thr && __expf(l - gmx) >= pthr ? __expf((l - gmx) * invT) : 0.f; };
  float mine = 0.f;
  for (int i = i0; i < i1; ++i) mine += keep(lg[i]);
  // inclusive scan of per-thread sums (Hillis-Steele in LDS)
  scan[threadIdx.x] = mine;
  __syncthreads();
  for (int o = 1; o < ST; o <<= 1) {
    const float v = threadIdx.x >= (unsigned)o ? scan[threadIdx.x - o] : 0.f;
    __syncthreads();
    scan[threadIdx.x] += v;
    __syncthreads();
  }
  const float total = scan[ST - 1];
  const int32_t step = p.step ? p.step[0] : 0;
  const uint64_t r = mix64(p.seed ^ mix64(((uint64_t)step << 20) ^ (uint64_t)row));
  const float u = (float)((r >> 40) * (1.0 / 16777216.0)) * total;
  const float before = scan[threadIdx.x] - mine;
  __shared__ int pick;
  if (threadIdx.x == 0) pick = -1;   // fallback: global argmax below
  __syncthreads();
  if (mine > 0.f && u >= before && u < scan[threadIdx.x]) {
    float c = before;
    int sel = -1;
    for (int i = i0; i < i1; ++i) {
      c += keep(lg[i]);
      if (u < c) { sel = i; break; }
    }
    if (sel < 0) for (int i = i1 - 1; i >= i0; --i) if (keep(lg[i]) > 0.f) { sel = i; break; }
    pick = sel;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = pick;
    if (t < 0 || t >= n) {  // u landed on total (rounding): take the global argmax
      t = 0;
      for (int i = 0; i < n; ++i) if (lg[i] == gmx) { t = i; break; }
    }
    p.tokens[row] = t;
  }
}

__global__ __launch_bounds__(256) void penalize_kernel(const PenaltyParams p) {
  const int row = blockIdx.x;
  const int32_t* h = p.hist + (size_t)row * p.last_n;
  float* lg = p.logits + (size_t)row * p.ld;
  for (int i = threadIdx.x; i < p.last_n; i += blockDim.x) {
    const int t = h[i];
    if (t < 0 || t >= p.n) continue;
    int c = 0;
    bool first = true;
    for (int j = 0; j < p.last_n; ++j)
      if (h[j] == t) {
        ++c;
        first &= j >= i;
      }
    if (!first) continue;   // the first occurrence in the window owns the token
    float l = lg[t];
    l = l > 0.f ? l / p.repeat : l * p.repeat;
    lg[t] = l - (float)c * p.freq - p.presence;
  }
}

__global__ void hist_push_kernel(int32_t* hist, int32_t* cnt, int last_n, const int32_t* tokens, int M) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const int c = cnt[m];
  hist[(size_t)m * last_n + c % last_n] = tokens[m];
  cnt[m] = c + 1;
}

}  // namespace mpk

namespace mp {
void launch_penalize(const PenaltyParams& p, hipStream_t st) {
  hipLaunchKernelGGL(mpk::penalize_kernel, dim3(p.M), dim3(256), 0, st, p);
}
void launch_hist_push(int32_t* hist, int32_t* cnt, int last_n, const int32_t* tokens, int M, hipStream_t st) {
  hipLaunchKernelGGL(mpk::hist_push_kernel, dim3((M + 63) / 64), dim3(64), 0, st, hist, cnt, last_n, tokens, M);
}
void launch_sample(const SampleParams& p, hipStream_t st) {
  hipLaunchKernelGGL(mpk::sample_kernel, dim3(p.M), dim3(mpk::ST), 0, st, p);
}
}  // namespace mp
