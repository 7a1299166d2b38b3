// Device-side random initialisation of packed weights (synthetic random-init models for the
// benchmark: a 70B Q4_K model is generated straight into HBM in well under a second instead of
// writing/reading a 40 GB GGUF).  Quant bits are hash-random; block scales are set so that
// weights have ~unit-RMS-preserving magnitude (std ~ scale).
#include "kcommon.h"
#include "../runtime/qtypes.h"

namespace mpk {
using namespace mp;

__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
  return (uint32_t)x;
}
__device__ __forceinline__ uint16_t f2h(float f) { return __builtin_bit_cast(uint16_t, (f16)f); }

// one thread per 16 bytes of the packed buffer
__global__ void init_packed_kernel(uint8_t* W, size_t nbytes, int pt, float scale, uint64_t seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t off = i * 16;
  if (off >= nbytes) return;
  const int cb = chunk_bytes(pt);
  const int in_chunk = (int)(off % cb);
  uint32_t v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = hash32(seed * 0x9E3779B97F4A7C15ULL + i * 4 + k);
  if (pt == P_F16 || pt == P_BF16) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = ((v[k] & 0xFFFF) / 65536.f - 0.5f) * 3.4f * scale;
      const float b = ((v[k] >> 16) / 65536.f - 0.5f) * 3.4f * scale;
      v[k] = pt == P_F16 ? (uint32_t)f2h(a) | ((uint32_t)f2h(b) << 16)
                         : (__float_as_uint(a) >> 16) | (__float_as_uint(b) & 0xFFFF0000u);   // bf16 (truncated)
    }
  } else if (pt == P_Q4_K || pt == P_Q5_K) {
    const int hdr0 = pt == P_Q4_K ? 2048 : 2560;
    if (in_chunk >= hdr0) {   // [d, dmin, scales(12)] of one row
      const float nmax = pt == P_Q4_K ? 15.f : 31.f;
      const float d = scale * 3.4f / (nmax * 63.f);
      const float dmin = d * nmax * 0.5f;           // centres sc*q around m
      v[0] = (uint32_t)f2h(d) | ((uint32_t)f2h(dmin) << 16);
      // random 6-bit scales with mins = scales, so each sub-block is roughly zero-mean; header
      // layout of csrc/runtime/pack.cpp: v_g = sc | m << 6 | sc' << 12 | m' << 18, byte b at 4b + g
      const uint32_t rnd[2] = {v[1], v[2]};
      uint32_t out[3] = {0u, 0u, 0u};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const uint32_t s0 = (rnd[g >> 1] >> (16 * (g & 1))) & 63u, s1 = (rnd[g >> 1] >> (16 * (g & 1) + 6)) & 63u;
        const uint32_t vg = s0 | s0 << 6 | s1 << 12 | s1 << 18;
#pragma unroll
        for (int b = 0; b < 3; ++b) out[b] |= ((vg >> (8 * b)) & 0xFFu) << (8 * g);
      }
      v[1] = out[0]; v[2] = out[1]; v[3] = out[2];
    }
  } else if (pt == P_Q6_K) {
    if (in_chunk >= 3328) {   // d for 8 rows per 16 B
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint16_t h = f2h(scale * 3.4f / (32.f * 127.f));
        v[k] = (uint32_t)h | ((uint32_t)h << 16);
      }
    }
  } else if (pt == P_Q8_0) {
    if (in_chunk >= 4096) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint16_t h = f2h(scale * 1.7f / 127.f);
        v[k] = (uint32_t)h | ((uint32_t)h << 16);
      }
    }
  } else if (pt == P_Q4_0) {
    if (in_chunk >= 2048) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint16_t h = f2h(scale * 3.4f / 15.f);
        v[k] = (uint32_t)h | ((uint32_t)h << 16);
      }
    }
  }
  u32x4 o = {v[0], v[1], v[2], v[3]};
  *reinterpret_cast<u32x4*>(W + off) = o;
}

// raw GGUF-native rows (embedding table): random bytes, then fix the block scales
__global__ void init_raw_kernel(uint8_t* W, int64_t nblocks, int t, float scale, uint64_t seed) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nblocks) return;
  const int bb = block_bytes(t);
  uint8_t* p = W + b * bb;
  for (int i = 0; i < bb; ++i) p[i] = (uint8_t)hash32(seed ^ ((uint64_t)b * 1315423911ULL + i));
  uint16_t* h = reinterpret_cast<uint16_t*>(p);
  switch (t) {
    case T_Q8_0: h[0] = f2h(scale * 1.7f / 127.f); break;
    case T_Q4_0: h[0] = f2h(scale * 3.4f / 15.f); break;
    case T_Q4_K: case T_Q5_K: {
      const float nmax = t == T_Q4_K ? 15.f : 31.f;
      const float d = scale * 3.4f / (nmax * 63.f);
      h[0] = f2h(d); h[1] = f2h(d * nmax * 0.5f);
      for (int i = 0; i < 4; ++i) p[8 + i] = p[4 + i];
      break;
    }
    case T_Q6_K: *reinterpret_cast<uint16_t*>(p + 208) = f2h(scale * 3.4f / (32.f * 127.f)); break;
    case T_F16: h[0] = f2h(((hash32(seed + b) & 0xFFFF) / 65536.f - 0.5f) * 3.4f * scale); break;
    case T_BF16: h[0] = (uint16_t)(__float_as_uint(((hash32(seed + b) & 0xFFFF) / 65536.f - 0.5f) * 3.4f * scale) >> 16); break;
    case T_F32: *reinterpret_cast<float*>(p) = ((hash32(seed + b) & 0xFFFF) / 65536.f - 0.5f) * 3.4f * scale; break;
  }
}

}  // namespace mpk

namespace mp {
void launch_init_packed(uint8_t* W, size_t nbytes, int pt, float scale, uint64_t seed, hipStream_t st) {
  const size_t n16 = nbytes / 16;
  hipLaunchKernelGGL(mpk::init_packed_kernel, dim3((unsigned)((n16 + 255) / 256)), dim3(256), 0, st, W, nbytes, pt,
                     scale, seed);
}
void launch_init_raw(uint8_t* W, int64_t nblocks, int t, float scale, uint64_t seed, hipStream_t st) {
  hipLaunchKernelGGL(mpk::init_raw_kernel, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, st, W, nblocks, t,
                     scale, seed);
}
}  // namespace mp
