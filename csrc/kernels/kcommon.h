// Device-side helpers shared by all mipipe CDNA4 (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 f16;
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64

__device__ __forceinline__ half2_t as_h2(uint32_t u) { return __builtin_bit_cast(half2_t, u); }
__device__ __forceinline__ uint32_t as_u32(half2_t h) { return __builtin_bit_cast(uint32_t, h); }

__device__ __forceinline__ f32x4 mfma16x16x32(half8_t a, half8_t b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// bf16 MFMA operands travel in the same 16-byte containers as f16 ones (a half8_t holds the bits)
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
__device__ __forceinline__ half8_t h8_to_bf8(half8_t a) {   // 8 f16 -> 8 bf16 (round to nearest even)
  bf16x8_t r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (__bf16)(float)a[i];
  return __builtin_bit_cast(half8_t, r);
}
// Weight-type MFMA.  BF: bf16 weights (P_BF16) -- their fragments are the packed bf16 bits and the
// f16 activation fragment goes through x_op (-> bf16) first, so the product runs on the bf16 MFMA
// with bf16's full exponent range (no narrowing of the weights to f16).  !BF: f16 MFMA.
template <bool BF>
__device__ __forceinline__ half8_t x_op(half8_t a) {
  if constexpr (BF) return h8_to_bf8(a);
  else return a;
}
// activations staged once per workgroup in the MFMA's A format: f16, or bf16 for BF16 weights
// (converted from f32 directly where the staging computes them, from f16 where it copies them)
template <bool BF>
__device__ __forceinline__ u32x4 x8_pack(float v0, float v1, float v2, float v3, float v4, float v5, float v6, float v7) {
  if constexpr (BF) return __builtin_bit_cast(u32x4, bf16x8_t{(__bf16)v0, (__bf16)v1, (__bf16)v2, (__bf16)v3, (__bf16)v4,
                                                               (__bf16)v5, (__bf16)v6, (__bf16)v7});
  else return __builtin_bit_cast(u32x4, half8_t{(f16)v0, (f16)v1, (f16)v2, (f16)v3, (f16)v4, (f16)v5, (f16)v6, (f16)v7});
}
template <bool BF>
__device__ __forceinline__ u32x2 x4_pack(float v0, float v1, float v2, float v3) {
  typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
  typedef _Float16 half4_t __attribute__((ext_vector_type(4)));
  if constexpr (BF) return __builtin_bit_cast(u32x2, bf16x4_t{(__bf16)v0, (__bf16)v1, (__bf16)v2, (__bf16)v3});
  else return __builtin_bit_cast(u32x2, half4_t{(f16)v0, (f16)v1, (f16)v2, (f16)v3});
}
template <bool BF>
__device__ __forceinline__ u32x4 x8_from_h8(u32x4 v) {
  if constexpr (BF) return __builtin_bit_cast(u32x4, h8_to_bf8(__builtin_bit_cast(half8_t, v)));
  else return v;
}

template <bool BF>
__device__ __forceinline__ f32x4 mma(half8_t a, half8_t b, f32x4 c) {
  if constexpr (BF)
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ half8_t pack8(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  u32x4 v = {w0, w1, w2, w3};
  return __builtin_bit_cast(half8_t, v);
}

__device__ __forceinline__ u32x4 ld16(const void* p) { return *reinterpret_cast<const u32x4*>(p); }
// streamed-once weights: non-temporal 16-B load (MI355X_MICROARCH row nt-weights)
__device__ __forceinline__ u32x4 ld16_nt(const void* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ float h2f(uint16_t h) { return (float)__builtin_bit_cast(f16, h); }

// 6-bit scale/min of a Q4_K/Q5_K super-block, sub-block j (ggml get_scale_min_k4)
__device__ __forceinline__ void scale_min_k4(int j, const uint8_t* q, int& sc, int& m) {
  if (j < 4) { sc = q[j] & 63; m = q[j + 4] & 63; }
  else { sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4); }
}

__device__ __forceinline__ float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// f16 with saturation: the SwiGLU intermediate of layers with massive activations can pass f16's
// 65504; saturating keeps an inf (and the NaNs it breeds in the next GEMV) out of the pipeline
__device__ __forceinline__ f16 sat_f16(float v) { return (f16)fminf(fmaxf(v, -65504.f), 65504.f); }

// fp8 KV cache (kv_dtype "fp8"): OCP e4m3 bytes, converted with the gfx950 cvt instructions.
// e4m3 has no inf: stored values are clamped to its +-448 range first.
__device__ __forceinline__ uint32_t f8x2_pack(float a, float b) {   // -> bytes 0, 1 of the result
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false) & 0xFFFFu;
}
__device__ __forceinline__ half2_t f8x2_lo(uint32_t w) { return __builtin_amdgcn_cvt_scalef32_pk_f16_fp8((int)w, 1.0f, false); }
__device__ __forceinline__ half2_t f8x2_hi(uint32_t w) { return __builtin_amdgcn_cvt_scalef32_pk_f16_fp8((int)w, 1.0f, true); }
__device__ __forceinline__ half8_t f8x8_to_h8(u32x2 r) {   // 8 e4m3 bytes (element j = byte j) -> 8 f16
  const half2_t a = f8x2_lo(r.x), b = f8x2_hi(r.x), c = f8x2_lo(r.y), d = f8x2_hi(r.y);
  return half8_t{a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y};
}
