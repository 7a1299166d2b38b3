// Quantized-weight x int8-activation dot products for the CPU stage (SURVEY.md E10 / BASELINE
// config 1: the reference's layers that -ngl does not offload run on ggml-cpu, main.rs:49-50).
//
// The f32 path (dequantize a weight row, f32 dot) spent ~22 ms per Llama-3-8B layer on 16 threads
// (profiles/r10al_hybrid_ngl_speed.txt): every weight became 4 bytes of f32 traffic and a scalar-ish
// multiply.  Here the activation rows are quantized once per matmul into blocks of 32 int8 values
// with an f32 scale per block and the integer sums per 16 (Q8Act), and each weight block is
// multiplied in its stored integer form:
//   Q4_K / Q5_K   sum_j (d sc_j q_ji - dmin m_j) (dx_j x_ji)   -> d sc_j dx_j <u4/u5 . i8> - dmin m_j dx_j S_j
//   Q6_K          d sc_s dx (<u6 . i8> - 32 S_s) per 16-wide sub-block s
//   Q8_0          dw dx <i8 . i8>;   Q4_0   dw dx (<u4 . i8> - 8 S)
// Integer block dots run on AVX2 (vpmaddubsw unsigned x signed -> i16 pairs, vpmaddwd -> i32, one
// f32 FMA per 32-block into a vector accumulator; the unsigned operand never exceeds 63, so the i16
// pair sums cannot saturate), with a portable scalar form that gives the same integer sums.  The
// activation scale is per 32 values (finer than a per-256 q8 block), so the result differs from the
// f32 dot only by the int8 rounding of x (relative ~1e-3 per GEMV).
//
// Host-only: hipcc runs a device pass over every runtime .cpp, so the intrinsics are compiled only
// for the host, and the AVX2 forms are picked at run time (__builtin_cpu_supports).
#include "cpu_qdot.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "qtypes.h"

#if !defined(__HIP_DEVICE_COMPILE__) && defined(__x86_64__)
#include <immintrin.h>
#define MP_QDOT_X86 1
#endif

namespace mp {

namespace {

inline float h2f(const uint8_t* p) {
  _Float16 h;
  std::memcpy(&h, p, 2);
  return (float)h;
}

// Q4_K / Q5_K packed 6-bit (scale, min) of sub-block j (GGUF scales[12])
inline void kscale(const uint8_t* s, int j, int& sc, int& m) {
  if (j < 4) {
    sc = s[j] & 63;
    m = s[j + 4] & 63;
  } else {
    sc = (s[j + 4] & 15) | ((s[j - 4] >> 6) << 4);
    m = (s[j + 4] >> 4) | ((s[j] >> 6) << 4);
  }
}

// ---------------------------------------------------------------- scalar reference forms
// (also the fallback on hosts without AVX2; the integer sums are exact, so both forms agree up
// to the f32 summation order)

float dot_q8_0_scalar(const uint8_t* w, const Q8Act& x, int64_t K) {
  float s = 0.f;
  for (int64_t b = 0; b < K / 32; ++b) {
    const uint8_t* blk = w + 34 * b;
    const int8_t* q = reinterpret_cast<const int8_t*>(blk + 2);
    const int8_t* a = x.q + 32 * b;
    int acc = 0;
    for (int i = 0; i < 32; ++i) acc += q[i] * a[i];
    s += h2f(blk) * x.d[b] * (float)acc;
  }
  return s;
}

float dot_q4_0_scalar(const uint8_t* w, const Q8Act& x, int64_t K) {
  float s = 0.f;
  for (int64_t b = 0; b < K / 32; ++b) {
    const uint8_t* blk = w + 18 * b;
    const int8_t* a = x.q + 32 * b;
    int acc = 0;
    for (int i = 0; i < 16; ++i) acc += (blk[2 + i] & 15) * a[i] + (blk[2 + i] >> 4) * a[16 + i];
    acc -= 8 * (x.s[2 * b] + x.s[2 * b + 1]);
    s += h2f(blk) * x.d[b] * (float)acc;
  }
  return s;
}

template <bool Q5>
float dot_q45k_scalar(const uint8_t* w, const Q8Act& x, int64_t K) {
  constexpr int BB = Q5 ? 176 : 144;
  float s = 0.f;
  for (int64_t sb = 0; sb < K / 256; ++sb) {
    const uint8_t* blk = w + BB * sb;
    const float d = h2f(blk), dmin = h2f(blk + 2);
    const uint8_t* sc = blk + 4;
    const uint8_t* qh = blk + 16;
    const uint8_t* qs = blk + (Q5 ? 48 : 16);
    for (int j = 0; j < 8; ++j) {
      int scj, mj;
      kscale(sc, j, scj, mj);
      const int c = j >> 1, hi = j & 1;
      const int64_t xb = sb * 8 + j;
      const int8_t* a = x.q + 32 * xb;
      int acc = 0;
      for (int l = 0; l < 32; ++l) {
        int q = hi ? qs[32 * c + l] >> 4 : qs[32 * c + l] & 15;
        if (Q5 && (qh[l] >> j & 1)) q += 16;
        acc += q * a[l];
      }
      const int sx = x.s[2 * xb] + x.s[2 * xb + 1];
      s += x.d[xb] * (d * (float)scj * (float)acc - dmin * (float)mj * (float)sx);
    }
  }
  return s;
}

float dot_q6k_scalar(const uint8_t* w, const Q8Act& x, int64_t K) {
  float s = 0.f;
  for (int64_t sb = 0; sb < K / 256; ++sb) {
    const uint8_t* blk = w + 210 * sb;
    const float d = h2f(blk + 208);
    const int8_t* scs = reinterpret_cast<const int8_t*>(blk + 192);
    for (int h = 0; h < 2; ++h) {
      const uint8_t* ql = blk + 64 * h;
      const uint8_t* qh = blk + 128 + 32 * h;
      // element e in [0, 128) of this half: quarter t = e / 32, l = e % 32
      for (int t = 0; t < 4; ++t) {
        for (int half16 = 0; half16 < 2; ++half16) {
          int acc = 0;
          for (int l = 16 * half16; l < 16 * half16 + 16; ++l) {
            const int lo = t & 1 ? ql[l + 32] : ql[l];
            const int u = (t < 2 ? lo & 15 : lo >> 4) | (((qh[l] >> (2 * t)) & 3) << 4);
            acc += u * x.q[sb * 256 + 128 * h + 32 * t + l];
          }
          const int64_t s16 = (sb * 256 + 128 * h + 32 * t) / 16 + half16;
          acc -= 32 * x.s[s16];
          const int sc = scs[8 * h + 2 * t + half16];
          s += d * (float)sc * x.d[s16 / 2] * (float)acc;
        }
      }
    }
  }
  return s;
}

#ifdef MP_QDOT_X86
// ---------------------------------------------------------------- AVX2 forms
#define MP_AVX2 __attribute__((target("avx2,fma")))

MP_AVX2 inline float hsum8(__m256 v) {
  __m128 a = _mm_add_ps(_mm256_castps256_ps128(v), _mm256_extractf128_ps(v, 1));
  a = _mm_add_ps(a, _mm_movehl_ps(a, a));
  a = _mm_add_ss(a, _mm_movehdup_ps(a));
  return _mm_cvtss_f32(a);
}
// <u . s> over 32 bytes as 8 i32 lanes (u <= 63: the i16 pair sums stay below 2 * 63 * 128)
MP_AVX2 inline __m256i udot32(__m256i u, __m256i s) {
  return _mm256_madd_epi16(_mm256_maddubs_epi16(u, s), _mm256_set1_epi16(1));
}

MP_AVX2 float dot_q8_0_avx2(const uint8_t* w, const Q8Act& x, int64_t K) {
  __m256 acc = _mm256_setzero_ps();
  for (int64_t b = 0; b < K / 32; ++b) {
    const uint8_t* blk = w + 34 * b;
    const __m256i q = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(blk + 2));
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(x.q + 32 * b));
    // signed x signed through the unsigned form: |q| . (a * sign(q))
    const __m256i p = udot32(_mm256_sign_epi8(q, q), _mm256_sign_epi8(a, q));
    acc = _mm256_fmadd_ps(_mm256_cvtepi32_ps(p), _mm256_set1_ps(h2f(blk) * x.d[b]), acc);
  }
  return hsum8(acc);
}

MP_AVX2 float dot_q4_0_avx2(const uint8_t* w, const Q8Act& x, int64_t K) {
  __m256 acc = _mm256_setzero_ps();
  const __m256i m4 = _mm256_set1_epi8(15);
  float corr = 0.f;
  for (int64_t b = 0; b < K / 32; ++b) {
    const uint8_t* blk = w + 18 * b;
    const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(blk + 2));
    const __m256i u = _mm256_and_si256(_mm256_set_m128i(_mm_srli_epi16(v, 4), v), m4);   // lo 16 | hi 16
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(x.q + 32 * b));
    const float sc = h2f(blk) * x.d[b];
    acc = _mm256_fmadd_ps(_mm256_cvtepi32_ps(udot32(u, a)), _mm256_set1_ps(sc), acc);
    corr += sc * (float)(x.s[2 * b] + x.s[2 * b + 1]);
  }
  return hsum8(acc) - 8.f * corr;
}

template <bool Q5>
MP_AVX2 float dot_q45k_avx2(const uint8_t* w, const Q8Act& x, int64_t K) {
  constexpr int BB = Q5 ? 176 : 144;
  __m256 acc = _mm256_setzero_ps();
  const __m256i m4 = _mm256_set1_epi8(15);
  float mins = 0.f;
  for (int64_t sb = 0; sb < K / 256; ++sb) {
    const uint8_t* blk = w + BB * sb;
    const float d = h2f(blk), dmin = h2f(blk + 2);
    const uint8_t* scp = blk + 4;
    const uint8_t* qs = blk + (Q5 ? 48 : 16);
    int sc[8], mn[8];
    for (int j = 0; j < 8; ++j) kscale(scp, j, sc[j], mn[j]);
    __m256i hb;
    if constexpr (Q5) hb = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(blk + 16));
    const int64_t xb0 = sb * 8;
    for (int c = 0; c < 4; ++c) {
      const __m256i v = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(qs + 32 * c));
      __m256i lo = _mm256_and_si256(v, m4);
      __m256i hi = _mm256_and_si256(_mm256_srli_epi16(v, 4), m4);
      if constexpr (Q5) {   // bit j of qh[l] -> +16 on element l of sub-block j
        const __m256i one = _mm256_set1_epi8(1);
        const __m256i b0 = _mm256_and_si256(_mm256_srli_epi16(hb, 2 * c), one);
        const __m256i b1 = _mm256_and_si256(_mm256_srli_epi16(hb, 2 * c + 1), one);
        lo = _mm256_or_si256(lo, _mm256_slli_epi16(b0, 4));
        hi = _mm256_or_si256(hi, _mm256_slli_epi16(b1, 4));
      }
      const int j0 = 2 * c, j1 = 2 * c + 1;
      const __m256i a0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(x.q + 32 * (xb0 + j0)));
      const __m256i a1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(x.q + 32 * (xb0 + j1)));
      acc = _mm256_fmadd_ps(_mm256_cvtepi32_ps(udot32(lo, a0)), _mm256_set1_ps(d * (float)sc[j0] * x.d[xb0 + j0]), acc);
      acc = _mm256_fmadd_ps(_mm256_cvtepi32_ps(udot32(hi, a1)), _mm256_set1_ps(d * (float)sc[j1] * x.d[xb0 + j1]), acc);
    }
    for (int j = 0; j < 8; ++j)
      mins += dmin * (float)mn[j] * x.d[xb0 + j] * (float)(x.s[2 * (xb0 + j)] + x.s[2 * (xb0 + j) + 1]);
  }
  return hsum8(acc) - mins;
}

MP_AVX2 float dot_q6k_avx2(const uint8_t* w, const Q8Act& x, int64_t K) {
  __m256 acc = _mm256_setzero_ps();
  const __m256i m4 = _mm256_set1_epi8(15), m3 = _mm256_set1_epi8(3);
  float corr = 0.f;
  for (int64_t sb = 0; sb < K / 256; ++sb) {
    const uint8_t* blk = w + 210 * sb;
    const float d = h2f(blk + 208);
    const int8_t* scs = reinterpret_cast<const int8_t*>(blk + 192);
    for (int h = 0; h < 2; ++h) {
      const __m256i l0 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(blk + 64 * h));
      const __m256i l1 = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(blk + 64 * h + 32));
      const __m256i qh = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(blk + 128 + 32 * h));
      __m256i u[4];
      u[0] = _mm256_or_si256(_mm256_and_si256(l0, m4), _mm256_slli_epi16(_mm256_and_si256(qh, m3), 4));
      u[1] = _mm256_or_si256(_mm256_and_si256(l1, m4), _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(qh, 2), m3), 4));
      u[2] = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(l0, 4), m4),
                             _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(qh, 4), m3), 4));
      u[3] = _mm256_or_si256(_mm256_and_si256(_mm256_srli_epi16(l1, 4), m4),
                             _mm256_slli_epi16(_mm256_and_si256(_mm256_srli_epi16(qh, 6), m3), 4));
      for (int t = 0; t < 4; ++t) {
        const int64_t e0 = sb * 256 + 128 * h + 32 * t;   // first element of this 32-block
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(x.q + e0));
        // two 16-wide sub-blocks with their own scales: i32 lanes 0-3 are elements 0-15, 4-7 are 16-31
        const __m256i p = udot32(u[t], a);
        const float dx = x.d[e0 / 32];
        const float s0 = d * (float)scs[8 * h + 2 * t] * dx, s1 = d * (float)scs[8 * h + 2 * t + 1] * dx;
        const __m256 scale = _mm256_setr_ps(s0, s0, s0, s0, s1, s1, s1, s1);
        acc = _mm256_fmadd_ps(_mm256_cvtepi32_ps(p), scale, acc);
        corr += s0 * (float)x.s[e0 / 16] + s1 * (float)x.s[e0 / 16 + 1];
      }
    }
  }
  return hsum8(acc) - 32.f * corr;
}
#endif

bool have_avx2() {
#ifdef MP_QDOT_X86
  static const bool ok = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return ok;
#else
  return false;
#endif
}

}  // namespace

bool qdot_supported(int type) {
  return type == T_Q8_0 || type == T_Q4_0 || type == T_Q4_K || type == T_Q5_K || type == T_Q6_K;
}

int64_t qdot_block(int type) { return type == T_Q8_0 || type == T_Q4_0 ? 32 : 256; }

void quantize_q8_rows(const float* X, int ldx, int M, int64_t K, Q8Buf& buf) {
  if (K % 32) throw std::runtime_error("quantize_q8_rows: K must be a multiple of 32");
  buf.K = K;
  buf.M = M;
  buf.q.resize((size_t)M * K);
  buf.d.resize((size_t)M * (K / 32));
  buf.s.resize((size_t)M * (K / 16));
  for (int m = 0; m < M; ++m) {
    const float* x = X + (size_t)m * ldx;
    int8_t* q = buf.q.data() + (size_t)m * K;
    float* d = buf.d.data() + (size_t)m * (K / 32);
    int32_t* s = buf.s.data() + (size_t)m * (K / 16);
    for (int64_t b = 0; b < K / 32; ++b) {
      float amax = 0.f;
      for (int i = 0; i < 32; ++i) amax = std::max(amax, std::fabs(x[32 * b + i]));
      const float db = amax / 127.f;
      const float id = db > 0.f ? 1.f / db : 0.f;
      d[b] = db;
      int s0 = 0, s1 = 0;
      for (int i = 0; i < 32; ++i) {
        const int v = (int)std::nearbyint(x[32 * b + i] * id);
        q[32 * b + i] = (int8_t)std::max(-127, std::min(127, v));
        (i < 16 ? s0 : s1) += q[32 * b + i];
      }
      s[2 * b] = s0;
      s[2 * b + 1] = s1;
    }
  }
}

float qdot_row(int type, const uint8_t* w, const Q8Act& x, int64_t K) {
  if (K % qdot_block(type)) throw std::runtime_error("qdot_row: K not a multiple of the block");
#ifdef MP_QDOT_X86
  if (have_avx2()) {
    switch (type) {
      case T_Q8_0: return dot_q8_0_avx2(w, x, K);
      case T_Q4_0: return dot_q4_0_avx2(w, x, K);
      case T_Q4_K: return dot_q45k_avx2<false>(w, x, K);
      case T_Q5_K: return dot_q45k_avx2<true>(w, x, K);
      case T_Q6_K: return dot_q6k_avx2(w, x, K);
    }
  }
#endif
  return qdot_row_scalar(type, w, x, K);
}

float qdot_row_scalar(int type, const uint8_t* w, const Q8Act& x, int64_t K) {
  switch (type) {
    case T_Q8_0: return dot_q8_0_scalar(w, x, K);
    case T_Q4_0: return dot_q4_0_scalar(w, x, K);
    case T_Q4_K: return dot_q45k_scalar<false>(w, x, K);
    case T_Q5_K: return dot_q45k_scalar<true>(w, x, K);
    case T_Q6_K: return dot_q6k_scalar(w, x, K);
  }
  throw std::runtime_error("qdot_row: unsupported type");
}

}  // namespace mp
