// Quantized-weight x int8-activation dot products for the CPU stage (cpu_qdot.cpp).
#pragma once
#include <cstdint>
#include <vector>

namespace mp {

// activation rows quantized to int8 blocks of 32: x ~= d[b] * q[32 b + i]; s = integer sums per 16
struct Q8Buf {
  std::vector<int8_t> q;
  std::vector<float> d;
  std::vector<int32_t> s;
  int64_t K = 0;
  int M = 0;
};
// one row of a Q8Buf
struct Q8Act {
  const int8_t* q;
  const float* d;
  const int32_t* s;
};
inline Q8Act q8_row(const Q8Buf& b, int m) {
  return Q8Act{b.q.data() + (size_t)m * b.K, b.d.data() + (size_t)m * (b.K / 32), b.s.data() + (size_t)m * (b.K / 16)};
}

// ggml types with an integer dot (Q8_0, Q4_0, Q4_K, Q5_K, Q6_K) and their block length in weights
bool qdot_supported(int ggml_type);
int64_t qdot_block(int ggml_type);
// X [M][ldx] f32 -> buf (K a multiple of 32)
void quantize_q8_rows(const float* X, int ldx, int M, int64_t K, Q8Buf& buf);
// dot of one GGUF weight row (K weights of ggml_type) with a quantized activation row; the AVX2 form
// when the host has it, else the scalar one (same integer sums)
float qdot_row(int ggml_type, const uint8_t* w, const Q8Act& x, int64_t K);
float qdot_row_scalar(int ggml_type, const uint8_t* w, const Q8Act& x, int64_t K);

}  // namespace mp
