// ggml block types (GGUF) and mipipe's MI355X-native packed weight layout.
//
// Packed layout ("T16"): a weight W[N][K] (row n = output feature) is cut into tiles of 16 rows
// and super-blocks of 256 k.  Tile t's super-blocks are contiguous, so one wavefront streams a
// tile with 16-B-per-lane coalesced loads.  Inside a (tile, super-block) chunk the bytes are
// arranged so that lane l = 16*g + r (g = l>>4, r = l&15) of a wave gets, with ONE 16-B load per
// 128-k half, exactly the 32 quantized weights of row r that feed its B-operand fragments of four
// consecutive v_mfma_f32_16x16x32_f16 (k = 128h + 32s + 8g + j, s = 0..3, j = 0..7).  Nibble order
// inside a dword lets ((w >> 4i) & 0x000F000F) | 0x64006400 produce a packed f16 pair (1024+q)
// directly.  Bytes per chunk equal 16 x the ggml block bytes (no bandwidth overhead), except F16
// which stores plain f16.
#pragma once
#include <stdint.h>
#include <stddef.h>

#if defined(__HIPCC__)
#define MP_HD __host__ __device__
#else
#define MP_HD
#endif

namespace mp {

enum GgmlType : int {
  T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q4_1 = 3, T_Q5_0 = 6, T_Q5_1 = 7, T_Q8_0 = 8, T_Q8_1 = 9,
  T_Q2_K = 10, T_Q3_K = 11, T_Q4_K = 12, T_Q5_K = 13, T_Q6_K = 14, T_Q8_K = 15, T_BF16 = 30,
};

inline const char* type_name(int t) {
  switch (t) {
    case T_F32: return "F32"; case T_F16: return "F16"; case T_BF16: return "BF16";
    case T_Q8_0: return "Q8_0"; case T_Q4_0: return "Q4_0"; case T_Q4_K: return "Q4_K";
    case T_Q5_K: return "Q5_K"; case T_Q6_K: return "Q6_K"; default: return "?";
  }
}

// elements per block, bytes per block; 0 if unsupported
MP_HD inline int block_elems(int t) {
  switch (t) {
    case T_F32: case T_F16: case T_BF16: return 1;
    case T_Q8_0: case T_Q4_0: return 32;
    case T_Q4_K: case T_Q5_K: case T_Q6_K: return 256;
    default: return 0;
  }
}
MP_HD inline int block_bytes(int t) {
  switch (t) {
    case T_F32: return 4; case T_F16: case T_BF16: return 2;
    case T_Q8_0: return 34; case T_Q4_0: return 18;
    case T_Q4_K: return 144; case T_Q5_K: return 176; case T_Q6_K: return 210;
    default: return 0;
  }
}
inline size_t row_bytes(int t, int64_t n) { return (size_t)(n / block_elems(t)) * block_bytes(t); }

// Packed kernel types (what the GEMV/GEMM kernels stream).  F32 weights are packed as F16; BF16
// weights stay bf16 (P_BF16, same chunk layout as F16): no narrowing at pack time, the kernels run
// the bf16 MFMA on them.  P_I8 is not a GGUF type: per-row int8 re-quantized weights (one f32 scale
// per output row, kept beside the matrix) for the int8-activation GEMM prototype (gemm3.hip, K15).
enum PackType : int { P_F16 = 0, P_Q8_0 = 1, P_Q4_K = 2, P_Q5_K = 3, P_Q6_K = 4, P_Q4_0 = 5, P_BF16 = 6, P_I8 = 7 };
constexpr bool is16(int p) { return p == P_F16 || p == P_BF16; }

inline int pack_type_of(int ggml_type) {
  switch (ggml_type) {
    case T_F32: case T_F16: return P_F16;
    case T_BF16: return P_BF16;
    case T_Q8_0: return P_Q8_0; case T_Q4_0: return P_Q4_0;
    case T_Q4_K: return P_Q4_K; case T_Q5_K: return P_Q5_K; case T_Q6_K: return P_Q6_K;
    default: return -1;
  }
}

// bytes of one (16-row tile, 256-k super-block) chunk
constexpr int chunk_bytes(int p) {
  return is16(p) ? 8192 : p == P_Q8_0 ? 4352 : p == P_Q4_K ? 2304 : p == P_Q5_K ? 2816
       : p == P_Q6_K ? 3360 : p == P_Q4_0 ? 2304 : p == P_I8 ? 4096 : 0;
}

inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

struct PackedDims {
  int64_t N, K, N_pad, K_pad, ntiles, nsb;
  size_t bytes;
};

inline PackedDims packed_dims(int ptype, int64_t N, int64_t K) {
  PackedDims d;
  d.N = N; d.K = K;
  d.N_pad = round_up(N, 16);
  d.K_pad = round_up(K, 256);
  d.ntiles = d.N_pad / 16;
  d.nsb = d.K_pad / 256;
  d.bytes = (size_t)d.ntiles * d.nsb * chunk_bytes(ptype);
  return d;
}

}  // namespace mp
