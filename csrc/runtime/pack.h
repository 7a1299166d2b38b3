// Host-side repacking of GGUF block tensors into the T16 device layout (qtypes.h).
#pragma once
#include <stdint.h>
#include <functional>

#include "qtypes.h"

namespace mp {

// Source row accessor: GGUF-native bytes of row n (K elements of `ggml_type`), or nullptr for a
// zero (padding) row.
using RowFn = std::function<const uint8_t*(int64_t n)>;

// Pack N x K (ggml row-major, row = output feature) into dst (packed_dims(...).bytes bytes).
// Multi-threaded over tiles.  Returns the packed type (PackType).
int pack_t16(int ggml_type, int64_t N, int64_t K, const RowFn& row, uint8_t* dst, int n_threads = 0);
// tiles [tile0, tile1) only (a contiguous byte range of the tile-major image), into dst
int pack_t16_tiles(int ggml_type, int64_t N, int64_t K, const RowFn& row, uint8_t* dst, int64_t tile0, int64_t tile1,
                   int n_threads = 0);

// Row n of the gate/up interleaved matrix (2F rows): tile t rows 0-7 = gate rows 8t..8t+7,
// rows 8-15 = up rows 8t..8t+7.
inline int64_t gateup_src_row(int64_t n, bool* is_up) {
  const int64_t t = n / 16, r = n % 16;
  *is_up = r >= 8;
  return t * 8 + (r & 7);
}

// Dequantize one GGUF-native row (K elements) to f32 (host reference path / CPU backend).
void dequant_row(int ggml_type, const uint8_t* src, float* dst, int64_t K);

float f16_to_f32(uint16_t h);
uint16_t f32_to_f16(float f);

}  // namespace mp
