#include "pack.h"

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <thread>
#include <vector>

// host-only multiversioning (hipcc also runs a device pass over this file, which has no clones)
#if defined(__HIP_DEVICE_COMPILE__)
#define MP_HOST_AVX2_CLONES
#else
#define MP_HOST_AVX2_CLONES __attribute__((target_clones("avx2", "default")))
#endif

namespace mp {

float f16_to_f32(uint16_t h) {
  _Float16 v;
  std::memcpy(&v, &h, 2);
  return (float)v;
}
uint16_t f32_to_f16(float f) {
  _Float16 v = (_Float16)f;
  uint16_t h;
  std::memcpy(&h, &v, 2);
  return h;
}
static inline float bf16f(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
static inline uint16_t rd16(const uint8_t* p) { uint16_t v; std::memcpy(&v, p, 2); return v; }

static inline void get_scale_min_k4(int j, const uint8_t* q, int& d, int& m) {
  if (j < 4) { d = q[j] & 63; m = q[j + 4] & 63; }
  else { d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4); }
}

// quant field extractors (w = 0..255 inside a 256 super-block)
static inline int q4k_nib(const uint8_t* b, int w) {
  const uint8_t* qs = b + 16;
  const int c = w / 64, l = w % 64;
  return l < 32 ? (qs[32 * c + l] & 15) : (qs[32 * c + l - 32] >> 4);
}
static inline int q5k_val(const uint8_t* b, int w) {
  const uint8_t* qh = b + 16;
  const uint8_t* qs = b + 48;
  const int c = w / 64, l = w % 64;
  const int lo = l < 32 ? (qs[32 * c + l] & 15) : (qs[32 * c + l - 32] >> 4);
  const int hi = (qh[l & 31] >> (2 * c + (l >= 32))) & 1;
  return lo | (hi << 4);
}
static inline int q6k_val(const uint8_t* b, int w) {
  const int n = w / 128, rr = w % 128, k = rr / 32, l = rr % 32;
  const uint8_t* ql = b + 64 * n;
  const uint8_t* qh = b + 128 + 32 * n;
  const int lo = k == 0 ? (ql[l] & 15) : k == 1 ? (ql[l + 32] & 15) : k == 2 ? (ql[l] >> 4) : (ql[l + 32] >> 4);
  const int hi = (qh[l] >> (2 * k)) & 3;
  return lo | (hi << 4);
}

// Position of weight w (0..255 of a super-block) of tile row r: MFMA i = 4h + s of lane 16g + r,
// element j, with w = 64g + 32h + 8s + j (the T16 k-mapping, csrc/kernels/dequant.h): lane group
// g owns the quarter [64g, 64g + 64) of the super-block.
struct Pos { int h, s, lane, j; };
static inline Pos pos_of(int w, int r) {
  Pos p;
  const int g = w / 64;
  p.h = (w % 64) / 32;
  p.s = (w % 32) / 8;
  p.j = w % 8;
  p.lane = 16 * g + r;
  return p;
}

// Q4_K / Q5_K header: (d, dmin) as in GGUF, then the 6-bit scales/mins regrouped per lane group g
// as v_g = sc(2g) | m(2g) << 6 | sc(2g+1) << 12 | m(2g+1) << 18, byte b of v_g at byte 4 + 4b + g
static void pack_kquarter_header(const uint8_t* src, uint8_t* dst) {
  std::memcpy(dst, src, 4);
  for (int g = 0; g < 4; ++g) {
    int s0, m0, s1, m1;
    get_scale_min_k4(2 * g, src + 4, s0, m0);
    get_scale_min_k4(2 * g + 1, src + 4, s1, m1);
    const uint32_t v = (uint32_t)s0 | (uint32_t)m0 << 6 | (uint32_t)s1 << 12 | (uint32_t)m1 << 18;
    for (int b = 0; b < 3; ++b) dst[4 + 4 * b + g] = (uint8_t)(v >> (8 * b));
  }
}
static inline void put_nib(uint8_t* chunk, const Pos& p, int v) {
  uint8_t* dw = chunk + p.h * 1024 + p.lane * 16 + p.s * 4;
  const int pos = (p.j & 1) * 4 + (p.j >> 1);   // nibble position inside the dword
  uint8_t& byte = dw[pos / 2];
  byte |= (uint8_t)((v & 15) << ((pos & 1) * 4));
}

static void pack_chunk(int t, int pt, const uint8_t* src, int64_t K, int64_t k0, uint8_t* chunk, int r) {
  // src: row bytes at k0 (super-block start); K: total row length (elements)
  switch (pt) {
    case P_Q4_K: {
      for (int w = 0; w < 256; ++w) put_nib(chunk, pos_of(w, r), q4k_nib(src, w));
      pack_kquarter_header(src, chunk + 2048 + 16 * r);
      break;
    }
    case P_Q5_K: {
      for (int w = 0; w < 256; ++w) {
        const Pos p = pos_of(w, r);
        const int v = q5k_val(src, w);
        put_nib(chunk, p, v & 15);
        uint8_t* qh = chunk + 2048 + p.h * 256 + p.lane * 4;
        const int bit = 8 * p.s + (p.j & 1) * 4 + (p.j >> 1);
        qh[bit / 8] |= (uint8_t)(((v >> 4) & 1) << (bit % 8));
      }
      pack_kquarter_header(src, chunk + 2560 + 16 * r);
      break;
    }
    case P_Q6_K: {
      for (int w = 0; w < 256; ++w) {
        const Pos p = pos_of(w, r);
        const int v = q6k_val(src, w);
        put_nib(chunk, p, v & 15);
        uint8_t* qh = chunk + 2048 + p.h * 512 + p.lane * 8;
        const int i = p.j >> 1;
        const int bit = 16 * p.s + ((p.j & 1) ? 8 + 2 * i : 2 * i);
        qh[bit / 8] |= (uint8_t)(((v >> 4) & 3) << (bit % 8));
      }
      std::memcpy(chunk + 3072 + 16 * r, src + 192, 16);
      std::memcpy(chunk + 3328 + 2 * r, src + 208, 2);
      break;
    }
    case P_Q8_0: {
      for (int b = 0; b < 8; ++b) {
        if (k0 + 32 * b >= K) break;
        const uint8_t* blk = src + 34 * b;
        std::memcpy(chunk + 4096 + 16 * r + 2 * b, blk, 2);
        for (int l = 0; l < 32; ++l) {
          const int w = 32 * b + l;
          const Pos p = pos_of(w, r);
          chunk[p.h * 2048 + p.lane * 32 + p.s * 8 + p.j] = (uint8_t)((int)(int8_t)blk[2 + l] + 128);
        }
      }
      break;
    }
    case P_Q4_0: {
      for (int b = 0; b < 8; ++b) {
        if (k0 + 32 * b >= K) break;
        const uint8_t* blk = src + 18 * b;
        std::memcpy(chunk + 2048 + 16 * r + 2 * b, blk, 2);
        for (int l = 0; l < 32; ++l) {
          const int v = l < 16 ? (blk[2 + l] & 15) : (blk[2 + l - 16] >> 4);
          put_nib(chunk, pos_of(32 * b + l, r), v);
        }
      }
      break;
    }
    case P_BF16: {   // bits as stored in the GGUF (T_BF16 only)
      for (int w = 0; w < 256 && k0 + w < K; ++w) {
        const Pos p = pos_of(w, r);
        std::memcpy(chunk + p.h * 4096 + p.s * 1024 + p.lane * 16 + p.j * 2, src + 2 * w, 2);
      }
      break;
    }
    case P_F16: {
      for (int w = 0; w < 256 && k0 + w < K; ++w) {
        float v;
        if (t == T_F32) std::memcpy(&v, src + 4 * w, 4);
        else if (t == T_F16) v = f16_to_f32(rd16(src + 2 * w));
        else v = bf16f(rd16(src + 2 * w));
        const Pos p = pos_of(w, r);
        const uint16_t h = f32_to_f16(v);
        std::memcpy(chunk + p.h * 4096 + p.s * 1024 + p.lane * 16 + p.j * 2, &h, 2);
      }
      break;
    }
  }
}

int pack_t16(int t, int64_t N, int64_t K, const RowFn& row, uint8_t* dst, int n_threads) {
  const int pt = pack_type_of(t);
  if (pt < 0) throw std::runtime_error(std::string("pack: unsupported ggml type ") + type_name(t));
  return pack_t16_tiles(t, N, K, row, dst, 0, packed_dims(pt, N, K).ntiles, n_threads);
}

// tiles [tile0, tile1) of the T16 image (tile-major, so the range is one contiguous byte run
// starting at tile0 * nsb * chunk_bytes) into dst
int pack_t16_tiles(int t, int64_t N, int64_t K, const RowFn& row, uint8_t* dst, int64_t tile0, int64_t tile1,
                   int n_threads) {
  const int pt = pack_type_of(t);
  if (pt < 0) throw std::runtime_error(std::string("pack: unsupported ggml type ") + type_name(t));
  const PackedDims d = packed_dims(pt, N, K);
  const int cb = chunk_bytes(pt);
  const int be = block_elems(t), bb = block_bytes(t);
  if (K % be) throw std::runtime_error("pack: K not a block multiple");
  if (tile0 < 0 || tile1 > d.ntiles || tile0 > tile1) throw std::runtime_error("pack: bad tile range");
  std::memset(dst, 0, (size_t)(tile1 - tile0) * d.nsb * cb);
  auto work = [&](int64_t t0, int64_t t1) {
    for (int64_t tile = t0; tile < t1; ++tile) {
      for (int r = 0; r < 16; ++r) {
        const int64_t n = tile * 16 + r;
        if (n >= N) break;
        const uint8_t* src = row(n);
        if (!src) continue;
        for (int64_t sb = 0; sb < d.nsb; ++sb) {
          const int64_t k0 = sb * 256;
          uint8_t* chunk = dst + (size_t)((tile - tile0) * d.nsb + sb) * cb;
          const uint8_t* s = src + (size_t)(k0 / be) * bb;
          pack_chunk(t, pt, s, K, k0, chunk, r);
        }
      }
    }
  };
  const int64_t nt = tile1 - tile0;
  if (n_threads <= 0) n_threads = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  if (nt < 64 || n_threads == 1) {
    work(tile0, tile1);
  } else {
    std::vector<std::thread> th;
    const int64_t per = (nt + n_threads - 1) / n_threads;
    for (int i = 0; i < n_threads; ++i) {
      const int64_t a = tile0 + i * per, b = std::min<int64_t>(tile1, a + per);
      if (a < b) th.emplace_back(work, a, b);
    }
    for (auto& x : th) x.join();
  }
  return pt;
}

// (host code: an AVX2 clone chosen at load time where the CPU has it -- no FMA, so both clones round
// alike -- and the baseline x86-64 one elsewhere)
MP_HOST_AVX2_CLONES void dequant_row(int t, const uint8_t* src, float* dst, int64_t K) {
  switch (t) {
    case T_F32: std::memcpy(dst, src, K * 4); return;
    case T_F16: for (int64_t i = 0; i < K; ++i) dst[i] = f16_to_f32(rd16(src + 2 * i)); return;
    case T_BF16: for (int64_t i = 0; i < K; ++i) dst[i] = bf16f(rd16(src + 2 * i)); return;
    case T_Q8_0:
      for (int64_t b = 0; b < K / 32; ++b) {
        const uint8_t* blk = src + 34 * b;
        const float d = f16_to_f32(rd16(blk));
        for (int l = 0; l < 32; ++l) dst[32 * b + l] = d * (float)(int8_t)blk[2 + l];
      }
      return;
    case T_Q4_0:
      for (int64_t b = 0; b < K / 32; ++b) {
        const uint8_t* blk = src + 18 * b;
        const float d = f16_to_f32(rd16(blk));
        for (int l = 0; l < 16; ++l) {
          dst[32 * b + l] = d * (float)((blk[2 + l] & 15) - 8);
          dst[32 * b + l + 16] = d * (float)((blk[2 + l] >> 4) - 8);
        }
      }
      return;
    case T_Q4_K: case T_Q5_K:
      // per 64-element group: two sub-block scales hoisted out of the element loop (the same float
      // arithmetic as the per-element form: (d * sc) * q - dmin * m)
      for (int64_t b = 0; b < K / 256; ++b) {
        const uint8_t* blk = src + (t == T_Q4_K ? 144 : 176) * b;
        const float d = f16_to_f32(rd16(blk)), dmin = f16_to_f32(rd16(blk + 2));
        const uint8_t* __restrict__ qh = blk + 16;             // Q5_K high bits
        const uint8_t* __restrict__ qs = blk + (t == T_Q4_K ? 16 : 48);
        float* __restrict__ o = dst + 256 * b;   // (restrict: the byte loads may not alias the stores)
        for (int c = 0; c < 4; ++c) {
          int s0, m0, s1, m1;
          get_scale_min_k4(2 * c, blk + 4, s0, m0);
          get_scale_min_k4(2 * c + 1, blk + 4, s1, m1);
          const float d0 = d * s0, n0 = dmin * m0, d1 = d * s1, n1 = dmin * m1;
          const uint8_t* __restrict__ q = qs + 32 * c;
          if (t == T_Q4_K) {
            for (int l = 0; l < 32; ++l) {
              o[64 * c + l] = d0 * (q[l] & 15) - n0;
              o[64 * c + 32 + l] = d1 * (q[l] >> 4) - n1;
            }
          } else {
            for (int l = 0; l < 32; ++l) {
              o[64 * c + l] = d0 * ((q[l] & 15) | (((qh[l] >> (2 * c)) & 1) << 4)) - n0;
              o[64 * c + 32 + l] = d1 * ((q[l] >> 4) | (((qh[l] >> (2 * c + 1)) & 1) << 4)) - n1;
            }
          }
        }
      }
      return;
    case T_Q6_K:
      for (int64_t b = 0; b < K / 256; ++b) {
        const uint8_t* blk = src + 210 * b;
        const float d = f16_to_f32(rd16(blk + 208));
        const int8_t* sc = reinterpret_cast<const int8_t*>(blk + 192);
        float* __restrict__ o = dst + 256 * b;
        for (int n = 0; n < 2; ++n) {
          const uint8_t* __restrict__ ql = blk + 64 * n;
          const uint8_t* __restrict__ qh = blk + 128 + 32 * n;
          for (int k = 0; k < 4; ++k) {
            const int w0 = 128 * n + 32 * k;
            const float ds0 = d * sc[w0 / 16], ds1 = d * sc[w0 / 16 + 1];
            const uint8_t* __restrict__ qq = ql + (k & 1) * 32;
            for (int l = 0; l < 32; ++l) {
              const int lo = (k < 2) ? (qq[l] & 15) : (qq[l] >> 4);
              const int v = lo | (((qh[l] >> (2 * k)) & 3) << 4);
              o[w0 + l] = (l < 16 ? ds0 : ds1) * (float)(v - 32);
            }
          }
        }
      }
      return;
  }
  throw std::runtime_error(std::string("dequant_row: unsupported type ") + type_name(t));
}

}  // namespace mp
