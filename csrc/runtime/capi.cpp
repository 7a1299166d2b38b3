// C ABI of libmipipe.so (consumed by the python package through ctypes and by the C++ tools).
// Every entry point catches exceptions, records the message (mp_last_error) and returns an
// error code / nullptr.
#include <hip/hip_runtime.h>
#include "tuning.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <string>
#include <atomic>
#include <mutex>
#include <thread>

#include "cpu_qdot.h"
#include "engine.h"
#include "probe.h"
#include "model.h"
#include "gguf.h"
#include "hip_stage.h"
#include "json.h"
#include "kernels_api.h"
#include "log.h"
#include "pack.h"
#include "tokenizer.h"
#include "transport.h"

using namespace mp;

static thread_local std::string g_err;
static thread_local std::string g_str;

#define API_TRY try {
#define API_CATCH(ret)                 \
  }                                    \
  catch (const std::exception& e) {    \
    g_err = e.what();                  \
    return ret;                        \
  }

extern "C" {

const char* mp_last_error() { return g_err.c_str(); }
int mp_version() { return 1; }
void mp_log_level(int lvl) { log_set_level(lvl); }
void mp_log_file(const char* path) { log_set_file(path ? path : ""); }

// ------------------------------------------------------------------ host utilities
int64_t mp_packed_bytes(int type, int64_t N, int64_t K) {
  const int pt = pack_type_of(type);
  if (pt < 0) return -1;
  return (int64_t)packed_dims(pt, N, K).bytes;
}
int mp_pack_type(int type) { return pack_type_of(type); }

int mp_pack_t16(int type, int64_t N, int64_t K, const uint8_t* src, int64_t src_row_bytes, uint8_t* dst,
                int gateup_interleave) {
  API_TRY
  if (gateup_interleave) {
    // src holds gate rows [0, N/2) then up rows [N/2, N)
    const int64_t F = N / 2;
    pack_t16(type, N, K, [&](int64_t n) -> const uint8_t* {
      bool up;
      const int64_t r = gateup_src_row(n, &up);
      if (r >= F) return nullptr;
      return src + (up ? F + r : r) * src_row_bytes;
    }, dst);
  } else {
    pack_t16(type, N, K, [&](int64_t n) -> const uint8_t* { return src + n * src_row_bytes; }, dst);
  }
  return 0;
  API_CATCH(-1)
}

int mp_dequant_row(int type, const uint8_t* src, float* dst, int64_t K) {
  API_TRY
  dequant_row(type, src, dst, K);
  return 0;
  API_CATCH(-1)
}

// CPU integer dot (cpu_qdot.cpp): y[n] = <row n of W (N rows of K weights of ggml type), q8(x)>, the
// dispatched (AVX2 when present) and the scalar form; returns 1 if the type has an integer dot
int mp_qdot_rows(int type, const uint8_t* W, int64_t N, int64_t K, const float* x, float* y, float* y_scalar) {
  API_TRY
  if (!qdot_supported(type)) return 0;
  Q8Buf b;
  quantize_q8_rows(x, (int)K, 1, K, b);
  const size_t rb = row_bytes(type, K);
  for (int64_t n = 0; n < N; ++n) {
    y[n] = qdot_row(type, W + n * rb, q8_row(b, 0), K);
    if (y_scalar) y_scalar[n] = qdot_row_scalar(type, W + n * rb, q8_row(b, 0), K);
  }
  return 1;
  API_CATCH(-1)
}

int mp_partition(const double* cost, int L, double first_extra, double last_extra, const double* speed, int S,
                 int mode, int32_t* out_ranges) {
  API_TRY
  std::vector<double> c(cost, cost + L), sp(speed, speed + S);
  auto r = partition_layers(c, first_extra, last_extra, sp, (SplitMode)mode);
  for (int s = 0; s < S; ++s) { out_ranges[2 * s] = r[s].layer_begin; out_ranges[2 * s + 1] = r[s].layer_end; }
  return 0;
  API_CATCH(-1)
}

// ------------------------------------------------------------------ GGUF
void* mp_gguf_open(const char* path) {
  API_TRY
  return new GgufFile(path);
  API_CATCH(nullptr)
}
void mp_gguf_close(void* h) { delete static_cast<GgufFile*>(h); }

const char* mp_gguf_json(void* h) {
  API_TRY
  auto* f = static_cast<GgufFile*>(h);
  Json j = Json::object();
  j["version"] = (int)f->version();
  Json kv = Json::object();
  for (auto& it : f->kv()) {
    const GgufValue& v = it.second;
    if (v.type == GV_STRING) kv[it.first] = Json(v.s);
    else if (v.type == GV_ARRAY) {
      Json a = Json::object();
      a["array_len"] = (int64_t)(v.elem_type == GV_STRING ? v.strs.size() : v.nums.size());
      a["elem_type"] = (int)v.elem_type;
      kv[it.first] = a;
    } else if (v.type == GV_F32 || v.type == GV_F64) kv[it.first] = Json(v.f);
    else kv[it.first] = Json((int64_t)v.i);
  }
  j["kv"] = kv;
  Json ts = Json::array();
  for (auto& t : f->tensors()) {
    Json o = Json::object();
    o["name"] = t.name;
    Json ne = Json::array();
    for (auto x : t.ne) ne.push(Json((int64_t)x));
    o["ne"] = ne;
    o["type"] = t.type;
    o["offset"] = (int64_t)t.offset;
    o["nbytes"] = (int64_t)t.nbytes;
    ts.push(o);
  }
  j["tensors"] = ts;
  g_str = j.dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}

const char* mp_model_config_json(const char* gguf_path) {
  API_TRY
  GgufFile f(gguf_path);
  ModelConfig c = ModelConfig::from_gguf(f);
  Json j = Json::object();
  j["n_layer"] = c.n_layer; j["d_model"] = c.d_model; j["n_head"] = c.n_head; j["n_head_kv"] = c.n_head_kv;
  j["head_dim"] = c.head_dim; j["d_ff"] = c.d_ff; j["vocab"] = c.vocab; j["rope_base"] = (double)c.rope_base;
  j["eps"] = (double)c.eps; j["n_expert"] = c.n_expert; j["n_expert_used"] = c.n_expert_used;
  j["rope_freqs"] = c.rope_freqs; j["tied_output"] = c.tied_output;
  j["arch"] = c.arch; j["rope_neox"] = c.rope_neox; j["qkv_bias"] = c.qkv_bias;
  g_str = j.dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}

// ------------------------------------------------------------------ kernel ops (tests)
int mp_op_gemm(int ptype, int epi, const void* W, int ntiles, int nsb, const void* X, int ldx, int M, void* Y,
               int ldy, void* H, int ldh, int n_valid, void* stream) {
  API_TRY
  GemvParams p{};
  p.W = (const uint8_t*)W; p.X = (const f16*)X; p.ldx = ldx; p.M = M; p.Y = (float*)Y; p.ldy = ldy;
  p.H = (f16*)H; p.ldh = ldh; p.ntiles = ntiles; p.nsb = nsb; p.n_valid = n_valid;
  launch_gemm(ptype, epi, p, (hipStream_t)stream);
  return 0;
  API_CATCH(-1)
}

int mp_op_gemm3(int ptype, int epi, const void* W, int ntiles, int nsb, const void* X, int ldx, int M, void* Y,
                int ldy, void* H, int ldh, int n_valid, int allow_split, void* stream) {
  API_TRY
  GemvParams p{};
  p.W = (const uint8_t*)W; p.X = (const f16*)X; p.ldx = ldx; p.M = M; p.Y = (float*)Y; p.ldy = ldy;
  p.H = (f16*)H; p.ldh = ldh; p.ntiles = ntiles; p.nsb = nsb; p.n_valid = n_valid;
  launch_gemm3(ptype, epi, p, (hipStream_t)stream, allow_split != 0);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_gemm4(int ptype, int epi, const void* W, int ntiles, int nsb, const void* X, int ldx, int M, void* Y,
                int ldy, void* H, int ldh, int n_valid, int allow_split, void* stream) {
  API_TRY
  GemvParams p{};
  p.W = (const uint8_t*)W; p.X = (const f16*)X; p.ldx = ldx; p.M = M; p.Y = (float*)Y; p.ldy = ldy;
  p.H = (f16*)H; p.ldh = ldh; p.ntiles = ntiles; p.nsb = nsb; p.n_valid = n_valid;
  if (!launch_gemm4(ptype, epi, p, (hipStream_t)stream, allow_split != 0)) throw std::runtime_error("gemm4: unsupported type");
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

// MoE (K13): device-side top-k routing of router logits [M][ld] into per-expert slot lists
int mp_op_moe_route(const void* logits, int ld, int M, int E, int k, void* counts, void* lists, int list_cap,
                    void* weights, void* stream) {
  API_TRY
  MoeRouteParams rp{};
  rp.logits = (const float*)logits; rp.ld = ld; rp.M = M; rp.E = E; rp.k = k;
  rp.counts = (int32_t*)counts; rp.lists = (int32_t*)lists; rp.list_cap = list_cap; rp.weights = (float*)weights;
  launch_moe_route(rp, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

// grouped expert GEMM (gemm4 MoE mode): SWIGLU (gate/up of every routed slot into H[slot]) or ATOMIC
// (down: router-weighted into Y[slot / k]); W = E packed matrices, estride bytes apart
int mp_op_moe_gemm4(int ptype, int epi, const void* W, int64_t estride, int ntiles, int nsb, const void* X, int ldx,
                    int x_per_slot, int M, int E, int k, const void* counts, const void* lists, int list_cap,
                    const void* weights, void* Y, int ldy, void* H, int ldh, int n_valid, void* stream) {
  API_TRY
  MoeGemvParams q{};
  q.W = (const uint8_t*)W; q.estride = (size_t)estride; q.ntiles = ntiles; q.nsb = nsb;
  q.X = (const f16*)X; q.ldx = ldx; q.x_per_slot = x_per_slot; q.M = M; q.E = E; q.k = k;
  q.counts = (const int32_t*)counts; q.lists = (const int32_t*)lists; q.list_cap = list_cap;
  q.weights = (const float*)weights; q.Y = (float*)Y; q.ldy = ldy; q.H = (f16*)H; q.ldh = ldh; q.n_valid = n_valid;
  if (!launch_moe_gemm4(ptype, epi, q, (hipStream_t)stream)) throw std::runtime_error("moe_gemm4: unsupported type/epilogue");
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

// router logits [M][ld] = X [M][ldx] . R [E][K]^T (dense f16 router)
int mp_op_router_logits(const void* X, int ldx, const void* R, int K, int E, int M, void* out, int ld, void* stream) {
  API_TRY
  launch_router_logits((const f16*)X, ldx, (const f16*)R, K, E, M, (float*)out, ld, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

// split-K with partial stores + the fixed-order reduction into Y; returns the split count, 0 when
// the shape does not split (nothing launched)
int mp_op_gemm4_splitk(int ptype, const void* W, int ntiles, int nsb, const void* X, int ldx, int M, void* Y, int ldy,
                       int n_valid, void* scratch, int64_t scratch_n, void* stream) {
  API_TRY
  GemvParams p{};
  p.W = (const uint8_t*)W; p.X = (const f16*)X; p.ldx = ldx; p.M = M; p.Y = (float*)Y; p.ldy = ldy;
  p.ntiles = ntiles; p.nsb = nsb; p.n_valid = n_valid;
  int ns = 0;
  if (!launch_gemm4_splitk(ptype, p, (float*)scratch, (size_t)scratch_n, (hipStream_t)stream, true, &ns)) return 0;
  HIP_OK(hipGetLastError());
  return ns;
  API_CATCH(-1)
}

// A/B overrides of gemm3 through the knob registry (0 = auto; split_wg 0 = the default 256 of the
// GEMM2_SPLIT_WG knob both GEMMs share)
int mp_set_gemm3_tuning(int bm, int bn, int nsplit, int split_wg) {
  API_TRY
  // 0 = back to the process's own value (environment or default), not a hard-coded one
  auto put = [](const char* k, int v) { v > 0 ? set_knob(k, v) : reset_knob(k); };
  put("GEMM3_BM", bm);
  put("GEMM3_BN", bn);
  put("GEMM3_SPLIT", nsplit);
  put("GEMM2_SPLIT_WG", split_wg);
  return 0;
  API_CATCH(-1)
}

// int8-activation GEMM prototype (K15): X f16 [M][ldx] -> int8 rows Q [M][ldq] + row scales xs;
// then Y = xs[m] ws[n] sum_k Q[m][k] W8[n][k] on v_mfma_i32_16x16x64_i8 (W: P_I8 chunks)
int mp_op_quant_i8(const void* X, int ldx, int M, int K, void* Q, int ldq, void* xs, void* stream) {
  API_TRY
  launch_quant_rows_i8((const f16*)X, ldx, M, K, (int8_t*)Q, ldq, (float*)xs, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_gemm3_i8(int epi, const void* W, int ntiles, int nsb, const void* Q, int ldq, int M, void* Y, int ldy,
                   void* H, int ldh, int n_valid, const void* xs, const void* ws, int allow_split, void* stream) {
  API_TRY
  GemvParams p{};
  p.W = (const uint8_t*)W; p.X = (const f16*)Q; p.ldx = ldq; p.M = M; p.Y = (float*)Y; p.ldy = ldy;
  p.H = (f16*)H; p.ldh = ldh; p.ntiles = ntiles; p.nsb = nsb; p.n_valid = n_valid;
  p.xscale = (const float*)xs; p.wscale = (const float*)ws;
  launch_gemm3(P_I8, epi, p, (hipStream_t)stream, allow_split != 0);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_set_knob(const char* name, int value) {
  API_TRY
  set_knob(name, value);
  return 0;
  API_CATCH(-1)
}

// back to the knob's MIPIPE_* environment value, else its default
int mp_reset_knob(const char* name) {
  API_TRY
  reset_knob(name);
  return 0;
  API_CATCH(-1)
}

int mp_op_gemv(int ptype, int epi, const void* W, int ntiles, int nsb, const void* X, int ldx, int M, void* Y,
               int ldy, void* H, int ldh, int n_valid, int nsplit, void* stream) {
  API_TRY
  GemvParams p{};
  p.W = (const uint8_t*)W; p.X = (const f16*)X; p.ldx = ldx; p.M = M; p.Y = (float*)Y; p.ldy = ldy;
  p.H = (f16*)H; p.ldh = ldh; p.ntiles = ntiles; p.nsb = nsb; p.n_valid = n_valid;
  if (M > 64) {
    for (int r0 = 0; r0 < M; r0 += 64) {
      GemvParams q = p;
      q.M = std::min(64, M - r0);
      q.X = p.X + (size_t)r0 * ldx;
      if (q.Y) q.Y = p.Y + (size_t)r0 * ldy;
      if (q.H) q.H = p.H + (size_t)r0 * ldh;
      launch_gemv(ptype, epi, q, nsplit, (hipStream_t)stream);
    }
  } else {
    launch_gemv(ptype, epi, p, nsplit, (hipStream_t)stream);
  }
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

void mp_set_gemv_tpw(int t) { set_gemv_tpw(t); }

int mp_init_packed(void* W, size_t nbytes, int ptype, float scale, uint64_t seed, void* stream) {
  API_TRY
  launch_init_packed((uint8_t*)W, nbytes, ptype, scale, seed, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_unpack(int ptype, const void* W, int ntiles, int nsb, void* out, int ldo, void* stream) {
  API_TRY
  launch_unpack(ptype, (const uint8_t*)W, ntiles, nsb, (f16*)out, ldo, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

// decode GEMV (gemv2.hip) with its optional fusions: Xf/gamma (deferred RMSNorm of the f32 rows Xf,
// M <= 4, X unused; ATOMIC publishes sum(x^2) per row to ssq), bias (added once per output),
// zero/zero_n (cleared after the GEMV)
int mp_op_gemv_fused(int ptype, int epi, const void* W, int ntiles, int nsb, const void* X, int ldx, int M, void* Y,
                     int ldy, void* H, int ldh, int n_valid, int nsplit, const void* Xf, int ldxf, const void* gamma,
                     float eps, int d_norm, void* ssq, const void* bias, void* zero, int64_t zero_n, void* stream) {
  API_TRY
  GemvParams p{};
  p.W = (const uint8_t*)W; p.X = (const f16*)X; p.ldx = ldx; p.M = M; p.Y = (float*)Y; p.ldy = ldy;
  p.H = (f16*)H; p.ldh = ldh; p.ntiles = ntiles; p.nsb = nsb; p.n_valid = n_valid;
  p.Xf = (const float*)Xf; p.ldxf = ldxf; p.gamma = (const float*)gamma; p.eps = eps; p.d_norm = d_norm;
  p.ssq = (float*)ssq; p.bias = (const float*)bias; p.zero = (float*)zero; p.zero_n = zero_n;
  launch_gemv(ptype, epi, p, nsplit, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

// small-M GEMV (gemvs.hip, M <= 4): Xf/gamma fuse the RMSNorm of the f32 rows Xf; ATOMIC adds into Y
// (read-modify-write at one k-split, atomics above); G / nsplit 0 = the launcher's own plan
int mp_op_gemvs(int ptype, int epi, const void* W, int ntiles, int nsb, const void* X, int ldx, int M, void* Y,
                int ldy, void* H, int ldh, int n_valid, const void* Xf, int ldxf, const void* gamma, float eps,
                int d_norm, const void* bias, int G, int nsplit, int deterministic, void* stream) {
  API_TRY
  GemvParams p{};
  p.W = (const uint8_t*)W; p.X = (const f16*)X; p.ldx = ldx; p.M = M; p.Y = (float*)Y; p.ldy = ldy;
  p.H = (f16*)H; p.ldh = ldh; p.ntiles = ntiles; p.nsb = nsb; p.n_valid = n_valid;
  p.Xf = (const float*)Xf; p.ldxf = ldxf; p.gamma = (const float*)gamma; p.eps = eps; p.d_norm = d_norm;
  p.bias = (const float*)bias;
  launch_gemvs(ptype, epi, p, deterministic != 0, (hipStream_t)stream, G, nsplit);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_rmsnorm(const void* x, int ldx, const void* w, int d, float eps, void* out, int ldo, int M, void* stream) {
  API_TRY
  launch_rmsnorm((const float*)x, ldx, (const float*)w, d, eps, (f16*)out, ldo, M, nullptr, 0, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_embed(int type, const void* table, int64_t row_bytes, int d, const void* tokens, int M, void* x, int ldx,
                void* stream) {
  API_TRY
  launch_embed(type, (const uint8_t*)table, row_bytes, d, (const int32_t*)tokens, M, (float*)x, ldx,
               (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_rope_kv(const void* qkv, int ldqkv, int M, int Hq, int Hkv, int hd, int Dp, const void* pos,
                  const void* slot, const void* block_table, int max_pages, const void* rope_cs, float q_scale,
                  void* q_out, void* k_cache, void* v_cache, void* stream) {
  API_TRY
  RopeKvParams p{};
  p.qkv = (const float*)qkv; p.ldqkv = ldqkv; p.M = M; p.Hq = Hq; p.Hkv = Hkv; p.hd = hd; p.Dp = Dp;
  p.pos = (const int32_t*)pos; p.slot = (const int32_t*)slot; p.block_table = (const int32_t*)block_table;
  p.max_pages = max_pages; p.rope_cs = (const float2*)rope_cs; p.q_scale = q_scale; p.q_out = (f16*)q_out;
  p.k_cache = (f16*)k_cache; p.v_cache = (f16*)v_cache;
  launch_rope_kv(p, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_attention(const void* q, const void* kvlen, const void* slot, const void* block_table, int max_pages,
                    const void* k_cache, const void* v_cache, int M, int Hq, int Hkv, int hd, int Dp, int tq,
                    int split_len, int n_split, void* o_part, void* ml_part, void* out, int ldo, void* stream) {
  API_TRY
  AttnParams p{};
  p.q = (const f16*)q; p.kvlen = (const int32_t*)kvlen; p.slot = (const int32_t*)slot;
  p.block_table = (const int32_t*)block_table; p.max_pages = max_pages; p.k_cache = (const f16*)k_cache;
  p.v_cache = (const f16*)v_cache; p.M = M; p.Hq = Hq; p.Hkv = Hkv; p.hd = hd; p.Dp = Dp; p.tq = tq;
  p.split_len = split_len; p.n_split = n_split; p.o_part = (float*)o_part; p.ml_part = (float*)ml_part;
  p.out = (f16*)out; p.ldo = ldo;
  launch_attention(p, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

// prefill flash attention over a packed chunk: segs = (row0, T) pairs of consecutive rows of one
// sequence each; the tiles are cut here exactly as the engine cuts them
int mp_op_attn_prefill(const void* q, const void* pos, const void* slot, const void* block_table, int max_pages,
                       const void* k_cache, const void* v_cache, int Hq, int Hkv, int hd, int Dp, const int32_t* segs,
                       int n_segs, void* out, int ldo, int n_split, int split_pages, void* o_part, void* ml_part,
                       int M, void* stream) {
  API_TRY
  PrefillAttnParams p{};
  p.q = (const f16*)q; p.pos = (const int32_t*)pos; p.slot = (const int32_t*)slot;
  p.block_table = (const int32_t*)block_table; p.max_pages = max_pages;
  p.k_cache = (const f16*)k_cache; p.v_cache = (const f16*)v_cache;
  p.Hq = Hq; p.Hkv = Hkv; p.hd = hd; p.Dp = Dp; p.out = (f16*)out; p.ldo = ldo;
  p.M = M; p.n_split = n_split; p.split_pages = split_pages; p.o_part = (float*)o_part; p.ml_part = (float*)ml_part;
  const int bt = prefill_attn_rows_per_tile(Hq / Hkv);
  for (int s = 0; s < n_segs; ++s)
    for (int r = 0; r < segs[2 * s + 1]; r += bt) {
      if (p.n_tiles == kPrefillAttnMaxTiles) { launch_attn_prefill(p, (hipStream_t)stream); p.n_tiles = 0; }
      p.tiles[p.n_tiles++] = (uint32_t)(segs[2 * s] + r) | ((uint32_t)std::min(bt, segs[2 * s + 1] - r) << 16);
    }
  launch_attn_prefill(p, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_argmax(const void* logits, int ld, int n, int M, void* tokens, void* part, void* counters, void* stream) {
  API_TRY
  // part [M][kArgmaxChunks][2] f32 + counters [M] zeroed int32 select the two-level kernel
  ArgmaxScratch sc{(float*)part, (int32_t*)counters, M};
  launch_argmax((const float*)logits, ld, n, M, (int32_t*)tokens, (hipStream_t)stream, part ? &sc : nullptr);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_sample(const void* logits, int ld, int n, int M, float temp, int top_k, float top_p, float min_p,
                 uint64_t seed, const void* step, void* tokens, void* stream) {
  API_TRY
  SampleParams p{};
  p.logits = (const float*)logits; p.ld = ld; p.n = n; p.M = M; p.temp = temp; p.top_k = top_k; p.top_p = top_p;
  p.min_p = min_p; p.seed = seed; p.step = (const int32_t*)step; p.tokens = (int32_t*)tokens;
  launch_sample(p, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_penalize(void* logits, int ld, int n, int M, const void* hist, int last_n, float repeat, float freq,
                   float presence, void* stream) {
  API_TRY
  PenaltyParams p{};
  p.logits = (float*)logits; p.ld = ld; p.n = n; p.M = M; p.hist = (const int32_t*)hist; p.last_n = last_n;
  p.repeat = repeat; p.freq = freq; p.presence = presence;
  launch_penalize(p, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

int mp_op_hist_push(void* hist, void* cnt, int last_n, const void* tokens, int M, void* stream) {
  API_TRY
  launch_hist_push((int32_t*)hist, (int32_t*)cnt, last_n, (const int32_t*)tokens, M, (hipStream_t)stream);
  HIP_OK(hipGetLastError());
  return 0;
  API_CATCH(-1)
}

// ------------------------------------------------------------------ tokenizer
void* mp_tok_open(const char* gguf_path) {
  API_TRY
  GgufFile f(gguf_path);
  return new Tokenizer(Tokenizer::from_gguf(f));
  API_CATCH(nullptr)
}
void mp_tok_close(void* h) { delete static_cast<Tokenizer*>(h); }
int mp_tok_encode(void* h, const char* text, int add_bos, int parse_special, int32_t* out, int cap) {
  API_TRY
  auto ids = static_cast<Tokenizer*>(h)->encode(text, add_bos != 0, parse_special != 0);
  const int n = (int)ids.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = ids[i];
  return n;
  API_CATCH(-1)
}
int mp_tok_piece(void* h, int32_t id, char* buf, int cap) {
  API_TRY
  const std::string s = static_cast<Tokenizer*>(h)->piece(id);
  const int n = (int)s.size();
  if (n <= cap) std::memcpy(buf, s.data(), n);
  return n;
  API_CATCH(-1)
}
int mp_tok_decode(void* h, const int32_t* ids, int n, char* buf, int cap) {
  API_TRY
  const std::string s = static_cast<Tokenizer*>(h)->decode(std::vector<int32_t>(ids, ids + n));
  const int len = (int)s.size();
  if (len <= cap) std::memcpy(buf, s.data(), len);
  return len;
  API_CATCH(-1)
}
int mp_tok_info(void* h, int32_t* out) {  // vocab, bos, eos, eot
  API_TRY
  auto* t = static_cast<Tokenizer*>(h);
  out[0] = t->n_vocab(); out[1] = t->bos(); out[2] = t->eos(); out[3] = t->eot();
  return 0;
  API_CATCH(-1)
}
// pre-tokenizer split (tests): returns pieces joined by '\x1f'
const char* mp_tok_pretokenize(const char* text, int max_digits) {
  API_TRY
  g_str.clear();
  for (auto& p : Tokenizer::llama3_pretokenize(text, max_digits > 0 ? max_digits : 3)) { g_str += p; g_str += '\x1f'; }
  return g_str.c_str();
  API_CATCH(nullptr)
}

// ------------------------------------------------------------------ engine
void* mp_engine_create(const char* json_cfg) {
  API_TRY
  return new Engine(Json::parse(json_cfg));
  API_CATCH(nullptr)
}
void mp_engine_destroy(void* h) {
  try { delete static_cast<Engine*>(h); } catch (...) {}
}
const char* mp_engine_info(void* h) {
  API_TRY
  g_str = static_cast<Engine*>(h)->info().dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
const char* mp_engine_health(void* h) {
  API_TRY
  g_str = static_cast<Engine*>(h)->health().dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
// checkpoint / resume (Engine::save_state / load_state); returns a JSON summary
const char* mp_engine_save_state(void* h, const char* dir) {
  API_TRY
  g_str = static_cast<Engine*>(h)->save_state(dir).dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
const char* mp_engine_load_state(void* h, const char* dir) {
  API_TRY
  g_str = static_cast<Engine*>(h)->load_state(dir).dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
int mp_engine_trace(void* h, int on, const char* path) {
  API_TRY
  Engine* e = static_cast<Engine*>(h);
  if (path && *path) e->write_trace(path);
  else e->enable_trace(on != 0);
  return 0;
  API_CATCH(-1)
}
// Generate for a batch of prompts. prompts: concatenated token ids, lens[n]. out: [n][n_predict]
// returns JSON stats string
const char* mp_engine_generate(void* h, const int32_t* prompt_tokens, const int32_t* lens, int n_seq, int n_predict,
                               int32_t* out_tokens) {
  API_TRY
  std::vector<std::vector<int32_t>> prompts;
  size_t off = 0;
  for (int i = 0; i < n_seq; ++i) {
    prompts.emplace_back(prompt_tokens + off, prompt_tokens + off + lens[i]);
    off += lens[i];
  }
  std::vector<std::vector<int32_t>> outs;
  Json stats = static_cast<Engine*>(h)->generate(prompts, n_predict, &outs);
  for (int i = 0; i < n_seq; ++i)
    for (int j = 0; j < n_predict; ++j) out_tokens[(size_t)i * n_predict + j] = j < (int)outs[i].size() ? outs[i][j] : -1;
  g_str = stats.dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
// Speculative (prompt-lookup) greedy generation: same layout as mp_engine_generate; draft_max tokens
// drafted per sequence per verify round from its last ngram-gram.  Returns JSON stats.
const char* mp_engine_spec_generate(void* h, const int32_t* prompt_tokens, const int32_t* lens, int n_seq,
                                    int n_predict, int draft_max, int ngram, int32_t* out_tokens) {
  API_TRY
  std::vector<std::vector<int32_t>> prompts;
  size_t off = 0;
  for (int i = 0; i < n_seq; ++i) {
    prompts.emplace_back(prompt_tokens + off, prompt_tokens + off + lens[i]);
    off += lens[i];
  }
  std::vector<std::vector<int32_t>> outs;
  Json stats = static_cast<Engine*>(h)->spec_generate(prompts, n_predict, draft_max, ngram, &outs);
  for (int i = 0; i < n_seq; ++i)
    for (int j = 0; j < n_predict; ++j) out_tokens[(size_t)i * n_predict + j] = j < (int)outs[i].size() ? outs[i][j] : -1;
  g_str = stats.dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
// Benchmark decode loop: n_warmup + n_steps decode steps of every micro-batch after a prefill of
// prompt_len synthetic tokens. Returns JSON stats.
const char* mp_engine_bench(void* h, int prompt_len, int n_warmup, int n_steps) {
  API_TRY
  g_str = static_cast<Engine*>(h)->bench(prompt_len, n_warmup, n_steps).dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
// fine-grained control (bench.py drives the timed region itself)
int mp_engine_start(void* h, const int32_t* prompt_tokens, const int32_t* lens, int n_seq) {
  API_TRY
  std::vector<std::vector<int32_t>> prompts;
  size_t off = 0;
  for (int i = 0; i < n_seq; ++i) {
    prompts.emplace_back(prompt_tokens + off, prompt_tokens + off + lens[i]);
    off += lens[i];
  }
  static_cast<Engine*>(h)->start(prompts);
  return 0;
  API_CATCH(-1)
}
// continuous batching: prefill prompts into the given sequence slots between decode rounds
int mp_engine_admit(void* h, const int32_t* slots, const int32_t* prompt_tokens, const int32_t* lens, int n_seq) {
  API_TRY
  std::vector<std::vector<int32_t>> prompts;
  std::vector<int> sl;
  size_t off = 0;
  for (int i = 0; i < n_seq; ++i) {
    prompts.emplace_back(prompt_tokens + off, prompt_tokens + off + lens[i]);
    off += lens[i];
    sl.push_back(slots[i]);
  }
  static_cast<Engine*>(h)->admit(sl, prompts);
  return 0;
  API_CATCH(-1)
}
int mp_engine_release(void* h, int slot) {
  API_TRY
  static_cast<Engine*>(h)->release(slot);
  return 0;
  API_CATCH(-1)
}
const char* mp_engine_decode(void* h, int k) {
  API_TRY
  StepStats ss = static_cast<Engine*>(h)->decode_steps(k);
  Json j = Json::object();
  j["wall_ms"] = ss.wall_ms;
  Json a = Json::array();
  for (double v : ss.token_ms) a.push(Json(v));
  j["token_ms"] = a;
  g_str = j.dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
// copy generated tokens: out[n_seq][cap]; returns tokens per sequence (min over sequences)
int mp_engine_tokens(void* h, int32_t* out, int n_seq, int cap) {
  API_TRY
  auto t = static_cast<Engine*>(h)->tokens();
  int n = 0;   // longest sequence (rows padded with -1: admitted sequences are shorter)
  for (int i = 0; i < n_seq && i < (int)t.size(); ++i) {
    n = std::max<int>(n, std::min<int>(cap, (int)t[i].size()));
    for (int j = 0; j < cap; ++j) out[(size_t)i * cap + j] = j < (int)t[i].size() ? t[i][j] : -1;
  }
  return n;
  API_CATCH(-1)
}
// debug: logits of the last decode/prefill of a micro-batch (last stage, rank-local)
int mp_engine_logits(void* h, int mb, float* out, int rows) {
  API_TRY
  return static_cast<Engine*>(h)->copy_logits(mb, out, rows);
  API_CATCH(-1)
}
// stage partitioner (model.cpp) on its own: {"layer_cost": [...], "first_extra", "last_extra",
// "device_speed": [...] (one per stage), "split": "even"|"mem"|"cost"} -> [[begin, end], ...]
const char* mp_plan_partition(const char* cfg) {
  API_TRY
  const Json j = Json::parse(cfg);
  std::vector<double> cost, speed;
  for (const Json& v : j["layer_cost"].arr()) cost.push_back(v.num());
  for (const Json& v : j["device_speed"].arr()) speed.push_back(v.num());
  const auto specs = partition_layers(cost, j.get_num("first_extra", 0.0), j.get_num("last_extra", 0.0), speed,
                                      parse_split_mode(j.get_str("split", "cost")));
  Json out = Json::array();
  for (const auto& s : specs) {
    Json r = Json::array();
    r.push(s.layer_begin);
    r.push(s.layer_end);
    out.push(r);
  }
  g_str = out.dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}
// multi-process rendezvous helpers: unique id bytes for RCCL
// Halda-style device profile (probe.h): out[0] HBM read GB/s, out[1] Q4_K decode GEMV GB/s;
// device < 0: the host (CPU backend)
int mp_device_probe(int device, double* out2) {
  API_TRY
  const DeviceProfile d = device < 0 ? probe_host() : probe_device(device);
  out2[0] = d.hbm_read_gbps;
  out2[1] = d.gemv_gbps;
  return 0;
  API_CATCH(-1)
}

int mp_rccl_unique_id(uint8_t* out128) {
  API_TRY
  return rccl_unique_id(out128);
  API_CATCH(-1)
}

// RCCL transport self-test (ws = 1): a 1-rank communicator on `device` and the
// engine's RcclLink looping every size in `sizes` back to itself (grouped ncclSend/ncclRecv on one
// stream), `iters` times each, checking every byte.  Returns a JSON report.
// LocalLink posted-queue self-test on one device: a sender thread cycles n_bufs buffers (message i
// filled with the value i + 1, each buffer reused only after Link::wait_consumed of its previous
// message) while a receiver thread takes the messages with recv_delay_us of host delay before each
// (a slow receiver: the sender runs ahead until the kDepth queue pushes back).  Returns the number of
// received words that do not hold their message's value (0: ordered, no buffer reused too early),
// or -1 on an error.
int mp_local_link_selftest(int device, int n_msgs, int64_t bytes, int n_bufs, int recv_delay_us) {
  API_TRY
  HIP_OK(hipSetDevice(device));
  if (n_msgs <= 0 || n_bufs <= 0 || bytes < 4 || bytes % 4) throw std::runtime_error("selftest: bad arguments");
  LocalLink link(device, device);
  link.set_timeout(60);
  std::vector<void*> bufs(n_bufs);
  for (auto& b : bufs) HIP_OK(hipMalloc(&b, bytes));
  void* rb = nullptr;
  HIP_OK(hipMalloc(&rb, bytes));
  hipStream_t ss, rs;
  HIP_OK(hipStreamCreateWithFlags(&ss, hipStreamNonBlocking));
  HIP_OK(hipStreamCreateWithFlags(&rs, hipStreamNonBlocking));
  std::atomic<int> bad{0};
  std::string err;
  std::mutex emu;
  std::thread snd([&] {
    try {
      HIP_OK(hipSetDevice(device));
      std::vector<uint64_t> seq(n_bufs, 0);
      for (int i = 0; i < n_msgs; ++i) {
        const int k = i % n_bufs;
        link.wait_consumed(seq[k], ss);   // the buffer's previous message has left it
        HIP_OK(hipMemsetD32Async((hipDeviceptr_t)bufs[k], i + 1, bytes / 4, ss));
        link.send(bufs[k], bytes, ss);
        seq[k] = link.last_seq();
      }
      HIP_OK(hipStreamSynchronize(ss));
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> l(emu);
      err = e.what();
      link.abort();
    }
  });
  std::thread rcv([&] {
    try {
      HIP_OK(hipSetDevice(device));
      std::vector<int32_t> h(bytes / 4);
      for (int i = 0; i < n_msgs; ++i) {
        if (recv_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(recv_delay_us));
        link.recv(rb, bytes, rs);
        HIP_OK(hipMemcpyAsync(h.data(), rb, bytes, hipMemcpyDeviceToHost, rs));
        HIP_OK(hipStreamSynchronize(rs));
        for (int32_t v : h) bad += v != i + 1;
      }
    } catch (const std::exception& e) {
      std::lock_guard<std::mutex> l(emu);
      err = e.what();
      link.abort();
    }
  });
  snd.join();
  rcv.join();
  for (auto b : bufs) (void)hipFree(b);
  (void)hipFree(rb);
  (void)hipStreamDestroy(ss);
  (void)hipStreamDestroy(rs);
  if (!err.empty()) throw std::runtime_error("local link selftest: " + err);
  return bad.load();
  API_CATCH(-1)
}

const char* mp_rccl_selftest(int device, const int64_t* sizes, int n_sizes, int iters) {
  API_TRY
  HIP_OK(hipSetDevice(device));
  std::vector<void*> comms;
  std::string err;
  if (!rccl_init_all({device}, &comms, &err)) throw std::runtime_error("RCCL init failed: " + err);
  RcclLink link(comms[0], 0, 0, device);
  hipStream_t st;
  HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  Json rep = Json::object();
  rep["rccl_version"] = std::string(rccl_version_string());
  Json res = Json::array();
  int64_t maxb = 0;
  for (int i = 0; i < n_sizes; ++i) maxb = std::max<int64_t>(maxb, sizes[i]);
  void *src = nullptr, *dst = nullptr;
  HIP_OK(hipMalloc(&src, std::max<int64_t>(maxb, 16)));
  HIP_OK(hipMalloc(&dst, std::max<int64_t>(maxb, 16)));
  std::vector<uint8_t> h(maxb), back(maxb);
  bool ok = true;
  for (int i = 0; i < n_sizes; ++i) {
    const size_t b = (size_t)sizes[i];
    double ms = 0;
    for (int it = 0; it < iters; ++it) {
      for (size_t k = 0; k < b; ++k) h[k] = (uint8_t)((k * 131 + it * 7 + i) & 0xFF);
      HIP_OK(hipMemcpy(src, h.data(), b, hipMemcpyHostToDevice));
      HIP_OK(hipMemset(dst, 0, b));
      const auto t0 = std::chrono::steady_clock::now();
      rccl_group_begin();
      link.send(src, b, st);
      link.recv(dst, b, st);
      rccl_group_end();
      HIP_OK(hipStreamSynchronize(st));
      ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      HIP_OK(hipMemcpy(back.data(), dst, b, hipMemcpyDeviceToHost));
      if (std::memcmp(back.data(), h.data(), b) != 0) ok = false;
    }
    Json r = Json::object();
    r["bytes"] = (double)b;
    r["avg_ms"] = ms / std::max(1, iters);
    res.push(r);
  }
  rep["results"] = res;
  rep["ok"] = ok;
  rep["bytes_sent"] = (double)link.bytes_sent;
  rep["msgs_sent"] = (double)link.msgs_sent;
  (void)hipFree(src);
  (void)hipFree(dst);
  (void)hipStreamDestroy(st);
  g_str = rep.dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}

// RCCL / compute CU-sharing proxy (1 rank): enqueue `iters` grouped self send/recv of `bytes` on a
// side stream of `device` and return at once; the caller times its GEMMs on its own stream while
// the RCCL kernels run, then mp_rccl_loop_wait reports the loop's wall time.  A 1-rank stand-in for
// a pipeline stage whose activation send/recv shares the CUs with the next micro-batch's GEMMs
// (tools/rccl_overlap_probe.py).
namespace {
struct RcclLoop {
  void* comm = nullptr;
  RcclLink* link = nullptr;
  hipStream_t st = nullptr;
  void *src = nullptr, *dst = nullptr;
  size_t cap = 0;
  hipEvent_t a = nullptr, b = nullptr;
  int device = -1;
};
RcclLoop g_loop;
}  // namespace

int mp_rccl_loop_start(int device, int64_t bytes, int iters) {
  API_TRY
  HIP_OK(hipSetDevice(device));
  if (g_loop.device != device) {
    std::vector<void*> comms;
    std::string err;
    if (!rccl_init_all({device}, &comms, &err)) throw std::runtime_error("RCCL init failed: " + err);
    g_loop.comm = comms[0];
    g_loop.link = new RcclLink(g_loop.comm, 0, 0, device);
    HIP_OK(hipStreamCreateWithFlags(&g_loop.st, hipStreamNonBlocking));
    HIP_OK(hipEventCreate(&g_loop.a));
    HIP_OK(hipEventCreate(&g_loop.b));
    g_loop.device = device;
  }
  if ((size_t)bytes > g_loop.cap) {
    if (g_loop.src) (void)hipFree(g_loop.src);
    if (g_loop.dst) (void)hipFree(g_loop.dst);
    HIP_OK(hipMalloc(&g_loop.src, (size_t)bytes));
    HIP_OK(hipMalloc(&g_loop.dst, (size_t)bytes));
    HIP_OK(hipMemset(g_loop.src, 0x3c, (size_t)bytes));
    g_loop.cap = (size_t)bytes;
  }
  HIP_OK(hipEventRecord(g_loop.a, g_loop.st));
  for (int i = 0; i < iters; ++i) {
    rccl_group_begin();
    g_loop.link->send(g_loop.src, (size_t)bytes, g_loop.st);
    g_loop.link->recv(g_loop.dst, (size_t)bytes, g_loop.st);
    rccl_group_end();
  }
  HIP_OK(hipEventRecord(g_loop.b, g_loop.st));
  return 0;
  API_CATCH(-1)
}

double mp_rccl_loop_wait() {
  API_TRY
  if (g_loop.device < 0) throw std::runtime_error("mp_rccl_loop_wait: no loop started");
  HIP_OK(hipSetDevice(g_loop.device));
  HIP_OK(hipEventSynchronize(g_loop.b));
  float ms = 0;
  HIP_OK(hipEventElapsedTime(&ms, g_loop.a, g_loop.b));
  return ms;
  API_CATCH(-1.0)
}

// can RCCL put `n` ranks of one communicator on these devices (e.g. the same GPU twice)?
const char* mp_rccl_probe_devices(const int* devices, int n) {
  API_TRY
  std::vector<void*> comms;
  std::string err;
  const bool ok = rccl_init_all(std::vector<int>(devices, devices + n), &comms, &err);
  for (void* c : comms) rccl_comm_destroy(c);
  Json r = Json::object();
  r["ok"] = ok;
  r["error"] = err;
  g_str = r.dump();
  return g_str.c_str();
  API_CATCH(nullptr)
}

}  // extern "C"
