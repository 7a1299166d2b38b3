#include "hip_stage.h"

#include <functional>
#include "tuning.h"

#include <chrono>
#include <cstring>

#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "gguf.h"
#include "log.h"
#include "pack.h"

namespace mp {

void launch_prefill_meta(int32_t* pos, int32_t* kvlen, int32_t* slot, int p0, int T, int s, hipStream_t st);

SyntheticTypes SyntheticTypes::from_ftype(const std::string& ftype_in, int layer, int n_layer) {
  std::string f = ftype_in;
  for (auto& c : f) c = (char)toupper(c);
  SyntheticTypes t;
  auto all = [&](int ty) { t.embd = t.q = t.k = t.v = t.o = t.gate = t.up = t.down = t.out = ty; };
  auto more_bits = [&](int i, int n) { return i < n / 8 || i >= 7 * n / 8 || (i - n / 8) % 3 == 2; };
  if (f == "F16") all(T_F16);
  else if (f == "BF16") all(T_BF16);
  else if (f == "F32") all(T_F32);
  else if (f == "Q8_0") all(T_Q8_0);
  else if (f == "Q6_K") all(T_Q6_K);
  else if (f == "Q5_K" || f == "Q5_K_M") { all(T_Q5_K); t.out = T_Q6_K; }
  else if (f == "Q4_0") all(T_Q4_0);
  else if (f == "Q4_K" || f == "Q4_K_S") { all(T_Q4_K); t.out = T_Q6_K; }
  else if (f == "Q4_K_M") {
    all(T_Q4_K);
    t.out = T_Q6_K;
    if (more_bits(layer, n_layer)) { t.v = T_Q6_K; t.down = T_Q6_K; }
  } else throw std::runtime_error("unknown synthetic ftype " + ftype_in);
  if (f == "Q5_K_M" && more_bits(layer, n_layer)) { t.v = T_Q6_K; t.down = T_Q6_K; }
  return t;
}

HipStage::HipStage(const ModelConfig& cfg, const StageSpec& spec, const StageOptions& opt)
    : cfg_(cfg), spec_(spec), opt_(opt) {
  HIP_OK(hipSetDevice(spec_.device));
  HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  if (opt_.max_ctx % 64) opt_.max_ctx = (int)round_up(opt_.max_ctx, 64);
  if (opt_.prefill_chunk < 1) opt_.prefill_chunk = 1;
  layers_.resize(spec_.layer_end - spec_.layer_begin);
  Dp_ = cfg_.padded_head_dim();
  Kd_ = (int)round_up(cfg_.d_model, 256);
  Ko_ = (int)round_up(cfg_.q_dim(), 256);
  Kff_ = (int)round_up(cfg_.d_ff, 256);
  qkv_n_ = cfg_.q_dim() + 2 * cfg_.kv_dim();
}

HipStage::~HipStage() {
  (void)hipSetDevice(spec_.device);
  destroy_graphs();
  for (void* p : allocs_) (void)hipFree(p);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void* HipStage::dmalloc(size_t bytes) {
  void* p = nullptr;
  HIP_OK(hipMalloc(&p, std::max<size_t>(bytes, 256)));
  allocs_.push_back(p);
  return p;
}

float* HipStage::upload_f32(const float* h, size_t n) {
  float* d = (float*)dmalloc(n * sizeof(float));
  HIP_OK(hipMemcpy(d, h, n * sizeof(float), hipMemcpyHostToDevice));
  weight_bytes_ += n * sizeof(float);
  return d;
}

// ---- weight upload (load_gguf): T16 packing on host threads into pinned double-buffered staging,
// hipMemcpyAsync on a dedicated stream, so packing piece i+1 overlaps the DMA of piece i (v1
// packed into pageable memory and then blocked in a synchronous hipMemcpy per tensor)
void HipStage::stage_begin() {
  if (stg_.buf[0]) return;
  stg_.cap = (size_t)256 << 20;
  for (int b = 0; b < 2; ++b) {
    HIP_OK(hipHostMalloc((void**)&stg_.buf[b], stg_.cap, hipHostMallocDefault));
    HIP_OK(hipEventCreateWithFlags(&stg_.ev[b], hipEventDisableTiming));
    stg_.busy[b] = false;
  }
  HIP_OK(hipStreamCreateWithFlags(&stg_.st, hipStreamNonBlocking));
  stg_.cur = 0;
  stg_.bytes = 0;
  stg_.t0 = std::chrono::steady_clock::now();
}

void HipStage::stage_end() {
  if (!stg_.buf[0]) return;
  HIP_OK(hipStreamSynchronize(stg_.st));
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - stg_.t0).count();
  upload_gbps_ = s > 0 ? stg_.bytes / s / 1e9 : 0.0;
  MP_LOGI("stage %d: uploaded %.2f GiB of packed weights in %.2f s (%.2f GB/s incl. packing)", spec_.stage,
          stg_.bytes / 1073741824.0, s, upload_gbps_);
  for (int b = 0; b < 2; ++b) {
    HIP_OK(hipEventDestroy(stg_.ev[b]));
    HIP_OK(hipHostFree(stg_.buf[b]));
    stg_.buf[b] = nullptr;
  }
  HIP_OK(hipStreamDestroy(stg_.st));
  stg_.st = nullptr;
}

// dst[0, bytes) <- fill(host, off, n) piece by piece through the staging buffers
void HipStage::stage_put(uint8_t* dst, size_t bytes, size_t granule,
                         const std::function<void(uint8_t*, size_t, size_t)>& fill) {
  const bool own = !stg_.buf[0];
  if (own) stage_begin();
  const size_t piece = std::max(granule, stg_.cap / granule * granule);
  if (piece > stg_.cap) throw std::runtime_error("stage_put: granule larger than the staging buffer");
  for (size_t off = 0; off < bytes; off += piece) {
    const size_t n = std::min(piece, bytes - off);
    const int b = stg_.cur;
    if (stg_.busy[b]) HIP_OK(hipEventSynchronize(stg_.ev[b]));   // its previous DMA has drained
    fill(stg_.buf[b], off, n);
    HIP_OK(hipMemcpyAsync(dst + off, stg_.buf[b], n, hipMemcpyHostToDevice, stg_.st));
    HIP_OK(hipEventRecord(stg_.ev[b], stg_.st));
    stg_.busy[b] = true;
    stg_.cur ^= 1;
    stg_.bytes += n;
  }
  if (own) stage_end();
}

PackedMat HipStage::upload_packed(int t, int64_t N, int64_t K, const std::function<const uint8_t*(int64_t)>& row) {
  PackedMat m;
  m.ptype = pack_type_of(t);
  if (m.ptype < 0) throw std::runtime_error(std::string("unsupported weight type ") + type_name(t));
  m.dims = packed_dims(m.ptype, N, K);
  m.d = (uint8_t*)dmalloc(m.dims.bytes);
  const size_t tile_b = (size_t)m.dims.nsb * chunk_bytes(m.ptype);
  stage_put(m.d, m.dims.bytes, tile_b, [&](uint8_t* h, size_t off, size_t n) {
    pack_t16_tiles(t, N, K, row, h, (int64_t)(off / tile_b), (int64_t)((off + n) / tile_b));
  });
  weight_bytes_ += m.dims.bytes;
  return m;
}

PackedMat HipStage::upload_packed_experts(int t, int E, int64_t N, int64_t K, size_t* stride,
                                          const std::function<const uint8_t*(int, int64_t)>& row) {
  PackedMat m;
  m.ptype = pack_type_of(t);
  if (m.ptype < 0) throw std::runtime_error(std::string("unsupported expert type ") + type_name(t));
  m.dims = packed_dims(m.ptype, N, K);
  *stride = m.dims.bytes;
  m.d = (uint8_t*)dmalloc(m.dims.bytes * E);
  const size_t tile_b = (size_t)m.dims.nsb * chunk_bytes(m.ptype);
  for (int e = 0; e < E; ++e)
    stage_put(m.d + (size_t)e * m.dims.bytes, m.dims.bytes, tile_b, [&](uint8_t* h, size_t off, size_t n) {
      pack_t16_tiles(t, N, K, [&](int64_t r) { return row(e, r); }, h, (int64_t)(off / tile_b),
                     (int64_t)((off + n) / tile_b));
    });
  weight_bytes_ += m.dims.bytes * E;
  return m;
}

PackedMat HipStage::alloc_packed_random(int t, int64_t N, int64_t K, uint64_t seed) {
  PackedMat m;
  m.ptype = pack_type_of(t);
  m.dims = packed_dims(m.ptype, N, K);
  m.d = (uint8_t*)dmalloc(m.dims.bytes);
  launch_init_packed(m.d, m.dims.bytes, m.ptype, 1.0f / std::sqrt((float)K), seed, stream_);
  weight_bytes_ += m.dims.bytes;
  return m;
}

static std::vector<float> tensor_f32(const GgufTensor& t) {
  std::vector<float> v(t.nelem());
  const int64_t K = t.ne[0];
  const size_t rb = row_bytes(t.type, K);
  for (int64_t r = 0; r < t.nelem() / K; ++r) dequant_row(t.type, t.data + r * rb, v.data() + r * K, K);
  return v;
}

void HipStage::load_gguf(const GgufFile& f) {
  HIP_OK(hipSetDevice(spec_.device));
  stage_begin();
  auto need = [&](const std::string& n) -> const GgufTensor& {
    const GgufTensor* t = f.tensor(n);
    if (!t) throw std::runtime_error("missing tensor " + n);
    return *t;
  };
  auto rows_of = [](const GgufTensor& t) {
    const size_t rb = row_bytes(t.type, t.ne[0]);
    return [&t, rb](int64_t n) -> const uint8_t* { return t.data + n * rb; };
  };
  auto pack_mat = [&](const GgufTensor& t) { return upload_packed(t.type, t.ne[1], t.ne[0], rows_of(t)); };

  for (int li = spec_.layer_begin; li < spec_.layer_end; ++li) {
    LayerW& L = layers_[li - spec_.layer_begin];
    const std::string p = "blk." + std::to_string(li) + ".";
    {
      auto v = tensor_f32(need(p + "attn_norm.weight"));
      L.attn_norm = upload_f32(v.data(), v.size());
      auto w = tensor_f32(need(p + "ffn_norm.weight"));
      L.ffn_norm = upload_f32(w.data(), w.size());
    }
    const GgufTensor& tq = need(p + "attn_q.weight");
    const GgufTensor& tk = need(p + "attn_k.weight");
    const GgufTensor& tv = need(p + "attn_v.weight");
    // merge same-type q/k/v into one launch (tile-major layout concatenates)
    const GgufTensor* qkv[3] = {&tq, &tk, &tv};
    int off = 0;
    for (int i = 0; i < 3;) {
      int j = i + 1;
      while (j < 3 && pack_type_of(qkv[j]->type) == pack_type_of(qkv[i]->type) && qkv[j - 1]->ne[1] % 16 == 0 &&
             qkv[j]->type == qkv[i]->type)
        ++j;
      int64_t N = 0;
      std::vector<std::pair<const GgufTensor*, int64_t>> parts;
      for (int k = i; k < j; ++k) { parts.push_back({qkv[k], N}); N += qkv[k]->ne[1]; }
      const bool neox = cfg_.rope_neox;
      const int hd = cfg_.head_dim;
      auto rowfn = [&parts, &tq, &tk, neox, hd](int64_t n) -> const uint8_t* {
        for (auto it = parts.rbegin(); it != parts.rend(); ++it)
          if (n >= it->second) {
            const GgufTensor* t = it->first;
            int64_t r = n - it->second;
            if (neox && (t == &tq || t == &tk)) r = neox_src_row(r, hd);
            return t->data + r * row_bytes(t->type, t->ne[0]);
          }
        return nullptr;
      };
      MatSeg s;
      s.m = upload_packed(qkv[i]->type, N, qkv[i]->ne[0], rowfn);
      s.y_off = off;
      off += (int)N;
      L.qkv.push_back(s);
      i = j;
    }
    if (cfg_.qkv_bias) {
      std::vector<float> b(qkv_n_, 0.f);
      const char* nm[3] = {"attn_q.bias", "attn_k.bias", "attn_v.bias"};
      const int o[3] = {0, cfg_.q_dim(), cfg_.q_dim() + cfg_.kv_dim()};
      for (int i = 0; i < 3; ++i) {
        const std::vector<float> v = tensor_f32(need(p + nm[i]));
        for (size_t r = 0; r < v.size(); ++r)
          b[o[i] + r] = v[i < 2 && cfg_.rope_neox ? neox_src_row((long)r, cfg_.head_dim) : r];
      }
      L.qkv_bias = upload_f32(b.data(), b.size());
    }
    L.wo = pack_mat(need(p + "attn_output.weight"));
    if (cfg_.n_expert) {
      // Mixtral: router [E][d] + stacked experts (ffn_*_exps [E][F][d]) or legacy per-expert tensors
      L.moe = true;
      const int E = cfg_.n_expert;
      L.ex.router = pack_mat(need(p + "ffn_gate_inp.weight"));
      std::vector<const GgufTensor*> g(E), u(E), dn(E);
      const GgufTensor* sg = f.tensor(p + "ffn_gate_exps.weight");
      for (int e = 0; e < E; ++e) {
        if (sg) {
          g[e] = sg;
          u[e] = &need(p + "ffn_up_exps.weight");
          dn[e] = &need(p + "ffn_down_exps.weight");
        } else {
          const std::string s = "." + std::to_string(e) + ".weight";
          g[e] = &need(p + "ffn_gate" + s);
          u[e] = &need(p + "ffn_up" + s);
          dn[e] = &need(p + "ffn_down" + s);
        }
      }
      if (g[0]->type != u[0]->type) throw std::runtime_error("MoE gate/up types differ");
      const int64_t F = cfg_.d_ff, D = cfg_.d_model;
      // row n of expert e of a (possibly stacked) tensor
      auto erow = [&](const GgufTensor* t, int e, int64_t n, int64_t rows) -> const uint8_t* {
        const size_t rb = row_bytes(t->type, t->ne[0]);
        return t->data + ((sg ? (size_t)e * rows : 0) + n) * rb;
      };
      L.ex.gateup = upload_packed_experts(g[0]->type, E, 2 * F, D, &L.ex.gateup_stride,
                                          [&](int e, int64_t n) -> const uint8_t* {
                                            bool up;
                                            const int64_t r = gateup_src_row(n, &up);
                                            if (r >= F) return nullptr;
                                            return erow(up ? u[e] : g[e], e, r, F);
                                          });
      L.ex.down = upload_packed_experts(dn[0]->type, E, D, F, &L.ex.down_stride,
                                        [&](int e, int64_t n) { return erow(dn[e], e, n, D); });
      continue;
    }
    const GgufTensor& tg = need(p + "ffn_gate.weight");
    const GgufTensor& tu = need(p + "ffn_up.weight");
    if (tg.type == tu.type && cfg_.d_ff % 8 == 0) {
      L.fused_gateup = true;
      const size_t rb = row_bytes(tg.type, tg.ne[0]);
      const int64_t F = tg.ne[1];
      L.gateup = upload_packed(tg.type, 2 * F, tg.ne[0], [&](int64_t n) -> const uint8_t* {
        bool up;
        const int64_t r = gateup_src_row(n, &up);
        if (r >= F) return nullptr;
        return (up ? tu.data : tg.data) + r * rb;
      });
    } else {
      L.fused_gateup = false;
      L.gate = pack_mat(tg);
      L.up = pack_mat(tu);
    }
    L.down = pack_mat(need(p + "ffn_down.weight"));
  }
  const GgufTensor& te = need("token_embd.weight");
  if (spec_.first()) {
    embd_type_ = te.type;
    embd_row_bytes_ = row_bytes(te.type, te.ne[0]);
    embd_raw_ = (uint8_t*)dmalloc(te.nbytes);
    stage_put(embd_raw_, te.nbytes, 1, [&](uint8_t* h, size_t off, size_t n) { std::memcpy(h, te.data + off, n); });
    weight_bytes_ += te.nbytes;
  }
  if (spec_.last()) {
    auto v = tensor_f32(need("output_norm.weight"));
    out_norm_ = upload_f32(v.data(), v.size());
    const GgufTensor* to = f.tensor("output.weight");
    out_ = pack_mat(to ? *to : te);
  }
  rope_ff_.clear();
  if (const GgufTensor* rf = f.tensor("rope_freqs.weight")) rope_ff_ = tensor_f32(*rf);
  stage_end();
  HIP_OK(hipDeviceSynchronize());
}

void HipStage::init_synthetic(const std::string& ftype, uint64_t seed) {
  HIP_OK(hipSetDevice(spec_.device));
  const int d = cfg_.d_model, qd = cfg_.q_dim(), kvd = cfg_.kv_dim(), F = cfg_.d_ff;
  std::vector<float> ones(std::max(d, 1), 1.0f);
  for (int li = spec_.layer_begin; li < spec_.layer_end; ++li) {
    LayerW& L = layers_[li - spec_.layer_begin];
    const SyntheticTypes t = SyntheticTypes::from_ftype(ftype, li, cfg_.n_layer);
    const uint64_t s = seed * 1000003ULL + (uint64_t)li * 97;
    L.attn_norm = upload_f32(ones.data(), d);
    L.ffn_norm = upload_f32(ones.data(), d);
    int off = 0;
    if (t.q == t.k && t.k == t.v) {
      L.qkv.push_back({alloc_packed_random(t.q, qd + 2 * kvd, d, s + 1), 0});
    } else if (t.q == t.k) {
      L.qkv.push_back({alloc_packed_random(t.q, qd + kvd, d, s + 1), 0});
      L.qkv.push_back({alloc_packed_random(t.v, kvd, d, s + 2), qd + kvd});
    } else {
      L.qkv.push_back({alloc_packed_random(t.q, qd, d, s + 1), off});
      L.qkv.push_back({alloc_packed_random(t.k, kvd, d, s + 2), qd});
      L.qkv.push_back({alloc_packed_random(t.v, kvd, d, s + 3), qd + kvd});
    }
    L.wo = alloc_packed_random(t.o, d, qd, s + 4);
    if (cfg_.n_expert) {
      const int E = cfg_.n_expert;
      L.moe = true;
      L.ex.router = alloc_packed_random(T_F16, E, d, s + 7);
      auto experts = [&](int ty, int64_t N, int64_t K, size_t* stride, uint64_t sd) {
        PackedMat m;
        m.ptype = pack_type_of(ty);
        m.dims = packed_dims(m.ptype, N, K);
        *stride = m.dims.bytes;
        m.d = (uint8_t*)dmalloc(m.dims.bytes * E);
        launch_init_packed(m.d, m.dims.bytes * E, m.ptype, 1.0f / std::sqrt((float)K), sd, stream_);
        weight_bytes_ += m.dims.bytes * E;
        return m;
      };
      L.ex.gateup = experts(t.gate, 2 * F, d, &L.ex.gateup_stride, s + 5);
      L.ex.down = experts(t.down, d, F, &L.ex.down_stride, s + 6);
      continue;
    }
    L.fused_gateup = true;
    L.gateup = alloc_packed_random(t.gate, 2 * F, d, s + 5);
    L.down = alloc_packed_random(t.down, d, F, s + 6);
  }
  const SyntheticTypes t0 = SyntheticTypes::from_ftype(ftype, 0, cfg_.n_layer);
  if (spec_.first()) {
    embd_type_ = t0.embd;
    embd_row_bytes_ = row_bytes(embd_type_, d);
    const size_t nb = embd_row_bytes_ * (size_t)cfg_.vocab;
    embd_raw_ = (uint8_t*)dmalloc(nb);
    launch_init_raw(embd_raw_, (int64_t)(nb / block_bytes(embd_type_)), embd_type_, 1.0f, seed ^ 0xE3BD, stream_);
    weight_bytes_ += nb;
  }
  if (spec_.last()) {
    out_norm_ = upload_f32(ones.data(), d);
    out_ = alloc_packed_random(t0.out, cfg_.vocab, d, seed ^ 0x0F7);
  }
  HIP_OK(hipStreamSynchronize(stream_));
}

// int8_gemm: an int8 copy of every quantized projection (K15; the wide GEMMs then run gemm3<P_I8>):
// each matrix is unpacked to dense f16 in a temporary buffer and re-quantized per row
void HipStage::build_i8_copies() {
  auto each = [&](const std::function<void(PackedMat&)>& f) {
    for (LayerW& L : layers_) {
      if (L.moe) continue;
      for (MatSeg& sg : L.qkv) f(sg.m);
      f(L.wo);
      if (L.fused_gateup) f(L.gateup);
      else { f(L.gate); f(L.up); }
      f(L.down);
    }
  };
  size_t maxe = 0;
  each([&](PackedMat& m) {
    if (m.d && !is16(m.ptype)) maxe = std::max(maxe, (size_t)m.dims.ntiles * 16 * m.dims.nsb * 256);
  });
  if (!maxe) return;
  f16* tmp = nullptr;
  HIP_OK(hipMalloc(&tmp, maxe * 2));
  size_t bytes = 0;
  each([&](PackedMat& m) {
    if (!m.d || is16(m.ptype)) return;
    const int nt = (int)m.dims.ntiles, nsb = (int)m.dims.nsb;
    launch_unpack(m.ptype, m.d, nt, nsb, tmp, nsb * 256, stream_);
    m.i8 = (uint8_t*)dmalloc((size_t)nt * nsb * 4096);
    m.i8_ws = (float*)dmalloc((size_t)nt * 16 * 4);
    launch_requant_i8(tmp, nsb * 256, (int)m.dims.N, nt * 16, nsb, m.i8, m.i8_ws, stream_);
    bytes += (size_t)nt * nsb * 4096;
  });
  HIP_OK(hipStreamSynchronize(stream_));
  HIP_OK(hipFree(tmp));
  weight_bytes_ += bytes;
  MP_LOGI("stage %d: int8_gemm: %.2f GiB of per-row int8 weight copies", spec_.stage, bytes / 1073741824.0);
}

void HipStage::alloc_runtime() {
  HIP_OK(hipSetDevice(spec_.device));
  if (opt_.int8_gemm && opt_.prefill_gemm) build_i8_copies();
  // MoE routers as dense f16 (E x d x 2 B per layer: 64 KB at Mixtral): the router-logits kernel
  // reads them row-major, one launch of M / 4 workgroups for any micro-batch width
  for (LayerW& L : layers_) {
    if (!L.moe || !L.ex.router.d) continue;
    const PackedMat& r = L.ex.router;
    const size_t bytes = (size_t)r.dims.ntiles * 16 * r.dims.nsb * 256 * 2;
    L.ex.router_dense = (f16*)dmalloc(bytes);
    launch_unpack(r.ptype, r.d, (int)r.dims.ntiles, (int)r.dims.nsb, L.ex.router_dense, (int)r.dims.nsb * 256, stream_);
    weight_bytes_ += bytes;
  }
  HIP_OK(hipStreamSynchronize(stream_));
  const int B = opt_.mb_size, NM = opt_.n_mb;
  const int d = cfg_.d_model, Hq = cfg_.n_head, Hkv = cfg_.n_head_kv;
  scratch_rows_ = std::max(B, opt_.prefill_chunk);
  act_rows_ = scratch_rows_;
  auto zalloc = [&](size_t bytes) {
    void* p = dmalloc(bytes);
    HIP_OK(hipMemset(p, 0, bytes));
    return p;
  };
  xn_ = (f16*)zalloc((size_t)scratch_rows_ * Kd_ * 2);
  if (opt_.int8_gemm && opt_.prefill_gemm && std::max(B, opt_.prefill_chunk) > 64) {
    xq_ld_ = std::max({Kd_, Ko_, Kff_});
    xq_ = (int8_t*)zalloc((size_t)scratch_rows_ * xq_ld_);
    xqs_ = (float*)zalloc((size_t)scratch_rows_ * 4);
  }
  attn_ = (f16*)zalloc((size_t)scratch_rows_ * Ko_ * 2);
  h_ = (f16*)zalloc((size_t)scratch_rows_ * Kff_ * 2);
  // [64 floats: per-row sum of squares of the deferred qkv RMSNorm][rows][q|k|v] f32 split-K
  // accumulator; one contiguous range so the o-proj's zero side job clears both
  ssq_ = (float*)zalloc((64 + (size_t)scratch_rows_ * qkv_n_) * 4);
  qkv_ = ssq_ + 64;
  q_ = (f16*)zalloc((size_t)scratch_rows_ * Hq * Dp_ * 2);
  bool any_unfused = false;
  for (auto& L : layers_) any_unfused |= !L.fused_gateup;
  if (any_unfused) gu_ = (float*)zalloc((size_t)scratch_rows_ * 2 * cfg_.d_ff * 4);
  if (cfg_.n_expert) {
    if (cfg_.n_expert > 64 || cfg_.n_expert_used > 8 || cfg_.n_expert_used < 1)
      throw std::runtime_error("MoE: need n_expert <= 64 and 1 <= n_expert_used <= 8");
    const int k = cfg_.n_expert_used;
    moe_logits_ = (float*)zalloc((size_t)scratch_rows_ * 64 * 4);
    moe_counts_ = (int32_t*)zalloc(64 * 4);
    moe_lists_ = (int32_t*)zalloc((size_t)cfg_.n_expert * scratch_rows_ * k * 4);
    moe_w_ = (float*)zalloc((size_t)scratch_rows_ * k * 4);
    moe_h_ = (f16*)zalloc((size_t)scratch_rows_ * k * Kff_ * 2);
    if (opt_.deterministic) moe_yslot_ = (float*)zalloc((size_t)std::min(scratch_rows_, 64) * k * cfg_.d_model * 4);
  }
  if (spec_.last()) {
    logits_ld_ = (int)round_up(cfg_.vocab, 16);
    logits_ = (float*)zalloc((size_t)B * logits_ld_ * 4);
    am_.rows = std::max(B, opt_.prefill_chunk);
    am_.part = (float*)zalloc((size_t)am_.rows * kArgmaxChunks * 2 * 4);
    am_.counters = (int32_t*)zalloc((size_t)am_.rows * 4);
  }
  int split = opt_.attn_split_len;
  if (split <= 0) {
    // auto: enough (sequence, kv head, split) workgroups to cover the CUs, but >= 256 keys per
    // split (a split merge costs a publish/acquire round trip; short contexts use one split)
    const int target = knob(KNOB_ATTN_WG_TARGET);
    const int pairs = std::max(1, B * Hkv);
    const int want = std::max(1, std::min((target + pairs - 1) / pairs, (opt_.max_ctx + 255) / 256));
    split = (opt_.max_ctx + want - 1) / want;
  }
  split = std::max(128, (int)round_up(split, 128));
  // the fused decode attention merges at most 128 splits per (token, kv head) in LDS
  split = std::max(split, (int)round_up((opt_.max_ctx + 127) / 128, 128));
  opt_.attn_split_len = split;
  n_split_ = (int)((opt_.max_ctx + split - 1) / split);
  if (n_split_ > 1) {
    o_part_ = (float*)zalloc((size_t)n_split_ * B * Hq * Dp_ * 4);
    ml_part_ = (float*)zalloc((size_t)n_split_ * B * Hq * 2 * 4);
  }
  attn_cnt_ = (int32_t*)zalloc((size_t)std::max(B, 16) * Hkv * 4);
  if (opt_.prefill_flash && opt_.max_ctx > 256) {   // prefill KV-split partials (attn_prefill.hip)
    pf_opart_ = (float*)zalloc((size_t)kPrefillMaxSplit * opt_.prefill_chunk * Hq * Dp_ * 4);
    pf_ml_ = (float*)zalloc((size_t)kPrefillMaxSplit * opt_.prefill_chunk * Hq * 2 * 4);
  }
  if (opt_.gemm_splitk_store && opt_.prefill_gemm) {
    // split-K partials of the M > 64 GEMMs (decode micro-batches and prompt chunks wider than 64 rows)
    size_t need = 0;
    auto acc = [&](const PackedMat& m) {
      if (!m.d || is16(m.ptype)) return;
      for (int M : {opt_.mb_size, opt_.prefill_chunk}) {
        if (M <= 64) continue;
        const int ns = gemm4_splits(m.ptype, (int)m.dims.ntiles, (int)m.dims.nsb, M);
        if (ns > 1) need = std::max(need, (size_t)ns * M * m.dims.ntiles * 16);
      }
    };
    for (const LayerW& L : layers_) {
      for (const MatSeg& sg : L.qkv) acc(sg.m);
      acc(L.wo);
      acc(L.down);
    }
    if (need) sk_part_ = (float*)dmalloc(need * 4);
    sk_part_n_ = need;
  }
  if (opt_.deterministic) {
    // fixed-order split-K: the largest nsplit x rows x N of any ATOMIC GEMV call (<= 64 rows each)
    size_t need = 0;
    auto acc = [&](const PackedMat& m) {
      if (!m.d) return;
      for (int M : {1, 2, 3, 4, 8, 16, 32, 64}) {
        const int ns = det_splits((int)m.dims.ntiles, (int)m.dims.nsb, M, EPI_ATOMIC);
        if (ns > 1) need = std::max(need, (size_t)ns * M * m.dims.ntiles * 16);
      }
    };
    for (const LayerW& L : layers_) {
      for (const MatSeg& sg : L.qkv) acc(sg.m);
      acc(L.wo);
      acc(L.down);
      if (L.moe) acc(L.ex.router);
    }
    if (need) det_part_ = (float*)zalloc(need * 4);
    det_part_n_ = need;
  }
  // KV cache: a pool of kv_pages 64-token pages per layer + one TRASH page (id kv_pages) that
  // unmapped block-table entries point at (idle rows of a micro-batch still append K/V); the engine's
  // KvPager installs the table (set_block_table)
  const int n_slots = NM * B;
  max_pages_ = opt_.max_ctx / 64;
  n_pages_ = opt_.kv_pages > 0 ? opt_.kv_pages : n_slots * max_pages_;
  const size_t per = (size_t)(n_pages_ + 1) * Hkv * 64 * Dp_ * kv_eb();
  for (size_t i = 0; i < layers_.size(); ++i) {
    kc_.push_back((f16*)zalloc(per));
    vc_.push_back((f16*)zalloc(per));
    kv_bytes_ += 2 * per;
  }
  host_bt_.assign((size_t)n_slots * max_pages_, n_pages_);
  block_table_ = (int32_t*)dmalloc(host_bt_.size() * 4);
  HIP_OK(hipMemcpy(block_table_, host_bt_.data(), host_bt_.size() * 4, hipMemcpyHostToDevice));
  // RoPE table (NORM mode), Llama-3.1 frequency factors if present
  const int hd2 = cfg_.head_dim / 2;
  std::vector<float2> cs((size_t)opt_.max_ctx * hd2);
  for (int i = 0; i < hd2; ++i) {
    double inv = std::pow((double)cfg_.rope_base, -2.0 * i / cfg_.head_dim);
    if (!rope_ff_.empty()) inv /= rope_ff_[i];
    for (int p = 0; p < opt_.max_ctx; ++p) {
      const double a = p * inv;
      cs[(size_t)p * hd2 + i] = make_float2((float)std::cos(a), (float)std::sin(a));
    }
  }
  rope_cs_ = (float2*)dmalloc(cs.size() * sizeof(float2));
  HIP_OK(hipMemcpy(rope_cs_, cs.data(), cs.size() * sizeof(float2), hipMemcpyHostToDevice));
  // per micro-batch I/O
  for (int mb = 0; mb < NM; ++mb) {
    act_.push_back((float*)zalloc((size_t)act_rows_ * d * 4));
    tok_.push_back((int32_t*)zalloc(std::max(B, 16) * 4));
    pos_.push_back((int32_t*)zalloc(std::max(B, 16) * 4));
    kvlen_.push_back((int32_t*)zalloc(std::max(B, 16) * 4));
    std::vector<int32_t> sl(std::max(B, 16), 0);
    for (int b = 0; b < B; ++b) sl[b] = slot_of(mb, b);
    int32_t* sd = (int32_t*)dmalloc(sl.size() * 4);
    HIP_OK(hipMemcpy(sd, sl.data(), sl.size() * 4, hipMemcpyHostToDevice));
    slot_.push_back(sd);
  }
  step_ = (int32_t*)zalloc(16);
  pf_pos_ = (int32_t*)zalloc((size_t)opt_.prefill_chunk * 4);
  pf_kvlen_ = (int32_t*)zalloc((size_t)opt_.prefill_chunk * 4);
  pf_slot_ = (int32_t*)zalloc((size_t)opt_.prefill_chunk * 4);
  prompt_dev_ = (int32_t*)zalloc((size_t)n_slots * opt_.max_ctx * 4);
  if (spec_.last())
    for (int mb = 0; mb < NM; ++mb) last_h_.push_back((float*)zalloc((size_t)B * d * 4));
  HIP_OK(hipDeviceSynchronize());
  MP_LOGI("stage %d: layers %d-%d offloaded to GPU %d (%s), weights %.2f GiB, KV %.2f GiB (%d pages of 64 tokens; "
          "%d slots x <= %d ctx)",
          spec_.stage, spec_.layer_begin, spec_.layer_end - 1, spec_.device,
          spec_.first() && spec_.last() ? "embd+head" : spec_.first() ? "embd" : spec_.last() ? "head" : "mid",
          weight_bytes_ / 1073741824.0, kv_bytes_ / 1073741824.0, n_pages_, n_slots, opt_.max_ctx);
}

void HipStage::set_positions(int mb, const std::vector<int32_t>& pos) {
  HIP_OK(hipSetDevice(spec_.device));
  std::vector<int32_t> p(std::max(opt_.mb_size, 16), 0), k(std::max(opt_.mb_size, 16), 1);
  for (size_t i = 0; i < pos.size() && i < p.size(); ++i) { p[i] = pos[i]; k[i] = pos[i] + 1; }
  HIP_OK(hipMemcpyAsync(pos_[mb], p.data(), p.size() * 4, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipMemcpyAsync(kvlen_[mb], k.data(), k.size() * 4, hipMemcpyHostToDevice, stream_));
  HIP_OK(hipStreamSynchronize(stream_));
}

void HipStage::set_block_table(const std::vector<int32_t>& t) {
  if (t.size() != host_bt_.size()) throw std::runtime_error("set_block_table: size mismatch");
  for (int32_t e : t)
    if (e < 0 || e > n_pages_) throw std::runtime_error("set_block_table: page id out of range");
  HIP_OK(hipSetDevice(spec_.device));
  HIP_OK(hipStreamSynchronize(stream_));   // no launch may still read the old table
  host_bt_ = t;
  HIP_OK(hipMemcpy(block_table_, host_bt_.data(), host_bt_.size() * 4, hipMemcpyHostToDevice));
}

// KV of one slot: per layer the first ceil(n_tok / 64) pages of K, then of V, each page
// [Hkv][64][Dp] (K) / [Hkv][Dp][64] (V) f16 (or e4m3 bytes), located through the slot's block-table row
size_t HipStage::kv_state_bytes(int n_tok) const {
  const size_t page = (size_t)cfg_.n_head_kv * 64 * Dp_ * kv_eb();
  return kc_.size() * 2 * (size_t)((n_tok + 63) / 64) * page;
}

void HipStage::kv_export(int slot, int n_tok, std::vector<uint8_t>& out) {
  HIP_OK(hipSetDevice(spec_.device));
  const size_t page = (size_t)cfg_.n_head_kv * 64 * Dp_ * kv_eb();
  const int np = (n_tok + 63) / 64;
  const size_t base = out.size();
  out.resize(base + kv_state_bytes(n_tok));
  uint8_t* dst = out.data() + base;
  HIP_OK(hipStreamSynchronize(stream_));
  for (size_t li = 0; li < kc_.size(); ++li)
    for (f16* c : {kc_[li], vc_[li]})
      for (int k = 0; k < np; ++k) {
        const int32_t pg = host_bt_[(size_t)slot * max_pages_ + k];
        if (pg >= n_pages_) throw std::runtime_error("kv_export: slot has no page for its tokens");
        HIP_OK(hipMemcpy(dst, reinterpret_cast<const uint8_t*>(c) + (size_t)pg * page, page, hipMemcpyDeviceToHost));
        dst += page;
      }
}

void HipStage::kv_import(int slot, int n_tok, const uint8_t* data, size_t bytes) {
  if (bytes != kv_state_bytes(n_tok)) throw std::runtime_error("kv_import: size mismatch");
  HIP_OK(hipSetDevice(spec_.device));
  const size_t page = (size_t)cfg_.n_head_kv * 64 * Dp_ * kv_eb();
  const int np = (n_tok + 63) / 64;
  HIP_OK(hipStreamSynchronize(stream_));
  for (size_t li = 0; li < kc_.size(); ++li)
    for (f16* c : {kc_[li], vc_[li]})
      for (int k = 0; k < np; ++k) {
        const int32_t pg = host_bt_[(size_t)slot * max_pages_ + k];
        if (pg >= n_pages_) throw std::runtime_error("kv_import: slot has no page for its tokens");
        HIP_OK(hipMemcpy(reinterpret_cast<uint8_t*>(c) + (size_t)pg * page, data, page, hipMemcpyHostToDevice));
        data += page;
      }
}

uint64_t HipStage::sample_step() {
  HIP_OK(hipSetDevice(spec_.device));
  HIP_OK(hipStreamSynchronize(stream_));
  int32_t v = 0;
  HIP_OK(hipMemcpy(&v, step_, 4, hipMemcpyDeviceToHost));
  return (uint64_t)(uint32_t)v;
}

void HipStage::set_sample_step(uint64_t s) {
  HIP_OK(hipSetDevice(spec_.device));
  const int32_t v = (int32_t)s;
  HIP_OK(hipMemcpy(step_, &v, 4, hipMemcpyHostToDevice));
}

void HipStage::set_sampling(float temp, int top_k, float top_p, float min_p, uint64_t seed) {
  const bool changed = temp != temp_ || top_k != top_k_ || top_p != top_p_ || min_p != min_p_ || seed != seed_;
  Stage::set_sampling(temp, top_k, top_p, min_p, seed);
  if (changed && !graphs_.empty() && spec_.last()) capture_graphs();
}

void HipStage::set_penalties(int last_n, float repeat, float freq, float presence) {
  const bool changed = last_n != pen_last_n_ || repeat != pen_repeat_ || freq != pen_freq_ || presence != pen_presence_;
  Stage::set_penalties(last_n, repeat, freq, presence);
  if (!spec_.last()) return;
  ensure_hist();
  if (changed && !graphs_.empty()) capture_graphs();
}

void HipStage::ensure_hist() {
  if (!penalties_on() || (hist_ && hist_n_ == pen_last_n_)) return;
  const size_t rows = (size_t)opt_.n_mb * opt_.mb_size;
  hist_ = (int32_t*)dmalloc(rows * pen_last_n_ * 4);
  HIP_OK(hipMemset(hist_, 0xFF, rows * pen_last_n_ * 4));   // -1: empty
  if (!hist_cnt_) hist_cnt_ = (int32_t*)dmalloc(rows * 4);
  HIP_OK(hipMemset(hist_cnt_, 0, rows * 4));
  hist_n_ = pen_last_n_;
}

void HipStage::set_history(int mb, const std::vector<std::vector<int32_t>>& seqs) {
  if (!spec_.last() || !penalties_on()) return;
  ensure_hist();
  const int B = opt_.mb_size, n = hist_n_;
  std::vector<int32_t> h((size_t)B * n, -1), cnt(B, 0);
  for (int b = 0; b < B && b < (int)seqs.size(); ++b) {
    const auto& q = seqs[b];
    const int take = std::min<int>(n, (int)q.size());
    for (int i = 0; i < take; ++i) h[(size_t)b * n + i] = q[q.size() - take + i];
    cnt[b] = take;
  }
  HIP_OK(hipSetDevice(spec_.device));
  HIP_OK(hipMemcpy(hist_ + (size_t)mb * B * n, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  HIP_OK(hipMemcpy(hist_cnt_ + (size_t)mb * B, cnt.data(), cnt.size() * 4, hipMemcpyHostToDevice));
}

void HipStage::gemv(const PackedMat& m, int epi, const f16* X, int ldx, int M, float* Y, int ldy, f16* H, int ldh,
                    int n_valid, bool allow_split, hipStream_t st, const GemvParams* extras) {
  // up to 64 rows (decode micro-batches, short prompt chunks): the dequant GEMV, 1-4 MFMA row
  // groups per weight fragment; longer prompt chunks: MFMA GEMM, weights read once per 64 rows
  // exception: the large gate/up GEMVs that run two tiles per wave (>= 192 workgroups of 16
  // tiles) beat the 64x64-tile GEMM per 64 rows (70B: 4 x 73.6 us vs 410 us per 256-row chunk;
  // profiles/r1g_prefill_gemm_vs_gemv.txt)
  // v2 GEMM (128 rows x 256 columns per workgroup, the decode GEMV's dequant + LDS-shared rows):
  // every shape, f16 weights excepted (they take the 64 x 64 GEMM)
  // v3 GEMM (gemm3.hip: 128|256 x 128|256 workgroup tiles, each weight element dequantized once
  // per workgroup, cross-stage MFMA stream): every type, 16-bit weights included
  // (round 3, before v4) v2 for the quantized types, v3 for 16-bit weights (v2 has no 16-bit path).  Measured in
  // the 70B mb256 round: v3 wins the gate/up on some boxes and loses it on others (212 vs 249 us in
  // profiles/r6h_engine_gemm_v2_v3.txt, 268 us in r6j_gemm_select.txt), and loses o/down (114 vs 98),
  // qkv (72 vs 69) and the Q6_K LM head (1162 vs 639) everywhere; bench.py A/B in one run:
  // v2 5402 tok/s, v3 for gate/up only 5204-5217, v3 everywhere 4867 (r6j)
  // auto for quantized weights, per epilogue (r8a, profiles/r8a_gemm_microbench.txt, 70B at M = 256):
  // the whole-K SwiGLU / store GEMMs (gate/up, LM head) take v4 (gate/up 297 vs 316 us, Q6_K head
  // 724 vs 820), the split-K accumulating ones (qkv, o, down) keep v2.  (v4 there too,
  // prefill_gemm_v=4, ran 70B mb256 at 5953-5970 vs 5764 tok/s but 8B mb256 at 27.3k vs 29.4k, prompt
  // processing 2-5 % slower, and missed the 70B-width oracle at row 128 after two decode rounds
  // (NMSE 1.1e-3): profiles/r8s_v4_everywhere.txt -- not the default)
  // round 5: with the tail-stage hazard gone (tools/isa_lint.py) and the saddr DMA, gemm4 takes the
  // split-K shapes too: 70B mb256 a tie (5797 / 5786 vs 5800 / 5776), 8B mb256 30401 vs 29709
  // (profiles/r10d_splitk_ab_and_prof.txt)
  // (round 6: the 128-row gemm2 form is retired; prefill_gemm_v = 2 takes gemm4)
  const int gv = opt_.prefill_gemm_v == 2 ? 4 : opt_.prefill_gemm_v != 0 ? opt_.prefill_gemm_v : is16(m.ptype) ? 3 : 4;
  const bool wide_swiglu = epi == EPI_SWIGLU && m.dims.ntiles / 16 >= 192;
  const bool v3 = gv == 3;
  if (M > 64 && opt_.prefill_gemm && m.i8 && xq_ && X) {
    // int8_gemm: x rows quantized per row, int8 MFMA against the re-quantized copy (gemm3<P_I8>)
    const int K = (int)m.dims.nsb * 256;
    if (X != xq_src_ || M != xq_rows_) {   // not already quantized by norm_x / the previous GEMM on X
      launch_quant_rows_i8(X, ldx, M, K, xq_, xq_ld_, xqs_, st);
      xq_src_ = X;
      xq_rows_ = M;
    }
    GemvParams p{};
    p.W = m.i8; p.X = reinterpret_cast<const f16*>(xq_); p.ldx = xq_ld_; p.M = M; p.Y = Y; p.ldy = ldy; p.H = H; p.ldh = ldh;
    p.ntiles = (int)m.dims.ntiles; p.nsb = (int)m.dims.nsb; p.n_valid = n_valid;
    p.xscale = xqs_; p.wscale = m.i8_ws;
    launch_gemm3(P_I8, epi, p, st, allow_split && !opt_.deterministic);
    return;
  }
  if (M > 64 && opt_.prefill_gemm && gv == 4 && gemm4_supported(m.ptype)) {
    // v4 GEMM (gemm4.hip: 32x32x16 MFMA): split-K shapes store per-split partials like v2 (into the
    // residual x: absorbed by the next RMSNorm), the rest run whole-K
    GemvParams p{};
    p.W = m.d; p.X = X; p.ldx = ldx; p.M = M; p.Y = Y; p.ldy = ldy; p.H = H; p.ldh = ldh;
    p.ntiles = (int)m.dims.ntiles; p.nsb = (int)m.dims.nsb; p.n_valid = n_valid;
    const bool sk = opt_.gemm_splitk_store && sk_part_ && epi == EPI_ATOMIC && allow_split;
    const bool defer = sk && Y == sk_defer_;
    if (sk) flush_sk(st);
    int ns = 0;
    if (sk && launch_gemm4_splitk(m.ptype, p, sk_part_, sk_part_n_, st, !defer, &ns)) {
      if (defer) sk_pend_ = SkPending{Y, M, n_valid, ldy, ns, p.ntiles * 16, (int64_t)M * p.ntiles * 16};
    } else {
      launch_gemm4(m.ptype, epi, p, st, allow_split && !opt_.deterministic);
    }
    return;
  }
  if (M > 64 && opt_.prefill_gemm && (v3 || !wide_swiglu)) {
    GemvParams p{};
    p.W = m.d; p.X = X; p.ldx = ldx; p.M = M; p.Y = Y; p.ldy = ldy; p.H = H; p.ldh = ldh;
    p.ntiles = (int)m.dims.ntiles; p.nsb = (int)m.dims.nsb; p.n_valid = n_valid;
    if (v3) launch_gemm3(m.ptype, epi, p, st, allow_split && !opt_.deterministic);
    else launch_gemm(m.ptype, epi, p, st);   // the types gemm4 does not take (Q4_0), or prefill_gemm_v = 1
    return;
  }
  for (int r0 = 0; r0 < M; r0 += 64) {
    GemvParams p{};
    if (extras) {   // fused norm / bias / zero-fill: small M only (one pass of this loop)
      p.Xf = extras->Xf; p.ldxf = extras->ldxf; p.gamma = extras->gamma; p.eps = extras->eps;
      p.d_norm = extras->d_norm; p.bias = extras->bias; p.zero = extras->zero; p.zero_n = extras->zero_n;
      p.ssq = extras->ssq;
    }
    p.W = m.d;
    p.X = X + (size_t)r0 * ldx;
    p.ldx = ldx;
    p.M = std::min(64, M - r0);
    p.Y = Y ? Y + (size_t)r0 * ldy : nullptr;
    p.ldy = ldy;
    p.H = H ? H + (size_t)r0 * ldh : nullptr;
    p.ldh = ldh;
    p.ntiles = (int)m.dims.ntiles;
    p.nsb = (int)m.dims.nsb;
    p.n_valid = n_valid;
    const int nsplit = allow_split ? gemv_auto_split(p.ntiles, p.nsb, p.M, epi) : 1;
    const int ns = det_splits(p.ntiles, p.nsb, p.M, epi, allow_split);
    if (opt_.deterministic && epi == EPI_ATOMIC && ns > 1) {
      // split s stores its partial to det_part_[s]; then one fixed-order reduction adds them into Y
      const int ldp = p.ntiles * 16;
      if ((size_t)ns * p.M * ldp > det_part_n_) throw std::runtime_error("deterministic split-K scratch too small");
      GemvParams q = p;
      q.Y = det_part_; q.ldy = ldp; q.split_stride = (int64_t)p.M * ldp;
      launch_gemv(m.ptype, EPI_STORE, q, ns, st);
      launch_splitk_reduce(det_part_, ns, (int64_t)p.M * ldp, ldp, p.M, n_valid, p.Y, ldy, st);
      continue;
    }
    launch_gemv(m.ptype, epi, p, nsplit, st);
  }
}

void HipStage::flush_sk(hipStream_t st) {
  if (!sk_pend_.x) return;
  launch_splitk_reduce(sk_part_, sk_pend_.ns, sk_pend_.ss, sk_pend_.ldp, sk_pend_.M, sk_pend_.n, sk_pend_.x, sk_pend_.ldy, st);
  sk_pend_ = SkPending{};
}

void HipStage::norm_x(float* x, const float* w, int M, float* zero, int64_t zero_n, hipStream_t st, const float* bias,
                      int bias_n) {
  const int d = cfg_.d_model;
  const bool pend = sk_pend_.x == x && sk_pend_.M == M && sk_pend_.n == d && sk_pend_.ldy == d;
  // int8_gemm: the wide GEMMs reading xn_ take its int8 rows from this launch (no separate quant)
  const bool q8 = xq_ && M > 64 && M <= scratch_rows_;
  if ((pend || q8) && d <= 8192 && (d & 3) == 0) {
    launch_rmsnorm_acc(x, d, w, d, cfg_.eps, xn_, Kd_, M, zero, zero_n, pend ? sk_part_ : nullptr, sk_pend_.ns,
                       sk_pend_.ss, sk_pend_.ldp, st, bias, bias_n, q8 ? xq_ : nullptr, xq_ld_, q8 ? xqs_ : nullptr);
    if (pend) sk_pend_ = SkPending{};
    xq_src_ = q8 ? (const void*)xn_ : nullptr;
    xq_rows_ = M;
    return;
  }
  flush_sk(st);
  launch_rmsnorm(x, d, w, d, cfg_.eps, xn_, Kd_, M, zero, zero_n, st, bias, bias_n);
  xq_src_ = nullptr;
}

void HipStage::moe_ffn(const LayerW& L, int M, hipStream_t st, float* x) {
  // > 64 tokens (wide decode micro-batches, prompt chunks): ONE grouped GEMM per projection over
  // every routed expert (gemm4.hip MoE mode: each expert's weights read once per call, its rows
  // gathered into 128/256-row MFMA tiles).  The deterministic mode keeps the slices (its per-slot
  // combine buffer holds 64 tokens).
  if (M > 64 && opt_.prefill_gemm && opt_.moe_gemm && !opt_.deterministic && gemm4_supported(L.ex.gateup.ptype) &&
      gemm4_supported(L.ex.down.ptype))
    return moe_ffn_rows(L, 0, M, st, x, true);
  // otherwise slices of <= 64 tokens, so every slice takes the workgroup-shared MoE GEMV (weights
  // streamed once per 64 tokens, not once per 16 routed rows as in v1)
  const bool v1 = knob(KNOB_MOE_V) == 1;
  const int step = v1 ? M : 64;
  for (int r0 = 0; r0 < M; r0 += step) moe_ffn_rows(L, r0, std::min(step, M - r0), st, x);
}

void HipStage::moe_ffn_rows(const LayerW& L, int r0, int M, hipStream_t st, float* x, bool grouped) {
  const int E = cfg_.n_expert, k = cfg_.n_expert_used, d = cfg_.d_model, F = cfg_.d_ff;
  const f16* xn = xn_ + (size_t)r0 * Kd_;
  float* logits = moe_logits_ + (size_t)r0 * 64;
  // router logits [M][E]: one 16-row tile, so split-K over the super-blocks (atomics into the
  // buffer the ffn RMSNorm cleared) instead of one serial workgroup (28.5 us -> a few us per layer)
  if (L.ex.router_dense && Kd_ >= (int)L.ex.router.dims.nsb * 256)
    launch_router_logits(xn, Kd_, L.ex.router_dense, (int)L.ex.router.dims.nsb * 256, E, M, logits, 64, st);
  else
    gemv(L.ex.router, EPI_ATOMIC, xn, Kd_, M, logits, 64, nullptr, 0, E, true, st);
  MoeRouteParams rp{};
  rp.logits = logits; rp.ld = 64; rp.M = M; rp.E = E; rp.k = k;
  rp.counts = moe_counts_; rp.lists = moe_lists_; rp.list_cap = scratch_rows_ * k; rp.weights = moe_w_;
  launch_moe_route(rp, st);
  MoeGemvParams gp{};
  gp.W = L.ex.gateup.d; gp.estride = L.ex.gateup_stride;
  gp.ntiles = (int)L.ex.gateup.dims.ntiles; gp.nsb = (int)L.ex.gateup.dims.nsb;
  gp.X = xn; gp.ldx = Kd_; gp.x_per_slot = 0; gp.k = k;
  gp.counts = moe_counts_; gp.lists = moe_lists_; gp.list_cap = rp.list_cap; gp.E = E;
  gp.H = moe_h_; gp.ldh = Kff_; gp.n_valid = F; gp.M = M;
  if (grouped) {
    MoeGemvParams dp = gp;
    dp.W = L.ex.down.d; dp.estride = L.ex.down_stride;
    dp.ntiles = (int)L.ex.down.dims.ntiles; dp.nsb = (int)L.ex.down.dims.nsb;
    dp.X = moe_h_; dp.ldx = Kff_; dp.x_per_slot = 1; dp.H = nullptr; dp.ldh = 0;
    dp.Y = x + (size_t)r0 * d; dp.ldy = d; dp.weights = moe_w_; dp.n_valid = d;
    if (!launch_moe_gemm4(L.ex.gateup.ptype, EPI_SWIGLU, gp, st) || !launch_moe_gemm4(L.ex.down.ptype, EPI_ATOMIC, dp, st))
      throw std::runtime_error("moe_ffn: grouped GEMM does not support the expert weight type");
    return;
  }
  launch_moe_gemv(L.ex.gateup.ptype, EPI_SWIGLU, gp, 1, st);
  MoeGemvParams dp = gp;
  dp.W = L.ex.down.d; dp.estride = L.ex.down_stride;
  dp.ntiles = (int)L.ex.down.dims.ntiles; dp.nsb = (int)L.ex.down.dims.nsb;
  dp.X = moe_h_; dp.ldx = Kff_; dp.x_per_slot = 1; dp.H = nullptr; dp.ldh = 0;
  dp.Y = x + (size_t)r0 * d; dp.ldy = d; dp.weights = moe_w_; dp.n_valid = d;
  if (opt_.deterministic) dp.Yslot = moe_yslot_;   // per-slot outputs, combined in expert-rank order below
  // only ~k/E of the expert grid is busy: size the split for the active experts
  const int active = std::min(E, M * k);
  // v1 (M > 64): one tile per 1-wave workgroup, ~4096 of them; v2: 8-tile workgroups, ~1024 of
  // them across the active experts
  const int nsplit = M <= 64 ? std::max(1, std::min(dp.nsb / 4, 1024 / std::max(1, (dp.ntiles + 7) / 8 * active)))
                             : std::max(1, std::min(dp.nsb / 4, 4096 / std::max(1, dp.ntiles * active)));
  launch_moe_gemv(L.ex.down.ptype, EPI_ATOMIC, dp, nsplit, st);
  if (opt_.deterministic) launch_moe_combine(moe_yslot_, d, k, M, d, x + (size_t)r0 * d, d, st);
}

// split count launch_gemv will actually use (deterministic mode reproduces its rounding)
int HipStage::det_splits(int ntiles, int nsb, int M, int epi, bool allow_split) const {
  if (!allow_split) return 1;
  int ns = std::max(1, gemv_auto_split(ntiles, nsb, M, epi));
  const int per = (nsb + ns - 1) / ns;
  return (nsb + per - 1) / per;
}

void HipStage::layer_forward(int li, int M, float* x, const int32_t* pos, const int32_t* kvlen,
                             const int32_t* slot, bool decode, hipStream_t st) {
  const LayerW& L = layers_[li];
  const int d = cfg_.d_model;
  if (small_path(M)) {
    // gemvs: RMSNorms fused into the qkv / gate-up GEMVs, complete outputs per workgroup (q|k|v
    // stored with its bias, o / down added into the residual by their single owner)
    const bool two = knob(KNOB_GEMVS2) != 0;
    // decode: RoPE and the KV append in the qkv GEMV's epilogue (QkvAppend), so the attention starts
    // from rotated q and a complete cache (no dependent position -> page -> append chain of its own)
    const bool pre = decode && opt_.fused_attn && knob(KNOB_ATTN_PRE) && !opt_.deterministic &&
                     attn_decode_pre_ok(decode_attn_params(li, M, pos, slot, false));
    QkvAppend qa{};
    if (pre) {
      qa.pos = pos; qa.slot0 = dec_slot0_; qa.block_table = block_table_; qa.max_pages = max_pages_;
      qa.rope_cs = rope_cs_; qa.k_cache = kc_[li]; qa.v_cache = vc_[li];
      qa.Hq = cfg_.n_head; qa.Hkv = cfg_.n_head_kv; qa.hd = cfg_.head_dim; qa.Dp = Dp_; qa.kv_fp8 = opt_.kv_fp8;
    }
    const int first = L.qkv.size() == 2 && gemvs2_supported(L.qkv[1].m.ptype, L.qkv[0].m.ptype) ? 1 : 0;
    if (two && L.qkv.size() == 2 && gemvs2_supported(L.qkv[first].m.ptype, L.qkv[1 - first].m.ptype) &&
        L.qkv[0].m.dims.nsb == L.qkv[1].m.dims.nsb) {
      // mixed-type q+k | v (Q4_K_M's Q6_K attn_v): both segments in one launch
      GemvParams ps[2];
      for (int i = 0; i < 2; ++i) {
        const MatSeg& sg = L.qkv[i == 0 ? first : 1 - first];
        GemvParams& q = ps[i];
        q.W = sg.m.d; q.M = M; q.Y = qkv_ + sg.y_off; q.ldy = qkv_n_;
        q.ntiles = (int)sg.m.dims.ntiles; q.nsb = (int)sg.m.dims.nsb; q.n_valid = (int)sg.m.dims.N;
        q.bias = L.qkv_bias ? L.qkv_bias + sg.y_off : nullptr;
        q.Xf = x; q.ldxf = d; q.gamma = L.attn_norm; q.eps = cfg_.eps; q.d_norm = d;
        if (pre) { q.qa = qa; q.qa.col0 = (int)sg.y_off; }
      }
      launch_gemvs2(L.qkv[first].m.ptype, L.qkv[1 - first].m.ptype, ps[0], ps[1], st);
    } else {
      for (const MatSeg& s : L.qkv) {
        QkvAppend q = qa;
        q.col0 = (int)s.y_off;
        gemv_small(s.m, EPI_STORE, nullptr, 0, x, L.attn_norm, M, qkv_ + s.y_off, qkv_n_, nullptr, 0, (int)s.m.dims.N,
                   L.qkv_bias ? L.qkv_bias + s.y_off : nullptr, st, pre ? &q : nullptr);
      }
    }
    if (!(decode && attention_o(li, M, pos, slot, x, st, pre))) {
      attention(li, M, pos, kvlen, slot, decode, st, false, pre);
      gemv_small(L.wo, EPI_ATOMIC, attn_, Ko_, nullptr, nullptr, M, x, d, nullptr, 0, d, nullptr, st);
    }
    if (L.moe) {
      launch_rmsnorm(x, d, L.ffn_norm, d, cfg_.eps, xn_, Kd_, M, moe_logits_, (int64_t)M * 64, st);
      xq_src_ = nullptr;
      moe_ffn(L, M, st, x);
      return;
    }
    if (L.fused_gateup) {
      gemv_small(L.gateup, EPI_SWIGLU, nullptr, 0, x, L.ffn_norm, M, nullptr, 0, h_, Kff_, cfg_.d_ff, nullptr, st);
    } else {
      const int F = cfg_.d_ff;
      gemv_small(L.gate, EPI_STORE, nullptr, 0, x, L.ffn_norm, M, gu_, 2 * F, nullptr, 0, F, nullptr, st);
      gemv_small(L.up, EPI_STORE, nullptr, 0, x, L.ffn_norm, M, gu_ + F, 2 * F, nullptr, 0, F, nullptr, st);
      launch_swiglu(gu_, 2 * F, F, M, h_, Kff_, st);
    }
    gemv_small(L.down, EPI_ATOMIC, h_, Kff_, nullptr, nullptr, M, x, d, nullptr, 0, d, nullptr, st);
    return;
  }
  // M <= 4 (fuse_norm): the RMSNorms are folded into the consuming GEMVs (gemv2.hip deferred
  // norm).  qkv: the split-K GEMV publishes per-row sums of squares to ssq_ and the fused decode
  // attention applies rsqrt and the bias when it reads q|k|v.  The o-proj then clears ssq_ + the
  // q|k|v accumulator (invariant: zero outside [qkv GEMV, o-proj]; unfused forwards clear it after
  // their last layer).
  const bool small = fuse_norm(M);
  const bool qkv_deferred = small && decode && opt_.fused_attn;
  GemvParams nx{};
  nx.Xf = x; nx.ldxf = d; nx.eps = cfg_.eps; nx.d_norm = d;
  if (qkv_deferred) {
    for (const MatSeg& s : L.qkv) {
      GemvParams e = nx;
      e.gamma = L.attn_norm;
      e.ssq = &s == &L.qkv[0] ? ssq_ : nullptr;   // the sums of squares once per row
      gemv(s.m, EPI_ATOMIC, nullptr, 0, M, qkv_ + s.y_off, qkv_n_, nullptr, 0, (int)s.m.dims.N, true, st, &e);
    }
  } else {
    norm_x(x, L.attn_norm, M, qkv_, (int64_t)M * qkv_n_, st, L.qkv_bias, qkv_n_);
    for (const MatSeg& s : L.qkv)
      gemv(s.m, EPI_ATOMIC, xn_, Kd_, M, qkv_ + s.y_off, qkv_n_, nullptr, 0, (int)s.m.dims.N, true, st);
  }
  attention(li, M, pos, kvlen, slot, decode, st, qkv_deferred);
  if (small) {
    GemvParams z{};
    z.zero = ssq_; z.zero_n = 64 + (int64_t)M * qkv_n_;
    gemv(L.wo, EPI_ATOMIC, attn_, Ko_, M, x, d, nullptr, 0, d, true, st, &z);
  } else {
    sk_defer_ = x;
    gemv(L.wo, EPI_ATOMIC, attn_, Ko_, M, x, d, nullptr, 0, d, true, st);
    sk_defer_ = nullptr;
    if (opt_.fused_norm && li + 1 == (int)layers_.size())
      HIP_OK(hipMemsetAsync(ssq_, 0, (64 + (size_t)M * qkv_n_) * 4, st));
  }
  const bool ffn_fused = small && !L.moe;
  // MoE: the same launch clears the router logits, which the router GEMV then accumulates split-K
  if (!ffn_fused) norm_x(x, L.ffn_norm, M, L.moe ? moe_logits_ : nullptr, L.moe ? (int64_t)M * 64 : 0, st);
  if (L.moe) {
    moe_ffn(L, M, st, x);
    return;
  }
  GemvParams fx = nx;
  fx.gamma = L.ffn_norm;
  const GemvParams* fe = ffn_fused ? &fx : nullptr;
  const f16* xin = ffn_fused ? nullptr : xn_;
  if (L.fused_gateup) {
    gemv(L.gateup, EPI_SWIGLU, xin, Kd_, M, nullptr, 0, h_, Kff_, cfg_.d_ff, false, st, fe);
  } else {
    const int F = cfg_.d_ff;
    gemv(L.gate, EPI_STORE, xin, Kd_, M, gu_, 2 * F, nullptr, 0, F, false, st, fe);
    gemv(L.up, EPI_STORE, xin, Kd_, M, gu_ + F, 2 * F, nullptr, 0, F, false, st, fe);
    launch_swiglu(gu_, 2 * F, F, M, h_, Kff_, st);
  }
  sk_defer_ = x;   // absorbed by the next layer's attention norm (or flushed after the last layer)
  gemv(L.down, EPI_ATOMIC, h_, Kff_, M, x, d, nullptr, 0, d, true, st);
  sk_defer_ = nullptr;
}

// single-stream decode: attention + o-projection in one launch (attention.hip attn_o_kernel) while
// the context is short enough for every workgroup of a kv head to compute that head's attention
// itself; false: the caller runs the two-kernel path
bool HipStage::attention_o(int li, int M, const int32_t* pos, const int32_t* slot, float* x, hipStream_t st, bool pre) {
  const LayerW& L = layers_[li];
  if (!opt_.fused_attn || opt_.deterministic || opt_.attn_o_max_ctx <= 0 || opt_.max_ctx > opt_.attn_o_max_ctx)
    return false;
  DecodeAttnParams dp{};
  dp.qkv = qkv_; dp.ldqkv = qkv_n_; dp.pos = pos; dp.slot = slot; dp.block_table = block_table_;
    dp.slot0 = dec_slot0_;   // decode only
  dp.max_pages = max_pages_; dp.rope_cs = rope_cs_; dp.q_scale = 1.0f / std::sqrt((float)cfg_.head_dim);
  dp.k_cache = kc_[li]; dp.v_cache = vc_[li]; dp.M = M; dp.Hq = cfg_.n_head; dp.Hkv = cfg_.n_head_kv;
  dp.kv_fp8 = opt_.kv_fp8;
  dp.pre = pre;   // q rotated and K / V appended by the qkv GEMV
  // one split over the whole context (every workgroup of a kv head runs that head's attention)
  dp.hd = cfg_.head_dim; dp.Dp = Dp_; dp.split_len = (int)round_up(opt_.max_ctx, 128); dp.n_split = 1;
  dp.o_part = o_part_; dp.ml_part = ml_part_; dp.counters = attn_cnt_; dp.out = attn_; dp.ldo = Ko_;
  AttnOParams op{};
  op.W = L.wo.d; op.ptype = L.wo.ptype; op.ntiles = (int)L.wo.dims.ntiles; op.nsb = (int)L.wo.dims.nsb;
  op.Y = x; op.ldy = cfg_.d_model; op.n_valid = cfg_.d_model;
  if (!attn_o_supported(dp, op)) return false;
  launch_attn_o(dp, op, st);
  return true;
}

// the fused decode attention's parameters for layer li (decode rows: slots dec_slot0_ + t)
DecodeAttnParams HipStage::decode_attn_params(int li, int M, const int32_t* pos, const int32_t* slot,
                                              bool qkv_deferred) const {
  const LayerW& L = layers_[li];
  DecodeAttnParams dp{};
  dp.qkv = qkv_; dp.ldqkv = qkv_n_; dp.pos = pos; dp.slot = slot; dp.block_table = block_table_;
  dp.slot0 = dec_slot0_;
  dp.max_pages = max_pages_; dp.rope_cs = rope_cs_; dp.q_scale = 1.0f / std::sqrt((float)cfg_.head_dim);
  dp.k_cache = kc_[li]; dp.v_cache = vc_[li]; dp.M = M; dp.Hq = cfg_.n_head; dp.Hkv = cfg_.n_head_kv;
  dp.kv_fp8 = opt_.kv_fp8;
  dp.hd = cfg_.head_dim; dp.Dp = Dp_; dp.split_len = opt_.attn_split_len; dp.n_split = n_split_;
  dp.o_part = o_part_; dp.ml_part = ml_part_; dp.counters = attn_cnt_; dp.out = attn_; dp.ldo = Ko_;
  if (qkv_deferred) { dp.ssq = ssq_; dp.eps = cfg_.eps; dp.d_model = cfg_.d_model; dp.bias = L.qkv_bias; }
  return dp;
}

void HipStage::attention(int li, int M, const int32_t* pos, const int32_t* kvlen, const int32_t* slot, bool decode,
                         hipStream_t st, bool qkv_deferred, bool pre) {
  if (decode && opt_.fused_attn) {
    DecodeAttnParams dp = decode_attn_params(li, M, pos, slot, qkv_deferred);
    dp.pre = pre;
#ifdef MIPIPE_TIMING_PROBES
    dp.probe = knob(KNOB_ATTN_PROBE);
#endif
    launch_attn_decode(dp, st);
  } else {
    RopeKvParams rp{};
    rp.qkv = qkv_; rp.ldqkv = qkv_n_; rp.M = M; rp.Hq = cfg_.n_head; rp.Hkv = cfg_.n_head_kv;
    rp.hd = cfg_.head_dim; rp.Dp = Dp_; rp.pos = pos; rp.slot = slot; rp.block_table = block_table_;
    rp.max_pages = max_pages_; rp.rope_cs = rope_cs_; rp.q_scale = 1.0f / std::sqrt((float)cfg_.head_dim);
    rp.q_out = q_; rp.k_cache = kc_[li]; rp.v_cache = vc_[li]; rp.kv_fp8 = opt_.kv_fp8;
    launch_rope_kv(rp, st);
    if (!decode && opt_.prefill_flash) {
      PrefillAttnParams pa{};
      pa.q = q_; pa.pos = pos; pa.slot = slot; pa.block_table = block_table_; pa.max_pages = max_pages_;
      pa.k_cache = kc_[li]; pa.v_cache = vc_[li]; pa.Hq = cfg_.n_head; pa.Hkv = cfg_.n_head_kv;
      pa.kv_fp8 = opt_.kv_fp8;
      pa.hd = cfg_.head_dim; pa.Dp = Dp_; pa.out = attn_; pa.ldo = Ko_;
      const int bt = prefill_attn_rows_per_tile(cfg_.n_head / cfg_.n_head_kv);
      auto add_rows = [&](int row0, int T) {
        for (int r = 0; r < T; r += bt) {
          if (pa.n_tiles == kPrefillAttnMaxTiles) { launch_attn_prefill(pa, st); pa.n_tiles = 0; }
          pa.tiles[pa.n_tiles++] = (uint32_t)(row0 + r) | ((uint32_t)std::min(bt, T - r) << 16);
        }
      };
      int pages_needed = 0, n_tiles = 0;
      if (segs_ && !segs_->empty()) {
        for (const PrefillSeg& sg : *segs_) {
          pages_needed = std::max(pages_needed, (sg.p0 + sg.T - 1) / 64 + 1);
          n_tiles += (sg.T + bt - 1) / bt;
        }
      }
      // long contexts: split every tile's pages over grid.z so the chunk fills the CUs; the LSE
      // merge runs in the same launcher (one workgroup list per launch, so only when it fits one)
      pa.M = M;
      if (pf_opart_ && n_tiles > 0 && n_tiles <= kPrefillAttnMaxTiles) {
        pa.n_split = prefill_attn_splits(n_tiles, cfg_.n_head_kv, pages_needed, kPrefillMaxSplit, &pa.split_pages);
        pa.o_part = pf_opart_; pa.ml_part = pf_ml_;
      }
      if (segs_ && !segs_->empty()) {
        int row = 0;
        for (const PrefillSeg& sg : *segs_) { add_rows(row, sg.T); row += sg.T; }
      } else {
        add_rows(0, M);
      }
      launch_attn_prefill(pa, st);
    } else {
    AttnParams ap{};
    ap.q = q_; ap.kvlen = kvlen; ap.slot = slot; ap.block_table = block_table_; ap.max_pages = max_pages_;
    if (opt_.kv_fp8) throw std::runtime_error("kv_dtype fp8: the unfused attention path reads f16 pages");
    ap.k_cache = kc_[li]; ap.v_cache = vc_[li]; ap.M = M; ap.Hq = cfg_.n_head; ap.Hkv = cfg_.n_head_kv;
    ap.hd = cfg_.head_dim; ap.Dp = Dp_; ap.max_kv = opt_.max_ctx; ap.out = attn_; ap.ldo = Ko_;
    if (decode) {
      ap.tq = 1;
      ap.split_len = opt_.attn_split_len;
      ap.n_split = n_split_;
      ap.o_part = o_part_; ap.ml_part = ml_part_;
    } else {
      const int G = cfg_.n_head / cfg_.n_head_kv;
      ap.tq = std::max(1, 16 / G);
      ap.split_len = (int)round_up(opt_.max_ctx, 128);
      ap.n_split = 1;
    }
    if (!decode && segs_ && segs_->size() > 1) {
      // packed prefill: a row group of the attention kernel must belong to one sequence
      int row = 0;
      for (const PrefillSeg& s : *segs_) {
        AttnParams a = ap;
        a.q = q_ + (size_t)row * cfg_.n_head * Dp_;
        a.kvlen = kvlen + row; a.slot = slot + row; a.M = s.T;
        a.out = attn_ + (size_t)row * Ko_;
        launch_attention(a, st);
        row += s.T;
      }
    } else {
      launch_attention(ap, st);
    }
    }
  }
}

void HipStage::gemv_small(const PackedMat& m, int epi, const f16* X, int ldx, const float* Xf, const float* gamma,
                          int M, float* Y, int ldy, f16* H, int ldh, int n_valid, const float* bias, hipStream_t st,
                          const QkvAppend* qa) {
  GemvParams p{};
  if (qa) p.qa = *qa;
  p.W = m.d; p.X = X; p.ldx = ldx; p.M = M; p.Y = Y; p.ldy = ldy; p.H = H; p.ldh = ldh;
  p.ntiles = (int)m.dims.ntiles; p.nsb = (int)m.dims.nsb; p.n_valid = n_valid; p.bias = bias;
  if (Xf) { p.Xf = Xf; p.ldxf = cfg_.d_model; p.gamma = gamma; p.eps = cfg_.eps; p.d_norm = cfg_.d_model; }
  const GemvsPlan pl = plan_gemvs(p.ntiles, p.nsb, M, epi, false, opt_.deterministic);
  if (!Xf && pl.lds + (size_t)pl.sb_per_split * 64 > 150 * 1024) {   // (+ the single-row form's table)
    // deterministic mode cannot split K over grid.y, so a wide K (70B down: 28672) with M >= 3
    // rows overflows LDS: take the v2 GEMV with its fixed-order split-K reduction instead
    gemv(m, epi, X, ldx, M, Y, ldy, H, ldh, n_valid, epi == EPI_ATOMIC, st);
    return;
  }
  launch_gemvs(m.ptype, epi, p, opt_.deterministic, st);
}

bool HipStage::fuse_norm(int M) const { return opt_.fused_norm && M <= 4; }

void HipStage::head(int mb, int M, const float* x, int32_t* tok_out, uint64_t salt, hipStream_t st) {
  const int d = cfg_.d_model;
  // (the LM head keeps the standalone norm: the deferred-norm GEMV variant needs ~50 more VGPRs,
  // which halves the head's occupancy: 90.5 vs 72.7 + 4.6 us at 8B, profiles/r2h_prof_8b_mb1.txt)
  if (small_path(M)) {
    gemv_small(out_, EPI_STORE, nullptr, 0, x, out_norm_, M, logits_, logits_ld_, nullptr, 0, cfg_.vocab, nullptr, st);
  } else {
    launch_rmsnorm(x, d, out_norm_, d, cfg_.eps, xn_, Kd_, M, nullptr, 0, st);
    xq_src_ = nullptr;
    gemv(out_, EPI_STORE, xn_, Kd_, M, logits_, logits_ld_, nullptr, 0, cfg_.vocab, false, st);
  }
  const bool pen = penalties_on() && hist_;
  int32_t* hist = pen ? hist_ + (size_t)mb * opt_.mb_size * hist_n_ : nullptr;
  if (pen) {
    PenaltyParams pp{};
    pp.logits = logits_; pp.ld = logits_ld_; pp.n = cfg_.vocab; pp.M = M;
    pp.hist = hist; pp.last_n = hist_n_; pp.repeat = pen_repeat_; pp.freq = pen_freq_; pp.presence = pen_presence_;
    launch_penalize(pp, st);
  }
  if (temp_ > 0.f) {
    SampleParams sp{};
    sp.logits = logits_; sp.ld = logits_ld_; sp.n = cfg_.vocab; sp.M = M;
    sp.temp = temp_; sp.top_k = top_k_; sp.top_p = top_p_; sp.min_p = min_p_;
    sp.seed = seed_ ^ (salt * 0x9E3779B97F4A7C15ULL); sp.step = step_; sp.tokens = tok_out;
    launch_sample(sp, st);
  } else {
    launch_argmax(logits_, logits_ld_, cfg_.vocab, M, tok_out, st, &am_);
  }
  if (pen) launch_hist_push(hist, hist_cnt_ + (size_t)mb * opt_.mb_size, hist_n_, tok_out, M, st);
}

void HipStage::prefill(int mb, const std::vector<PrefillSeg>& segs, hipStream_t st) {
  const int d = cfg_.d_model;
  float* x = act_[mb];
  int T = 0;
  for (const PrefillSeg& s : segs) {
    if (s.p0 + s.T > opt_.max_ctx) throw std::runtime_error("prompt exceeds context");
    const int sl = slot_of(mb, s.b);
    launch_prefill_meta(pf_pos_ + T, pf_kvlen_ + T, pf_slot_ + T, s.p0, s.T, sl, st);
    if (spec_.first())
      launch_embed(embd_type_, embd_raw_, (int64_t)embd_row_bytes_, d, prompt_dev_ + (size_t)sl * opt_.max_ctx + s.p0,
                   s.T, x + (size_t)T * d, d, st);
    T += s.T;
  }
  if (T > opt_.prefill_chunk) throw std::runtime_error("prefill chunk too large");
  segs_ = &segs;
  for (size_t li = 0; li < layers_.size(); ++li)
    layer_forward((int)li, T, x, pf_pos_, pf_kvlen_, pf_slot_, false, st);
  flush_sk(st);
  segs_ = nullptr;
  if (spec_.last() && !segs.empty() && segs[0].verify) {
    // speculative verification: LM head over every row of the chunk, greedy next token per row
    if (!vlogits_) {
      vlogits_ = (float*)dmalloc((size_t)opt_.prefill_chunk * logits_ld_ * 4);
      vtok_ = (int32_t*)dmalloc((size_t)opt_.n_mb * opt_.prefill_chunk * 4);
    }
    launch_rmsnorm(x, d, out_norm_, d, cfg_.eps, xn_, Kd_, T, nullptr, 0, st);
    xq_src_ = nullptr;
    gemv(out_, EPI_STORE, xn_, Kd_, T, vlogits_, logits_ld_, nullptr, 0, cfg_.vocab, false, st);
    launch_argmax(vlogits_, logits_ld_, cfg_.vocab, T, vtok_ + (size_t)mb * opt_.prefill_chunk, st, &am_);
  } else if (spec_.last()) {
    int row = 0;
    for (const PrefillSeg& s : segs) {
      row += s.T;
      if (s.last)
        HIP_OK(hipMemcpyAsync(last_h_[mb] + (size_t)s.b * d, x + (size_t)(row - 1) * d, (size_t)d * 4,
                              hipMemcpyDeviceToDevice, st));
    }
  }
}

void HipStage::copy_verify_tokens(int mb, int32_t* host, int n) {
  if (!vtok_ || n > opt_.prefill_chunk) throw std::runtime_error("no verify tokens");
  HIP_OK(hipSetDevice(spec_.device));
  HIP_OK(hipMemcpy(host, vtok_ + (size_t)mb * opt_.prefill_chunk, (size_t)n * 4, hipMemcpyDeviceToHost));
}

void HipStage::prefill_finish(int mb, hipStream_t st, const std::vector<int>* rows) {
  if (!spec_.last()) return;
  if (!rows) {
    head(mb, opt_.mb_size, last_h_[mb], tok_[mb], 1000003ULL + (uint64_t)mb, st);
    return;
  }
  if (!tok_tmp_) tok_tmp_ = (int32_t*)dmalloc((size_t)std::max(opt_.mb_size, 16) * 4);
  head(mb, opt_.mb_size, last_h_[mb], tok_tmp_, 1000003ULL + (uint64_t)mb, st);
  for (int b : *rows) HIP_OK(hipMemcpyAsync(tok_[mb] + b, tok_tmp_ + b, 4, hipMemcpyDeviceToDevice, st));
}

void HipStage::decode_eager(int mb, hipStream_t st) {
  const int B = opt_.mb_size;
  float* x = act_[mb];
  if (spec_.first())
    launch_embed(embd_type_, embd_raw_, (int64_t)embd_row_bytes_, cfg_.d_model, tok_[mb], B, x, cfg_.d_model, st);
  dec_slot0_ = slot_of(mb, 0);   // slot_[mb] holds slot_of(mb, b) = dec_slot0_ + b
  for (size_t li = 0; li < layers_.size(); ++li)
    layer_forward((int)li, B, x, pos_[mb], kvlen_[mb], slot_[mb], true, st);
  flush_sk(st);
  if (spec_.last()) head(mb, B, x, tok_[mb], (uint64_t)mb + 1, st);
  launch_advance(pos_[mb], kvlen_[mb], B, mb == 0 ? step_ : nullptr, st);
}

void HipStage::capture_graphs() {
  HIP_OK(hipSetDevice(spec_.device));
  destroy_graphs();
  if (!opt_.use_graphs) return;
  for (int mb = 0; mb < opt_.n_mb; ++mb) {
    hipGraph_t g;
    HIP_OK(hipStreamBeginCapture(stream_, hipStreamCaptureModeRelaxed));
    decode_eager(mb, stream_);
    HIP_OK(hipStreamEndCapture(stream_, &g));
    hipGraphExec_t ex;
    HIP_OK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    HIP_OK(hipGraphDestroy(g));
    graphs_.push_back(ex);
  }
}

void HipStage::destroy_graphs() {
  for (auto g : graphs_) (void)hipGraphExecDestroy(g);
  graphs_.clear();
}

void HipStage::decode(int mb, hipStream_t st) {
  if (!graphs_.empty()) HIP_OK(hipGraphLaunch(graphs_[mb], st));
  else decode_eager(mb, st);
}

}  // namespace mp
