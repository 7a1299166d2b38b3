#include "cpu_stage.h"

#include <unordered_map>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <random>
#include <stdexcept>
#include <thread>

#include <sched.h>
#include <cstdio>

#include "gguf.h"
#include "hip_stage.h"   // SyntheticTypes
#include "log.h"
#include "pack.h"
#include "qtypes.h"

// host-only multiversioning (hipcc also runs a device pass over this file, which has no clones)
#if defined(__HIP_DEVICE_COMPILE__)
#define MP_HOST_AVX2_CLONES
#else
#define MP_HOST_AVX2_CLONES __attribute__((target_clones("avx2", "default")))
#endif

namespace mp {

namespace {

std::vector<float> tensor_f32(const GgufTensor& t) {
  std::vector<float> v(t.nelem());
  const int64_t K = t.ne[0];
  const size_t rb = row_bytes(t.type, K);
  for (int64_t r = 0; r < t.nelem() / K; ++r) dequant_row(t.type, t.data + r * rb, v.data() + r * K, K);
  return v;
}

CpuMat mat_of(const GgufTensor& t, int64_t expert = -1) {
  CpuMat m;
  m.type = t.type;
  m.K = t.ne[0];
  m.N = t.ne[1];
  m.rb = row_bytes(t.type, m.K);
  m.data = t.data + (expert >= 0 ? (size_t)expert * m.N * m.rb : 0);
  return m;
}

inline void put_f16(uint8_t* p, float v) {
  const uint16_t h = f32_to_f16(v);
  std::memcpy(p, &h, 2);
}

// random blocks of a ggml type whose dequantised values are ~U(-scale, scale)-sized
void fill_random(int type, int64_t nblocks, float scale, uint64_t seed, uint8_t* dst) {
  std::mt19937_64 rng(seed);
  const size_t bb = block_bytes(type);
  for (size_t i = 0; i < (size_t)nblocks * bb; i += 8) {
    const uint64_t r = rng();
    std::memcpy(dst + i, &r, std::min<size_t>(8, (size_t)nblocks * bb - i));
  }
  std::uniform_real_distribution<float> u(-scale, scale);
  for (int64_t b = 0; b < nblocks; ++b) {
    uint8_t* p = dst + b * bb;
    switch (type) {
      case T_F32: { const float v = u(rng); std::memcpy(p, &v, 4); break; }
      case T_F16: put_f16(p, u(rng)); break;
      case T_BF16: { const float v = u(rng); uint32_t x; std::memcpy(&x, &v, 4); const uint16_t h = (uint16_t)(x >> 16); std::memcpy(p, &h, 2); break; }
      case T_Q8_0: put_f16(p, scale / 80.f); break;
      case T_Q4_0: put_f16(p, scale / 5.f); break;
      case T_Q4_K: case T_Q5_K:
        put_f16(p, scale / (type == T_Q4_K ? 300.f : 600.f));
        put_f16(p + 2, scale / 300.f);
        break;
      case T_Q6_K: put_f16(p + bb - 2, scale / 2000.f); break;
      default: throw std::runtime_error("cpu synthetic: unsupported type");
    }
  }
}

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ULL; x ^= x >> 27; x *= 0x94d049bb133111ebULL; x ^= x >> 31;
  return x;
}

}  // namespace

// CPUs this process may really use: the affinity mask and the cgroup quota (cpu.max), not the
// machine's count (a GPU box's container sees every CPU of the host but gets a 16-CPU share); one
// is left to the control plane (HTTP / session / link threads), since the pool's workers spin
int default_cpu_threads() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = std::min(n, CPU_COUNT(&cs));
  if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    long period = 0;
    if (std::fscanf(f, "%31s %ld", q, &period) == 2 && std::strcmp(q, "max") != 0 && period > 0) {
      const long quota = std::atol(q);
      if (quota > 0) n = std::min(n, (int)std::max(1L, (quota + period - 1) / period));
    }
    std::fclose(f);
  }
  return std::max(1, n > 3 ? n - 1 : n);
}

CpuStage::CpuStage(const ModelConfig& cfg, const StageSpec& spec, const StageOptions& opt)
    : cfg_(cfg), spec_(spec), opt_(opt) {
  int nt = opt_.threads > 0 ? opt_.threads : default_cpu_threads();
  pool_.reset(new ThreadPool(std::max(1, std::min(nt, 64))));
  layers_.resize(spec_.layer_end - spec_.layer_begin);
}

CpuStage::~CpuStage() = default;

CpuMat CpuStage::own_random(int type, int64_t N, int64_t K, uint64_t seed) {
  CpuMat m;
  m.type = type;
  m.N = N;
  m.K = K;
  m.rb = row_bytes(type, K);
  owned_.emplace_back(m.rb * N);
  // F32 fill_random writes one value per block: F32/F16/BF16 blocks are single elements
  fill_random(type, (int64_t)(m.rb * N / block_bytes(type)), 1.7f / std::sqrt((float)K), seed, owned_.back().data());
  m.data = owned_.back().data();
  weight_bytes_ += m.rb * N;
  return m;
}

void CpuStage::load_gguf(const GgufFile& f) {
  auto need = [&](const std::string& n) -> const GgufTensor& {
    const GgufTensor* t = f.tensor(n);
    if (!t) throw std::runtime_error("missing tensor " + n);
    return *t;
  };
  auto mat = [&](const std::string& n) {
    const GgufTensor& t = need(n);
    weight_bytes_ += t.nbytes;
    return mat_of(t);
  };
  for (int li = spec_.layer_begin; li < spec_.layer_end; ++li) {
    Layer& L = layers_[li - spec_.layer_begin];
    const std::string p = "blk." + std::to_string(li) + ".";
    L.attn_norm = tensor_f32(need(p + "attn_norm.weight"));
    if (cfg_.qkv_bias) {
      L.bq = tensor_f32(need(p + "attn_q.bias"));
      L.bk = tensor_f32(need(p + "attn_k.bias"));
      L.bv = tensor_f32(need(p + "attn_v.bias"));
    }
    L.ffn_norm = tensor_f32(need(p + "ffn_norm.weight"));
    L.q = mat(p + "attn_q.weight");
    L.k = mat(p + "attn_k.weight");
    L.v = mat(p + "attn_v.weight");
    L.o = mat(p + "attn_output.weight");
    if (cfg_.n_expert) {
      L.moe = true;
      L.router = mat(p + "ffn_gate_inp.weight");
      const GgufTensor* sg = f.tensor(p + "ffn_gate_exps.weight");
      for (int e = 0; e < cfg_.n_expert; ++e) {
        if (sg) {
          L.eg.push_back(mat_of(*sg, e));
          L.eu.push_back(mat_of(need(p + "ffn_up_exps.weight"), e));
          L.ed.push_back(mat_of(need(p + "ffn_down_exps.weight"), e));
        } else {
          const std::string s = "." + std::to_string(e) + ".weight";
          L.eg.push_back(mat(p + "ffn_gate" + s));
          L.eu.push_back(mat(p + "ffn_up" + s));
          L.ed.push_back(mat(p + "ffn_down" + s));
        }
      }
      if (sg)
        weight_bytes_ += sg->nbytes + need(p + "ffn_up_exps.weight").nbytes + need(p + "ffn_down_exps.weight").nbytes;
    } else {
      L.gate = mat(p + "ffn_gate.weight");
      L.up = mat(p + "ffn_up.weight");
      L.down = mat(p + "ffn_down.weight");
    }
  }
  const GgufTensor& te = need("token_embd.weight");
  if (spec_.first()) { embd_ = mat_of(te); weight_bytes_ += te.nbytes; }
  if (spec_.last()) {
    out_norm_ = tensor_f32(need("output_norm.weight"));
    const GgufTensor* to = f.tensor("output.weight");
    out_ = mat_of(to ? *to : te);
    weight_bytes_ += (to ? *to : te).nbytes;
  }
  inv_freq_.clear();
  const int hd2 = cfg_.head_dim / 2;
  std::vector<float> ff;
  if (const GgufTensor* rf = f.tensor("rope_freqs.weight")) ff = tensor_f32(*rf);
  for (int i = 0; i < hd2; ++i) {
    double inv = std::pow((double)cfg_.rope_base, -2.0 * i / cfg_.head_dim);
    if (!ff.empty()) inv /= ff[i];
    inv_freq_.push_back((float)inv);
  }
}

void CpuStage::init_synthetic(const std::string& ftype, uint64_t seed) {
  const int d = cfg_.d_model, qd = cfg_.q_dim(), kvd = cfg_.kv_dim(), F = cfg_.d_ff;
  for (int li = spec_.layer_begin; li < spec_.layer_end; ++li) {
    Layer& L = layers_[li - spec_.layer_begin];
    const SyntheticTypes t = SyntheticTypes::from_ftype(ftype, li, cfg_.n_layer);
    const uint64_t s = seed * 1000003ULL + (uint64_t)li * 97;
    L.attn_norm.assign(d, 1.f);
    L.ffn_norm.assign(d, 1.f);
    L.q = own_random(t.q, qd, d, s + 1);
    L.k = own_random(t.k, kvd, d, s + 2);
    L.v = own_random(t.v, kvd, d, s + 3);
    L.o = own_random(t.o, d, qd, s + 4);
    if (cfg_.n_expert) {
      L.moe = true;
      L.router = own_random(T_F32, cfg_.n_expert, d, s + 7);
      for (int e = 0; e < cfg_.n_expert; ++e) {
        L.eg.push_back(own_random(t.gate, F, d, s + 100 + 3 * e));
        L.eu.push_back(own_random(t.up, F, d, s + 101 + 3 * e));
        L.ed.push_back(own_random(t.down, d, F, s + 102 + 3 * e));
      }
    } else {
      L.gate = own_random(t.gate, F, d, s + 5);
      L.up = own_random(t.up, F, d, s + 8);
      L.down = own_random(t.down, d, F, s + 6);
    }
  }
  const SyntheticTypes t0 = SyntheticTypes::from_ftype(ftype, 0, cfg_.n_layer);
  if (spec_.first()) embd_ = own_random(t0.embd, cfg_.vocab, d, seed ^ 0xE3BD);
  if (spec_.last()) {
    out_norm_.assign(d, 1.f);
    out_ = own_random(t0.out, cfg_.vocab, d, seed ^ 0x0F7);
  }
  inv_freq_.clear();
  for (int i = 0; i < cfg_.head_dim / 2; ++i)
    inv_freq_.push_back((float)std::pow((double)cfg_.rope_base, -2.0 * i / cfg_.head_dim));
}

void CpuStage::alloc_runtime() {
  const int B = opt_.mb_size, NM = opt_.n_mb, d = cfg_.d_model;
  const int rows = std::max(B, opt_.prefill_chunk);
  const int n_slots = NM * B;
  // paged KV (kvpager.h): kv_pages pages of [64][kv_dim] f32 + the TRASH page, per layer
  max_pages_ = opt_.max_ctx / 64;
  n_pages_ = opt_.kv_pages > 0 ? opt_.kv_pages : n_slots * max_pages_;
  bt_.assign((size_t)n_slots * max_pages_, n_pages_);
  const size_t per = (size_t)(n_pages_ + 1) * 64 * cfg_.kv_dim();
  for (size_t i = 0; i < layers_.size(); ++i) {
    kc_.emplace_back(per, 0.f);
    vc_.emplace_back(per, 0.f);
    kv_bytes_ += 2 * per * 4;
  }
  for (int mb = 0; mb < NM; ++mb) {
    act_.emplace_back((size_t)rows * d, 0.f);
    tok_.emplace_back(std::max(B, 16), 0);
    pos_.emplace_back(std::max(B, 16), 0);
  }
  prompt_.assign((size_t)n_slots * opt_.max_ctx, 0);
  if (spec_.last())
    for (int mb = 0; mb < NM; ++mb) last_h_.emplace_back((size_t)B * d, 0.f);
  if (spec_.last()) logits_.assign((size_t)B * cfg_.vocab, 0.f);
  xn_.resize((size_t)rows * d);
  qkv_.resize((size_t)rows * (cfg_.q_dim() + 2 * cfg_.kv_dim()));
  att_.resize((size_t)rows * cfg_.q_dim());
  h_.resize((size_t)rows * cfg_.d_ff);
  gu_.resize((size_t)rows * 2 * cfg_.d_ff);
  MP_LOGI("stage %d: layers %d-%d on CPU (%d threads), weights %.2f GiB, KV %.2f GiB (%d pages of 64 tokens; "
          "%d slots x <= %d ctx)", spec_.stage, spec_.layer_begin, spec_.layer_end - 1, pool_->size(),
          weight_bytes_ / 1073741824.0, kv_bytes_ / 1073741824.0, n_pages_, n_slots, opt_.max_ctx);
}

void CpuStage::set_positions(int mb, const std::vector<int32_t>& pos) {
  std::fill(pos_[mb].begin(), pos_[mb].end(), 0);
  for (size_t i = 0; i < pos.size() && i < pos_[mb].size(); ++i) pos_[mb][i] = pos[i];
}

// dot product with 8 fixed-order partial sums (one AVX2 vector; no FMA contraction in either clone, so
// the AVX2 and baseline builds give the same bits)
MP_HOST_AVX2_CLONES static float dot8(const float* w, const float* x, int64_t K) {
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  int64_t k = 0;
  for (; k + 8 <= K; k += 8)
    for (int j = 0; j < 8; ++j) s[j] += w[k + j] * x[k + j];
  for (; k < K; ++k) s[0] += w[k] * x[k];
  return ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
}

void CpuStage::matmul(const CpuMat& W, const float* X, int ldx, int M, float* Y, int ldy, bool accumulate) {
  const int64_t K = W.K;
  if (opt_.cpu_q8 && qdot_supported(W.type) && K % qdot_block(W.type) == 0) {
    // the weights in their stored integer form against int8 activation blocks (cpu_qdot.cpp)
    quantize_q8_rows(X, ldx, M, K, xq_);
    pool_->parallel_for(W.N, [&](int64_t n0, int64_t n1) {
      for (int64_t n = n0; n < n1; ++n) {
        const uint8_t* wr = W.data + n * W.rb;
        for (int m = 0; m < M; ++m) {
          const float s = qdot_row(W.type, wr, q8_row(xq_, m), K);
          float& y = Y[(size_t)m * ldy + n];
          y = accumulate ? y + s : s;
        }
      }
    }, 16);
    return;
  }
  pool_->parallel_for(W.N, [&](int64_t n0, int64_t n1) {
    std::vector<float> w((size_t)K);
    for (int64_t n = n0; n < n1; ++n) {
      dequant_row(W.type, W.data + n * W.rb, w.data(), K);
      for (int m = 0; m < M; ++m) {
        const float s = dot8(w.data(), X + (size_t)m * ldx, K);
        float& y = Y[(size_t)m * ldy + n];
        y = accumulate ? y + s : s;
      }
    }
  }, 16);
}

void CpuStage::rmsnorm(const float* x, const std::vector<float>& w, float* y, int M) {
  const int d = cfg_.d_model;
  for (int m = 0; m < M; ++m) {
    const float* xr = x + (size_t)m * d;
    double ss = 0;
    for (int i = 0; i < d; ++i) ss += (double)xr[i] * xr[i];
    const float r = 1.0f / std::sqrt((float)(ss / d) + cfg_.eps);
    for (int i = 0; i < d; ++i) y[(size_t)m * d + i] = xr[i] * r * w[i];
  }
}

void CpuStage::layer_forward(int li, int M, float* x, const int32_t* pos, const int32_t* slot) {
  const Layer& L = layers_[li];
  const int d = cfg_.d_model, qd = cfg_.q_dim(), kvd = cfg_.kv_dim(), hd = cfg_.head_dim;
  const int Hq = cfg_.n_head, Hkv = cfg_.n_head_kv, G = Hq / Hkv, ctx = opt_.max_ctx;
  const int ldq = qd + 2 * kvd;
  rmsnorm(x, L.attn_norm, xn_.data(), M);
  matmul(L.q, xn_.data(), d, M, qkv_.data(), ldq, false);
  matmul(L.k, xn_.data(), d, M, qkv_.data() + qd, ldq, false);
  matmul(L.v, xn_.data(), d, M, qkv_.data() + qd + kvd, ldq, false);
  if (!L.bq.empty())
    for (int m = 0; m < M; ++m) {
      float* row = qkv_.data() + (size_t)m * ldq;
      for (int i = 0; i < qd; ++i) row[i] += L.bq[i];
      for (int i = 0; i < kvd; ++i) row[qd + i] += L.bk[i], row[qd + kvd + i] += L.bv[i];
    }
  // RoPE (GGUF Llama layout: adjacent pairs (2i, 2i+1); Qwen2 NEOX: (i, i + hd/2)) + KV append
  const int half = hd / 2, pstride = cfg_.rope_neox ? 1 : 2, poff = cfg_.rope_neox ? half : 1;
  for (int m = 0; m < M; ++m) {
    float* row = qkv_.data() + (size_t)m * ldq;
    const int p = pos[m];
    for (int h = 0; h < Hq + Hkv; ++h) {
      float* v = row + (size_t)h * hd;   // q heads then k heads (contiguous)
      for (int i = 0; i < half; ++i) {
        const float a = p * inv_freq_[i], c = std::cos(a), s = std::sin(a);
        float* e0 = v + pstride * i;
        float* e1 = e0 + poff;
        const float x0 = *e0, x1 = *e1;
        *e0 = x0 * c - x1 * s;
        *e1 = x0 * s + x1 * c;
      }
    }
    const size_t kv_off = kv_row(slot[m], p) * kvd;
    std::memcpy(&kc_[li][kv_off], row + qd, (size_t)kvd * 4);
    std::memcpy(&vc_[li][kv_off], row + qd + kvd, (size_t)kvd * 4);
  }
  // causal attention over the slot's cache (tokens of this chunk are already appended)
  const float scale = 1.0f / std::sqrt((float)hd);
  pool_->parallel_for((int64_t)M * Hq, [&](int64_t i0, int64_t i1) {
    std::vector<float> sc((size_t)ctx);
    for (int64_t i = i0; i < i1; ++i) {
      const int m = (int)(i / Hq), h = (int)(i % Hq), kh = h / G;
      const float* q = qkv_.data() + (size_t)m * ldq + (size_t)h * hd;
      const int n = pos[m] + 1;
      const float* kb = &kc_[li][(size_t)kh * hd];
      const float* vb = &vc_[li][(size_t)kh * hd];
      float mx = -INFINITY;
      for (int t = 0; t < n; ++t) {
        const float* k = kb + kv_row(slot[m], t) * kvd;
        float s = 0;
        for (int j = 0; j < hd; ++j) s += q[j] * k[j];
        sc[t] = s * scale;
        mx = std::max(mx, sc[t]);
      }
      float sum = 0;
      for (int t = 0; t < n; ++t) { sc[t] = std::exp(sc[t] - mx); sum += sc[t]; }
      float* o = att_.data() + (size_t)m * qd + (size_t)h * hd;
      std::fill(o, o + hd, 0.f);
      for (int t = 0; t < n; ++t) {
        const float p = sc[t] / sum;
        const float* v = vb + kv_row(slot[m], t) * kvd;
        for (int j = 0; j < hd; ++j) o[j] += p * v[j];
      }
    }
  });
  matmul(L.o, att_.data(), qd, M, x, d, true);
  rmsnorm(x, L.ffn_norm, xn_.data(), M);
  ffn(L, M, xn_.data(), x);
}

void CpuStage::ffn(const Layer& L, int M, const float* xn, float* x) {
  const int d = cfg_.d_model, F = cfg_.d_ff;
  auto swiglu = [&](const CpuMat& g, const CpuMat& u, const float* xin, int rows) {
    matmul(g, xin, d, rows, gu_.data(), 2 * F, false);
    matmul(u, xin, d, rows, gu_.data() + F, 2 * F, false);
    for (int m = 0; m < rows; ++m)
      for (int j = 0; j < F; ++j) {
        const float a = gu_[(size_t)m * 2 * F + j], b = gu_[(size_t)m * 2 * F + F + j];
        h_[(size_t)m * F + j] = a / (1.f + std::exp(-a)) * b;
      }
  };
  if (!L.moe) {
    swiglu(L.gate, L.up, xn, M);
    matmul(L.down, h_.data(), F, M, x, d, true);
    return;
  }
  const int E = cfg_.n_expert, k = cfg_.n_expert_used;
  std::vector<float> lg((size_t)M * E), y(d);
  matmul(L.router, xn, d, M, lg.data(), E, false);
  for (int m = 0; m < M; ++m) {
    const float* l = lg.data() + (size_t)m * E;
    std::vector<int> idx(E);
    for (int e = 0; e < E; ++e) idx[e] = e;
    std::partial_sort(idx.begin(), idx.begin() + k, idx.end(), [&](int a, int b) { return l[a] > l[b] || (l[a] == l[b] && a < b); });
    const float mx = l[idx[0]];
    float wsum = 0;
    std::vector<float> w(k);
    for (int j = 0; j < k; ++j) { w[j] = std::exp(l[idx[j]] - mx); wsum += w[j]; }
    for (int j = 0; j < k; ++j) {
      const int e = idx[j];
      swiglu(L.eg[e], L.eu[e], xn + (size_t)m * d, 1);
      matmul(L.ed[e], h_.data(), F, 1, y.data(), d, false);
      for (int i = 0; i < d; ++i) x[(size_t)m * d + i] += w[j] / wsum * y[i];
    }
  }
}

// llama.cpp sampler-chain semantics (same as the HIP sampler, csrc/kernels/sample.hip): top-k,
// top-p and min-p cut the T = 1 distribution, the draw uses temperature T
int CpuStage::sample_row(const float* lg, uint64_t salt, int row) {
  const int n = cfg_.vocab;
  if (temp_ <= 0.f) return (int)(std::max_element(lg, lg + n) - lg);
  std::vector<std::pair<float, int>> v(n);
  for (int i = 0; i < n; ++i) v[i] = {lg[i], i};
  std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first > b.first || (a.first == b.first && a.second < b.second); });
  int keep = (top_k_ > 0 && top_k_ < n) ? top_k_ : n;
  const float mx = v[0].first;
  std::vector<double> p1(keep);
  for (int i = 0; i < keep; ++i) p1[i] = std::exp((double)v[i].first - mx);
  if (top_p_ > 0.f && top_p_ < 1.f) {
    double tot = 0, c = 0;
    for (int i = 0; i < keep; ++i) tot += p1[i];
    int j = 0;
    while (j < keep) { c += p1[j++]; if (c >= top_p_ * tot) break; }
    keep = std::max(1, j);
  }
  if (min_p_ > 0) {
    int j = 0;
    while (j < keep && p1[j] >= min_p_) ++j;
    keep = std::max(1, j);
  }
  std::vector<double> p(keep);
  double sum = 0;
  for (int i = 0; i < keep; ++i) { p[i] = std::exp(((double)v[i].first - mx) / temp_); sum += p[i]; }
  const uint64_t r = mix64((seed_ ^ (salt * 0x9E3779B97F4A7C15ULL)) ^ mix64((step_ << 20) ^ (uint64_t)row));
  const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0) * sum;
  double c = 0;
  for (int i = 0; i < keep; ++i) {
    c += p[i];
    if (u < c) return v[i].second;
  }
  return v[keep - 1].second;
}

// KV of one slot: per layer, K rows then V rows [n_tok][kv_dim] f32 (gathered through the slot's
// block-table row)
size_t CpuStage::kv_state_bytes(int n_tok) const {
  return kc_.size() * 2 * (size_t)n_tok * cfg_.kv_dim() * 4;
}

size_t CpuStage::kv_row(int slot, int pos) const {
  return (size_t)bt_[(size_t)slot * max_pages_ + pos / 64] * 64 + pos % 64;
}

void CpuStage::set_block_table(const std::vector<int32_t>& t) {
  if (t.size() != bt_.size()) throw std::runtime_error("set_block_table: size mismatch");
  for (int32_t e : t)
    if (e < 0 || e > n_pages_) throw std::runtime_error("set_block_table: page id out of range");
  bt_ = t;
}

void CpuStage::kv_export(int slot, int n_tok, std::vector<uint8_t>& out) {
  const size_t row = (size_t)cfg_.kv_dim();
  for (size_t li = 0; li < kc_.size(); ++li)
    for (const auto* c : {&kc_[li], &vc_[li]})
      for (int t = 0; t < n_tok; ++t) {
        if (bt_[(size_t)slot * max_pages_ + t / 64] >= n_pages_) throw std::runtime_error("kv_export: unmapped page");
        const uint8_t* p = reinterpret_cast<const uint8_t*>(c->data() + kv_row(slot, t) * row);
        out.insert(out.end(), p, p + row * 4);
      }
}

void CpuStage::kv_import(int slot, int n_tok, const uint8_t* data, size_t bytes) {
  if (bytes != kv_state_bytes(n_tok)) throw std::runtime_error("kv_import: size mismatch");
  const size_t row = (size_t)cfg_.kv_dim();
  for (size_t li = 0; li < kc_.size(); ++li)
    for (auto* c : {&kc_[li], &vc_[li]})
      for (int t = 0; t < n_tok; ++t) {
        if (bt_[(size_t)slot * max_pages_ + t / 64] >= n_pages_) throw std::runtime_error("kv_import: unmapped page");
        std::memcpy(c->data() + kv_row(slot, t) * row, data, row * 4);
        data += row * 4;
      }
}

void CpuStage::set_history(int mb, const std::vector<std::vector<int32_t>>& seqs) {
  const int B = opt_.mb_size;
  if (hist_.empty()) hist_.resize((size_t)opt_.n_mb * B);
  for (int b = 0; b < B; ++b) {
    auto& h = hist_[(size_t)mb * B + b];
    h.clear();
    if (b < (int)seqs.size()) {
      const auto& q = seqs[b];
      const size_t take = std::min<size_t>(q.size(), (size_t)std::max(0, pen_last_n_));
      h.assign(q.end() - take, q.end());
    }
  }
}

void CpuStage::head(int mb, int M, const float* x, int32_t* tok_out, uint64_t salt) {
  rmsnorm(x, out_norm_, xn_.data(), M);
  matmul(out_, xn_.data(), cfg_.d_model, M, logits_.data(), cfg_.vocab, false);
  const bool pen = penalties_on();
  if (pen && hist_.empty()) hist_.resize((size_t)opt_.n_mb * opt_.mb_size);
  for (int m = 0; m < M; ++m) {
    float* lg = logits_.data() + (size_t)m * cfg_.vocab;
    std::vector<int32_t>* h = pen ? &hist_[(size_t)mb * opt_.mb_size + m] : nullptr;
    if (pen) {
      std::unordered_map<int32_t, int> cnt;
      for (int32_t t : *h) ++cnt[t];
      for (const auto& [t, c] : cnt) {
        if (t < 0 || t >= cfg_.vocab) continue;
        float l = lg[t];
        l = l > 0.f ? l / pen_repeat_ : l * pen_repeat_;
        lg[t] = l - (float)c * pen_freq_ - pen_presence_;
      }
    }
    tok_out[m] = sample_row(lg, salt, m);
    if (pen) {
      h->push_back(tok_out[m]);
      if ((int)h->size() > pen_last_n_) h->erase(h->begin());
    }
  }
}

void CpuStage::prefill(int mb, const std::vector<PrefillSeg>& segs, hipStream_t) {
  const int d = cfg_.d_model;
  float* x = act_[mb].data();
  std::vector<int32_t> pos, slot;
  for (const PrefillSeg& s : segs) {
    if (s.p0 + s.T > opt_.max_ctx) throw std::runtime_error("prompt exceeds context");
    const int sl = mb * opt_.mb_size + s.b;
    for (int t = 0; t < s.T; ++t) {
      const int row = (int)pos.size();
      pos.push_back(s.p0 + t);
      slot.push_back(sl);
      if (spec_.first()) {
        const int32_t tok = prompt_[(size_t)sl * opt_.max_ctx + s.p0 + t];
        if (tok < 0 || tok >= cfg_.vocab) throw std::runtime_error("token id out of range");
        dequant_row(embd_.type, embd_.data + (size_t)tok * embd_.rb, x + (size_t)row * d, d);
      }
    }
  }
  const int T = (int)pos.size();
  if (T > opt_.prefill_chunk) throw std::runtime_error("prefill chunk too large");
  // rows carry their own slot and position, so the packed chunk runs as one batch (the causal
  // mask per row is its position; other sequences' rows are in other slots)
  for (size_t li = 0; li < layers_.size(); ++li) layer_forward((int)li, T, x, pos.data(), slot.data());
  if (spec_.last() && !segs.empty() && segs[0].verify) {
    // speculative verification: greedy next token after every row of the chunk
    if (vtok_.size() < (size_t)opt_.n_mb) vtok_.resize(opt_.n_mb);
    std::vector<float> xn((size_t)T * d), lg((size_t)T * cfg_.vocab);
    rmsnorm(x, out_norm_, xn.data(), T);
    matmul(out_, xn.data(), d, T, lg.data(), cfg_.vocab, false);
    vtok_[mb].assign(T, 0);
    for (int m = 0; m < T; ++m) {
      const float* r = lg.data() + (size_t)m * cfg_.vocab;
      vtok_[mb][m] = (int32_t)(std::max_element(r, r + cfg_.vocab) - r);
    }
  } else if (spec_.last()) {
    int row = 0;
    for (const PrefillSeg& s : segs) {
      row += s.T;
      if (s.last) std::memcpy(last_h_[mb].data() + (size_t)s.b * d, x + (size_t)(row - 1) * d, (size_t)d * 4);
    }
  }
}

void CpuStage::copy_verify_tokens(int mb, int32_t* host, int n) {
  if ((size_t)mb >= vtok_.size() || (int)vtok_[mb].size() < n) throw std::runtime_error("no verify tokens");
  std::memcpy(host, vtok_[mb].data(), (size_t)n * 4);
}

void CpuStage::prefill_finish(int mb, hipStream_t, const std::vector<int>* rows) {
  if (!spec_.last()) return;
  if (!rows) {
    head(mb, opt_.mb_size, last_h_[mb].data(), tok_[mb].data(), 1000003ULL + (uint64_t)mb);
    return;
  }
  std::vector<int32_t> t(opt_.mb_size, 0);
  head(mb, opt_.mb_size, last_h_[mb].data(), t.data(), 1000003ULL + (uint64_t)mb);
  for (int b : *rows) tok_[mb][b] = t[b];
}

void CpuStage::decode(int mb, hipStream_t) {
  const int B = opt_.mb_size, d = cfg_.d_model;
  float* x = act_[mb].data();
  if (spec_.first())
    for (int b = 0; b < B; ++b) {
      const int32_t t = std::min(std::max(tok_[mb][b], 0), cfg_.vocab - 1);
      dequant_row(embd_.type, embd_.data + (size_t)t * embd_.rb, x + (size_t)b * d, d);
    }
  std::vector<int32_t> slot(B);
  for (int b = 0; b < B; ++b) slot[b] = mb * B + b;
  for (size_t li = 0; li < layers_.size(); ++li) layer_forward((int)li, B, x, pos_[mb].data(), slot.data());
  if (spec_.last()) head(mb, B, x, tok_[mb].data(), (uint64_t)mb + 1);
  for (int b = 0; b < B; ++b) pos_[mb][b] = std::min(pos_[mb][b] + 1, opt_.max_ctx - 1);
  if (mb == 0) ++step_;
}

}  // namespace mp
