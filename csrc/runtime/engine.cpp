#include "engine.h"
#include "probe.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <fstream>
#include <limits>
#include <map>
#include <sys/mman.h>
#include <unistd.h>
#include <sys/stat.h>
#include <numeric>
#include <stdexcept>

#include "cpu_stage.h"
#include "gguf.h"
#include "log.h"
#include "qtypes.h"

namespace mp {

namespace {
// host memory a CPU stage's KV pool may plan with: the "host_mem_gib" option, else MemAvailable from
// /proc/meminfo (physical pages as a fallback), instead of assuming a 64 GiB host
double host_mem_bytes(const Json& j) {
  const double opt = j.get_num("host_mem_gib", 0.0);
  if (opt > 0) return opt * (1 << 30);
  if (FILE* f = std::fopen("/proc/meminfo", "r")) {
    char key[64];
    long kb = 0;
    while (std::fscanf(f, "%63s %ld kB\n", key, &kb) == 2) {
      if (std::strcmp(key, "MemAvailable:") == 0) {
        std::fclose(f);
        return (double)kb * 1024.0;
      }
    }
    std::fclose(f);
  }
  const long pages = sysconf(_SC_PHYS_PAGES), psz = sysconf(_SC_PAGE_SIZE);
  return pages > 0 && psz > 0 ? (double)pages * (double)psz : 64.0 * (1 << 30);
}
}  // namespace

namespace {

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

ModelConfig config_from_json(const Json& j) {
  ModelConfig c;
  c.name = j.get_str("name", "synthetic");
  c.n_layer = j.get_int("n_layer", 0);
  c.d_model = j.get_int("d_model", 0);
  c.n_head = j.get_int("n_head", 0);
  c.n_head_kv = j.get_int("n_head_kv", c.n_head);
  c.d_ff = j.get_int("d_ff", 0);
  c.vocab = j.get_int("vocab", 32000);
  c.head_dim = j.get_int("head_dim", c.n_head ? c.d_model / c.n_head : 0);
  c.rope_base = (float)j.get_num("rope_base", 10000.0);
  c.eps = (float)j.get_num("eps", 1e-5);
  c.n_expert = j.get_int("n_expert", 0);
  c.n_expert_used = j.get_int("n_expert_used", 0);
  c.n_ctx_train = j.get_int("n_ctx_train", 2048);
  if (!c.n_layer || !c.d_model || !c.n_head || !c.d_ff) throw std::runtime_error("synthetic config incomplete");
  return c;
}

std::vector<uint8_t> unhex(const std::string& s) {
  std::vector<uint8_t> o(s.size() / 2);
  for (size_t i = 0; i < o.size(); ++i) o[i] = (uint8_t)std::stoi(s.substr(2 * i, 2), nullptr, 16);
  return o;
}

double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  const double idx = p * (v.size() - 1);
  const size_t i = (size_t)idx;
  const double f = idx - i;
  return i + 1 < v.size() ? v[i] * (1 - f) + v[i + 1] * f : v[i];
}

// decode-step bytes of one layer / the head (partition cost model: decode is HBM-bound)
double synth_layer_bytes(const ModelConfig& c, const std::string& ftype, int li) {
  const SyntheticTypes t = SyntheticTypes::from_ftype(ftype, li, c.n_layer);
  auto b = [](int ty, double n, double k) { return n * k * block_bytes(ty) / block_elems(ty); };
  const double d = c.d_model, q = c.q_dim(), kv = c.kv_dim(), f = c.d_ff;
  const double ffn = b(t.gate, f, d) + b(t.up, f, d) + b(t.down, d, f);
  return b(t.q, q, d) + b(t.k, kv, d) + b(t.v, kv, d) + b(t.o, d, q) + ffn * std::max(1, c.n_expert);
}

// int8_gemm (HipStage::build_i8_copies): an int8 copy of every quantized non-MoE projection, one
// byte per weight of the 16-row x 256-k padded packing plus a float row scale.  These bytes live
// next to the weights, so the KV budget and the --gpu-mem check must see them.
double i8_copy_bytes(int t, int64_t n, int64_t k) {
  if (t == T_F32 || t == T_F16 || t == T_BF16) return 0;
  const double np = (double)((n + 15) / 16 * 16), kp = (double)((k + 255) / 256 * 256);
  return np * kp + np * 4;
}

double synth_layer_i8_bytes(const ModelConfig& c, const std::string& ftype, int li) {
  if (c.n_expert > 0) return 0;   // MoE experts keep their own kernels (no copy)
  const SyntheticTypes t = SyntheticTypes::from_ftype(ftype, li, c.n_layer);
  const int64_t d = c.d_model, q = c.q_dim(), kv = c.kv_dim(), f = c.d_ff;
  return i8_copy_bytes(t.q, q, d) + i8_copy_bytes(t.k, kv, d) + i8_copy_bytes(t.v, kv, d) + i8_copy_bytes(t.o, d, q) +
         i8_copy_bytes(t.gate, f, d) + i8_copy_bytes(t.up, f, d) + i8_copy_bytes(t.down, d, f);
}

double gguf_layer_i8_bytes(const GgufFile& g, int li) {
  double b = 0;
  const std::string p = "blk." + std::to_string(li) + ".";
  if (g.tensor(p + "ffn_gate_inp.weight")) return 0;   // MoE layer: build_i8_copies skips it whole
  for (const char* nm : {"attn_q", "attn_k", "attn_v", "attn_output", "ffn_gate", "ffn_up", "ffn_down"}) {
    const GgufTensor* t = g.tensor(p + nm + ".weight");
    if (t && t->ne.size() >= 2) b += i8_copy_bytes(t->type, t->ne[1], t->ne[0]);
  }
  return b;
}

}  // namespace

Engine::Engine(const Json& j) : jcfg_(j) {
  const double t0 = now_ms();
  if (j.get_bool("verbose", false)) log_set_level(LOG_DEBUG);
  if (j.has("log_file")) log_set_file(j.get_str("log_file", ""));
  mode_ = j.get_str("mode", "local");
  cpu_ = j.get_str("backend", "hip") == "cpu";
  watchdog_s_ = j.get_num("watchdog_s", 600.0);
  if (j.has("fault")) fault_ = j["fault"];
  else if (const char* fe = std::getenv("MIPIPE_FAULT")) fault_ = Json::parse(fe);
  if (j.get_bool("trace", false)) enable_trace(true);
  M_ = std::max(1, j.get_int("n_mb", 1));
  B_ = std::max(1, j.get_int("mb_size", 1));
  // > 64 rows per micro-batch: the decode projections run on the prompt GEMM (gemm2, 128 rows per
  // workgroup), which turns the M = 64 GEMV's exposed MFMA issue into a throughput-bound GEMM
  if (B_ > 1024) throw std::runtime_error("mb_size > 1024 not supported");
  // max_ctx 0 or "auto": sized from HBM capacity after partitioning (below)
  const bool auto_ctx = (j.has("max_ctx") && j["max_ctx"].is_str() && j["max_ctx"].str() == "auto") ||
                        (j.has("max_ctx") && j["max_ctx"].is_num() && j["max_ctx"].num() == 0);
  max_ctx_ = auto_ctx ? 2048 : (int)round_up(std::max(64, j.get_int("max_ctx", 2048)), 64);
  chunk_ = std::max(16, j.get_int("prefill_chunk", 512));
  const std::string ftype = j.get_str("ftype", "Q4_K_M");
  const uint64_t seed = (uint64_t)j.get_num("seed", 1234);

  std::vector<double> layer_cost;
  std::vector<double> layer_extra;   // HBM bytes per layer beyond its weights (int8_gemm copies)
  const bool i8_copies = j.get_bool("int8_gemm", false) && j.get_bool("prefill_gemm", true) &&
                         j.get_str("backend", "hip") != "cpu";
  double head_cost = 0, embd_cost = 0;
  if (j.has("gguf")) {
    gguf_.reset(new GgufFile(j.get_str("gguf", "")));
    cfg_ = ModelConfig::from_gguf(*gguf_);
    for (int li = 0; li < cfg_.n_layer; ++li) {
      double bytes = 0;
      const std::string p = "blk." + std::to_string(li) + ".";
      for (auto& t : gguf_->tensors())
        if (t.name.compare(0, p.size(), p) == 0) bytes += (double)t.nbytes;
      layer_cost.push_back(bytes);
      layer_extra.push_back(i8_copies ? gguf_layer_i8_bytes(*gguf_, li) : 0.0);
    }
    const GgufTensor* out = gguf_->tensor("output.weight");
    head_cost = (double)(out ? out->nbytes : gguf_->tensor("token_embd.weight")->nbytes);
  } else if (j.has("synthetic")) {
    cfg_ = config_from_json(j["synthetic"]);
    for (int li = 0; li < cfg_.n_layer; ++li) {
      layer_cost.push_back(synth_layer_bytes(cfg_, ftype, li));
      layer_extra.push_back(i8_copies ? synth_layer_i8_bytes(cfg_, ftype, li) : 0.0);
    }
    const SyntheticTypes t = SyntheticTypes::from_ftype(ftype, 0, cfg_.n_layer);
    head_cost = (double)cfg_.vocab * cfg_.d_model * block_bytes(t.out) / block_elems(t.out);
  } else {
    throw std::runtime_error("engine config needs 'gguf' or 'synthetic'");
  }
  MP_LOGI("model: %s", cfg_.describe().c_str());

  // ---- partition
  if (mode_ == "mp") {
    S_ = j.get_int("world", 1);
    rank_ = j.get_int("rank", 0);
  } else {
    S_ = std::max(1, j.get_int("stages", 1));
  }
  // gpu_layers (llama-cli -ngl N, n_gpu_layers) below the layer count: like llama.cpp, the LAST N
  // layers (and the head) are offloaded -- to the `stages` GPU stages, partitioned as usual -- and
  // the first n_layer - N layers with the embedding run on a CPU stage in front of them (one more
  // stage; host links on both of its ends).  N <= 0 keeps the engine-wide backend, N >= n_layer
  // is the all-GPU engine (the reference's -ngl 99).
  const int ngl = j.get_int("gpu_layers", -1);
  hybrid_ = !cpu_ && ngl > 0 && ngl < cfg_.n_layer;
  if (hybrid_ && mode_ == "mp") throw std::runtime_error("gpu_layers < n_layer (hybrid CPU/GPU split) needs mode local");
  const int S_gpu = S_;
  if (hybrid_) S_ = S_gpu + 1;
  const int g0 = hybrid_ ? 1 : 0;   // first GPU stage
  // default prompt chunk: 2048 rows for a single GPU stage (the 128-row GEMM tiles then run 16 row
  // blocks per weight tile group: 8B 41.6k -> 59.0k, 70B 6.3k -> 6.9k prompt tok/s at 64 x 512
  // prompts), 512 when stages pipeline the chunks (finer chunks overlap the stages) or on CPU
  if (!j.has("prefill_chunk")) chunk_ = (S_ == 1 && j.get_str("backend", "hip") != "cpu") ? 2048 : 512;
  // KV cache element type: "f16" (default) or "fp8" (OCP e4m3 bytes: half the KV bytes per decode
  // step and twice the tokens per GiB; HIP backend, fused decode + flash prefill attention)
  const std::string kv_dtype = j.get_str("kv_dtype", "f16");
  if (kv_dtype != "f16" && kv_dtype != "fp8") throw std::runtime_error("kv_dtype must be f16 or fp8");
  const bool kv_fp8 = kv_dtype == "fp8";
  kv_fp8_ = kv_fp8;
  if (kv_fp8 && (j.get_str("backend", "hip") == "cpu" || !j.get_bool("fused_attn", true) || !j.get_bool("prefill_flash", true)))
    throw std::runtime_error("kv_dtype fp8 needs the HIP backend with fused_attn and prefill_flash");
  // devices of the GPU stages (a hybrid split's CPU stage 0 carries the first GPU's id, unused)
  std::vector<int> devices(S_);
  for (int s = g0; s < S_; ++s) devices[s] = s - g0;
  if (j.has("devices")) {
    auto& a = j["devices"].arr();
    for (int s = g0; s < S_; ++s) devices[s] = (int)a[(s - g0) % a.size()].num();
  }
  if (hybrid_) devices[0] = devices[1];
  if (mode_ == "mp") devices[rank_] = j.get_int("device", devices[rank_]);
  // per-stage speed for the cost partitioner: given (device_speed: [..]), or measured
  // (device_speed: "probe", Halda-style; mp mode: every rank must pass the same list, which
  // mipipe.parallel.init_from_torchrun(device_speed="probe") gathers over torch.distributed)
  // (hybrid: the speeds of the GPU stages, which split the offloaded layers among themselves)
  std::vector<double> speed(S_gpu, 1.0);
  if (j.has("device_speed") && j["device_speed"].is_str()) {
    if (j["device_speed"].str() != "probe") throw std::runtime_error("device_speed: a list or \"probe\"");
    if (mode_ == "mp") throw std::runtime_error("device_speed probe in mp mode: gather the list across ranks first");
    std::map<int, DeviceProfile> seen;
    for (int s = 0; s < S_gpu; ++s) {
      const int dv = devices[s + g0];
      if (!seen.count(dv)) seen[dv] = cpu_ ? probe_host() : probe_device(dv);
      speed[s] = seen[dv].speed();
    }
    // stages sharing one device (single-GPU emulation) split its speed
    std::map<int, int> share;
    for (int s = 0; s < S_gpu; ++s) share[devices[s + g0]]++;
    for (int s = 0; s < S_gpu; ++s) speed[s] /= share[devices[s + g0]];
  } else if (j.has("device_speed")) {
    for (int s = 0; s < S_gpu && s < (int)j["device_speed"].arr().size(); ++s) speed[s] = j["device_speed"].arr()[s].num();
  }
  device_speed_ = speed;
  const SplitMode split_mode = parse_split_mode(j.get_str("split", "cost"));
  if (hybrid_) {
    const int Lc = cfg_.n_layer - ngl;   // layers kept on the CPU
    std::vector<double> gcost(layer_cost.begin() + Lc, layer_cost.end());
    std::vector<StageSpec> g = partition_layers(gcost, 0.0, head_cost, speed, split_mode);
    StageSpec c;
    c.stage = 0; c.n_stages = S_; c.layer_begin = 0; c.layer_end = Lc;
    specs_.assign(1, c);
    for (StageSpec sp : g) {
      sp.stage += 1; sp.n_stages = S_; sp.layer_begin += Lc; sp.layer_end += Lc;
      specs_.push_back(sp);
    }
  } else {
    specs_ = partition_layers(layer_cost, embd_cost, head_cost, speed, split_mode);
  }
  for (int s = 0; s < S_; ++s) specs_[s].device = devices[s];
  // --gpu-mem (prima.cpp): per-GPU memory budget in GiB; caps the auto KV sizing and
  // is checked against every stage's weights + KV below (--force downgrades the failure to a warning)
  const double gpu_mem = j.get_num("gpu_mem_gib", 0.0) * 1073741824.0;
  if (auto_ctx) {
    // KV sized from HBM (288 GB per MI355X): every rank derives the same value from
    // the partition and the device capacity alone (no exchange needed in mp mode): the heaviest
    // stage's weights (+ embedding on stage 0, head on the last) and the most layers per stage
    // bound the per-slot context; kv_frac of the card, minus a reserve for activations/scratch.
    const double frac = j.get_num("kv_frac", 0.9);
    double cap_bytes = 64.0 * (1 << 30);   // CPU backend: 64 GiB
    if (!cpu_) {
      size_t fr = 0, tot = 0;
      HIP_OK(hipSetDevice(devices[mode_ == "mp" ? rank_ : 0]));
      HIP_OK(hipMemGetInfo(&fr, &tot));
      cap_bytes = (double)tot;
    }
    if (gpu_mem > 0) cap_bytes = std::min(cap_bytes, gpu_mem);
    const double embd_bytes = gguf_ && gguf_->tensor("token_embd.weight")
                                  ? (double)gguf_->tensor("token_embd.weight")->nbytes : head_cost;
    // stages sharing a GPU (single-GPU PP emulation, devices 0,0,..) share its memory: size from
    // the device carrying the most layers / weights, summed over its stages (mp mode: one GPU per
    // rank, every rank derives the same value)
    std::map<int, double> dev_w;
    std::map<int, int> dev_l, dev_n;
    for (auto& sp : specs_) {
      double w = 0;
      for (int li = sp.layer_begin; li < sp.layer_end; ++li) w += layer_cost[li] + layer_extra[li];
      if (sp.first()) w += embd_bytes;
      if (sp.last()) w += head_cost;
      const int key = stage_cpu(sp.stage) && hybrid_ ? -1 : mode_ == "mp" ? sp.stage : devices[sp.stage];   // -1: host
      dev_w[key] += w;
      dev_l[key] += sp.layer_end - sp.layer_begin;
      dev_n[key] += 1;
    }
    long ctx = std::numeric_limits<long>::max();
    double per_tok = 0;
    int lmax = 1;
    for (auto& e : dev_w) {
      const bool host = cpu_ || e.first == -1;   // CPU stages: f32 KV in host memory
      const int layers = std::max(1, dev_l[e.first]);
      const double pt = (double)layers * 2.0 * cfg_.n_head_kv * cfg_.padded_head_dim() * (host ? 4.0 : kv_fp8 ? 1.0 : 2.0);
      const double reserve =
          dev_n[e.first] * (4.0 * (1 << 30) + (double)M_ * std::max(chunk_, B_) * cfg_.d_model * 4.0 * 4);
      const double budget = frac * (host ? host_mem_bytes(j) : cap_bytes) - e.second - reserve;
      // paged KV: the pool holds the LIVE tokens of all slots (not n_slots x max_ctx)
      const long c = budget > 0 ? (long)(budget / pt) : 0;
      if (c < ctx) { ctx = c; per_tok = pt; lmax = layers; }
    }
    if (ctx < 64) throw std::runtime_error("max_ctx auto: no HBM left for the KV cache");
    kv_pages_ = (int)std::min<long>(ctx / 64, std::numeric_limits<int>::max() / 64);
    const long train = cfg_.n_ctx_train > 0 ? cfg_.n_ctx_train : 131072;
    const long per_seq = std::min((long)kv_pages_ * 64, std::min(train, (long)j.get_int("max_ctx_cap", 1 << 20)));
    max_ctx_ = (int)(per_seq / 64 * 64);
    MP_LOGI("max_ctx auto: KV pool of %d pages (%ld tokens, %.1f GiB on the GPU holding %d layers; device %.0f GiB) "
            "shared by %d slots, up to %d tokens per sequence",
            kv_pages_, (long)kv_pages_ * 64, per_tok * kv_pages_ * 64 / 1073741824.0, lmax, cap_bytes / 1073741824.0,
            M_ * B_, max_ctx_);
  } else {
    // explicit pool (kv_pool_tokens; e.g. oversubscribed slots), else every slot can hold max_ctx
    const long pool = j.get_int("kv_pool_tokens", 0);
    kv_pages_ = pool > 0 ? (int)((pool + 63) / 64) : M_ * B_ * (max_ctx_ / 64);
  }
  for (auto& sp : specs_)
    MP_LOGI("partition: stage %d <- layers [%d, %d) (%d layers)%s%s", sp.stage, sp.layer_begin, sp.layer_end,
            sp.layer_end - sp.layer_begin, sp.first() ? " +embd" : "", sp.last() ? " +head" : "");

  if (gpu_mem > 0) {
    // --gpu-mem is per GPU: add up weights + KV of every stage this process places on a device
    const double embd_b = gguf_ && gguf_->tensor("token_embd.weight")
                              ? (double)gguf_->tensor("token_embd.weight")->nbytes : head_cost;
    std::map<int, std::pair<double, double>> need;   // device -> (weights, kv)
    std::map<int, std::string> who;
    for (auto& sp : specs_) {
      if ((mode_ == "mp" && sp.stage != rank_) || (hybrid_ && stage_cpu(sp.stage))) continue;   // per GPU
      double w = 0;
      for (int li = sp.layer_begin; li < sp.layer_end; ++li) w += layer_cost[li] + layer_extra[li];
      if (sp.first()) w += embd_b;
      if (sp.last()) w += head_cost;
      const double kv = (double)(sp.layer_end - sp.layer_begin) * 2.0 * cfg_.n_head_kv * cfg_.padded_head_dim() *
                        (cpu_ ? 4.0 : kv_fp8 ? 1.0 : 2.0) * ((double)kv_pages_ + 1) * 64;
      auto& e = need[devices[sp.stage]];
      e.first += w;
      e.second += kv;
      std::string& ws = who[devices[sp.stage]];
      ws += (ws.empty() ? "" : ",") + std::to_string(sp.stage);
    }
    for (auto& e : need) {
      const double w = e.second.first, k = e.second.second;
      if (w + k > gpu_mem) {
        char msg[320];
        snprintf(msg, sizeof msg,
                 "GPU %d (stage %s) needs %.3f MiB (weights %.3f + KV %.3f) > --gpu-mem %.3f MiB",
                 e.first, who[e.first].c_str(), (w + k) / 1048576.0, w / 1048576.0, k / 1048576.0,
                 gpu_mem / 1048576.0);
        if (!j.get_bool("force", false)) throw std::runtime_error(std::string(msg) + " (use --force to proceed)");
        MP_LOGW("%s; --force: proceeding", msg);
      }
    }
  }
  // --prefetch: ask the kernel to read ahead the mmap'd GGUF ranges of the layers this
  // process uploads, so page-in overlaps the partition / allocation work instead of the upload loop
  if (gguf_ && j.get_bool("prefetch", false)) {
    const long pg = sysconf(_SC_PAGESIZE);
    size_t advised = 0;
    for (auto& t : gguf_->tensors()) {
      int li = -1;
      if (t.name.compare(0, 4, "blk.") == 0) li = std::atoi(t.name.c_str() + 4);
      bool mine = mode_ != "mp";
      for (auto& sp : specs_)
        if (sp.stage == rank_ || mode_ != "mp")
          mine = mine || (li >= 0 ? li >= sp.layer_begin && li < sp.layer_end : sp.first() || sp.last());
      if (!mine || !t.nbytes) continue;
      const uintptr_t a = (uintptr_t)t.data & ~(uintptr_t)(pg - 1);
      if (madvise((void*)a, (uintptr_t)t.data + t.nbytes - a, MADV_WILLNEED) == 0) advised += t.nbytes;
    }
    MP_LOGI("prefetch: madvise(WILLNEED) on %.2f GiB of GGUF tensor data", advised / 1073741824.0);
  }

  StageOptions so;
  so.n_mb = M_;
  so.mb_size = B_;
  so.max_ctx = max_ctx_;
  so.kv_pages = kv_pages_;
  so.prefill_chunk = chunk_;
  so.use_graphs = j.get_bool("graphs", true);
  so.attn_split_len = j.get_int("attn_split_len", 0);   // 0 = auto
  so.threads = j.get_int("threads", 0);
  {
    const std::string ca = j.get_str("cpu_act", "q8");
    if (ca != "q8" && ca != "f32") throw std::runtime_error("cpu_act must be q8 or f32");
    so.cpu_q8 = ca == "q8";
  }
  so.fused_attn = j.get_bool("fused_attn", true);
  so.attn_o_max_ctx = j.get_int("attn_o_max_ctx", 512);   // r11g: 8B mb1 attention + o 15.6 -> 12.4 us/layer
  so.prefill_gemm = j.get_bool("prefill_gemm", true);
  so.prefill_gemm_v = j.get_int("prefill_gemm_v", 0);
  so.gemm_splitk_store = j.get_bool("gemm_splitk_store", true);
  so.int8_gemm = j.get_bool("int8_gemm", false);
  so.deterministic = j.get_bool("deterministic", false);
  so.prefill_flash = j.get_bool("prefill_flash", true);
  so.kv_fp8 = j.get_str("kv_dtype", "f16") == "fp8";
  so.fused_norm = j.get_bool("fused_norm", false) && !so.deterministic;   // its sums of squares are atomics
  so.small_gemv = j.get_bool("small_gemv", true);
  so.moe_gemm = j.get_bool("moe_gemm", true);
  packed_prefill_ = j.get_bool("packed_prefill", true);
  prefix_cache_ = j.get_bool("prefix_cache", true);

  // ---- stages this process owns
  for (int s = 0; s < S_; ++s) {
    if (mode_ == "mp" && s != rank_) continue;
    auto w = std::make_unique<Worker>();
    w->device = specs_[s].device;
    w->cpu = stage_cpu(s);
    if (w->cpu) {
      w->stage.reset(new CpuStage(cfg_, specs_[s], so));
    } else {
      HIP_OK(hipSetDevice(w->device));
      w->stage.reset(new HipStage(cfg_, specs_[s], so));
    }
    if (gguf_) w->stage->load_gguf(*gguf_);
    else w->stage->init_synthetic(ftype, seed);
    w->stage->alloc_runtime();
    w->stage->set_sampling((float)j.get_num("temp", 0.0), j.get_int("top_k", 0), (float)j.get_num("top_p", 1.0),
                           (float)j.get_num("min_p", 0.0), seed);
    w->stage->set_penalties(j.get_int("repeat_last_n", 64), (float)j.get_num("repeat_penalty", 1.0),
                            (float)j.get_num("frequency_penalty", 0.0), (float)j.get_num("presence_penalty", 0.0));
    if (w->cpu) {
      w->ring_pending.assign(M_, false);
      workers_.push_back(std::move(w));
      continue;
    }
    HIP_OK(hipStreamCreateWithFlags(&w->send_st, hipStreamNonBlocking));
    HIP_OK(hipStreamCreateWithFlags(&w->recv_st, hipStreamNonBlocking));
    w->comp_ev.resize(M_); w->sent_ev.resize(M_); w->recv_ev.resize(M_);
    w->sent_valid.assign(M_, false);
    w->sent_seq.assign(M_, 0);
    for (int mb = 0; mb < M_; ++mb) {
      HIP_OK(hipEventCreateWithFlags(&w->comp_ev[mb], hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&w->sent_ev[mb], hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&w->recv_ev[mb], hipEventDisableTiming));
    }
    workers_.push_back(std::move(w));
  }
  build_links(j);
  for (auto& l : links_) l->set_timeout(j.get_num("link_timeout_s", 600.0));
  // Stage-boundary wire format: the residual stream is f32 inside a stage; between
  // GPUs it travels as bf16 by default (half the xGMI bytes: 16 KiB per 70B token) over RCCL and
  // over peer-copy LocalLinks, f32 elsewhere (same-GPU LocalLink emulation and TCP keep PP=S
  // bitwise equal to PP=1).  Every rank derives the same choice from the shared config.
  {
    const std::string ad = j.get_str("act_dtype", "auto");
    const std::string lk = S_ > 1 ? std::string(links_.empty() ? "none" : links_.front()->kind()) : "none";
    bool cross_gpu = false;
    for (auto& l : links_)
      if (auto* ll = dynamic_cast<LocalLink*>(l.get())) cross_gpu = cross_gpu || ll->peer();
    if (ad == "auto") act_dtype_ = (!cpu_ && (lk == "rccl" || cross_gpu)) ? ACT_BF16 : ACT_F32;
    else if (ad == "f32") act_dtype_ = ACT_F32;
    else if (ad == "f16") act_dtype_ = ACT_F16;
    else if (ad == "bf16") act_dtype_ = ACT_BF16;
    else throw std::runtime_error("act_dtype must be auto, f32, f16 or bf16");
    if (cpu_ || hybrid_) act_dtype_ = ACT_F32;   // host links carry the f32 residual
    if (act_dtype_ != ACT_F32 && S_ > 1) {
      const size_t wb = (size_t)std::max(chunk_, B_) * cfg_.d_model * 2;
      for (auto& w : workers_) {
        HIP_OK(hipSetDevice(w->device));
        for (int mb = 0; mb < M_; ++mb) {
          void *o = nullptr, *i = nullptr;
          HIP_OK(hipMalloc(&o, wb));
          HIP_OK(hipMalloc(&i, wb));
          w->wire_out.push_back(o);
          w->wire_in.push_back(i);
        }
      }
    }
    if (S_ > 1)
      MP_LOGI("stage boundary: %s activations, %.1f KiB per token", act_dtype_ == ACT_F32 ? "f32" : act_dtype_ == ACT_F16 ? "f16" : "bf16",
              cfg_.d_model * (act_dtype_ == ACT_F32 ? 4 : 2) / 1024.0);
  }
  pager_.init(M_ * B_, max_ctx_ / 64, kv_pages_);
  kv_sync();
  rounds_cap_ = max_ctx_ + 2;
  if (cpu_) {
    out_vec_.resize((size_t)rounds_cap_ * M_ * B_);
    out_host_ = out_vec_.data();
  } else {
    for (auto& w : workers_) {
      if (w->cpu) continue;
      HIP_OK(hipSetDevice(w->device));
      w->stage->capture_graphs();
    }
    HIP_OK(hipHostMalloc((void**)&out_host_, (size_t)rounds_cap_ * M_ * B_ * 4, hipHostMallocDefault));
  }
  std::memset(out_host_, 0xff, (size_t)rounds_cap_ * M_ * B_ * 4);
  load_ms_ = now_ms() - t0;
  MP_LOGI("engine ready: %d stage(s), %d micro-batch(es) x %d seq, ctx %d, load %.1f ms", S_, M_, B_, max_ctx_,
          load_ms_);
}

Engine::~Engine() {
  try {
    sync_all();
  } catch (...) {
  }
  for (auto& w : workers_) {
    if (w->cpu) {
      w->stage.reset();
      continue;
    }
    (void)hipSetDevice(w->device);
    if (bcast_dev_ && w.get() == workers_[0].get()) (void)hipFree(bcast_dev_);
    for (void* p : w->wire_out) (void)hipFree(p);
    for (void* p : w->wire_in) (void)hipFree(p);
    for (auto e : w->comp_ev) (void)hipEventDestroy(e);
    for (auto e : w->sent_ev) (void)hipEventDestroy(e);
    for (auto e : w->recv_ev) (void)hipEventDestroy(e);
    for (auto e : w->tok_ev) (void)hipEventDestroy(e);
    w->stage.reset();
    (void)hipStreamDestroy(w->send_st);
    (void)hipStreamDestroy(w->recv_st);
  }
  links_.clear();
  if (out_host_ && !cpu_) (void)hipHostFree(out_host_);
}

bool Engine::owns_last() const {
  for (auto& w : workers_) if (w->stage->spec().last()) return true;
  return false;
}
bool Engine::owns_first() const {
  for (auto& w : workers_) if (w->stage->spec().first()) return true;
  return false;
}

void Engine::build_links(const Json& j) {
  if (S_ == 1) return;
  // link i: stage i -> stage (i+1) % S (link S-1 is the token ring back to stage 0)
  if (mode_ == "local") {
    // "rccl": one 2-rank communicator per link direction from ncclCommInitAll (in-process, one host
    // thread per GPU).  RCCL refuses a communicator with two ranks on one GPU, and may be unusable
    // on a box; then the link falls back to the peer-copy LocalLink and says so (info()["links"]).
    // "auto": rccl when every stage has its own GPU, local otherwise.
    // (a hybrid split: host links everywhere; the GPU ends copy through host memory)
    std::string kind = cpu_ || hybrid_ ? "host" : j.get_str("link", "local");
    if (kind == "auto") {
      std::vector<int> d;
      for (auto& sp : specs_) d.push_back(sp.device);
      std::sort(d.begin(), d.end());
      kind = std::unique(d.begin(), d.end()) == d.end() ? "rccl" : "local";
    }
    for (int i = 0; i < S_; ++i) {
      const int a = i, b = (i + 1) % S_;
      if (kind == "host") {
        links_.emplace_back(new HostLink(std::max(4, M_ + 2)));
        workers_[a]->out = links_.back().get();
        workers_[b]->in = links_.back().get();
        continue;
      }
      if (kind == "rccl") {
        void *ca = nullptr, *cb = nullptr;
        try {
          rccl_make_pair(specs_[a].device, specs_[b].device, &ca, &cb);
        } catch (const std::exception& e) {
          link_fallback_ = std::string("rccl -> local: ") + e.what();
          MP_LOGW("link %d (GPU %d -> GPU %d): %s", i, specs_[a].device, specs_[b].device, link_fallback_.c_str());
          kind = "local";
        }
        if (kind == "rccl") {
          links_.emplace_back(new RcclLink(ca, 0, 1, specs_[a].device));   // sender end (rank 0 -> 1)
          Link* snd = links_.back().get();
          links_.emplace_back(new RcclLink(cb, 1, 0, specs_[b].device));   // receiver end
          Link* rcv = links_.back().get();
          workers_[a]->out = snd;
          workers_[b]->in = rcv;
          continue;
        }
      }
      links_.emplace_back(new LocalLink(specs_[a].device, specs_[b].device));
      workers_[a]->out = links_.back().get();
      workers_[b]->in = links_.back().get();
    }
    if (kind == "local" && !link_fallback_.empty()) {
      // a partial RCCL ring mixed with local links would be valid, but keep one transport per ring
      for (int i = 0; i < S_; ++i) {
        Link* o = workers_[i]->out;
        if (std::string(o->kind()) != "rccl") continue;
        links_.emplace_back(new LocalLink(specs_[i].device, specs_[(i + 1) % S_].device));
        workers_[i]->out = workers_[(i + 1) % S_]->in = links_.back().get();
      }
      std::vector<std::unique_ptr<Link>> keep;
      for (auto& l : links_)
        if (std::string(l->kind()) != "rccl") keep.push_back(std::move(l));
      links_ = std::move(keep);
    }
    MP_LOGI("links: %d x %s (token ring %d B per sequence)", S_, kind.c_str(), 4);
  } else if (cpu_ || j.get_str("link", "rccl") == "tcp") {
    // one TCP connection per link: receiver of link l (rank l+1) listens on base_port + l,
    // sender (rank l) connects to hosts[l+1].  Accept runs on a helper thread so the ring cannot
    // deadlock on connection order.
    const int base = j.get_int("base_port", 29600);
    std::vector<std::string> hosts(S_, "127.0.0.1");
    if (j.has("hosts"))
      for (int r = 0; r < S_ && r < (int)j["hosts"].arr().size(); ++r) hosts[r] = j["hosts"].arr()[r].str();
    if (j.has("next_host")) hosts[(rank_ + 1) % S_] = j.get_str("next_host", "127.0.0.1");   // prima.cpp --next
    const double to = j.get_num("connect_timeout", 120.0);
    const int in_l = (rank_ - 1 + S_) % S_, out_l = rank_;
    Worker& w = *workers_[0];
    std::unique_ptr<TcpLink> rx;
    std::exception_ptr err;
    std::thread acc([&] {
      try {
        rx = TcpLink::make_receiver(base + in_l, to);
      } catch (...) {
        err = std::current_exception();
      }
    });
    std::unique_ptr<TcpLink> tx;
    try {
      tx = TcpLink::make_sender(hosts[(rank_ + 1) % S_], base + out_l, to);
    } catch (...) {
      acc.join();
      throw;
    }
    acc.join();
    if (err) std::rethrow_exception(err);
    w.in = rx.get();
    w.out = tx.get();
    links_.emplace_back(std::move(rx));
    links_.emplace_back(std::move(tx));
    MP_LOGI("rank %d: TCP links in=%d (port %d) out=%d -> %s:%d", rank_, in_l, base + in_l, out_l,
            hosts[(rank_ + 1) % S_].c_str(), base + out_l);
  } else {
    const auto& ids = j["rccl_ids"].arr();
    if ((int)ids.size() != S_) throw std::runtime_error("mp mode needs one RCCL id per link");
    const int in_l = (rank_ - 1 + S_) % S_, out_l = rank_;
    Worker& w = *workers_[0];
    for (int l : {std::min(in_l, out_l), std::max(in_l, out_l)}) {
      auto id = unhex(ids[l].str());
      const bool sender = (l == out_l);
      // a 2-rank communicator per link direction (rank 0 sends, rank 1 receives): every link is
      // its own FIFO, so the ring cannot deadlock on RCCL's per-communicator ordering
      void* c = rccl_init_rank(id.data(), 2, sender ? 0 : 1, w.device);
      links_.emplace_back(new RcclLink(c, sender ? 0 : 1, sender ? 1 : 0, w.device));
      if (sender) w.out = links_.back().get();
      else w.in = links_.back().get();
    }
    MP_LOGI("rank %d: RCCL links in=%d out=%d on GPU %d", rank_, in_l, out_l, w.device);
  }
}

void Engine::post_ring_recv(Worker& w, int mb) {
  Stage& st = *w.stage;
  HIP_OK(hipEventRecord(w.comp_ev[mb], st.stream()));
  HIP_OK(hipStreamWaitEvent(w.recv_st, w.comp_ev[mb], 0));
  w.in->recv(st.tokens(mb), (size_t)B_ * 4, w.recv_st);
  HIP_OK(hipEventRecord(w.recv_ev[mb], w.recv_st));
}

// Fault injection: config "fault" (or env MIPIPE_FAULT, same JSON) =
//   {"stage": k, "delay_ms": d}          sleep d ms before every item of stage k
//   {"stage": k, "fail_at": n}           throw at the n-th item stage k runs
//   {"stage": k, "drop_send_at": n}      silently skip the n-th send of stage k (peer stalls ->
//                                        the watchdog / link timeouts must surface it)
bool Engine::fault_hook(Worker& w, const char* what) {
  if (!fault_.is_obj() || fault_.get_int("stage", -1) != w.stage->spec().stage) return false;
  const long n = w.items_seen;
  if (fault_.has("delay_ms")) std::this_thread::sleep_for(std::chrono::microseconds((long)(1000 * fault_.get_num("delay_ms", 0))));
  if (std::strcmp(what, "item") == 0 && fault_.get_int("fail_at", -1) == n)
    throw std::runtime_error("injected fault at item " + std::to_string(n) + " of stage " + std::to_string(w.stage->spec().stage));
  if (std::strcmp(what, "send") == 0 && fault_.get_int("drop_send_at", -1) == w.sends_seen++) {
    MP_LOGW("fault injection: dropping send %ld of stage %d", w.sends_seen - 1, w.stage->spec().stage);
    return true;
  }
  return false;
}

// timeline span (Chrome trace, --trace): HIP events on stream s, or host time for CPU stages
void Engine::span(Worker& w, hipStream_t s, int tid, const std::string& name, const std::function<void()>& body) {
  if (!trace_) return body();
  Worker::TraceRecT r;
  r.name = name;
  r.tid = tid;
  if (w.cpu) {
    r.ta = now_ms();
    body();
    r.tb = now_ms();
  } else {
    HIP_OK(hipEventCreate(&r.a));
    HIP_OK(hipEventRecord(r.a, s));
    body();
    HIP_OK(hipEventCreate(&r.b));
    HIP_OK(hipEventRecord(r.b, s));
  }
  w.tr.push_back(r);
}

// CPU stages: the same item schedule, blocking host transfers.  The first stage receives the
// ring token of micro-batch mb lazily (right before its next DECODE) and drains the ring at the
// end of the item list, like the GPU path's posted ring receives.
void Engine::run_items_cpu(Worker& w, const std::vector<Item>& items) {
  Stage& st = *w.stage;
  const bool first = st.spec().first(), last = st.spec().last();
  const size_t d4 = (size_t)cfg_.d_model * 4;
  auto recv = [&](int mb, void* buf, size_t bytes, const char* what) {
    span(w, nullptr, 2, std::string("recv ") + what + " mb" + std::to_string(mb), [&] { w.in->recv(buf, bytes, nullptr); });
  };
  auto send = [&](int mb, const void* buf, size_t bytes, const char* what) {
    if (fault_hook(w, "send")) return;
    span(w, nullptr, 1, std::string("send ") + what + " mb" + std::to_string(mb), [&] { w.out->send(buf, bytes, nullptr); });
  };
  for (const Item& it : items) {
    const int mb = it.mb;
    fault_hook(w, "item");
    ++w.items_seen;
    switch (it.kind) {
      case Item::PREFILL: {
        if (!first) recv(mb, st.act(mb), (size_t)it.T * d4, "act");
        span(w, nullptr, 0, "prefill mb" + std::to_string(mb) + " T" + std::to_string(it.T),
             [&] { st.prefill(mb, it.segs, nullptr); });
        if (!last) send(mb, st.act(mb), (size_t)it.T * d4, "act");
        break;
      }
      case Item::PREFILL_END: {
        if (last) {
          span(w, nullptr, 0, "prefill_head mb" + std::to_string(mb), [&] { st.prefill_finish(mb, nullptr, it.rows.empty() ? nullptr : &it.rows); });
          std::memcpy(out_host_ + (size_t)mb * B_, st.tokens(mb), (size_t)B_ * 4);
        }
        if (S_ > 1) {
          if (last) send(mb, st.tokens(mb), (size_t)B_ * 4, "tok");
          if (first) w.ring_pending[mb] = true;
        }
        break;
      }
      case Item::DECODE: {
        if (!first) recv(mb, st.act(mb), (size_t)B_ * d4, "act");
        else if (w.ring_pending[mb]) {
          recv(mb, st.tokens(mb), (size_t)B_ * 4, "tok");
          w.ring_pending[mb] = false;
        }
        span(w, nullptr, 0, "decode mb" + std::to_string(mb), [&] { st.decode(mb, nullptr); });
        if (last) {
          w.tok_t.push_back(now_ms());
          std::memcpy(out_host_ + ((size_t)((it.round + 1) % rounds_cap_) * M_ + mb) * B_, st.tokens(mb), (size_t)B_ * 4);
        }
        if (S_ > 1) {
          if (!last) send(mb, st.act(mb), (size_t)B_ * d4, "act");
          else send(mb, st.tokens(mb), (size_t)B_ * 4, "tok");
          if (first) w.ring_pending[mb] = true;
        }
        break;
      }
    }
    ++w.progress;
  }
  if (first && S_ > 1)
    for (int mb = 0; mb < M_; ++mb)
      if (w.ring_pending[mb]) {
        recv(mb, st.tokens(mb), (size_t)B_ * 4, "tok");
        w.ring_pending[mb] = false;
      }
}

void Engine::run_items(Worker& w, const std::vector<Item>& items) {
  if (w.cpu) return run_items_cpu(w, items);
  HIP_OK(hipSetDevice(w.device));
  Stage& st = *w.stage;
  hipStream_t cs = st.stream();
  const bool first = st.spec().first(), last = st.spec().last();
  const size_t d4 = (size_t)cfg_.d_model * 4;
  if (trace_ && !w.tr_base) {
    HIP_OK(hipEventCreate(&w.tr_base));
    HIP_OK(hipEventRecord(w.tr_base, cs));
    HIP_OK(hipEventSynchronize(w.tr_base));
    w.tr_base_ms = now_ms();
  }
  const bool wire = act_dtype_ != ACT_F32;
  // before a stream overwrites micro-batch mb's last sent buffer: its send has been issued (sent_ev)
  // and its bytes have left the buffer (Link::wait_consumed: LocalLink's posted queue)
  auto reuse_wait = [&](int mb, hipStream_t s) {
    if (!w.sent_valid[mb]) return;
    HIP_OK(hipStreamWaitEvent(s, w.sent_ev[mb], 0));
    w.out->wait_consumed(w.sent_seq[mb], s);
  };
  auto recv_into = [&](int mb, void* buf, size_t bytes) {
    reuse_wait(mb, w.recv_st);
    HIP_OK(hipEventRecord(w.comp_ev[mb], cs));
    HIP_OK(hipStreamWaitEvent(w.recv_st, w.comp_ev[mb], 0));
    // 2-byte wire: receive into the staging buffer, widen to the f32 residual on the compute stream
    void* dst = wire ? w.wire_in[mb] : buf;
    const size_t nb = wire ? bytes / 2 : bytes;
    span(w, w.recv_st, 2, "recv act mb" + std::to_string(mb), [&] { w.in->recv(dst, nb, w.recv_st); });
    HIP_OK(hipEventRecord(w.recv_ev[mb], w.recv_st));
    HIP_OK(hipStreamWaitEvent(cs, w.recv_ev[mb], 0));
    if (wire) launch_act_unpack(dst, static_cast<float*>(buf), (int64_t)(bytes / 4), act_dtype_, cs);
  };
  // a LocalLink send only records the ready event (the receiver copies): on the compute stream
  // itself, one cross-stream hop fewer per item than through the send stream (profiles/r12a trace)
  const bool send_direct = w.out && std::strcmp(w.out->kind(), "local") == 0;
  auto send_from = [&](int mb, const void* buf, size_t bytes) {
    if (fault_hook(w, "send")) return;
    hipStream_t ss = send_direct ? cs : w.send_st;
    if (!send_direct) {
      HIP_OK(hipEventRecord(w.comp_ev[mb], cs));
      HIP_OK(hipStreamWaitEvent(w.send_st, w.comp_ev[mb], 0));
    }
    span(w, ss, 1, std::string(last ? "send tok" : "send act") + " mb" + std::to_string(mb),
         [&] { w.out->send(buf, bytes, ss); });
    HIP_OK(hipEventRecord(w.sent_ev[mb], ss));
    w.sent_seq[mb] = w.out->last_seq();
    w.sent_valid[mb] = true;
  };
  // activations: narrowed to the wire format on the compute stream (the previous send of this
  // micro-batch's staging buffer is complete: the compute stream waited for sent_ev[mb])
  auto send_act = [&](int mb, const float* buf, size_t bytes) {
    if (!wire) return send_from(mb, buf, bytes);
    launch_act_pack(buf, w.wire_out[mb], (int64_t)(bytes / 4), act_dtype_, cs);
    send_from(mb, w.wire_out[mb], bytes / 2);
  };
  for (const Item& it : items) {
    const int mb = it.mb;
    fault_hook(w, "item");
    ++w.items_seen;
    switch (it.kind) {
      case Item::PREFILL: {
        const size_t bytes = (size_t)it.T * d4;
        if (!first) recv_into(mb, st.act(mb), bytes);
        else reuse_wait(mb, cs);
        span(w, cs, 0, "prefill mb" + std::to_string(mb) + " T" + std::to_string(it.T),
             [&] { st.prefill(mb, it.segs, cs); });
        if (!last) send_act(mb, st.act(mb), bytes);
        break;
      }
      case Item::PREFILL_END: {
        if (last) {
          span(w, cs, 0, "prefill_head mb" + std::to_string(mb), [&] { st.prefill_finish(mb, cs, it.rows.empty() ? nullptr : &it.rows); });
          HIP_OK(hipMemcpyAsync(out_host_ + (size_t)mb * B_, st.tokens(mb), (size_t)B_ * 4, hipMemcpyDeviceToHost,
                                cs));
        }
        if (S_ > 1) {
          if (last) send_from(mb, st.tokens(mb), (size_t)B_ * 4);
          if (first) post_ring_recv(w, mb);
        }
        break;
      }
      case Item::DECODE: {
        if (!first) recv_into(mb, st.act(mb), (size_t)B_ * d4);
        else if (S_ > 1) HIP_OK(hipStreamWaitEvent(cs, w.recv_ev[mb], 0));
        reuse_wait(mb, cs);
        span(w, cs, 0, "decode mb" + std::to_string(mb), [&] { st.decode(mb, cs); });
        if (last) {
          const size_t ev_i = (size_t)(it.round - rounds_done_) * M_ + mb;
          if (ev_i < w.tok_ev.size()) HIP_OK(hipEventRecord(w.tok_ev[ev_i], cs));
          HIP_OK(hipMemcpyAsync(out_host_ + ((size_t)((it.round + 1) % rounds_cap_) * M_ + mb) * B_, st.tokens(mb), (size_t)B_ * 4,
                                hipMemcpyDeviceToHost, cs));
        }
        if (S_ > 1) {
          if (!last) send_act(mb, st.act(mb), (size_t)B_ * d4);
          else send_from(mb, st.tokens(mb), (size_t)B_ * 4);
          if (first) post_ring_recv(w, mb);
        }
        break;
      }
    }
    ++w.progress;
  }
}

void Engine::run_all(const std::vector<Item>& items) {
  if (workers_.size() == 1) {
    try {
      run_items(*workers_[0], items);
    } catch (...) {
      failed_ = true;
      failed_stage_ = workers_[0]->stage->spec().stage;
      for (auto& l : links_) l->abort();
      throw;
    }
  } else {
    // persistent stage workers: one pool thread per owned stage (thread i always runs stage i, the
    // calling thread runs stage 0), created on the first multi-stage call and reused by every
    // decode round (the serving loop calls run_all once per round)
    if (!pool_ || pool_->size() != (int)workers_.size()) pool_.reset(new ThreadPool((int)workers_.size()));
    std::vector<std::exception_ptr> errs(workers_.size());
    std::atomic<int> first_err{-1};   // the root cause; the others are usually "link aborted"
    int dev0 = 0;
    if (!cpu_) HIP_OK(hipGetDevice(&dev0));
    pool_->parallel_for((int64_t)workers_.size(), [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) {
        try {
          run_items(*workers_[i], items);
        } catch (...) {
          errs[i] = std::current_exception();
          int expect = -1;
          first_err.compare_exchange_strong(expect, (int)i);
          for (auto& l : links_) l->abort();
        }
      }
    });
    if (!cpu_) (void)hipSetDevice(dev0);   // run_items set the calling thread's device to stage 0's
    if (first_err >= 0) {
      failed_ = true;
      failed_stage_ = workers_[first_err]->stage->spec().stage;
      std::rethrow_exception(errs[first_err]);
    }
  }
  sync_all();
  if (trace_) collect_trace();
}

void Engine::collect_trace() {
  for (auto& wp : workers_) {
    Worker& w = *wp;
    const int pid = w.stage->spec().stage;
    for (auto& r : w.tr) {
      double ta = r.ta, tb = r.tb;
      if (!w.cpu) {
        float ea = 0, eb = 0;
        HIP_OK(hipEventElapsedTime(&ea, w.tr_base, r.a));
        HIP_OK(hipEventElapsedTime(&eb, w.tr_base, r.b));
        ta = w.tr_base_ms + ea;
        tb = w.tr_base_ms + eb;
        (void)hipEventDestroy(r.a);
        (void)hipEventDestroy(r.b);
      }
      Json e = Json::object();
      e["name"] = r.name;
      e["ph"] = "X";
      e["pid"] = pid;
      e["tid"] = r.tid;
      e["ts"] = (ta - trace_t0_) * 1e3;
      e["dur"] = std::max(0.0, (tb - ta) * 1e3);
      trace_events_.push_back(e.dump());
    }
    w.tr.clear();
  }
}

void Engine::enable_trace(bool on) {
  trace_ = on;
  if (on && trace_t0_ == 0) trace_t0_ = now_ms();
}

void Engine::write_trace(const std::string& path) const {
  FILE* f = fopen(path.c_str(), "w");
  if (!f) throw std::runtime_error("cannot write trace " + path);
  fputs("{\"traceEvents\":[\n", f);
  static const char* tnames[3] = {"compute", "send", "recv"};
  bool firstl = true;
  for (auto& wp : workers_)
    for (int t = 0; t < 3; ++t) {
      Json m = Json::object();
      m["name"] = "thread_name";
      m["ph"] = "M";
      m["pid"] = wp->stage->spec().stage;
      m["tid"] = t;
      Json a = Json::object();
      a["name"] = std::string(tnames[t]);
      m["args"] = a;
      fprintf(f, "%s%s", firstl ? "" : ",\n", m.dump().c_str());
      firstl = false;
    }
  for (auto& e : trace_events_) {
    fprintf(f, "%s%s", firstl ? "" : ",\n", e.c_str());
    firstl = false;
  }
  fputs("\n]}\n", f);
  fclose(f);
}

Json Engine::health() const {
  Json j = Json::object();
  j["ok"] = !failed_;
  j["backend"] = cpu_ ? "cpu" : hybrid_ ? "hybrid" : "hip";
  j["prefix_reused_tokens"] = (int64_t)reused_tokens_;
  if (failed_stage_ >= 0) {
    j["failed_stage"] = failed_stage_;
    j["failed_device"] = specs_[failed_stage_].device;
  }
  Json st = Json::array();
  for (auto& w : workers_) {
    Json o = Json::object();
    o["stage"] = w->stage->spec().stage;
    o["backend"] = w->stage->backend_name();
    o["device"] = w->device;
    o["items_done"] = (int64_t)w->progress.load();
    if (w->out) {
      o["bytes_sent"] = (int64_t)w->out->bytes_sent;
      o["msgs_sent"] = (int64_t)w->out->msgs_sent;
      o["link"] = std::string(w->out->kind());
    }
    st.push(o);
  }
  j["stages"] = st;
  return j;
}

// Stream drain with a watchdog: a peer that never sends (dead process, dropped
// message) would otherwise hang hipStreamSynchronize on a posted receive forever.  After
// `watchdog_s` without completion the links are aborted (ncclCommAbort for RCCL) and the
// engine reports the stall.
// Failover (the reference design's auto-healing workers, PDF pp.6-7 §5.2-5.3):
// the config of an engine rebuilt WITHOUT the failed stage's device -- one stage fewer, the layers
// re-partitioned over the survivors by the same cost model; a single-stage engine is rebuilt in place.
Json Engine::failover_config(const Json& cfg, const Json& health) {
  Json c = cfg;
  c["fault"] = Json::object();   // an injected fault does not follow the engine across a rebuild
  const int S = cfg.get_int("stages", 1);   // GPU stages (a hybrid split puts its CPU stage 0 in front)
  if (!health.has("failed_stage") || S <= 1 || cfg.get_str("mode", "local") == "mp") return c;
  int bad = health.get_int("failed_stage", 0);
  if (health.get_str("backend", "") == "hybrid") {
    if (bad == 0) return c;   // the CPU stage: rebuilt in place
    bad -= 1;                 // index among the GPU stages
  }
  Json devs = Json::array();
  if (cfg.has("devices") && cfg["devices"].is_arr() && !cfg["devices"].arr().empty()) {
    const auto& a = cfg["devices"].arr();
    for (int s = 0; s < S; ++s)
      if (s != bad) devs.push(a[s % a.size()]);
  } else {
    for (int s = 0; s < S; ++s)
      if (s != bad) devs.push(Json((double)s));
  }
  c["stages"] = S - 1;
  c["devices"] = devs;
  if (cfg.has("device_speed") && cfg["device_speed"].is_arr()) {
    Json sp = Json::array();
    const auto& a = cfg["device_speed"].arr();
    for (int s = 0; s < S && s < (int)a.size(); ++s)
      if (s != bad) sp.push(a[s]);
    c["device_speed"] = sp;
  }
  MP_LOGW("failover: stage %d (device %d) lost; re-partitioning over %d stage(s)", bad,
          health.get_int("failed_device", -1), S - 1);
  return c;
}

// The links are idle between run_all calls (every item's sends were matched by the peer's
// receives, and sync_all drained the streams), so this pass cannot interleave with pipeline traffic.
void Engine::ring_bcast_from_last(std::vector<int32_t>& v) {
  if (mode_ != "mp" || S_ == 1 || v.empty()) return;
  Worker& w = *workers_[0];
  const int s = w.stage->spec().stage;
  const size_t bytes = v.size() * 4;
  const bool last = s == S_ - 1, fwd = s < S_ - 2;
  if (cpu_) {
    if (last) {
      w.out->send(v.data(), bytes, nullptr);
    } else {
      w.in->recv(v.data(), bytes, nullptr);
      if (fwd) w.out->send(v.data(), bytes, nullptr);
    }
    return;
  }
  HIP_OK(hipSetDevice(w.device));
  if (bcast_cap_ < v.size()) {
    if (bcast_dev_) HIP_OK(hipFree(bcast_dev_));
    HIP_OK(hipMalloc(&bcast_dev_, bytes));
    bcast_cap_ = v.size();
  }
  if (last) {
    HIP_OK(hipMemcpy(bcast_dev_, v.data(), bytes, hipMemcpyHostToDevice));
    w.out->send(bcast_dev_, bytes, w.send_st);
    w.out->wait_consumed(w.out->last_seq(), w.send_st);
    HIP_OK(hipStreamSynchronize(w.send_st));
  } else {
    w.in->recv(bcast_dev_, bytes, w.recv_st);
    HIP_OK(hipStreamSynchronize(w.recv_st));
    HIP_OK(hipMemcpy(v.data(), bcast_dev_, bytes, hipMemcpyDeviceToHost));
    if (fwd) {
      w.out->send(bcast_dev_, bytes, w.send_st);
      w.out->wait_consumed(w.out->last_seq(), w.send_st);
      HIP_OK(hipStreamSynchronize(w.send_st));
    }
  }
}

void Engine::sync_all() {
  if (cpu_) return;
  const double deadline = now_ms() + watchdog_s_ * 1e3;
  for (auto& w : workers_) {
    if (w->cpu) continue;
    HIP_OK(hipSetDevice(w->device));
    for (hipStream_t s : {w->stage->stream(), w->send_st, w->recv_st}) {
      for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) break;
        if (e != hipErrorNotReady) HIP_OK(e);
        if (now_ms() > deadline) {
          failed_ = true;
          failed_stage_ = w->stage->spec().stage;
          for (auto& l : links_) l->abort();
          throw std::runtime_error("pipeline watchdog: stage " + std::to_string(w->stage->spec().stage) +
                                   " made no progress for " + std::to_string((int)watchdog_s_) +
                                   " s (peer stalled or lost); links aborted");
        }
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    }
  }
}

void Engine::start(const std::vector<std::vector<int32_t>>& prompts) {
  if ((int)prompts.size() > M_ * B_) throw std::runtime_error("more prompts than micro-batch slots");
  prompts_ = prompts;
  gen_.assign(prompts.size(), {});
  rounds_done_ = 0;
  resumable_ = true;
  base_round_.assign((size_t)M_ * B_, 0);
  active_.assign((size_t)M_ * B_, 0);
  for (size_t i = 0; i < prompts.size(); ++i) active_[i] = 1;
  // KV pages: each prompt + its first decode position; slots without a prompt give theirs back
  // (a reused prefix keeps the pages it already owns)
  for (size_t i = prompts.size(); i < (size_t)M_ * B_; ++i) pager_.release((int)i);
  for (size_t i = 0; i < prompts.size(); ++i)
    if (!prompts[i].empty() && (int)prompts[i].size() < max_ctx_) kv_grant(i, (int)prompts[i].size() + 1);
  kv_sync();
  std::vector<Item> items;
  for (auto& w : workers_) {
    Stage& st = *w->stage;
    if (!w->cpu) HIP_OK(hipSetDevice(w->device));
    for (int mb = 0; mb < M_; ++mb) {
      std::vector<int32_t> pos(B_, 0);
      for (int b = 0; b < B_; ++b) {
        const size_t i = (size_t)mb * B_ + b;
        if (i < prompts.size()) pos[b] = (int)prompts[i].size();
      }
      st.set_positions(mb, pos);
    }
    if (st.spec().last()) {   // repetition-penalty windows start with the prompts (llama-cli accepts them)
      for (int mb = 0; mb < M_; ++mb) {
        std::vector<std::vector<int32_t>> seqs;
        for (int b = 0; b < B_ && (size_t)mb * B_ + b < prompts.size(); ++b) seqs.push_back(prompts[(size_t)mb * B_ + b]);
        st.set_history(mb, seqs);
      }
    }
    if (st.spec().first()) {
      for (size_t i = 0; i < prompts.size(); ++i) {
        if (prompts[i].empty() || (int)prompts[i].size() >= max_ctx_) throw std::runtime_error("bad prompt length");
        if (w->cpu) std::memcpy(st.prompt_buf() + i * max_ctx_, prompts[i].data(), prompts[i].size() * 4);
        else HIP_OK(hipMemcpy(st.prompt_buf() + i * max_ctx_, prompts[i].data(), prompts[i].size() * 4,
                              hipMemcpyHostToDevice));
      }
    }
  }
  {
    std::vector<size_t> seqs(prompts.size());
    std::iota(seqs.begin(), seqs.end(), (size_t)0);
    items = prefill_items(seqs, false);
  }
  slot_toks_.clear();   // KV content unknown until this prefill has completed
  run_all(items);
  started_ = true;
  if (owns_last())
    for (size_t i = 0; i < prompts.size(); ++i) gen_[i].push_back(out_host_[i]);
  slot_toks_ = prompts;
}

// tokens whose KV a slot holds after the last decode round: prompt + every generated token that went
// through a decode step (all but the newest).  The generated part is only known where the last
// stage lives, so a multi-process pipeline caches prompts only (every rank must agree on reuse).
void Engine::refresh_slot_cache() {
  slot_toks_ = prompts_;
  // a released slot's KV is not guaranteed (load_state restores active slots only; live idle rows
  // keep overwriting theirs): never offer it for prefix reuse
  for (size_t i = 0; i < slot_toks_.size(); ++i)
    if (i < active_.size() && !active_[i]) slot_toks_[i].clear();
  if (!resumable_ || !owns_first() || !owns_last()) return;
  for (size_t i = 0; i < slot_toks_.size() && i < gen_.size(); ++i) {
    const int since = rounds_done_ - (i < base_round_.size() ? base_round_[i] : 0);
    const size_t n = std::min(gen_[i].size(), (size_t)std::max(0, since));
    slot_toks_[i].insert(slot_toks_[i].end(), gen_[i].begin(), gen_[i].begin() + n);
  }
}

// ---------------------------------------------------------------- checkpoint / resume
// everything the saved KV bytes depend on: model shape, pipeline shape, and the KV element type
// (f32 on the CPU backend, f16 or fp8 e4m3 on HIP) -- a checkpoint written with one KV dtype must
// not be imported page by page into another
static Json state_fingerprint(const ModelConfig& c, int S, int M, int B, int max_ctx, bool cpu, bool kv_fp8) {
  Json f = Json::object();
  f["n_layer"] = c.n_layer; f["d_model"] = c.d_model; f["n_head"] = c.n_head; f["n_head_kv"] = c.n_head_kv;
  f["d_ff"] = c.d_ff; f["vocab"] = c.vocab; f["n_stages"] = S; f["n_mb"] = M; f["mb_size"] = B;
  f["max_ctx"] = max_ctx;
  f["kv_dtype"] = cpu ? "f32" : kv_fp8 ? "fp8" : "f16";
  return f;
}

Json Engine::save_state(const std::string& dir) {
  if (!started_) throw std::runtime_error("save_state before start");
  if (failed_) throw std::runtime_error("save_state after a pipeline fault");
  if (!resumable_) throw std::runtime_error("save_state: not supported after speculative decoding");
  ::mkdir(dir.c_str(), 0755);
  sync_all();
  const Json fp = state_fingerprint(cfg_, S_, M_, B_, max_ctx_, cpu_, kv_fp8_);
  // tokens already in each slot's KV: prompt + generated - 1 (the newest token is the next input)
  std::vector<int> n_tok((size_t)M_ * B_, 0);
  for (size_t i = 0; i < prompts_.size(); ++i)
    if (i < active_.size() && active_[i]) n_tok[i] = slot_pos(i);
  size_t total = 0;
  for (auto& wp : workers_) {
    Stage& st = *wp->stage;
    if (!wp->cpu) HIP_OK(hipSetDevice(wp->device));
    Json h = Json::object();
    h["magic"] = "mipipe-stage-state"; h["version"] = 1; h["fingerprint"] = fp;
    h["stage"] = st.spec().stage; h["layer_begin"] = st.spec().layer_begin; h["layer_end"] = st.spec().layer_end;
    h["backend"] = st.backend_name(); h["sample_step"] = (double)st.sample_step();
    Json lens = Json::array();
    for (int v : n_tok) lens.push(v);
    h["n_tok"] = lens;
    if (st.spec().first()) {   // current decode input of every row (received over the ring for S > 1)
      Json toks = Json::array();
      std::vector<int32_t> t(B_);
      for (int mb = 0; mb < M_; ++mb) {
        if (wp->cpu) std::memcpy(t.data(), st.tokens(mb), (size_t)B_ * 4);
        else HIP_OK(hipMemcpy(t.data(), st.tokens(mb), (size_t)B_ * 4, hipMemcpyDeviceToHost));
        for (int b = 0; b < B_; ++b) toks.push(t[b]);
      }
      h["tokens"] = toks;
    }
    std::vector<uint8_t> kv;
    for (size_t i = 0; i < n_tok.size(); ++i)
      if (n_tok[i] > 0) st.kv_export((int)i, n_tok[i], kv);
    h["kv_bytes"] = (double)kv.size();
    const std::string path = dir + "/stage" + std::to_string(st.spec().stage) + ".bin";
    std::ofstream f(path, std::ios::binary | std::ios::trunc);
    const std::string hs = h.dump() + "\n";
    f.write(hs.data(), (std::streamsize)hs.size());
    f.write(reinterpret_cast<const char*>(kv.data()), (std::streamsize)kv.size());
    if (!f) throw std::runtime_error("save_state: cannot write " + path);
    total += hs.size() + kv.size();
  }
  if (owns_last()) {
    Json sj = Json::object();
    sj["magic"] = "mipipe-session"; sj["version"] = 1; sj["fingerprint"] = fp; sj["rounds_done"] = rounds_done_;
    Json ps = Json::array(), gs = Json::array();
    for (size_t i = 0; i < prompts_.size(); ++i) {
      Json p = Json::array(), g = Json::array();
      for (int32_t t : prompts_[i]) p.push(t);
      for (int32_t t : gen_[i]) g.push(t);
      ps.push(p);
      gs.push(g);
    }
    sj["prompts"] = ps;
    sj["generated"] = gs;
    Json br = Json::array(), ac = Json::array();
    for (size_t i = 0; i < prompts_.size(); ++i) {
      br.push(i < base_round_.size() ? base_round_[i] : 0);
      ac.push(i < active_.size() && active_[i] ? 1 : 0);
    }
    sj["base_round"] = br;
    sj["active"] = ac;
    std::ofstream f(dir + "/session.json", std::ios::trunc);
    f << sj.dump() << "\n";
    if (!f) throw std::runtime_error("save_state: cannot write session.json");
  }
  MP_LOGI("state saved to %s: %zu sequences, %d rounds, %.1f MiB", dir.c_str(), prompts_.size(), rounds_done_,
          total / 1048576.0);
  Json r = Json::object();
  r["bytes"] = (double)total; r["rounds_done"] = rounds_done_; r["sequences"] = (int)prompts_.size();
  return r;
}

Json Engine::load_state(const std::string& dir) {
  auto slurp = [](const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("load_state: cannot read " + path);
    return std::string((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  };
  const Json fp = state_fingerprint(cfg_, S_, M_, B_, max_ctx_, cpu_, kv_fp8_);
  const Json sj = Json::parse(slurp(dir + "/session.json"));
  if (sj.get_str("magic", "") != "mipipe-session" || sj["fingerprint"].dump() != fp.dump())
    throw std::runtime_error("load_state: session was saved by a different model / pipeline shape");
  prompts_.clear();
  gen_.clear();
  for (const Json& p : sj["prompts"].arr()) {
    std::vector<int32_t> v;
    for (const Json& t : p.arr()) v.push_back((int32_t)t.num());
    prompts_.push_back(v);
  }
  for (const Json& g : sj["generated"].arr()) {
    std::vector<int32_t> v;
    for (const Json& t : g.arr()) v.push_back((int32_t)t.num());
    gen_.push_back(v);
  }
  rounds_done_ = sj.get_int("rounds_done", 0);
  // session.json is untrusted input: validate every index and size before it reaches a buffer
  if (prompts_.empty() || (int)prompts_.size() > M_ * B_ || gen_.size() != prompts_.size() || rounds_done_ < 0)
    throw std::runtime_error("load_state: bad session");
  if ((sj.has("base_round") && sj["base_round"].arr().size() != prompts_.size()) ||
      (sj.has("active") && sj["active"].arr().size() != prompts_.size()))
    throw std::runtime_error("load_state: bad session (base_round / active size)");
  auto check_ids = [&](const std::vector<int32_t>& v) {
    for (int32_t t : v)
      if (t < 0 || t >= cfg_.vocab) throw std::runtime_error("load_state: token id out of range");
  };
  for (size_t i = 0; i < prompts_.size(); ++i) {
    if (prompts_[i].empty() || (int)prompts_[i].size() >= max_ctx_)
      throw std::runtime_error("load_state: prompt length out of range");
    check_ids(prompts_[i]);
    check_ids(gen_[i]);
  }
  base_round_.assign((size_t)M_ * B_, 0);
  active_.assign((size_t)M_ * B_, 0);
  for (size_t i = 0; i < prompts_.size(); ++i) {
    base_round_[i] = sj.has("base_round") ? (int)sj["base_round"].arr()[i].num() : 0;
    active_[i] = sj.has("active") ? (char)sj["active"].arr()[i].num() : 1;
    if (base_round_[i] < 0 || base_round_[i] > rounds_done_)
      throw std::runtime_error("load_state: bad session (base_round)");
    if (active_[i] && slot_pos(i) >= max_ctx_) throw std::runtime_error("load_state: sequence longer than max_ctx");
  }
  // KV pages for the restored sequences (their KV bytes are imported page by page below)
  for (int i = 0; i < M_ * B_; ++i) pager_.release(i);
  for (size_t i = 0; i < prompts_.size(); ++i)
    if (active_[i]) kv_grant(i, slot_pos(i) + 1);
  kv_sync();
  for (auto& wp : workers_) {
    Stage& st = *wp->stage;
    if (!wp->cpu) HIP_OK(hipSetDevice(wp->device));
    const std::string path = dir + "/stage" + std::to_string(st.spec().stage) + ".bin";
    const std::string raw = slurp(path);
    const size_t nl = raw.find('\n');
    if (nl == std::string::npos) throw std::runtime_error("load_state: bad stage file " + path);
    const Json h = Json::parse(raw.substr(0, nl));
    if (h.get_str("magic", "") != "mipipe-stage-state" || h["fingerprint"].dump() != fp.dump() ||
        h.get_int("layer_begin", -1) != st.spec().layer_begin || h.get_int("layer_end", -1) != st.spec().layer_end ||
        h.get_str("backend", "") != st.backend_name())
      throw std::runtime_error("load_state: " + path + " does not match this stage (layers / backend / shape)");
    const uint8_t* kv = reinterpret_cast<const uint8_t*>(raw.data()) + nl + 1;
    const uint8_t* end = reinterpret_cast<const uint8_t*>(raw.data()) + raw.size();
    const auto& lens = h["n_tok"].arr();
    if ((int)lens.size() != M_ * B_) throw std::runtime_error("load_state: bad n_tok in " + path);
    // the KV payload must be exactly what this stage exports for those lengths (element size
    // included) and exactly what the file holds after its header
    size_t want_bytes = 0;
    for (size_t i = 0; i < lens.size(); ++i) {
      const int n = (int)lens[i].num();
      if (n > 0 && n < max_ctx_) want_bytes += st.kv_state_bytes(n);
    }
    if ((double)want_bytes != h.get_num("kv_bytes", -1) || want_bytes != (size_t)(end - kv))
      throw std::runtime_error("load_state: " + path + " KV payload size does not match this stage (kv dtype?)");
    for (size_t i = 0; i < lens.size(); ++i) {
      const int n = (int)lens[i].num();
      // the stage file must describe exactly the KV the session implies (active slots only)
      const int want = i < prompts_.size() && active_[i] ? slot_pos(i) : 0;
      if (n != want) throw std::runtime_error("load_state: " + path + " KV length disagrees with session.json");
      if (n <= 0) continue;
      if (n >= max_ctx_) throw std::runtime_error("load_state: sequence longer than max_ctx");
      const size_t nb = st.kv_state_bytes(n);
      if (kv + nb > end) throw std::runtime_error("load_state: truncated " + path);
      st.kv_import((int)i, n, kv, nb);
      kv += nb;
    }
    st.set_sample_step((uint64_t)h.get_num("sample_step", 0));
    for (int mb = 0; mb < M_; ++mb) {   // next decode position: prompt + rounds since admission
      std::vector<int32_t> pos(B_);
      for (int b = 0; b < B_; ++b) pos[b] = slot_pos((size_t)mb * B_ + b);
      st.set_positions(mb, pos);
    }
    if (st.spec().first()) {
      const auto& toks = h["tokens"].arr();
      if ((int)toks.size() != M_ * B_) throw std::runtime_error("load_state: missing first-stage tokens");
      std::vector<int32_t> t(B_);
      for (int mb = 0; mb < M_; ++mb) {
        for (int b = 0; b < B_; ++b) {
          t[b] = (int32_t)toks[(size_t)mb * B_ + b].num();
          if (t[b] < 0 || t[b] >= cfg_.vocab) throw std::runtime_error("load_state: token id out of range");
        }
        if (wp->cpu) std::memcpy(st.tokens(mb), t.data(), (size_t)B_ * 4);
        else HIP_OK(hipMemcpy(st.tokens(mb), t.data(), (size_t)B_ * 4, hipMemcpyHostToDevice));
      }
      for (size_t i = 0; i < prompts_.size(); ++i) {
        if (wp->cpu) std::memcpy(st.prompt_buf() + i * max_ctx_, prompts_[i].data(), prompts_[i].size() * 4);
        else HIP_OK(hipMemcpy(st.prompt_buf() + i * max_ctx_, prompts_[i].data(), prompts_[i].size() * 4,
                              hipMemcpyHostToDevice));
      }
      if (wp->cpu) std::fill(wp->ring_pending.begin(), wp->ring_pending.end(), false);
    }
    if (st.spec().last()) {   // penalty windows: prompt + accepted tokens
      for (int mb = 0; mb < M_; ++mb) {
        std::vector<std::vector<int32_t>> seqs;
        for (int b = 0; b < B_ && (size_t)mb * B_ + b < prompts_.size(); ++b) {
          const size_t i = (size_t)mb * B_ + b;
          std::vector<int32_t> q = prompts_[i];
          q.insert(q.end(), gen_[i].begin(), gen_[i].end());
          seqs.push_back(q);
        }
        st.set_history(mb, seqs);
      }
    }
  }
  started_ = true;
  resumable_ = true;
  refresh_slot_cache();
  MP_LOGI("state loaded from %s: %zu sequences, %d rounds", dir.c_str(), prompts_.size(), rounds_done_);
  Json r = Json::object();
  r["rounds_done"] = rounds_done_; r["sequences"] = (int)prompts_.size();
  return r;
}


// packed prefill of sequences `seqs` (slot indices): each micro-batch's prompts are cut into chunks
// of up to chunk_ rows that may hold several sequences, so each projection reads its weights once
// per chunk (not per sequence).  start(): every micro-batch gets a PREFILL_END (head over all its
// rows); admission: only the micro-batches of admitted slots, restricted to their rows.
std::vector<Item> Engine::prefill_items(const std::vector<size_t>& seqs, bool admission) {
  std::vector<Item> items;
  std::vector<std::vector<size_t>> by_mb(M_);
  for (size_t i : seqs) by_mb[i / B_].push_back(i);
  for (int mb = 0; mb < M_; ++mb) {
    if (admission && by_mb[mb].empty()) continue;
    std::sort(by_mb[mb].begin(), by_mb[mb].end());
    Item it{Item::PREFILL};
    it.mb = mb;
    auto flush = [&] {
      if (it.T > 0) items.push_back(it);
      it.segs.clear();
      it.T = 0;
    };
    for (size_t i : by_mb[mb]) {
      const int b = (int)(i % B_);
      const int n = (int)prompts_[i].size();
      // prefix cache: the slot's KV already holds the tokens of slot_toks_[i]; only the part after
      // the common prefix is prefilled (at least the last prompt token, whose row feeds the head)
      int reuse = 0;
      if (prefix_cache_ && i < slot_toks_.size()) {
        const auto& c = slot_toks_[i];
        const size_t lim = std::min(c.size(), (size_t)n - 1);
        while ((size_t)reuse < lim && c[reuse] == prompts_[i][reuse]) ++reuse;
      }
      reused_tokens_ += reuse;
      for (int p0 = reuse; p0 < n;) {
        const int take = std::min(chunk_ - it.T, n - p0);
        PrefillSeg sg;
        sg.b = b; sg.p0 = p0; sg.T = take; sg.last = p0 + take >= n;
        it.segs.push_back(sg);
        it.T += take;
        p0 += take;
        if (it.T == chunk_ || !packed_prefill_) flush();
      }
    }
    flush();
    Item e{Item::PREFILL_END};
    e.mb = mb;
    if (admission)
      for (size_t i : by_mb[mb]) e.rows.push_back((int)(i % B_));
    items.push_back(e);
  }
  return items;
}

void Engine::push_positions(int mb) {
  std::vector<int32_t> pos(B_);
  for (int b = 0; b < B_; ++b) pos[b] = slot_pos((size_t)mb * B_ + b);
  for (auto& w : workers_) {
    if (!w->cpu) HIP_OK(hipSetDevice(w->device));
    w->stage->set_positions(mb, pos);
  }
}

void Engine::release(int slot) {
  if (slot >= 0 && slot < (int)active_.size()) active_[slot] = 0;
  if (slot >= 0 && slot < M_ * B_) pager_.release(slot);   // table pushed before the next engine call
}

void Engine::kv_grant(size_t slot, int n_tokens) {
  if (pager_.ensure((int)slot, n_tokens)) return;
  throw std::runtime_error("KV page pool exhausted: slot " + std::to_string(slot) + " needs " +
                           std::to_string((n_tokens + 63) / 64) + " pages, owns " +
                           std::to_string(pager_.owned((int)slot)) + ", " + std::to_string(pager_.free_pages()) +
                           " of " + std::to_string(pager_.n_pages()) + " free (kv_pool_tokens / max_ctx auto)");
}

void Engine::kv_sync() {
  if (!pager_.dirty()) return;
  for (auto& w : workers_) {
    if (!w->cpu) HIP_OK(hipSetDevice(w->device));
    w->stage->set_block_table(pager_.table());
  }
  pager_.clean();
}

void Engine::admit(const std::vector<int>& slots, const std::vector<std::vector<int32_t>>& prompts) {
  if (!started_) throw std::runtime_error("admit before start");
  if (!resumable_) throw std::runtime_error("admit after speculative decoding");
  if (slots.size() != prompts.size()) throw std::runtime_error("admit: one prompt per slot");
  const size_t NS = (size_t)M_ * B_;
  if (prompts_.size() < NS) { prompts_.resize(NS); gen_.resize(NS); }
  base_round_.resize(NS, 0);
  active_.resize(NS, 0);
  std::vector<size_t> seqs;
  std::vector<char> mbs(M_, 0);
  for (size_t k = 0; k < slots.size(); ++k) {
    const int i = slots[k];
    if (i < 0 || (size_t)i >= NS) throw std::runtime_error("admit: bad slot");
    if (active_[i]) throw std::runtime_error("admit: slot " + std::to_string(i) + " is busy");
    if (prompts[k].empty() || (int)prompts[k].size() >= max_ctx_) throw std::runtime_error("bad prompt length");
    kv_grant((size_t)i, (int)prompts[k].size() + 1);
    prompts_[i] = prompts[k];
    gen_[i].clear();
    base_round_[i] = rounds_done_;
    active_[i] = 1;
    seqs.push_back((size_t)i);
    mbs[i / B_] = 1;
  }
  kv_sync();
  for (auto& w : workers_) {
    Stage& st = *w->stage;
    if (!w->cpu) HIP_OK(hipSetDevice(w->device));
    if (st.spec().first())
      for (size_t i : seqs) {
        if (w->cpu) std::memcpy(st.prompt_buf() + i * max_ctx_, prompts_[i].data(), prompts_[i].size() * 4);
        else HIP_OK(hipMemcpy(st.prompt_buf() + i * max_ctx_, prompts_[i].data(), prompts_[i].size() * 4,
                              hipMemcpyHostToDevice));
      }
  }
  for (int mb = 0; mb < M_; ++mb)
    if (mbs[mb]) push_positions(mb);
  std::vector<Item> items = prefill_items(seqs, true);
  slot_toks_.clear();
  run_all(items);
  if (owns_last())
    for (size_t i : seqs) gen_[i].push_back(out_host_[i]);
  // the head pushed a token into the penalty window of every row of these micro-batches: re-seed
  // them from the host (prompt + accepted tokens)
  for (auto& w : workers_)
    if (w->stage->spec().last())
      for (int mb = 0; mb < M_; ++mb)
        if (mbs[mb]) {
          std::vector<std::vector<int32_t>> hs;
          for (int b = 0; b < B_; ++b) {
            const size_t i = (size_t)mb * B_ + b;
            std::vector<int32_t> q = prompts_[i];
            q.insert(q.end(), gen_[i].begin(), gen_[i].end());
            hs.push_back(q);
          }
          w->stage->set_history(mb, hs);
        }
  refresh_slot_cache();
}

StepStats Engine::decode_steps(int k) {
  if (!started_) throw std::runtime_error("decode_steps before start");
  if (k + 1 >= rounds_cap_) throw std::runtime_error("decode_steps: too many rounds in one call");
  // running sequences must fit their slot's KV pages; idle rows (which still compute) restart at
  // position 0 before they could run past them
  for (size_t i = 0; i < (size_t)M_ * B_; ++i) {
    const bool act = i < active_.size() && active_[i];
    if (slot_pos(i) + k + 1 <= max_ctx_) continue;
    if (act) throw std::runtime_error("context capacity exhausted (prompt + generated tokens > max_ctx)");
    if (i < prompts_.size()) prompts_[i].clear();
    if (base_round_.size() < (size_t)M_ * B_) base_round_.resize((size_t)M_ * B_, 0);
    base_round_[i] = rounds_done_;
    push_positions((int)(i / B_));
  }
  // KV pages for the k positions every running sequence is about to write
  for (size_t i = 0; i < (size_t)M_ * B_; ++i)
    if (i < active_.size() && active_[i]) kv_grant(i, slot_pos(i) + k + 1);
  kv_sync();
  for (auto& w : workers_)
    if (w->stage->spec().last() && w->cpu) {
      w->tok_t.clear();
    } else if (w->stage->spec().last()) {
      HIP_OK(hipSetDevice(w->device));
      for (auto e : w->tok_ev) (void)hipEventDestroy(e);
      w->tok_ev.assign((size_t)k * M_, nullptr);
      for (auto& e : w->tok_ev) HIP_OK(hipEventCreate(&e));
    }
  std::vector<Item> items;
  for (int r = 0; r < k; ++r)
    for (int mb = 0; mb < M_; ++mb) {
      Item it{Item::DECODE};
      it.mb = mb;
      it.round = rounds_done_ + r;
      items.push_back(it);
    }
  const double t0 = now_ms();
  run_all(items);
  StepStats ss;
  ss.wall_ms = now_ms() - t0;
  for (auto& w : workers_)
    if (w->stage->spec().last() && w->cpu) {
      for (size_t i = M_; i < w->tok_t.size(); ++i) ss.token_ms.push_back(w->tok_t[i] - w->tok_t[i - M_]);
    } else if (w->stage->spec().last()) {
      for (int r = 1; r < k; ++r)
        for (int mb = 0; mb < M_; ++mb) {
          float ms = 0;
          HIP_OK(hipEventElapsedTime(&ms, w->tok_ev[(size_t)(r - 1) * M_ + mb], w->tok_ev[(size_t)r * M_ + mb]));
          ss.token_ms.push_back(ms);
        }
    }
  if (owns_last())
    for (int r = 0; r < k; ++r)
      for (size_t i = 0; i < prompts_.size(); ++i) {
        const int32_t t = out_host_[(size_t)((rounds_done_ + r + 1) % rounds_cap_) * M_ * B_ + i];
        gen_[i].push_back(t);
        if (on_token) on_token((int)i, t);
      }
  rounds_done_ += k;
  refresh_slot_cache();
  return ss;
}

std::vector<std::vector<int32_t>> Engine::tokens() const { return gen_; }

Json Engine::generate(const std::vector<std::vector<int32_t>>& prompts, int n_predict,
                      std::vector<std::vector<int32_t>>* out) {
  const double t0 = now_ms();
  start(prompts);
  const double t1 = now_ms();
  StepStats ss;
  if (n_predict > 1) ss = decode_steps(n_predict - 1);
  const double t2 = now_ms();
  if (out) *out = gen_;
  size_t n_prompt = 0;
  for (auto& p : prompts) n_prompt += p.size();
  Json j = Json::object();
  j["prefill_ms"] = t1 - t0;
  j["decode_ms"] = t2 - t1;
  j["n_prompt_tokens"] = (int64_t)n_prompt;
  j["n_decode_tokens"] = (int64_t)(prompts.size() * std::max(0, n_predict - 1));
  j["prompt_tok_s"] = n_prompt / std::max(1e-9, (t1 - t0) / 1e3);
  j["decode_tok_s"] = prompts.size() * std::max(0, n_predict - 1) / std::max(1e-9, (t2 - t1) / 1e3);
  j["p50_ms"] = pct(ss.token_ms, 0.5);
  j["p90_ms"] = pct(ss.token_ms, 0.9);
  j["p99_ms"] = pct(ss.token_ms, 0.99);
  return j;
}

// Draft for prompt-lookup decoding: the tokens that followed the most recent earlier occurrence
// of the context's last g-gram (g = ngram .. 1), at most k of them.
static std::vector<int32_t> lookup_draft(const std::vector<int32_t>& ctx, int k, int ngram) {
  const int n = (int)ctx.size();
  for (int g = std::min(ngram, n - 1); g >= 1; --g)
    for (int s = n - g - 1; s >= 0; --s)
      if (std::equal(ctx.begin() + s, ctx.begin() + s + g, ctx.end() - g)) {
        const int from = s + g;
        if (from < n) return std::vector<int32_t>(ctx.begin() + from, ctx.begin() + std::min(n, from + k));
      }
  return {};
}

// Speculative decoding by prompt lookup (llama.cpp's `llama-lookup`; the design report's
// speculative decoding, PDF p.12 / SURVEY.md D10).  Every round, each sequence drafts up to
// `draft_max` tokens from its own context (lookup_draft), and ONE verify chunk per micro-batch
// scores [last token, draft...] at positions pos .. pos+k through the whole pipeline on the
// prefill path (causal attention against the KV cache; every projection one GEMV/GEMM over all
// rows, i.e. the weights are streamed once for k+1 tokens of every sequence).  The last stage
// returns the greedy token after each row; the host accepts the longest agreeing draft prefix
// plus the target's own next token, so the output equals plain greedy decoding.  KV rows written
// for rejected draft positions are overwritten by the next chunk (attention reads [0, kvlen)).
Json Engine::spec_generate(const std::vector<std::vector<int32_t>>& prompts, int n_predict, int draft_max,
                           int ngram, std::vector<std::vector<int32_t>>* out) {
  // one process per stage (mode "mp"): every rank runs this same loop; the last stage's tokens
  // reach the other ranks over the ring after each verify pass (ring_bcast_from_last), so every rank
  // drafts, grants KV and builds the identical next verify chunk
  const bool mp = mode_ == "mp" && S_ > 1;
  if (!mp && (int)workers_.size() != S_) throw std::runtime_error("speculative decoding needs every stage in this process");
  if (jcfg_.get_num("temp", 0.0) > 0.0) throw std::runtime_error("speculative decoding is greedy (temp 0)");
  if (jcfg_.get_num("repeat_penalty", 1.0) != 1.0 || jcfg_.get_num("frequency_penalty", 0.0) != 0.0 ||
      jcfg_.get_num("presence_penalty", 0.0) != 0.0)
    throw std::runtime_error("speculative decoding runs without repetition penalties");
  // one verify chunk per micro-batch: B sequences x (k + 1) rows <= prefill chunk
  const int k = std::max(1, std::min(draft_max, chunk_ / B_ - 1));
  if (k < 1 || chunk_ / B_ < 2) throw std::runtime_error("prefill chunk too small for speculative decoding");
  ngram = std::max(1, ngram);
  Worker* wf = nullptr;
  Worker* wl = nullptr;
  for (auto& w : workers_) {
    if (w->stage->spec().first()) wf = w.get();
    if (w->stage->spec().last()) wl = w.get();
  }
  const double t0 = now_ms();
  start(prompts);
  resumable_ = false;   // sequences advance by different amounts: positions are not prompt + rounds
  slot_toks_.clear();   // the verify chunks write draft rows past the accepted tokens
  const double t1 = now_ms();
  const size_t n = prompts.size();
  if (mp) {   // the first token of every sequence is known where the last stage lives
    std::vector<int32_t> ft(n, 0);
    if (owns_last())
      for (size_t i = 0; i < n; ++i) ft[i] = gen_[i][0];
    ring_bcast_from_last(ft);
    if (!owns_last())
      for (size_t i = 0; i < n; ++i) gen_[i].assign(1, ft[i]);
  }
  if (on_token)
    for (size_t i = 0; i < n; ++i) on_token((int)i, gen_[i][0]);
  std::vector<std::vector<int32_t>> ctx(n);
  for (size_t i = 0; i < n; ++i) {
    ctx[i] = prompts[i];
    ctx[i].insert(ctx[i].end(), gen_[i].begin(), gen_[i].end());
  }
  long rounds = 0, drafted = 0, accepted = 0;
  std::vector<int32_t> vt(chunk_);
  for (;;) {
    std::vector<Item> items;
    std::vector<std::vector<int32_t>> chunk(n);
    for (int mb = 0; mb < M_; ++mb) {
      Item it{Item::PREFILL};
      it.mb = mb;
      for (int b = 0; b < B_; ++b) {
        const size_t i = (size_t)mb * B_ + b;
        if (i >= n || (int)gen_[i].size() >= n_predict || (int)ctx[i].size() >= max_ctx_) continue;
        if (keep_going && !keep_going((int)i)) continue;
        const int pos = (int)ctx[i].size() - 1;   // the last token is not in the KV cache yet
        std::vector<int32_t> d = lookup_draft(ctx[i], k, ngram);
        const int room = std::min(max_ctx_ - pos - 1, n_predict - (int)gen_[i].size() - 1);
        if ((int)d.size() > room) d.resize(std::max(0, room));
        chunk[i].push_back(ctx[i].back());
        chunk[i].insert(chunk[i].end(), d.begin(), d.end());
        kv_grant(i, pos + (int)chunk[i].size());
        drafted += (long)d.size();
        if (!wf) {
        } else if (wf->cpu) {
          std::memcpy(wf->stage->prompt_buf() + i * max_ctx_ + pos, chunk[i].data(), chunk[i].size() * 4);
        } else {
          HIP_OK(hipSetDevice(wf->device));
          HIP_OK(hipMemcpy(wf->stage->prompt_buf() + i * max_ctx_ + pos, chunk[i].data(), chunk[i].size() * 4,
                           hipMemcpyHostToDevice));
        }
        PrefillSeg sg;
        sg.b = b; sg.p0 = pos; sg.T = (int)chunk[i].size(); sg.last = true; sg.verify = true;
        it.segs.push_back(sg);
        it.T += sg.T;
      }
      if (it.T > 0) items.push_back(it);
    }
    if (items.empty()) break;
    kv_sync();
    run_all(items);
    ++rounds;
    // the target's greedy token after every verify row, all items back to back
    size_t n_rows = 0;
    for (const Item& it : items) n_rows += (size_t)it.T;
    if (vt.size() < n_rows) vt.resize(n_rows);
    std::vector<int32_t> all(n_rows, 0);
    if (wl) {
      size_t off = 0;
      for (const Item& it : items) {
        if (!wl->cpu) HIP_OK(hipSetDevice(wl->device));
        wl->stage->copy_verify_tokens(it.mb, all.data() + off, it.T);
        off += (size_t)it.T;
      }
    }
    if (mp) ring_bcast_from_last(all);
    size_t off = 0;
    for (const Item& it : items) {
      std::copy(all.begin() + off, all.begin() + off + it.T, vt.begin());
      off += (size_t)it.T;
      int row = 0;
      for (const PrefillSeg& sg : it.segs) {
        const size_t i = (size_t)it.mb * B_ + sg.b;
        const std::vector<int32_t>& c = chunk[i];
        int a = 0;   // accepted draft tokens: c[1 + a] agrees with the target's token after row a
        while (1 + a < (int)c.size() && c[1 + a] == vt[row + a]) ++a;
        accepted += a;
        for (int j = 0; j <= a; ++j) {
          const int32_t t = vt[row + j];   // = c[1 + j] for j < a, the target's own token at j = a
          gen_[i].push_back(t);
          ctx[i].push_back(t);
          if (on_token) on_token((int)i, t);
        }
        if ((int)gen_[i].size() > n_predict) gen_[i].resize(n_predict);
        row += sg.T;
      }
    }
  }
  started_ = false;   // positions on the devices no longer follow the decode schedule
  const double t2 = now_ms();
  if (out) *out = gen_;
  size_t n_prompt = 0, n_gen = 0;
  for (auto& p : prompts) n_prompt += p.size();
  for (auto& g : gen_) n_gen += g.size() > 0 ? g.size() - 1 : 0;
  Json j = Json::object();
  j["prefill_ms"] = t1 - t0;
  j["decode_ms"] = t2 - t1;
  j["n_prompt_tokens"] = (int64_t)n_prompt;
  j["n_decode_tokens"] = (int64_t)n_gen;
  j["decode_tok_s"] = n_gen / std::max(1e-9, (t2 - t1) / 1e3);
  j["verify_rounds"] = (int64_t)rounds;
  j["draft_max"] = k;
  j["drafted"] = (int64_t)drafted;
  j["accepted"] = (int64_t)accepted;
  j["acceptance"] = drafted ? (double)accepted / drafted : 0.0;
  j["tokens_per_round"] = rounds ? (double)n_gen / rounds / std::max<size_t>(1, n) : 0.0;
  return j;
}

Json Engine::bench(int prompt_len, int warmup, int steps) {
  std::vector<std::vector<int32_t>> prompts(M_ * B_);
  uint32_t h = 12345;
  for (auto& p : prompts) {
    p.resize(prompt_len);
    for (auto& t : p) { h = h * 1664525u + 1013904223u; t = (int32_t)(h % (uint32_t)cfg_.vocab); }
  }
  const double t0 = now_ms();
  start(prompts);
  const double t1 = now_ms();
  if (warmup > 0) decode_steps(warmup);
  StepStats ss = decode_steps(steps);
  Json j = Json::object();
  const double toks = (double)steps * M_ * B_;
  j["decode_tok_s"] = toks / (ss.wall_ms / 1e3);
  j["wall_ms"] = ss.wall_ms;
  j["ms_per_round"] = ss.wall_ms / std::max(1, steps);
  j["p50_ms"] = pct(ss.token_ms, 0.5);
  j["p90_ms"] = pct(ss.token_ms, 0.9);
  j["p99_ms"] = pct(ss.token_ms, 0.99);
  j["prefill_ms"] = t1 - t0;
  j["prompt_tok_s"] = (double)prompt_len * M_ * B_ / ((t1 - t0) / 1e3);
  return j;
}

int Engine::copy_logits(int mb, float* out, int rows) {
  (void)mb;
  for (auto& w : workers_)
    if (w->stage->spec().last()) {
      if (w->cpu) {
        for (int r = 0; r < rows; ++r)
          std::memcpy(out + (size_t)r * cfg_.vocab, w->stage->logits_ptr() + (size_t)r * w->stage->logits_ld(),
                      (size_t)cfg_.vocab * 4);
        return 0;
      }
      HIP_OK(hipSetDevice(w->device));
      HIP_OK(hipStreamSynchronize(w->stage->stream()));
      HIP_OK(hipMemcpy2D(out, (size_t)cfg_.vocab * 4, w->stage->logits_ptr(), (size_t)w->stage->logits_ld() * 4,
                         (size_t)cfg_.vocab * 4, rows, hipMemcpyDeviceToHost));
      return 0;
    }
  return -1;
}

Json Engine::info() const {
  Json j = Json::object();
  j["n_stages"] = S_;
  j["n_mb"] = M_;
  j["mb_size"] = B_;
  j["max_ctx"] = max_ctx_;
  j["kv_pages"] = kv_pages_;
  {
    Json ds = Json::array();
    for (double v : device_speed_) ds.push(v);
    j["device_speed"] = ds;
  }
  j["kv_free_pages"] = pager_.free_pages();
  j["mode"] = mode_;
  j["backend"] = cpu_ ? "cpu" : hybrid_ ? "hybrid" : "hip";
  j["load_ms"] = load_ms_;
  Json st = Json::array();
  for (auto& s : specs_) {
    Json o = Json::object();
    o["stage"] = s.stage;
    o["layer_begin"] = s.layer_begin;
    o["layer_end"] = s.layer_end;
    o["device"] = s.device;
    st.push(o);
  }
  j["stages"] = st;
  Json m = Json::object();
  m["n_layer"] = cfg_.n_layer; m["d_model"] = cfg_.d_model; m["vocab"] = cfg_.vocab;
  m["n_head"] = cfg_.n_head; m["n_head_kv"] = cfg_.n_head_kv; m["d_ff"] = cfg_.d_ff;
  j["model"] = m;
  size_t wb = 0, kb = 0;
  for (auto& w : workers_) { wb += w->stage->weight_bytes(); kb += w->stage->kv_bytes(); }
  j["weight_bytes_local"] = (int64_t)wb;
  j["kv_bytes_local"] = (int64_t)kb;
  // the data plane as the transports report it: what each local stage sends and receives over,
  // the communicator sizes RCCL itself returns, and the bytes one token moves across a boundary
  Json ls = Json::array();
  for (auto& w : workers_) {
    for (int dir = 0; dir < 2; ++dir) {
      const Link* l = dir ? w->in : w->out;
      if (!l) continue;
      Json o = Json::object();
      o["stage"] = w->stage->spec().stage;
      o["dir"] = dir ? "in" : "out";
      o["kind"] = std::string(l->kind());
      o["comm_nranks"] = l->comm_nranks();
      o["bytes"] = (int64_t)l->bytes_sent;
      o["msgs"] = (int64_t)l->msgs_sent;
      ls.push(o);
    }
  }
  j["links"] = ls;
  if (!link_fallback_.empty()) j["link_fallback"] = link_fallback_;
  const int ab = act_dtype_ == ACT_F32 ? 4 : 2;
  j["act_dtype"] = act_dtype_ == ACT_F32 ? "f32" : act_dtype_ == ACT_F16 ? "f16" : "bf16";
  j["wire_bytes_per_token"] = S_ > 1 ? (int64_t)cfg_.d_model * ab : 0;   // per stage boundary
  return j;
}

}  // namespace mp
