#include "model.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <sstream>
#include <stdexcept>

#include "gguf.h"

namespace mp {

ModelConfig ModelConfig::from_gguf(const GgufFile& f) {
  ModelConfig c;
  c.arch = f.get_str("general.architecture", "llama");
  c.name = f.get_str("general.name", "");
  const std::string a = c.arch + ".";
  if (c.arch != "llama" && c.arch != "qwen2") throw std::runtime_error("unsupported architecture: " + c.arch);
  c.rope_neox = c.arch == "qwen2";
  c.qkv_bias = f.tensor("blk.0.attn_q.bias") != nullptr;
  c.n_layer = (int)f.get_int(a + "block_count", 0);
  c.d_model = (int)f.get_int(a + "embedding_length", 0);
  c.n_head = (int)f.get_int(a + "attention.head_count", 0);
  c.n_head_kv = (int)f.get_int(a + "attention.head_count_kv", c.n_head);
  c.d_ff = (int)f.get_int(a + "feed_forward_length", 0);
  c.n_ctx_train = (int)f.get_int(a + "context_length", 2048);
  c.rope_base = (float)f.get_float(a + "rope.freq_base", 10000.0);
  c.eps = (float)f.get_float(a + "attention.layer_norm_rms_epsilon", 1e-5);
  c.n_expert = (int)f.get_int(a + "expert_count", 0);
  c.n_expert_used = (int)f.get_int(a + "expert_used_count", 0);
  c.head_dim = (int)f.get_int(a + "rope.dimension_count", c.n_head ? c.d_model / c.n_head : 0);
  const GgufTensor* emb = f.tensor("token_embd.weight");
  if (!emb) throw std::runtime_error("missing token_embd.weight");
  c.vocab = (int)f.get_int(a + "vocab_size", emb->ne.size() > 1 ? emb->ne[1] : 0);
  c.rope_freqs = f.tensor("rope_freqs.weight") != nullptr;
  c.tied_output = f.tensor("output.weight") == nullptr;
  if (!c.n_layer || !c.d_model || !c.n_head || !c.d_ff || !c.vocab)
    throw std::runtime_error("incomplete llama hyper-parameters in GGUF");
  if (c.n_head % c.n_head_kv) throw std::runtime_error("n_head not a multiple of n_head_kv");
  if (c.head_dim > 128) throw std::runtime_error("head_dim > 128 unsupported");
  if (c.n_head / c.n_head_kv > 16) throw std::runtime_error("GQA group > 16 unsupported");
  return c;
}

std::string ModelConfig::describe() const {
  std::ostringstream o;
  o << "arch=" << arch << " n_layer=" << n_layer << " d_model=" << d_model << " n_head=" << n_head
    << " n_head_kv=" << n_head_kv << " head_dim=" << head_dim << " d_ff=" << d_ff << " vocab=" << vocab
    << " rope_base=" << rope_base;
  if (n_expert) o << " n_expert=" << n_expert << " n_expert_used=" << n_expert_used;
  if (rope_neox) o << " rope=neox";
  if (qkv_bias) o << " qkv_bias";
  return o.str();
}

SplitMode parse_split_mode(const std::string& s) {
  if (s == "even") return SPLIT_EVEN;
  if (s == "mem" || s == "memory") return SPLIT_MEM;
  if (s == "cost" || s == "halda") return SPLIT_COST;
  throw std::runtime_error("unknown split mode: " + s);
}

std::vector<StageSpec> partition_layers(const std::vector<double>& cost, double first_extra, double last_extra,
                                        const std::vector<double>& dev_speed, SplitMode mode) {
  const int L = (int)cost.size();
  const int S = (int)dev_speed.size();
  if (S < 1) throw std::runtime_error("partition: no stages");
  if (S > L) throw std::runtime_error("partition: more stages than layers");
  std::vector<StageSpec> out(S);
  if (mode == SPLIT_EVEN) {
    int b = 0;
    for (int s = 0; s < S; ++s) {
      const int n = L / S + (s < L % S ? 1 : 0);
      out[s].layer_begin = b;
      out[s].layer_end = b + n;
      b += n;
    }
  } else {
    // Contiguous partition minimising max_s cost_s / speed_s (DP, O(S L^2)).
    // SPLIT_MEM ignores the embedding/head extras (pure weight-bytes balance).
    const double fe = mode == SPLIT_COST ? first_extra : 0.0;
    const double le = mode == SPLIT_COST ? last_extra : 0.0;
    std::vector<double> pre(L + 1, 0.0);
    for (int i = 0; i < L; ++i) pre[i + 1] = pre[i] + cost[i];
    const double INF = std::numeric_limits<double>::infinity();
    // best[s][j]: minimal max-cost placing layers [0, j) on stages [0, s]
    std::vector<std::vector<double>> best(S, std::vector<double>(L + 1, INF));
    std::vector<std::vector<int>> arg(S, std::vector<int>(L + 1, -1));
    auto seg = [&](int s, int a, int b) {
      double c = pre[b] - pre[a];
      if (s == 0) c += fe;
      if (s == S - 1) c += le;
      return c / std::max(dev_speed[s], 1e-9);
    };
    for (int j = 1; j <= L; ++j) best[0][j] = seg(0, 0, j);
    for (int s = 1; s < S; ++s)
      for (int j = s + 1; j <= L; ++j)
        for (int i = s; i < j; ++i) {
          const double v = std::max(best[s - 1][i], seg(s, i, j));
          if (v < best[s][j]) { best[s][j] = v; arg[s][j] = i; }
        }
    int j = L;
    for (int s = S - 1; s >= 0; --s) {
      const int i = s == 0 ? 0 : arg[s][j];
      out[s].layer_begin = i;
      out[s].layer_end = j;
      j = i;
    }
  }
  for (int s = 0; s < S; ++s) { out[s].stage = s; out[s].n_stages = S; out[s].device = s; }
  return out;
}

}  // namespace mp
