// Model hyper-parameters (from GGUF metadata) and the pipeline stage partitioner.
//
// Partitioner = the new build's answer to llama.cpp's layer->device assignment (E4: -ngl +
// tensor_split by free memory, upstream; not in mount) and to the PDF's Halda scheduler
// (D2, PDF p.5 / p.8): contiguous layer ranges per stage, minimising the slowest stage's cost
// where cost = bytes streamed per decode step / device bandwidth weight, with the token
// embedding charged to stage 0 and the LM head to the last stage.
#pragma once
#include <string>
#include <vector>

namespace mp {

class GgufFile;

struct ModelConfig {
  std::string arch = "llama";
  std::string name;
  int n_layer = 0, d_model = 0, n_head = 0, n_head_kv = 0, head_dim = 0, d_ff = 0, vocab = 0;
  int n_ctx_train = 0;
  float rope_base = 10000.f, eps = 1e-5f;
  int n_expert = 0, n_expert_used = 0;
  bool rope_freqs = false;
  bool tied_output = false;
  // Qwen2 family (arch "qwen2"): q/k/v projections carry biases, and RoPE rotates the pairs
  // (i, i + hd/2) ("NEOX" mode) instead of (2i, 2i+1).  The stages permute the rows of Wq / Wk
  // (and the q/k biases) per head at load time, new row 2i <- i, 2i+1 <- i + hd/2 (neox_src_row),
  // which turns NEOX rotation into the adjacent-pair rotation the kernels implement; q.k is
  // invariant under the shared permutation and V is untouched, so no kernel changes.
  bool rope_neox = false;
  bool qkv_bias = false;

  int q_dim() const { return n_head * head_dim; }
  int kv_dim() const { return n_head_kv * head_dim; }
  int padded_head_dim() const { return head_dim <= 64 ? 64 : 128; }
  static ModelConfig from_gguf(const GgufFile& f);
  std::string describe() const;
};

// source row of permuted q/k row r (rope_neox): within a head of hd rows, 2i <- i, 2i+1 <- i + hd/2
inline long neox_src_row(long r, int hd) {
  const long h = r / hd, j = r % hd;
  return h * hd + ((j & 1) ? j / 2 + hd / 2 : j / 2);
}

struct StageSpec {
  int stage = 0, n_stages = 1;
  int layer_begin = 0, layer_end = 0;   // [begin, end)
  int device = 0;
  bool first() const { return stage == 0; }
  bool last() const { return stage == n_stages - 1; }
};

enum SplitMode { SPLIT_EVEN = 0, SPLIT_MEM = 1, SPLIT_COST = 2 };
SplitMode parse_split_mode(const std::string& s);

// layer_cost[i]: cost units of layer i; first_extra / last_extra: embedding / head cost;
// dev_speed[s]: relative throughput of stage s's device (1.0 = reference). Returns S ranges.
std::vector<StageSpec> partition_layers(const std::vector<double>& layer_cost, double first_extra,
                                        double last_extra, const std::vector<double>& dev_speed,
                                        SplitMode mode);

}  // namespace mp
