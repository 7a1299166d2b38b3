// CpuStage: a pipeline stage on the host CPU.  Same Stage contract as HipStage (contiguous layer
// range, per-micro-batch activations, KV cache per sequence slot, prefill chunks + decode steps),
// computed in f32 directly from the GGUF bytes (weights stay in the mmap, rows are dequantised
// on the fly into a per-thread buffer).
//
// Roles: BASELINE.json config 1 (the reference's "single-stage via orchestrator on the CPU
// backend", llama.cpp CPU path, `README.md:49` of the reference), the CPU test vehicle of the
// whole pipeline runtime (multi-stage, multi-process over TCP) on machines without a GPU, and a
// second numerical oracle (independent of the HIP kernels) for the engine tests.
#pragma once
#include <memory>
#include <vector>

#include "model.h"
#include "cpu_qdot.h"
#include "stage.h"
#include "threadpool.h"

namespace mp {

struct CpuMat {
  const uint8_t* data = nullptr;   // N rows of row_bytes(type, K)
  int type = 0;
  int64_t N = 0, K = 0;
  size_t rb = 0;
};

class CpuStage : public Stage {
 public:
  CpuStage(const ModelConfig& cfg, const StageSpec& spec, const StageOptions& opt);
  ~CpuStage() override;

  bool is_gpu() const override { return false; }
  const StageSpec& spec() const override { return spec_; }
  hipStream_t stream() const override { return nullptr; }
  void load_gguf(const GgufFile& f) override;
  void init_synthetic(const std::string& ftype, uint64_t seed) override;
  void alloc_runtime() override;

  float* act(int mb) override { return act_[mb].data(); }
  int32_t* tokens(int mb) override { return tok_[mb].data(); }
  int32_t* prompt_buf() override { return prompt_.data(); }
  void set_positions(int mb, const std::vector<int32_t>& pos) override;
  void prefill(int mb, const std::vector<PrefillSeg>& segs, hipStream_t st) override;
  void prefill_finish(int mb, hipStream_t st, const std::vector<int>* rows = nullptr) override;
  void copy_verify_tokens(int mb, int32_t* host, int n) override;
  void decode(int mb, hipStream_t st) override;
  const float* logits_ptr() const override { return logits_.data(); }
  int logits_ld() const override { return cfg_.vocab; }
  size_t weight_bytes() const override { return weight_bytes_; }
  size_t kv_bytes() const override { return kv_bytes_; }

 private:
  struct Layer {
    std::vector<float> attn_norm, ffn_norm;
    CpuMat q, k, v, o, gate, up, down;
    std::vector<float> bq, bk, bv;   // Qwen2 q/k/v biases (empty: none)
    bool moe = false;
    CpuMat router;
    std::vector<CpuMat> eg, eu, ed;   // experts
  };
  // Y[m][n] (+)= sum_k W[n][k] X[m][k]
  void matmul(const CpuMat& W, const float* X, int ldx, int M, float* Y, int ldy, bool accumulate);
  void rmsnorm(const float* x, const std::vector<float>& w, float* y, int M);
  void layer_forward(int li, int M, float* x, const int32_t* pos, const int32_t* slot);
  void ffn(const Layer& L, int M, const float* xn, float* x);
  void head(int mb, int M, const float* x, int32_t* tok_out, uint64_t salt);
  void set_history(int mb, const std::vector<std::vector<int32_t>>& seqs) override;
  void kv_export(int slot, int n_tok, std::vector<uint8_t>& out) override;
  void set_block_table(const std::vector<int32_t>& table) override;
  void kv_import(int slot, int n_tok, const uint8_t* data, size_t bytes) override;
  size_t kv_state_bytes(int n_tok) const override;
  uint64_t sample_step() override { return step_; }
  void set_sample_step(uint64_t s) override { step_ = s; }
  const char* backend_name() const override { return "cpu"; }
  int sample_row(const float* logits, uint64_t salt, int row);
  CpuMat own_random(int type, int64_t N, int64_t K, uint64_t seed);

  ModelConfig cfg_;
  StageSpec spec_;
  StageOptions opt_;
  std::unique_ptr<ThreadPool> pool_;
  std::vector<std::vector<uint8_t>> owned_;
  size_t weight_bytes_ = 0, kv_bytes_ = 0;
  std::vector<Layer> layers_;
  CpuMat embd_, out_;
  std::vector<float> out_norm_;
  std::vector<float> inv_freq_;
  // KV: [layer][slot][ctx][kv_dim]
  std::vector<std::vector<float>> kc_, vc_;   // per layer: (kv_pages + 1) pages of [64][kv_dim]
  std::vector<int32_t> bt_;                    // block table [n_slots][max_pages] (kvpager.h)
  int max_pages_ = 0, n_pages_ = 0;
  size_t kv_row(int slot, int pos) const;      // page row of (slot, position)
  // per micro-batch
  std::vector<std::vector<float>> act_;
  std::vector<std::vector<int32_t>> tok_, pos_;
  std::vector<int32_t> prompt_;
  std::vector<std::vector<float>> last_h_;   // last stage: [mb][B][d] final prompt rows
  std::vector<std::vector<int32_t>> vtok_;   // last stage: [mb][rows] greedy tokens of a verify chunk
  std::vector<float> logits_;
  // scratch
  std::vector<float> xn_, qkv_, att_, h_, gu_;
  Q8Buf xq_;   // matmul: the activation rows as int8 blocks (cpu_q8)
  uint64_t step_ = 0;
  std::vector<std::vector<int32_t>> hist_;   // per slot: accepted tokens, most recent last
};

}  // namespace mp
