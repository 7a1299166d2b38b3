// Stage interface: one pipeline stage (contiguous layer range) on one device.
//   HipStage: MI355X, hand-written HIP kernels, hipGraph decode (hip_stage.h)
//   CpuStage: host reference / plumbing backend (BASELINE.json config 1: "single-stage via
//             orchestrator on the CPU backend"; also the CPU test vehicle of the pipeline runtime)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "model.h"

namespace mp {

class GgufFile;

struct StageOptions {
  int n_mb = 1;             // micro-batches in flight
  int mb_size = 1;          // sequences per micro-batch
  int max_ctx = 2048;       // KV capacity per sequence (multiple of 64)
  int prefill_chunk = 512;  // max tokens per prefill chunk (8B: 31.5k prompt tok/s vs 24.3k at 256)
  bool use_graphs = true;
  int attn_split_len = 0;   // decode flash-decoding split length (multiple of 128; 0 = auto)
  int threads = 0;          // CPU backend worker threads (0 = hardware concurrency)
  bool cpu_q8 = true;       // CPU backend: quantized weights x int8 activation blocks (cpu_qdot.cpp); false: f32
                            // dequant + f32 dot (exact to the fp32 oracle)
  bool fused_attn = true;   // decode: one fused RoPE + KV-append + attention + merge kernel
  int attn_o_max_ctx = 512;   // single-stream decode: attention + o-projection in one launch up to this max_ctx (0 = off)
  bool prefill_gemm = true; // prompt chunks > 16 rows: MFMA dequant-GEMM instead of 16-row GEMVs
  bool int8_gemm = false;   // M > 64 GEMMs on v_mfma_i32_16x16x64_i8: per-row int8 activations x per-row int8
                            // re-quantized weights (+1 B/weight of HBM; reduced precision, opt-in)
  bool gemm_splitk_store = true;   // M > 64 split-K GEMMs: per-split partial stores + a fixed-order reduction
                                   // (into the residual: absorbed by the next RMSNorm) instead of float atomics
  int prefill_gemm_v = 0;    // 0: auto (quantized: v4 for gate/up and the LM head, v2 for the split-K projections;
                             // 16-bit: v3); 4: gemm4 (32x32x16); 3: gemm3; 2: gemm2 (128 x 256); 1: 64 x 64
  bool prefill_flash = true; // prompt chunks: the LDS-tiled prefill flash attention (attn_prefill.hip)
  bool kv_fp8 = false;       // kv_dtype "fp8": KV pages hold OCP e4m3 bytes
  int kv_pages = 0;          // KV pool pages per stage (64 tokens each; 0: n_slots x max_ctx / 64)
  bool deterministic = false;  // split-K and MoE partials reduced in a fixed order (no float atomics
                               // on shared outputs): bitwise-reproducible logits, PP=1 == PP=S
  bool fused_norm = false;  // M <= 4 rows: deferred RMSNorm folded into the qkv / gate-up GEMVs (gemv2.hip);
                            // off by default: 8B mb1 470.7 vs 473.7 tok/s, 70B mb1 92.5 vs 104.8 (r2i)
  bool moe_gemm = true;     // M > 64 MoE FFN on the grouped expert GEMM (gemm4.hip) instead of 64-row GEMV slices
  bool small_gemv = true;   // M <= 4 rows: the gemvs kernels (gemvs.hip: x staged once per workgroup,
                            // RMSNorm fused into the qkv / gate-up / LM-head GEMVs, in-workgroup split-K)
};

struct PrefillSeg {
  int b = 0;          // sequence row within the micro-batch
  int p0 = 0;         // first position of this segment
  int T = 0;          // tokens
  bool last = false;  // ends the prompt
  bool verify = false;  // speculative verification chunk: the last stage scores EVERY row (greedy
                        // argmax after each row -> verify_tokens), nothing is kept for prefill_finish
};

class Stage {
 public:
  virtual ~Stage() = default;
  virtual bool is_gpu() const = 0;
  virtual const StageSpec& spec() const = 0;
  virtual hipStream_t stream() const = 0;                 // nullptr on CPU
  virtual void load_gguf(const GgufFile& f) = 0;
  virtual void init_synthetic(const std::string& ftype, uint64_t seed) = 0;
  virtual void alloc_runtime() = 0;
  virtual void capture_graphs() {}

  // per micro-batch buffers (device memory for HIP, host memory for CPU)
  virtual float* act(int mb) = 0;          // [rows][d] f32 residual in/out
  virtual int32_t* tokens(int mb) = 0;     // [mb_size]
  virtual int32_t* prompt_buf() = 0;       // [n_slots][max_ctx] token ids (first stage)
  virtual void set_positions(int mb, const std::vector<int32_t>& pos) = 0;
  // Packed prefill: one chunk = segments of several sequences of micro-batch mb (rows stacked in
  // segment order, sum of T <= prefill_chunk).  The projections run as ONE GEMM over all rows
  // (weights read once per chunk, not per sequence); attention runs per segment.  The first
  // stage embeds the tokens from prompt_buf(); for a segment with `last` set, the last stage
  // keeps the final row's hidden state for prefill_finish().
  virtual void prefill(int mb, const std::vector<PrefillSeg>& segs, hipStream_t st) = 0;
  // last stage: LM head + sampling over the kept rows -> tokens(mb)[b] for every sequence of mb;
  // with `rows`, only those rows' tokens change (continuous batching admits sequences into some
  // rows while the others are mid-generation)
  virtual void prefill_finish(int mb, hipStream_t st, const std::vector<int>* rows = nullptr) = 0;
  virtual void decode(int mb, hipStream_t st) = 0;
  // last stage, after a prefill() of verify segments of micro-batch mb: the greedy next token after
  // each of the chunk's n rows (row order = segment order) -> host
  virtual void copy_verify_tokens(int mb, int32_t* host, int n) = 0;
  virtual const float* logits_ptr() const = 0;   // last computed logits (device/host)
  virtual int logits_ld() const = 0;
  virtual size_t weight_bytes() const = 0;
  virtual size_t kv_bytes() const = 0;
  // sampling configuration for the last stage (temp <= 0: greedy)
  virtual void set_sampling(float temp, int top_k, float top_p, float min_p, uint64_t seed) {
    temp_ = temp; top_k_ = top_k; top_p_ = top_p; min_p_ = min_p; seed_ = seed;
  }
  // repetition penalties (llama.cpp penalties sampler, applied before the cuts): every distinct
  // token among the last `last_n` accepted tokens of a sequence (prompt included) with count c
  // gets l = l > 0 ? l / repeat : l * repeat, then l -= c * freq + presence
  virtual void set_penalties(int last_n, float repeat, float freq, float presence) {
    pen_last_n_ = last_n < 0 ? 0 : last_n; pen_repeat_ = repeat; pen_freq_ = freq; pen_presence_ = presence;
  }
  bool penalties_on() const {
    return pen_last_n_ > 0 && (pen_repeat_ != 1.f || pen_freq_ != 0.f || pen_presence_ != 0.f);
  }
  // last stage: seed the penalty window of micro-batch mb (row b <- seqs[b], its last tokens)
  virtual void set_history(int mb, const std::vector<std::vector<int32_t>>& seqs) { (void)mb; (void)seqs; }

  // Checkpoint / resume (the reference has none beyond re-reading the GGUF):
  // the KV of sequence slot `slot` (= mb * mb_size + row) for positions [0, n_tok) of every layer
  // of this stage as opaque bytes in the backend's own layout (HIP: bf16-class f16 pages, CPU:
  // f32 rows), appended to `out`; kv_import writes the same bytes back.  Called with the stage
  // idle (between decode_steps calls).
  virtual void kv_export(int slot, int n_tok, std::vector<uint8_t>& out) = 0;
  // paged KV (kvpager.h): the block table [n_slots][max_ctx / 64] of page ids (kv_pages = TRASH),
  // installed between engine calls (the stage's stream is idle or synchronised first)
  virtual void set_block_table(const std::vector<int32_t>& table) = 0;
  virtual void kv_import(int slot, int n_tok, const uint8_t* data, size_t bytes) = 0;
  virtual size_t kv_state_bytes(int n_tok) const = 0;   // bytes kv_export appends for n_tok
  // sampling step counter (seeds the per-row RNG streams of the sampler)
  virtual uint64_t sample_step() = 0;
  virtual void set_sample_step(uint64_t s) = 0;
  virtual const char* backend_name() const = 0;

 protected:
  float temp_ = 0.f, top_p_ = 1.f, min_p_ = 0.f;
  int top_k_ = 0;
  uint64_t seed_ = 0;
  int pen_last_n_ = 64;
  float pen_repeat_ = 1.f, pen_freq_ = 0.f, pen_presence_ = 0.f;
};

}  // namespace mp
