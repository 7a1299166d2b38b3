// HipStage: one pipeline stage on one MI355X = a contiguous layer range, its packed weights in
// HBM, its share of the paged KV cache, per-micro-batch I/O buffers and one captured hipGraph per
// micro-batch for the decode step (E5/E6/E9 of SURVEY.md §2.2, MI355X-native).
#pragma once
#include <hip/hip_runtime.h>

#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <chrono>
#include <vector>

#include "kernels_api.h"
#include "model.h"
#include "qtypes.h"
#include "stage.h"

namespace mp {

class GgufFile;

#define HIP_OK(x)                                                                                  \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + \
                                                   " at " + __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)

// ggml types of the 2-D weights when initialising a synthetic model on device
struct SyntheticTypes {
  int embd = T_Q4_K, q = T_Q4_K, k = T_Q4_K, v = T_Q4_K, o = T_Q4_K, gate = T_Q4_K, up = T_Q4_K,
      down = T_Q4_K, out = T_Q6_K;
  static SyntheticTypes from_ftype(const std::string& ftype, int layer, int n_layer);
};

struct PackedMat {
  uint8_t* d = nullptr;
  int ptype = -1;
  PackedDims dims{};
  uint8_t* i8 = nullptr;    // int8_gemm: per-row int8 re-quantized copy (P_I8 chunks) ...
  float* i8_ws = nullptr;   // ... and its row scales
  size_t bytes() const { return dims.bytes; }
};

struct MatSeg {  // one launch of a (possibly merged) projection
  PackedMat m;
  int y_off = 0;  // output column offset
};

struct ExpertW {  // MoE layer weights (Mixtral); experts stored back to back
  PackedMat gateup;            // E interleaved gate/up matrices, stride gateup_stride bytes
  size_t gateup_stride = 0;
  PackedMat down;              // E down matrices
  size_t down_stride = 0;
  PackedMat router;            // [E][d] router (f16 packed)
  f16* router_dense = nullptr;  // the router unpacked to dense f16 [E_pad][nsb*256] (launch_router_logits)
};

struct LayerW {
  float* attn_norm = nullptr;
  float* ffn_norm = nullptr;
  std::vector<MatSeg> qkv;
  float* qkv_bias = nullptr;  // [q | k | v] f32 (Qwen2), q/k rows NEOX-permuted like the weights
  PackedMat wo;
  bool fused_gateup = true;
  PackedMat gateup;           // interleaved (fused SwiGLU)
  PackedMat gate, up;         // unfused fallback
  PackedMat down;
  bool moe = false;
  ExpertW ex;
};

class HipStage : public Stage {
 public:
  HipStage(const ModelConfig& cfg, const StageSpec& spec, const StageOptions& opt);
  ~HipStage() override;

  bool is_gpu() const override { return true; }
  void load_gguf(const GgufFile& f) override;
  void init_synthetic(const std::string& ftype, uint64_t seed) override;
  void alloc_runtime() override;   // KV cache, buffers, rope tables (after weights)

  const StageSpec& spec() const override { return spec_; }
  const ModelConfig& cfg() const { return cfg_; }
  hipStream_t stream() const override { return stream_; }
  int device() const { return spec_.device; }

  float* act(int mb) override { return act_[mb]; }          // [act_rows][d] f32 residual in/out
  int32_t* tokens(int mb) override { return tok_[mb]; }     // [mb_size] (first: input, last: output)
  int32_t* prompt_buf() override { return prompt_dev_; }
  int act_rows() const { return act_rows_; }
  int slot_of(int mb, int b) const { return mb * opt_.mb_size + b; }
  int dec_slot0_ = -1;   // decode: slot of row 0 of the micro-batch being recorded (decode attention)

  // positions of micro-batch mb (host values) before decode; kvlen = pos + 1
  void set_positions(int mb, const std::vector<int32_t>& pos) override;

  // packed prefill chunk (see Stage::prefill) and the head over the kept last rows
  void prefill(int mb, const std::vector<PrefillSeg>& segs, hipStream_t st) override;
  void prefill_finish(int mb, hipStream_t st, const std::vector<int>* rows = nullptr) override;
  void copy_verify_tokens(int mb, int32_t* host, int n) override;

  // One decode step for micro-batch mb (graph replay if captured).
  void decode(int mb, hipStream_t st) override;
  void capture_graphs() override;
  void destroy_graphs();
  // sampling parameters are baked into the decode graphs: re-capture when they change
  void set_sampling(float temp, int top_k, float top_p, float min_p, uint64_t seed) override;
  void set_penalties(int last_n, float repeat, float freq, float presence) override;
  void set_history(int mb, const std::vector<std::vector<int32_t>>& seqs) override;

  size_t weight_bytes() const override { return weight_bytes_; }
  size_t kv_bytes() const override { return kv_bytes_; }
  void kv_export(int slot, int n_tok, std::vector<uint8_t>& out) override;
  void set_block_table(const std::vector<int32_t>& table) override;
  void kv_import(int slot, int n_tok, const uint8_t* data, size_t bytes) override;
  size_t kv_state_bytes(int n_tok) const override;
  uint64_t sample_step() override;
  void set_sample_step(uint64_t s) override;
  const char* backend_name() const override { return "hip"; }
  const float* logits_ptr() const override { return logits_; }
  int logits_ld() const override { return logits_ld_; }

  // decode body without graph (captured by capture_graphs)
  void decode_eager(int mb, hipStream_t st);

 private:
  void layer_forward(int li, int M, float* x, const int32_t* pos, const int32_t* kvlen, const int32_t* slot,
                     bool decode, hipStream_t st);
  void moe_ffn(const LayerW& L, int M, hipStream_t st, float* x);
  void moe_ffn_rows(const LayerW& L, int r0, int M, hipStream_t st, float* x, bool grouped = false);
  bool fuse_norm(int M) const;
  void build_i8_copies();
  int8_t* xq_ = nullptr; float* xqs_ = nullptr; int xq_ld_ = 0;   // int8_gemm: quantized activation rows
  const void* xq_src_ = nullptr; int xq_rows_ = 0;   // the f16 rows xq_ currently holds (set by norm_x / the quant)
  bool attention_o(int li, int M, const int32_t* pos, const int32_t* slot, float* x, hipStream_t st, bool pre = false);
  void attention(int li, int M, const int32_t* pos, const int32_t* kvlen, const int32_t* slot, bool decode,
                 hipStream_t st, bool qkv_deferred, bool pre = false);
  DecodeAttnParams decode_attn_params(int li, int M, const int32_t* pos, const int32_t* slot, bool qkv_deferred) const;
  bool small_path(int M) const { return opt_.small_gemv && M <= 4; }
  // gemvs (M <= 4): Xf != nullptr fuses the RMSNorm of the f32 rows Xf with gamma
  void gemv_small(const PackedMat& m, int epi, const f16* X, int ldx, const float* Xf, const float* gamma, int M,
                  float* Y, int ldy, f16* H, int ldh, int n_valid, const float* bias, hipStream_t st,
                  const QkvAppend* qa = nullptr);
  size_t kv_eb() const { return opt_.kv_fp8 ? 1 : 2; }   // bytes per cached K/V element
  int det_splits(int ntiles, int nsb, int M, int epi, bool allow_split = true) const;   // RMSNorm folded into the consuming GEMVs at this row count
  void flush_sk(hipStream_t st);
  // RMSNorm of the residual x into xn_ (absorbing pending split-K partials of x first)
  void norm_x(float* x, const float* w, int M, float* zero, int64_t zero_n, hipStream_t st, const float* bias = nullptr,
              int bias_n = 0);
  void gemv(const PackedMat& m, int epi, const f16* X, int ldx, int M, float* Y, int ldy, f16* H, int ldh,
            int n_valid, bool allow_split, hipStream_t st,
            const GemvParams* extras = nullptr);
  void head(int mb, int M, const float* x, int32_t* tok_out, uint64_t salt, hipStream_t st);
  void ensure_hist();
  // pinned double-buffered weight staging (load_gguf)
  struct Staging {
    uint8_t* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool busy[2] = {false, false};
    size_t cap = 0, bytes = 0;
    int cur = 0;
    hipStream_t st = nullptr;
    std::chrono::steady_clock::time_point t0;
  } stg_;
  double upload_gbps_ = 0;
  void stage_begin();
  void stage_end();
  void stage_put(uint8_t* dst, size_t bytes, size_t granule, const std::function<void(uint8_t*, size_t, size_t)>& fill);
  PackedMat upload_packed(int ggml_type, int64_t N, int64_t K, const std::function<const uint8_t*(int64_t)>& row);
  // E matrices of N x K packed back to back (MoE experts); row(e, n)
  PackedMat upload_packed_experts(int ggml_type, int E, int64_t N, int64_t K, size_t* stride,
                                  const std::function<const uint8_t*(int, int64_t)>& row);
  PackedMat alloc_packed_random(int ggml_type, int64_t N, int64_t K, uint64_t seed);
  float* upload_f32(const float* h, size_t n);
  void* dmalloc(size_t bytes);

  ModelConfig cfg_;
  StageSpec spec_;
  StageOptions opt_;
  hipStream_t stream_ = nullptr;
  std::vector<void*> allocs_;
  size_t weight_bytes_ = 0, kv_bytes_ = 0;

  // weights
  std::vector<LayerW> layers_;
  uint8_t* embd_raw_ = nullptr; int embd_type_ = 0; size_t embd_row_bytes_ = 0;
  float* out_norm_ = nullptr;
  PackedMat out_;

  // dims
  int Kd_ = 0, Ko_ = 0, Kff_ = 0, qkv_n_ = 0, Dp_ = 0;
  int act_rows_ = 0, scratch_rows_ = 0;

  // scratch (shared by micro-batches: compute is serial on the stage's stream)
  static constexpr int kPrefillMaxSplit = 8;
  float* pf_opart_ = nullptr; float* pf_ml_ = nullptr;   // prefill attention KV-split partials
  float* det_part_ = nullptr; size_t det_part_n_ = 0;   // deterministic split-K partials
  float* moe_yslot_ = nullptr;                           // deterministic MoE per-slot down outputs
  float* ssq_ = nullptr;   // [64] deferred-norm sums of squares, immediately followed by qkv_
  f16* xn_ = nullptr; float* qkv_ = nullptr; f16* q_ = nullptr; f16* attn_ = nullptr; f16* h_ = nullptr;
  float* gu_ = nullptr;   // unfused gate|up f32
  float* logits_ = nullptr; int logits_ld_ = 0;
  ArgmaxScratch am_{nullptr, nullptr, 0};   // two-level argmax partials / arrival counters
  float* sk_part_ = nullptr; size_t sk_part_n_ = 0;   // gemm_splitk_store: per-split GEMM partials
  // split-K partials of the last o / down GEMM not yet added into the residual x: the next RMSNorm
  // of x absorbs them (norm_x), anything else reading x first calls flush_sk
  struct SkPending { float* x = nullptr; int M = 0, n = 0, ldy = 0, ns = 0, ldp = 0; int64_t ss = 0; };
  SkPending sk_pend_;
  float* sk_defer_ = nullptr;   // gemv(): ATOMIC GEMMs into this buffer defer their reduction
  float* o_part_ = nullptr; float* ml_part_ = nullptr; int n_split_ = 1;
  int32_t* attn_cnt_ = nullptr;   // fused decode attention: split arrival counters
  // MoE scratch
  float* moe_logits_ = nullptr; int32_t* moe_counts_ = nullptr; int32_t* moe_lists_ = nullptr;
  float* moe_w_ = nullptr; f16* moe_h_ = nullptr;
  // KV
  std::vector<f16*> kc_, vc_;
  int32_t* block_table_ = nullptr; int max_pages_ = 0; int n_pages_ = 0;   // paged KV (kvpager.h)
  std::vector<int32_t> host_bt_;                                            // host copy of the table
  float2* rope_cs_ = nullptr;
  std::vector<float> rope_ff_;
  // per-mb I/O
  std::vector<float*> act_;
  std::vector<int32_t*> tok_, pos_, kvlen_, slot_;
  int32_t* step_ = nullptr;
  int32_t* tok_tmp_ = nullptr;   // row-selective prefill_finish
  // repetition-penalty windows (last stage): [n_mb][mb_size][hist_n_] token ring, -1 = empty,
  // and the per-row count of accepted tokens (ring position)
  int32_t* hist_ = nullptr;
  int32_t* hist_cnt_ = nullptr;
  int hist_n_ = 0;
  // prefill metadata
  int32_t* pf_pos_ = nullptr; int32_t* pf_kvlen_ = nullptr; int32_t* pf_slot_ = nullptr;
  int32_t* prompt_dev_ = nullptr;
  std::vector<float*> last_h_;                       // last stage: [mb][B][d] final prompt rows
  float* vlogits_ = nullptr;                          // last stage, speculative verify: [chunk][logits_ld_]
  int32_t* vtok_ = nullptr;                           // [n_mb][chunk] greedy token after each verify row
  const std::vector<PrefillSeg>* segs_ = nullptr;    // segments of the prefill in progress
  // graphs
  std::vector<hipGraphExec_t> graphs_;
};

// device random init (init.hip)
void launch_init_packed(uint8_t* W, size_t nbytes, int pt, float scale, uint64_t seed, hipStream_t st);
void launch_init_raw(uint8_t* W, int64_t nblocks, int t, float scale, uint64_t seed, hipStream_t st);

}  // namespace mp
