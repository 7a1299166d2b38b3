// Engine = model + partition + stage workers + links + the micro-batched piped-ring scheduler.
//
// This replaces, MI355X-first, what the reference assembles from `llama-cli --rpc ... -ngl 99`
// (orchestrator/src/main.rs:35-57): llama.cpp's backend scheduler runs the layer splits of the two
// rpc-servers strictly one after the other (E7).  Here every stage owns a GPU and
// runs concurrently: M micro-batches circulate through the S stages (activations forward,
// sampled token ids from the last stage back to the first: the PDF's "piped-ring", D1), each
// stage overlaps its sends/receives (dedicated comm streams, events) with the compute of the
// other micro-batches.
//
// Modes (config "mode"):
//   "local" : all stages in this process, one host thread each; devices from "devices" (may
//             repeat a device for single-GPU PP emulation); links "local" (D2D) or "rccl".
//   "mp"    : one stage per process (torch.distributed / torchrun launch): config carries
//             "world", "rank" and the RCCL unique ids of the links this rank participates in.
#pragma once
#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hip_stage.h"
#include "json.h"
#include "kvpager.h"
#include "model.h"
#include "threadpool.h"
#include "transport.h"

namespace mp {

class GgufFile;

struct Item {
  enum Kind { PREFILL, PREFILL_END, DECODE } kind;
  int mb = 0;
  int T = 0;                      // PREFILL: total rows of the packed chunk
  std::vector<PrefillSeg> segs;   // PREFILL: sequences (segments) packed into the chunk
  int round = 0;
  std::vector<int> rows;          // PREFILL_END of an admission: only these rows get a new token
};

struct StepStats {
  std::vector<double> token_ms;   // inter-token latency samples (per micro-batch per round)
  double wall_ms = 0;
};

class Engine {
 public:
  explicit Engine(const Json& cfg);
  ~Engine();

  Json info() const;
  const ModelConfig& model() const { return cfg_; }
  int n_stages() const { return S_; }
  int n_mb() const { return M_; }
  int mb_size() const { return B_; }
  int max_ctx() const { return max_ctx_; }
  int kv_pages() const { return kv_pages_; }
  // config of a replacement engine after a fault: the failed stage's device dropped, layers
  // re-partitioned over the survivors (see engine.cpp)
  static Json failover_config(const Json& cfg, const Json& health);
  int kv_free_pages() const { return pager_.free_pages(); }
  double load_ms() const { return load_ms_; }
  bool owns_last() const;
  bool owns_first() const;

  // assign prompts to slots (sequence i -> mb i / B, row i % B), prefill them, produce token 0
  void start(const std::vector<std::vector<int32_t>>& prompts);
  // run k decode rounds (every micro-batch once per round); blocks until the GPU work is done
  StepStats decode_steps(int k);
  // generated tokens so far per sequence (valid where the last stage lives)
  std::vector<std::vector<int32_t>> tokens() const;

  // Continuous batching: between decode rounds, prefill new sequences into the
  // given sequence slots (slot = mb * mb_size + row) while the other slots keep their state; each
  // admitted slot gets its first token like start().  release() marks a slot idle (its row keeps
  // computing garbage until re-admitted; its position is recycled before it could leave the slot's
  // KV pages).  Every process of a multi-process pipeline must make the same calls.
  void admit(const std::vector<int>& slots, const std::vector<std::vector<int32_t>>& prompts);
  void release(int slot);
  int32_t last_token(int slot) const { return slot < (int)gen_.size() && !gen_[slot].empty() ? gen_[slot].back() : -1; }
  int slot_position(int slot) const { return slot_pos((size_t)slot); }
  bool started() const { return started_; }
  bool slot_active(int slot) const { return slot >= 0 && slot < (int)active_.size() && active_[slot]; }

  Json generate(const std::vector<std::vector<int32_t>>& prompts, int n_predict,
                std::vector<std::vector<int32_t>>* out);
  // Speculative decoding by prompt lookup (greedy; every stage in this process): see engine.cpp
  Json spec_generate(const std::vector<std::vector<int32_t>>& prompts, int n_predict, int draft_max, int ngram,
                     std::vector<std::vector<int32_t>>* out);
  Json bench(int prompt_len, int warmup, int steps);
  int copy_logits(int mb, float* out, int rows);
  // Chrome-trace timeline of compute / send / recv spans per stage
  void enable_trace(bool on);
  void write_trace(const std::string& path) const;
  // heartbeat counters + link byte counters per owned stage; "ok" false after a fault
  Json health() const;
  // Checkpoint / resume of a running generation: between decode_steps calls,
  // write every owned stage's KV shard (only the used positions of each sequence), its current
  // input tokens and sampler step to <dir>/stage<k>.bin, and the sequences (prompts, generated
  // tokens, rounds done) to <dir>/session.json (by the owner of the last stage).  load_state on an
  // engine built with the same model / partition / micro-batch shape continues the generation
  // exactly where it stopped (greedy and seeded sampling alike).
  Json save_state(const std::string& dir);
  Json load_state(const std::string& dir);

  // streaming hook: called on the host (from the worker of the last stage) after each round
  // with (sequence index, token) pairs
  std::function<void(int seq, int32_t tok)> on_token;
  // spec_generate: a sequence for which this returns false is finished (e.g. end of generation)
  std::function<bool(int seq)> keep_going;
  const Json& config() const { return jcfg_; }

 private:
  struct Worker {
    std::unique_ptr<Stage> stage;
    Link* in = nullptr;    // activations from s-1 (or ring tokens from S-1 for s = 0)
    Link* out = nullptr;   // activations to s+1 (or ring tokens to 0 for s = S-1)
    hipStream_t send_st = nullptr, recv_st = nullptr;
    std::vector<hipEvent_t> comp_ev, sent_ev, recv_ev;
    std::vector<bool> sent_valid;
    std::vector<uint64_t> sent_seq;   // Link::last_seq() of each micro-batch's last send
    std::vector<hipEvent_t> tok_ev;   // last stage: per (round, mb) timing events
    std::vector<double> tok_t;        // CPU backend: host timestamps of the same
    std::vector<bool> ring_pending;   // CPU backend, first stage: ring token not yet received
    std::atomic<long> progress{0};   // items completed (heartbeat)
    long items_seen = 0, sends_seen = 0;
    struct TraceRecT { std::string name; int tid = 0; hipEvent_t a = nullptr, b = nullptr; double ta = 0, tb = 0; };
    std::vector<TraceRecT> tr;
    hipEvent_t tr_base = nullptr;
    double tr_base_ms = 0;
    int device = 0;
    bool cpu = false;   // CpuStage (backend "cpu", or the host stage of a hybrid -ngl split)
    // act_dtype != f32: per micro-batch device staging of the 2-byte wire format
    std::vector<void*> wire_out, wire_in;
  };

  void build_links(const Json& cfg);
  void run_items(Worker& w, const std::vector<Item>& items);
  void run_items_cpu(Worker& w, const std::vector<Item>& items);
  void span(Worker& w, hipStream_t s, int tid, const std::string& name, const std::function<void()>& body);
  bool fault_hook(Worker& w, const char* what);
  void collect_trace();
  void run_all(const std::vector<Item>& items);
  void post_ring_recv(Worker& w, int mb);
  void sync_all();
  // multi-process pipeline: the last stage's host vector (same length on every rank) reaches every
  // rank over the idle ring (S-1 -> 0 -> 1 -> .. -> S-2); no-op in local mode
  void ring_bcast_from_last(std::vector<int32_t>& v);

  Json jcfg_;
  ModelConfig cfg_;
  std::vector<StageSpec> specs_;
  int S_ = 1, M_ = 1, B_ = 1;
  int max_ctx_ = 2048, chunk_ = 256;
  std::string mode_ = "local";
  int rank_ = 0;
  std::vector<std::unique_ptr<Worker>> workers_;   // owned stages (all in local mode)
  std::vector<std::unique_ptr<Link>> links_;
  std::unique_ptr<GgufFile> gguf_;
  // sequences
  std::vector<std::vector<int32_t>> prompts_;
  std::vector<std::vector<int32_t>> gen_;          // generated tokens per sequence
  int32_t* out_host_ = nullptr;                    // pinned [rounds_cap][M*B]
  std::vector<int32_t> out_vec_;                   // CPU backend storage of out_host_
  bool cpu_ = false;          // every stage on the CPU backend
  bool hybrid_ = false;       // gpu_layers (-ngl N) < n_layer: stage 0 on the CPU, the rest on GPUs
  bool stage_cpu(int s) const { return cpu_ || (hybrid_ && s == 0); }
  bool kv_fp8_ = false;      // kv_dtype "fp8" (checkpoint fingerprint: the KV bytes' element type)
  bool trace_ = false, failed_ = false;
  bool packed_prefill_ = true;   // several sequences per prefill chunk (config "packed_prefill")
  int act_dtype_ = 0;            // stage-boundary activation wire format (ActDtype; config "act_dtype")
  std::string link_fallback_;    // why local mode's requested RCCL links became LocalLinks (empty: none)
  double trace_t0_ = 0, watchdog_s_ = 600;
  std::vector<std::string> trace_events_;
  Json fault_;
  int rounds_cap_ = 0, rounds_done_ = 0;
  bool started_ = false;
  bool resumable_ = true;   // false after spec_generate (per-sequence positions)
  int32_t* bcast_dev_ = nullptr;   // ring_bcast_from_last device staging (RCCL / device links)
  size_t bcast_cap_ = 0;
  // prefix cache (config "prefix_cache", default on): per slot, the tokens its KV holds; start()
  // prefills only what follows the common prefix (multi-turn chat re-sends the whole history)
  bool prefix_cache_ = true;
  std::vector<std::vector<int32_t>> slot_toks_;
  long reused_tokens_ = 0;
  void refresh_slot_cache();
  // per slot: the round at which its sequence was admitted, and whether one is running
  std::vector<int> base_round_;
  std::vector<char> active_;
  KvPager pager_;            // paged KV: one logical table, installed on every stage
  int kv_pages_ = 0;         // pool pages per stage
  std::vector<double> device_speed_;
  int failed_stage_ = -1;    // stage whose worker raised the fault (health()["failed_stage"])   // partitioner weights per stage (given or probed)
  void kv_grant(size_t slot, int n_tokens);   // throws when the pool is exhausted
  void kv_sync();            // push a changed table to the stages (between engine calls)
  int slot_pos(size_t i) const {
    return (i < prompts_.size() ? (int)prompts_[i].size() : 0) + rounds_done_ - (i < base_round_.size() ? base_round_[i] : 0);
  }
  void push_positions(int mb);
  std::vector<Item> prefill_items(const std::vector<size_t>& seqs, bool admission);
  double load_ms_ = 0;
  // persistent stage-worker threads of run_all (declared last: joined before anything they use
  // is destroyed)
  std::unique_ptr<ThreadPool> pool_;
};

}  // namespace mp
