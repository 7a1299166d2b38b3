// Session = engine + tokenizer + the text-level generation loop shared by mi-cli and the
// orchestrator (the role llama-cli's main loop plays for the reference):
// tokenize, prefill, decode token by token, stream UTF-8-safe pieces, stop at end-of-generation
// or n_predict, cancel on request (client disconnect), and the llama.cpp-style perf summary.
#pragma once
#include <functional>
#include <memory>
#include <string>
#include <vector>

#include "engine.h"
#include "tokenizer.h"

namespace mp {

// complete-UTF-8 emitter: push() returns the bytes up to the last whole character, keeps the rest
struct Utf8Acc {
  std::string buf;
  std::string push(const std::string& b);
};
double session_now_ms();

struct GenRequest {
  std::string prompt;
  int n_predict = 200;
  // receives text pieces (complete UTF-8); return false to cancel this sequence
  std::function<bool(const std::string& piece)> on_piece;
};

struct GenResult {
  int n_prompt = 0, n_gen = 0;
  double prefill_ms = 0, decode_ms = 0;
  std::string text;
  std::string stop;   // "eog" | "length" | "cancelled" | "context"
  std::vector<int32_t> tokens;
};

class Session {
 public:
  // gguf may be empty (synthetic model: byte-level stand-in tokenizer)
  Session(Engine& eng, const std::string& gguf_path);
  ~Session();
  Engine& engine() { return *eng_; }
  int capacity() const { return eng_->n_mb() * eng_->mb_size(); }
  // Failover for serve(): called with the error of a failed engine call; returns a replacement
  // engine (e.g. re-partitioned without the failed stage's GPU, Engine::failover_config) or nullptr
  // to give up.  The running requests are then re-admitted as prompt + tokens generated so far and
  // keep streaming.  At most `max_failovers` per serve() call.
  void set_fault_handler(std::function<Engine*(const std::string& error)> h, int max_failovers = 4) {
    on_fault_ = std::move(h);
    max_failovers_ = max_failovers;
  }
  int failovers() const { return failovers_; }
  std::vector<int32_t> encode(const std::string& text) const;
  std::string piece(int32_t id) const;
  bool is_eog(int32_t id) const;

  // runs up to capacity() requests together (one sequence slot each)
  std::vector<GenResult> run(std::vector<GenRequest>& reqs);

  // Continuous batching (single-process pipelines): between decode rounds, `next(free)` is asked
  // for up to `free` new requests (non-blocking), which are admitted into idle sequence slots while
  // the running ones keep decoding; `done(request, result)` fires as each request finishes (EOG,
  // n_predict, cancellation, context).  Returns when nothing runs and next() has nothing.
  struct Served {
    GenRequest req;
    std::function<void(GenResult&)> done;
  };
  void serve(const std::function<std::vector<Served>(int free)>& next);
  // llama.cpp-style summary lines (prompt eval / eval / total)
  static std::string perf_summary(const GenResult& r, double load_ms);

 private:
  Engine* eng_;
  std::function<Engine*(const std::string&)> on_fault_;
  int max_failovers_ = 0, failovers_ = 0;
  std::unique_ptr<GgufFile> gguf_;
  std::unique_ptr<Tokenizer> tok_;
};

}  // namespace mp
