// Shared command-line handling of mi-cli and the orchestrator: llama-cli flag spellings
// (reference `orchestrator/src/main.rs:38-53`: -m -p -n -c --rpc -ngl --verbose --log-file) plus
// the pipeline flags of SURVEY.md §5.6, mapped onto the engine's JSON config.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "json.h"

namespace mp {

struct CliOptions {
  Json eng = Json::object();  // engine config
  std::string prompt = "Once upon a time";
  int n_predict = 200;        // reference: -n 200 (main.rs:44)
  int ngl = -1;               // -1 (no -ngl): every layer on the GPUs; reference -ngl 99 (main.rs:50) means the
                              // same; 0 = CPU backend; 0 < N < n_layer: hybrid (the first n_layer - N on the CPU)
  bool verbose = false;
  bool echo_prompt = true;
  bool bench = false;
  int bench_prompt = 128, bench_warmup = 3, bench_steps = 20;
  std::string trace;
  std::string rpc;            // --rpc host:port,... (without --world): stage workers to attach to (rpc.h)
  std::string master;         // --master HOST: this process's address as the workers see it (rpc.h)
  std::map<std::string, std::string> extra;   // tool-specific flags (--port, --static, ...)
};

inline std::vector<std::string> split_list(const std::string& s, char sep = ',') {
  std::vector<std::string> o;
  std::stringstream ss(s);
  std::string t;
  while (std::getline(ss, t, sep))
    if (!t.empty()) o.push_back(t);
  return o;
}

inline std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot read " + path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// synthetic architectures (random-init weights, no checkpoint needed)
inline Json synthetic_arch(const std::string& name) {
  Json s = Json::object();
  auto set = [&](const char* nm, int L, int d, int h, int kv, int ff, int V, double base, int E = 0, int k = 0) {
    s["name"] = nm; s["n_layer"] = L; s["d_model"] = d; s["n_head"] = h; s["n_head_kv"] = kv; s["d_ff"] = ff;
    s["vocab"] = V; s["rope_base"] = base;
    if (E) { s["n_expert"] = E; s["n_expert_used"] = k; }
  };
  if (name == "llama3-70b") set("Llama-3-70B", 80, 8192, 64, 8, 28672, 128256, 500000.0);
  else if (name == "llama3-8b") set("Llama-3-8B", 32, 4096, 32, 8, 14336, 128256, 500000.0);
  else if (name == "tinyllama") set("TinyLlama-1.1B", 22, 2048, 32, 4, 5632, 32000, 10000.0);
  else if (name == "mixtral-8x7b") set("Mixtral-8x7B", 32, 4096, 32, 8, 14336, 32000, 1000000.0, 8, 2);
  else if (name == "stories15m") set("stories15M", 6, 288, 6, 6, 768, 32000, 10000.0);
  else throw std::runtime_error("unknown synthetic model " + name +
                                " (llama3-70b, llama3-8b, tinyllama, mixtral-8x7b, stories15m)");
  return s;
}

inline void print_common_usage(FILE* f) {
  fprintf(f,
          "model:\n"
          "  -m, --model FILE          GGUF model (llama/mistral/mixtral architectures)\n"
          "  --synthetic NAME          random-init model instead of -m (llama3-70b, llama3-8b, tinyllama,\n"
          "                            mixtral-8x7b, stories15m); --ftype Q4_K_M|Q4_K|Q5_K_M|Q6_K|Q8_0|F16\n"
          "generation:\n"
          "  -p, --prompt TEXT         prompt (default \"Once upon a time\")\n"
          "  -f, --file FILE           read the prompt from a file\n"
          "  -n, --n-predict N         tokens to generate (default 200)\n"
          "  -c, --ctx-size N          context per sequence (default 2048)\n"
          "  --temp T --top-k K --top-p P --min-p P --seed S   sampling (default greedy, temp 0)\n"
          "  --repeat-penalty R --repeat-last-n N --frequency-penalty F --presence-penalty P\n"
          "                            penalties over the last N tokens (default 1.0 / 64 / 0 / 0)\n"
          "  --sampling greedy         force greedy\n"
          "  --draft-max K             speculative decoding by prompt lookup: up to K drafted tokens per\n"
          "                            verify round (greedy; --lookup-ngram N, default 3)\n"
          "placement / pipeline:\n"
          "  -ngl, --n-gpu-layers N    layers offloaded to the GPU stages (default: all); 0 = CPU backend;\n"
          "                            0 < N < n_layer: the first n_layer - N layers run on a CPU stage in front\n"
          "  --stages N, --pp N        pipeline stages (one GPU each)\n"
          "  --devices 0,1,..          GPU of each stage (repeat a GPU to emulate PP on one device)\n"
          "  --micro-batches M         micro-batches in flight;  --mb-size B sequences per micro-batch\n"
          "  --split even|mem|cost     layer partitioner (default cost)\n"
          "  --link local|rccl|tcp     stage transport;  --prefill-chunk N;  --no-graphs;  --threads N\n"
          "  --cpu-act q8|f32          CPU stages: integer dots on int8 activation blocks (default) or f32\n"
          "  --no-prefix-cache         prefill every request in full (no KV reuse of a common prefix)\n"
          "  --kv-pool TOKENS          paged KV pool per stage;  --kv-dtype f16|fp8 (-ctk/-ctv) KV cache element type\n"
          "  --int8-gemm               batches > 64 rows on the int8 MFMA (per-row int8 activations and weights:\n"
          "                            faster, reduced precision);  --deterministic  bitwise-reproducible logits\n"
          "  --world N --rank R        one process per stage (multi-process / multi-host)\n"
          "  --next HOST --master HOST --base-port P   TCP ring neighbours (prima.cpp style)\n"
          "  --gpu-mem GiB [--force]   per-GPU memory budget (caps auto KV; fail if a stage exceeds it)\n"
          "  --prefetch                madvise(WILLNEED) the GGUF ranges this process uploads\n"
          "  --rpc host:port,...       stage workers (mi-cli --rpc-server PORT) to attach to; with --world: the\n"
          "                            hosts of the stage processes; no worker answering: one local stage per entry\n"
          "logging:\n"
          "  --verbose, --log-file FILE, --trace FILE (Chrome trace of the pipeline)\n");
}

// Parses the shared flags; unknown flags are offered to `extra_flag(name, next_value_fn)` which
// returns true if it consumed them.
inline CliOptions parse_cli(int argc, char** argv,
                            const std::function<bool(const std::string&, const std::function<std::string()>&)>&
                                extra_flag = nullptr) {
  CliOptions o;
  Json& e = o.eng;
  e["max_ctx"] = 2048;
  std::string synthetic, devices, rpc, next, master;
  int stages = 0, world = 0, rank = -1;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
      return argv[++i];
    };
    if (a == "-m" || a == "--model") e["gguf"] = val();
    else if (a == "--synthetic") synthetic = val();
    else if (a == "--ftype") e["ftype"] = val();
    else if (a == "-p" || a == "--prompt") o.prompt = val();
    else if (a == "-f" || a == "--file") o.prompt = read_file(val());
    else if (a == "-n" || a == "--n-predict") o.n_predict = std::atoi(val().c_str());
    else if (a == "-c" || a == "--ctx-size") e["max_ctx"] = std::atoi(val().c_str());
    else if (a == "-ngl" || a == "--n-gpu-layers" || a == "--gpu-layers") o.ngl = std::atoi(val().c_str());
    else if (a == "--temp") e["temp"] = std::atof(val().c_str());
    else if (a == "--top-k") e["top_k"] = std::atoi(val().c_str());
    else if (a == "--top-p") e["top_p"] = std::atof(val().c_str());
    else if (a == "--min-p") e["min_p"] = std::atof(val().c_str());
    else if (a == "--repeat-penalty") e["repeat_penalty"] = std::atof(val().c_str());
    else if (a == "--repeat-last-n") e["repeat_last_n"] = std::atoi(val().c_str());
    else if (a == "--frequency-penalty") e["frequency_penalty"] = std::atof(val().c_str());
    else if (a == "--presence-penalty") e["presence_penalty"] = std::atof(val().c_str());
    else if (a == "--seed" || a == "-s") e["seed"] = std::atof(val().c_str());
    else if (a == "--sampling") { if (val() == "greedy") e["temp"] = 0.0; }
    else if (a == "--stages" || a == "--pp") stages = std::atoi(val().c_str());
    else if (a == "--devices") devices = val();
    else if (a == "--micro-batches") e["n_mb"] = std::atoi(val().c_str());
    else if (a == "--mb-size") e["mb_size"] = std::atoi(val().c_str());
    else if (a == "--split") e["split"] = val();
    else if (a == "--link") e["link"] = val();
    else if (a == "--prefill-chunk" || a == "-ub" || a == "--ubatch-size") e["prefill_chunk"] = std::atoi(val().c_str());
    else if (a == "--no-graphs") e["graphs"] = false;
    else if (a == "--draft-max" || a == "--draft") e["draft_max"] = std::atoi(val().c_str());   // prompt-lookup speculation
    else if (a == "--lookup-ngram") e["lookup_ngram"] = std::atoi(val().c_str());
    else if (a == "--threads" || a == "-t") e["threads"] = std::atoi(val().c_str());
    else if (a == "--cpu-act") e["cpu_act"] = val();   // CPU stages: q8 (integer dots, default) | f32
    else if (a == "--world") world = std::atoi(val().c_str());
    else if (a == "--rank") rank = std::atoi(val().c_str());
    else if (a == "--next") next = val();
    else if (a == "--master") master = val();
    else if (a == "--prefetch") e["prefetch"] = true;
    else if (a == "--gpu-mem") e["gpu_mem_gib"] = std::atof(val().c_str());
    else if (a == "--kv-pool") e["kv_pool_tokens"] = std::atoi(val().c_str());   // paged KV pool (tokens per stage)
    else if (a == "--kv-dtype" || a == "-ctk" || a == "--cache-type-k" || a == "-ctv" || a == "--cache-type-v")
      e["kv_dtype"] = val();                                                     // f16 | fp8 (K and V together)
    else if (a == "--force") e["force"] = true;
    else if (a == "--int8-gemm") e["int8_gemm"] = true;
    else if (a == "--deterministic") e["deterministic"] = true;
    else if (a == "--base-port") e["base_port"] = std::atoi(val().c_str());
    else if (a == "--rpc") rpc = val();
    else if (a == "--device") e["device"] = std::atoi(val().c_str());
    else if (a == "--verbose" || a == "-v") { o.verbose = true; e["verbose"] = true; }
    else if (a == "--log-file") e["log_file"] = val();
    else if (a == "--no-prefix-cache") e["prefix_cache"] = false;
    else if (a == "--trace") o.trace = val();
    else if (a == "--no-display-prompt") o.echo_prompt = false;
    else if (a == "--bench") o.bench = true;
    else if (a == "--bench-prompt") o.bench_prompt = std::atoi(val().c_str());
    else if (a == "--bench-warmup") o.bench_warmup = std::atoi(val().c_str());
    else if (a == "--bench-steps") o.bench_steps = std::atoi(val().c_str());
    else if (extra_flag && extra_flag(a, val)) continue;
    else throw std::runtime_error("unknown flag " + a);
  }
  if (!synthetic.empty()) e["synthetic"] = synthetic_arch(synthetic);
  if (!e.has("gguf") && !e.has("synthetic")) throw std::runtime_error("need -m FILE or --synthetic NAME");
  if (o.ngl == 0) e["backend"] = "cpu";
  else if (o.ngl > 0) e["gpu_layers"] = o.ngl;   // explicit -ngl only: >= n_layer puts every layer on the GPUs
  if (stages > 0) e["stages"] = stages;
  if (!devices.empty()) {
    Json d = Json::array();
    for (auto& s : split_list(devices)) d.push(std::atoi(s.c_str()));
    e["devices"] = d;
    if (stages == 0) e["stages"] = (int)d.arr().size();
  }
  if (world > 0) {
    if (rank < 0 || rank >= world) throw std::runtime_error("--rank must be in [0, --world)");
    e["mode"] = "mp";
    e["world"] = world;
    e["rank"] = rank;
    if (!e.has("link")) e["link"] = "tcp";
    Json hosts = Json::array();
    auto rl = split_list(rpc);
    for (int r = 0; r < world; ++r) {
      std::string h = r < (int)rl.size() ? rl[r] : (r == 0 && !master.empty() ? master : "127.0.0.1");
      const auto c = h.find(':');
      if (c != std::string::npos) h = h.substr(0, c);
      hosts.push(h);
    }
    e["hosts"] = hosts;
    if (!next.empty()) e["next_host"] = next;
  } else if (!rpc.empty() && stages == 0) {
    // llama-cli --rpc lists remote workers (rpc.h attaches to them when they answer); without
    // workers every stage is a local GPU: one stage per entry
    e["stages"] = (int)split_list(rpc).size();
    o.rpc = rpc;
  }
  o.master = master;
  return o;
}

// Emits only complete UTF-8 sequences (the reference's 64-byte stdout reads split multi-byte
// characters into U+FFFD)
class Utf8Stream {
 public:
  std::string push(const std::string& bytes) {
    buf_ += bytes;
    size_t cut = buf_.size();
    // find start of a trailing incomplete sequence
    for (size_t k = 1; k <= 4 && k <= buf_.size(); ++k) {
      const unsigned char c = (unsigned char)buf_[buf_.size() - k];
      if ((c & 0xC0) == 0x80) continue;   // continuation byte
      int need = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1;
      if (need > (int)k) cut = buf_.size() - k;
      break;
    }
    std::string out = buf_.substr(0, cut);
    buf_.erase(0, cut);
    return out;
  }
  std::string flush() {
    std::string o;
    o.swap(buf_);
    return o;
  }

 private:
  std::string buf_;
};

}  // namespace mp
