// orchestrator: the HTTP front-end (reference `orchestrator/src/main.rs`, SURVEY.md C1-C10, D5, D7,
// D12), C++ instead of Rust/axum and with the engine IN-PROCESS: the model is loaded once at
// start-up (the reference spawns a fresh llama-cli per request and reloads the GGUF every time,
// `main.rs:35-57`).
//
//   POST /chat        {"prompt": str, "n_predict"?: int} -> text/event-stream of
//                     data: {"msg_type": "log"|"token", "content": str}   (main.rs:23-27,97)
//                     keep-alive comment every 1 s (main.rs:97); generation is cancelled when the
//                     client disconnects (the reference lets the child run on, main.rs:77,91)
//   POST /completion  {"prompt", "n_predict"} -> {"content", "response", "tokens_predicted", ...}
//                     (the PDF's proxy design, p.9-10, llama-server style)
//   GET  /metrics     Prometheus text (requests, tokens, tok/s, p50/p90/p99 per token, stage
//                     heartbeats, link bytes)
//   GET  /health      engine health JSON
//   GET  /models      registered models ({"data": [{"id", "loaded", "source"}]}); requests pick one
//                     with "model": NAME (--model-alias NAME=PATH|synthetic:NAME, PDF p.7 item 3:
//                     multi-model management), at most --max-models engines resident (LRU)
//   GET  /*           static files (default ./static, index.html at /) (main.rs:104)
//   CORS: Access-Control-Allow-Origin * on every response, OPTIONS preflight (main.rs:105)
//   errors as axum's Json extractor: 415 (not application/json), 400 (bad JSON), 422 (no
//   "prompt" string), 405 (wrong method), 404; optional --api-key (401) and --rate-limit (429)
//
// Concurrency: connection thread per client; one generation thread batches up to
// n_mb * mb_size queued requests for the same model into one engine run (request-level batching,
// SURVEY.md D5).  A failed run whose engine reports a fault (stage exception, link abort, watchdog)
// is answered with an error and the engine is rebuilt from its config (the design report's worker
// auto-restart, PDF p.6-7 / SURVEY.md D6).
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/socket.h>
#include <poll.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cerrno>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "cli_common.h"
#include "engine.h"
#include "log.h"
#include "session.h"

using namespace mp;

namespace {

double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------------------------ events / jobs
struct Event {
  std::string type;      // "log" | "token" | "end"
  std::string content;
};

struct Job {
  std::string prompt;
  std::string model;   // "" = the default model
  int n_predict = 200;
  double enqueued_ms = 0;   // fairness between models (serve_model)
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Event> q;
  bool done = false;
  std::atomic<bool> cancelled{false};
  GenResult result;
  void push(Event e) {
    {
      std::lock_guard<std::mutex> l(mu);
      q.push_back(std::move(e));
    }
    cv.notify_all();
  }
  void finish() {
    {
      std::lock_guard<std::mutex> l(mu);
      done = true;
    }
    cv.notify_all();
  }
};

struct Metrics {
  std::mutex mu;
  uint64_t requests = 0, completed = 0, cancelled = 0, errors = 0, prompt_tokens = 0, gen_tokens = 0;
  double last_decode_tok_s = 0, last_prefill_tok_s = 0;
  std::vector<double> token_ms;   // recent per-token latencies
  void add_latency(double ms) {
    token_ms.push_back(ms);
    if (token_ms.size() > 4096) token_ms.erase(token_ms.begin(), token_ms.begin() + 2048);
  }
};

double pctl(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (v.size() - 1) + 0.5))];
}

// ------------------------------------------------------------------ server state
struct ModelSlot {
  std::string name, source;
  Json cfg;
  std::unique_ptr<Engine> eng;
  std::unique_ptr<Session> sess;
  double last_used = 0;
  int restarts = 0;
};

struct Server {
  Engine* eng = nullptr;     // the default model's engine (models[0])
  std::vector<std::unique_ptr<ModelSlot>> models;
  int max_models = 2;        // resident engines (the default one included)
  std::mutex eng_mu;         // engine swaps (restart / load) vs /health and /metrics readers
  bool ready = false;        // start-up finished (later logs are not replayed to new requests)
  bool mock = false;
  bool continuous = true;    // continuous batching (--no-continuous: one batch per engine run)
  int mock_delay_ms = 2;
  int capacity = 1;
  int default_n = 200;
  std::string static_dir = "static";
  std::string api_key;
  int rate_limit = 0;   // requests per minute per client IP (0 = off)
  std::mutex rl_mu;
  std::map<std::string, std::deque<double>> rl_hist;
  std::vector<std::string> startup_logs;
  std::mutex jobs_mu;
  std::condition_variable jobs_cv;
  std::deque<std::shared_ptr<Job>> pending;
  std::vector<std::shared_ptr<Job>> active;
  std::mutex active_mu;
  Metrics metrics;
  std::atomic<bool> stop{false};
  std::atomic<int> connections{0};
  // a request for another model that has waited this long stops admission into the model being
  // served; its live requests drain and the generation loop switches models (no starvation)
  double switch_after_ms = 2000;
  // --spawn-cli: the reference's process model (main.rs:35-57) -- every request runs a CLI child
  // (mi-cli with the model flags this server was started with); its stdout streams as "token"
  // messages, its stderr lines as "log" messages; a client disconnect kills the child
  std::string spawn_cli;
  std::vector<std::string> cli_args;
};

Server* g_srv = nullptr;

void broadcast_log(const std::string& line) {
  if (!g_srv) return;
  std::lock_guard<std::mutex> l(g_srv->active_mu);
  for (auto& j : g_srv->active) j->push({"log", line});
}

// mock generation (no model): echoes words for API tests (SURVEY.md T6 "mock engine")
GenResult mock_run(Job& j, int delay_ms) {
  GenResult r;
  r.n_prompt = (int)j.prompt.size();
  std::vector<std::string> words = {" once", " upon", " a", " time", " there", " was", " a", " pipeline", ".",
                                    " \xc3\xa7", "\xc4\x9f", " \xf0\x9f\x9a\x80"};
  const double t0 = now_ms();
  for (int i = 0; i < j.n_predict; ++i) {
    if (j.cancelled) { r.stop = "cancelled"; break; }
    const std::string& w = words[i % words.size()];
    r.text += w;
    r.n_gen++;
    j.push({"token", w});
    std::this_thread::sleep_for(std::chrono::milliseconds(delay_ms));
  }
  if (r.stop.empty()) r.stop = "length";
  r.decode_ms = now_ms() - t0;
  return r;
}

ModelSlot* find_model(Server& S, const std::string& name) {
  if (name.empty()) return S.models.empty() ? nullptr : S.models[0].get();
  for (auto& m : S.models)
    if (m->name == name) return m.get();
  return nullptr;
}

void load_slot(Server& S, ModelSlot& m) {
  const bool dflt = &m == S.models[0].get();
  {
    std::lock_guard<std::mutex> l(S.eng_mu);
    if (dflt) S.eng = nullptr;
    m.sess.reset();
    m.eng.reset();
  }
  std::unique_ptr<Engine> e(new Engine(m.cfg));
  std::unique_ptr<Session> ss(new Session(*e, m.cfg.get_str("gguf", "")));
  std::lock_guard<std::mutex> l(S.eng_mu);
  m.eng = std::move(e);
  m.sess = std::move(ss);
  if (dflt) S.eng = m.eng.get();
}

// generation thread only: the slot of `name`, loaded (evicting the least recently used other
// model when more than max_models engines would be resident)
ModelSlot* acquire_model(Server& S, const std::string& name) {
  ModelSlot* m = find_model(S, name);
  if (!m) throw std::runtime_error("unknown model " + name);
  if (!m->eng) {
    int resident = 0;
    for (auto& x : S.models) resident += x->eng ? 1 : 0;
    while (resident >= S.max_models) {
      ModelSlot* lru = nullptr;
      for (size_t i = 1; i < S.models.size(); ++i)
        if (S.models[i]->eng && (!lru || S.models[i]->last_used < lru->last_used)) lru = S.models[i].get();
      if (!lru) break;
      MP_LOGI("orchestrator: unloading model %s", lru->name.c_str());
      std::lock_guard<std::mutex> l(S.eng_mu);
      lru->sess.reset();
      lru->eng.reset();
      --resident;
    }
    MP_LOGI("orchestrator: loading model %s (%s)", m->name.c_str(), m->source.c_str());
    load_slot(S, *m);
  }
  m->last_used = now_ms();
  return m;
}

// per-request bookkeeping once a generation ends (both scheduling modes)
void record_result(Server& S, Job& j, const GenResult& r, double load_ms) {
  j.result = r;
  const std::string perf = Session::perf_summary(r, load_ms);
  j.push({"log", perf});
  fputs(perf.c_str(), stderr);
  std::lock_guard<std::mutex> l(S.metrics.mu);
  S.metrics.completed++;
  if (r.stop == "cancelled") S.metrics.cancelled++;
  S.metrics.prompt_tokens += r.n_prompt;
  S.metrics.gen_tokens += r.n_gen;
  if (r.decode_ms > 0 && r.n_gen > 1) {
    S.metrics.last_decode_tok_s = (r.n_gen - 1) * 1e3 / r.decode_ms;
    S.metrics.add_latency(r.decode_ms / (r.n_gen - 1));
  }
  if (r.prefill_ms > 0) S.metrics.last_prefill_tok_s = r.n_prompt * 1e3 / r.prefill_ms;
}

// the engine is poisoned (aborted links, failed stage): rebuild it; injected faults are a one-shot
// test hook and are not re-armed
void restart_if_failed(Server& S, ModelSlot* slot) {
  if (!slot || !slot->eng || slot->eng->health().get_bool("ok", true)) return;
  slot->cfg["fault"] = Json::object();
  try {
    load_slot(S, *slot);
    slot->restarts++;
    MP_LOGW("orchestrator: engine of model %s restarted after a fault (%d restarts)", slot->name.c_str(),
            slot->restarts);
  } catch (const std::exception& e2) {
    MP_LOGE("orchestrator: engine restart failed: %s", e2.what());
  }
}

// Continuous batching (default): requests for `model` are admitted into free sequence slots between
// decode rounds while the running ones keep generating; each finishes (and frees its slot) on its own.
void serve_model(Server& S, ModelSlot* slot, const std::string& model) {
  const double turn_start = now_ms();
  auto next = [&](int free) {
    std::vector<std::shared_ptr<Job>> taken;
    {
      std::lock_guard<std::mutex> l(S.jobs_mu);
      // each model gets a turn of at least switch_after_ms before another model's waiting request
      // can end it (otherwise two busy models would hand the turn back and forth, admitting nothing)
      const double now = now_ms();
      if (now - turn_start > S.switch_after_ms)
        for (auto& pj : S.pending)
          if (pj->model != model && now - pj->enqueued_ms > S.switch_after_ms) return std::vector<Session::Served>{};
      for (auto it = S.pending.begin(); it != S.pending.end() && (int)taken.size() < free;) {
        if ((*it)->model == model) {
          taken.push_back(*it);
          it = S.pending.erase(it);
        } else {
          ++it;
        }
      }
    }
    std::vector<Session::Served> out;
    for (auto& j : taken) {
      {
        std::lock_guard<std::mutex> l(S.active_mu);
        S.active.push_back(j);
      }
      j->push({"log", "orchestrator: request accepted (continuous batching, " + std::to_string(free) + " free slots)\n"});
      for (auto& sl : S.startup_logs) j->push({"log", sl});
      Session::Served sv;
      sv.req.prompt = j->prompt;
      sv.req.n_predict = j->n_predict;
      Job* jp = j.get();
      sv.req.on_piece = [jp](const std::string& p) {
        if (jp->cancelled) return false;
        jp->push({"token", p});
        return true;
      };
      std::shared_ptr<Job> keep = j;
      sv.done = [&S, slot, keep](GenResult& r) {
        record_result(S, *keep, r, slot->eng->load_ms());
        {
          std::lock_guard<std::mutex> l(S.active_mu);
          S.active.erase(std::remove(S.active.begin(), S.active.end(), keep), S.active.end());
        }
        keep->finish();
      };
      out.push_back(std::move(sv));
    }
    return out;
  };
  // failover: a stage fault mid-generation rebuilds the engine without the failed stage's GPU
  // (layers re-partitioned over the survivors) and the running requests continue on it
  slot->sess->set_fault_handler([&S, slot](const std::string& err) -> Engine* {
    if (!slot->eng) return nullptr;
    const Json cfg2 = Engine::failover_config(slot->cfg, slot->eng->health());
    MP_LOGW("orchestrator: engine of model %s faulted (%s); failing over", slot->name.c_str(), err.c_str());
    // free the faulted engine's weights and KV on the surviving GPUs BEFORE the replacement sizes
    // and allocates its own there (it carries more layers per GPU and an auto-sized KV pool)
    std::unique_ptr<Engine> old;
    bool dflt = false;
    {
      std::lock_guard<std::mutex> l(S.eng_mu);
      dflt = S.eng == slot->eng.get();
      if (dflt) S.eng = nullptr;
      old = std::move(slot->eng);
    }
    old.reset();
    std::unique_ptr<Engine> e(new Engine(cfg2));
    std::lock_guard<std::mutex> l(S.eng_mu);
    slot->eng = std::move(e);
    slot->cfg = cfg2;
    slot->restarts++;
    if (dflt) S.eng = slot->eng.get();
    return slot->eng.get();
  });
  try {
    slot->sess->serve(next);
  } catch (const std::exception& e) {
    MP_LOGE("generation failed: %s", e.what());
    std::vector<std::shared_ptr<Job>> left;
    {
      std::lock_guard<std::mutex> l(S.active_mu);
      left.swap(S.active);
    }
    {
      std::lock_guard<std::mutex> l(S.metrics.mu);
      S.metrics.errors += left.size();
    }
    for (auto& j : left) {
      j->push({"log", std::string("error: ") + e.what() + "\n"});
      j->finish();
    }
    restart_if_failed(S, slot);
  }
}

void generation_loop(Server& S) {
  std::string last_model;
  bool have_last = false;
  while (!S.stop) {
    std::vector<std::shared_ptr<Job>> batch;
    ModelSlot* slot = nullptr;
    std::string model;
    {
      std::unique_lock<std::mutex> l(S.jobs_mu);
      S.jobs_cv.wait_for(l, std::chrono::milliseconds(200), [&] { return !S.pending.empty() || S.stop; });
      if (S.pending.empty()) continue;
      // the oldest request's model, except that the oldest request of ANOTHER model than the one
      // served last goes first once it has waited switch_after_ms (serve_model stopped for it)
      model = S.pending.front()->model;
      const double now = now_ms();
      if (have_last)
        for (auto& pj : S.pending)
          if (pj->model != last_model && now - pj->enqueued_ms > S.switch_after_ms) {
            model = pj->model;
            break;
          }
    }
    last_model = model;
    have_last = true;
    int cap = S.capacity;
    if (!S.mock) {
      try {
        slot = acquire_model(S, model);
        cap = slot->sess->capacity();
      } catch (const std::exception& e) {
        MP_LOGE("orchestrator: model %s unavailable: %s", model.c_str(), e.what());
        std::shared_ptr<Job> j;
        {
          std::lock_guard<std::mutex> l(S.jobs_mu);
          j = S.pending.front();
          S.pending.pop_front();
        }
        j->push({"log", std::string("error: ") + e.what() + "\n"});
        j->finish();
        continue;
      }
    }
    if (!S.mock && S.continuous && slot->cfg.get_int("draft_max", 0) <= 0) {
      serve_model(S, slot, model);
      continue;
    }
    {
      // the oldest request's model; later requests for other models keep their place in the queue
      std::lock_guard<std::mutex> l(S.jobs_mu);
      for (auto it = S.pending.begin(); it != S.pending.end() && (int)batch.size() < cap;) {
        if ((*it)->model == model) {
          batch.push_back(*it);
          it = S.pending.erase(it);
        } else {
          ++it;
        }
      }
    }
    if (batch.empty()) continue;
    {
      std::lock_guard<std::mutex> l(S.active_mu);
      S.active = batch;
    }
    for (auto& j : batch) {
      j->push({"log", "orchestrator: request accepted (" + std::to_string(batch.size()) + " in this batch)\n"});
      for (auto& s : S.startup_logs) j->push({"log", s});
    }
    try {
      std::vector<GenResult> res;
      if (S.mock) {
        for (auto& j : batch) res.push_back(mock_run(*j, S.mock_delay_ms));
      } else {
        std::vector<GenRequest> reqs(batch.size());
        for (size_t i = 0; i < batch.size(); ++i) {
          reqs[i].prompt = batch[i]->prompt;
          reqs[i].n_predict = batch[i]->n_predict;
          Job* jp = batch[i].get();
          reqs[i].on_piece = [jp](const std::string& p) {
            if (jp->cancelled) return false;
            jp->push({"token", p});
            return true;
          };
        }
        res = slot->sess->run(reqs);
      }
      for (size_t i = 0; i < batch.size(); ++i) record_result(S, *batch[i], res[i], slot ? slot->eng->load_ms() : 0.0);
    } catch (const std::exception& e) {
      MP_LOGE("generation failed: %s", e.what());
      {
        std::lock_guard<std::mutex> l(S.metrics.mu);
        S.metrics.errors += batch.size();
      }
      for (auto& j : batch) j->push({"log", std::string("error: ") + e.what() + "\n"});
      restart_if_failed(S, slot);
    }
    {
      std::lock_guard<std::mutex> l(S.active_mu);
      S.active.clear();
    }
    for (auto& j : batch) j->finish();
  }
}

// ------------------------------------------------------------------ HTTP
struct Request {
  std::string method, path, query, version;
  std::map<std::string, std::string> headers;   // lower-case keys
  std::string body;
  std::string peer;
  std::string header(const std::string& k) const {
    auto it = headers.find(k);
    return it == headers.end() ? "" : it->second;
  }
};

bool write_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t w = ::send(fd, s.data() + off, s.size() - off, MSG_NOSIGNAL);
    if (w <= 0) return false;
    off += (size_t)w;
  }
  return true;
}

std::string lower(std::string s) {
  for (auto& c : s) c = (char)tolower((unsigned char)c);
  return s;
}

const char* status_text(int code) {
  switch (code) {
    case 200: return "OK";
    case 204: return "No Content";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 413: return "Payload Too Large";
    case 415: return "Unsupported Media Type";
    case 422: return "Unprocessable Entity";
    case 429: return "Too Many Requests";
    case 500: return "Internal Server Error";
    case 503: return "Service Unavailable";
  }
  return "Unknown";
}

const char* kCors =
    "Access-Control-Allow-Origin: *\r\n"
    "Access-Control-Allow-Methods: GET, POST, OPTIONS\r\n"
    "Access-Control-Allow-Headers: *\r\n";

void respond(int fd, int code, const std::string& ctype, const std::string& body, const std::string& extra = "") {
  std::string h = "HTTP/1.1 " + std::to_string(code) + " " + status_text(code) + "\r\n";
  if (!ctype.empty()) h += "Content-Type: " + ctype + "\r\n";
  h += "Content-Length: " + std::to_string(body.size()) + "\r\n";
  h += kCors;
  h += extra;
  h += "Connection: close\r\n\r\n";
  write_all(fd, h + body);
}

void respond_text(int fd, int code, const std::string& msg) { respond(fd, code, "text/plain; charset=utf-8", msg); }

// 1 = request read, 0 = connection closed / oversized, -1 = malformed (answer 400)
int read_request(int fd, Request& r) {
  std::string buf;
  char tmp[8192];
  size_t hdr_end = std::string::npos;
  while ((hdr_end = buf.find("\r\n\r\n")) == std::string::npos) {
    ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
    if (n <= 0) return 0;
    buf.append(tmp, (size_t)n);
    if (buf.size() > (1 << 20)) return 0;
  }
  const std::string head = buf.substr(0, hdr_end);
  r.body = buf.substr(hdr_end + 4);
  size_t eol = head.find("\r\n");
  const std::string line = head.substr(0, eol);
  size_t a = line.find(' '), b = line.rfind(' ');
  if (a == std::string::npos || b == a) return 0;
  r.method = line.substr(0, a);
  std::string target = line.substr(a + 1, b - a - 1);
  r.version = line.substr(b + 1);
  const size_t q = target.find('?');
  r.path = target.substr(0, q);
  if (q != std::string::npos) r.query = target.substr(q + 1);
  size_t pos = eol == std::string::npos ? head.size() : eol + 2;
  while (pos < head.size()) {
    size_t e = head.find("\r\n", pos);
    if (e == std::string::npos) e = head.size();
    const std::string h = head.substr(pos, e - pos);
    const size_t c = h.find(':');
    if (c != std::string::npos) {
      std::string v = h.substr(c + 1);
      while (!v.empty() && (v[0] == ' ' || v[0] == '\t')) v.erase(0, 1);
      r.headers[lower(h.substr(0, c))] = v;
    }
    pos = e + 2;
  }
  size_t cl = 0;
  const std::string clh = r.header("content-length");
  if (!clh.empty()) {
    // strict decimal: a malformed or out-of-range value is a 400, never an exception on this thread
    errno = 0;
    char* end = nullptr;
    const unsigned long long v = std::strtoull(clh.c_str(), &end, 10);
    if (clh[0] < '0' || clh[0] > '9' || errno == ERANGE || !end || *end != '\0') return -1;
    if (v > (8ull << 20)) return 0;
    cl = (size_t)v;
  }
  while (r.body.size() < cl) {
    ssize_t n = ::recv(fd, tmp, sizeof(tmp), 0);
    if (n <= 0) return 0;
    r.body.append(tmp, (size_t)n);
  }
  r.body.resize(cl);
  return 1;
}

std::string mime_of(const std::string& p) {
  auto ends = [&](const char* s) { return p.size() >= strlen(s) && p.compare(p.size() - strlen(s), strlen(s), s) == 0; };
  if (ends(".html") || ends(".htm")) return "text/html; charset=utf-8";
  if (ends(".js")) return "application/javascript";
  if (ends(".css")) return "text/css";
  if (ends(".json")) return "application/json";
  if (ends(".png")) return "image/png";
  if (ends(".svg")) return "image/svg+xml";
  if (ends(".ico")) return "image/x-icon";
  return "application/octet-stream";
}

void serve_static(Server& S, int fd, const Request& r) {
  std::string p = r.path == "/" ? "/index.html" : r.path;
  if (p.find("..") != std::string::npos) return respond_text(fd, 404, "Not Found");
  const std::string full = S.static_dir + p;
  struct stat stt;
  if (stat(full.c_str(), &stt) != 0 || !S_ISREG(stt.st_mode)) return respond_text(fd, 404, "Not Found");
  try {
    const std::string body = read_file(full);
    respond(fd, 200, mime_of(full), r.method == "HEAD" ? "" : body);
  } catch (...) {
    respond_text(fd, 404, "Not Found");
  }
}

// axum Json<ChatRequest> extractor semantics (main.rs:18-21)
bool parse_prompt_body(int fd, const Request& r, std::string* prompt, int* n_predict, int def_n,
                       std::string* model = nullptr) {
  if (lower(r.header("content-type")).find("application/json") == std::string::npos) {
    respond_text(fd, 415, "Expected request with `Content-Type: application/json`");
    return false;
  }
  Json j;
  try {
    j = Json::parse(r.body);
  } catch (const std::exception& e) {
    respond_text(fd, 400, std::string("Failed to parse the request body as JSON: ") + e.what());
    return false;
  }
  if (!j.is_obj() || !j.has("prompt") || !j["prompt"].is_str()) {
    respond_text(fd, 422, "Failed to deserialize the JSON body into the target type: missing field `prompt`");
    return false;
  }
  *prompt = j["prompt"].str();
  *n_predict = j.get_int("n_predict", def_n);
  if (*n_predict < 0) *n_predict = def_n;
  if (model) *model = j.get_str("model", "");
  return true;
}

bool authorized(Server& S, int fd, const Request& r) {
  if (!S.api_key.empty()) {
    const std::string a = r.header("authorization"), k = r.header("x-api-key");
    if (a != "Bearer " + S.api_key && k != S.api_key) {
      respond_text(fd, 401, "Unauthorized");
      return false;
    }
  }
  if (S.rate_limit > 0) {
    std::lock_guard<std::mutex> l(S.rl_mu);
    auto& h = S.rl_hist[r.peer];
    const double t = now_ms();
    while (!h.empty() && t - h.front() > 60000) h.pop_front();
    if ((int)h.size() >= S.rate_limit) {
      respond(fd, 429, "text/plain; charset=utf-8", "Too Many Requests", "Retry-After: 60\r\n");
      return false;
    }
    h.push_back(t);
  }
  return true;
}

bool known_model(Server& S, int fd, std::string* model) {
  if (S.mock || model->empty()) return true;
  if (ModelSlot* m = find_model(S, *model)) {
    if (m == S.models[0].get()) model->clear();   // the default model under its own name
    return true;
  }
  respond(fd, 404, "application/json", "{\"error\":\"unknown model\"}");
  return false;
}

// one request = one child process (spawn-cli mode)
void spawn_job(Server& S, std::shared_ptr<Job> job) {
  std::vector<std::string> av{S.spawn_cli};
  av.insert(av.end(), S.cli_args.begin(), S.cli_args.end());
  for (const char* a : {"-p", "", "-n", "", "--no-display-prompt"}) av.push_back(a);
  av[av.size() - 4] = job->prompt;
  av[av.size() - 2] = std::to_string(job->n_predict);
  int out[2], err[2];
  if (pipe(out) != 0 || pipe(err) != 0) {
    job->push({"log", std::string("error: pipe: ") + strerror(errno) + "\n"});
    job->finish();
    return;
  }
  const double t0 = now_ms();
  const pid_t pid = fork();
  if (pid == 0) {   // child: exec before touching anything else (no GPU state in this process)
    dup2(out[1], 1);
    dup2(err[1], 2);
    close(out[0]); close(out[1]); close(err[0]); close(err[1]);
    std::vector<char*> cv;
    for (auto& a : av) cv.push_back(const_cast<char*>(a.c_str()));
    cv.push_back(nullptr);
    execv(cv[0], cv.data());
    fprintf(stderr, "exec %s: %s\n", cv[0], strerror(errno));
    _exit(127);
  }
  close(out[1]);
  close(err[1]);
  if (pid < 0) {
    close(out[0]); close(err[0]);
    job->push({"log", std::string("error: fork: ") + strerror(errno) + "\n"});
    job->finish();
    return;
  }
  Utf8Acc acc;
  std::string line, text;
  pollfd fds[2] = {{out[0], POLLIN, 0}, {err[0], POLLIN, 0}};
  int open_fds = 2;
  bool killed = false;
  char buf[4096];
  while (open_fds > 0) {
    if (job->cancelled && !killed) { kill(pid, SIGTERM); killed = true; }
    if (poll(fds, 2, 100) < 0 && errno != EINTR) break;
    for (int k = 0; k < 2; ++k) {
      if (fds[k].fd < 0 || !(fds[k].revents & (POLLIN | POLLHUP | POLLERR))) continue;
      const ssize_t n = read(fds[k].fd, buf, sizeof(buf));
      if (n <= 0) { close(fds[k].fd); fds[k].fd = -1; --open_fds; continue; }
      if (k == 0) {   // token stream (UTF-8 safe pieces, like the reference's stdout pump)
        const std::string p = acc.push(std::string(buf, (size_t)n));
        if (!p.empty()) { text += p; job->push({"token", p}); }
      } else {        // log lines (stderr), line by line
        line.append(buf, (size_t)n);
        size_t nl;
        while ((nl = line.find('\n')) != std::string::npos) {
          job->push({"log", line.substr(0, nl + 1)});
          line.erase(0, nl + 1);
        }
      }
    }
  }
  if (!acc.buf.empty()) { text += acc.buf; job->push({"token", acc.buf}); }
  if (!line.empty()) job->push({"log", line + "\n"});
  int status = 0;
  waitpid(pid, &status, 0);
  GenResult r;
  r.text = text;
  r.stop = killed ? "cancelled" : (WIFEXITED(status) && WEXITSTATUS(status) == 0 ? "length" : "error");
  r.decode_ms = now_ms() - t0;
  job->result = r;
  {
    std::lock_guard<std::mutex> l(S.metrics.mu);
    if (r.stop == "length") S.metrics.completed++;
    else if (killed) S.metrics.cancelled++;
    else S.metrics.errors++;
  }
  job->finish();
}

std::shared_ptr<Job> submit(Server& S, const std::string& prompt, int n, const std::string& model = "") {
  auto job = std::make_shared<Job>();
  job->prompt = prompt;
  job->n_predict = n;
  job->model = model;
  {
    std::lock_guard<std::mutex> l(S.metrics.mu);
    S.metrics.requests++;
  }
  printf("request: %s\n", prompt.c_str());   // reference main.rs:32 request log
  fflush(stdout);
  if (!S.spawn_cli.empty()) {   // a child process per request, no engine in this process
    std::thread(spawn_job, std::ref(S), job).detach();
    return job;
  }
  {
    std::lock_guard<std::mutex> l(S.jobs_mu);
    job->enqueued_ms = now_ms();
    S.pending.push_back(job);
  }
  S.jobs_cv.notify_all();
  return job;
}

std::string sse_event(const Event& e) {
  Json m = Json::object();
  m["msg_type"] = e.type;
  m["content"] = e.content;
  return "data: " + m.dump() + "\n\n";
}

std::string chunk(const std::string& s) {
  char h[32];
  snprintf(h, sizeof(h), "%zx\r\n", s.size());
  return std::string(h) + s + "\r\n";
}

void handle_chat(Server& S, int fd, const Request& r) {
  std::string prompt;
  int n = S.default_n;
  std::string model;
  if (!parse_prompt_body(fd, r, &prompt, &n, S.default_n, &model) || !known_model(S, fd, &model)) return;
  auto job = submit(S, prompt, n, model);
  std::string h = "HTTP/1.1 200 OK\r\nContent-Type: text/event-stream\r\nCache-Control: no-cache\r\n";
  h += kCors;
  h += "Transfer-Encoding: chunked\r\nConnection: close\r\n\r\n";
  if (!write_all(fd, h)) { job->cancelled = true; return; }
  double last = now_ms();
  for (;;) {
    std::vector<Event> evs;
    bool done;
    {
      std::unique_lock<std::mutex> l(job->mu);
      job->cv.wait_for(l, std::chrono::milliseconds(100), [&] { return !job->q.empty() || job->done; });
      while (!job->q.empty()) {
        evs.push_back(std::move(job->q.front()));
        job->q.pop_front();
      }
      done = job->done;
    }
    std::string out;
    for (auto& e : evs) out += sse_event(e);
    if (out.empty() && now_ms() - last >= 1000.0) out = ":\n\n";   // keep-alive (main.rs:97)
    if (!out.empty()) {
      if (!write_all(fd, chunk(out))) {   // client went away: stop generating for it
        job->cancelled = true;
        return;
      }
      last = now_ms();
    }
    if (done && evs.empty()) break;
  }
  write_all(fd, "0\r\n\r\n");
}

void handle_completion(Server& S, int fd, const Request& r) {
  std::string prompt;
  int n = 128;   // PDF p.10: n_predict 128
  std::string model;
  if (!parse_prompt_body(fd, r, &prompt, &n, 128, &model) || !known_model(S, fd, &model)) return;
  auto job = submit(S, prompt, n, model);
  {
    std::unique_lock<std::mutex> l(job->mu);
    job->cv.wait(l, [&] { return job->done; });
  }
  const GenResult& g = job->result;
  Json o = Json::object();
  o["content"] = g.text;
  o["response"] = g.text;
  o["tokens_predicted"] = g.n_gen;
  o["tokens_evaluated"] = g.n_prompt;
  o["stop_reason"] = g.stop;
  Json t = Json::object();
  t["prompt_ms"] = g.prefill_ms;
  t["predicted_ms"] = g.decode_ms;
  t["predicted_per_second"] = g.n_gen > 1 && g.decode_ms > 0 ? (g.n_gen - 1) * 1e3 / g.decode_ms : 0.0;
  o["timings"] = t;
  respond(fd, 200, "application/json", o.dump());
}

void handle_metrics(Server& S, int fd) {
  std::string m;
  char b[512];
  {
    std::lock_guard<std::mutex> l(S.metrics.mu);
    auto& M = S.metrics;
    snprintf(b, sizeof(b),
             "# TYPE mipipe_requests_total counter\nmipipe_requests_total %llu\n"
             "# TYPE mipipe_requests_completed_total counter\nmipipe_requests_completed_total %llu\n"
             "# TYPE mipipe_requests_cancelled_total counter\nmipipe_requests_cancelled_total %llu\n"
             "# TYPE mipipe_request_errors_total counter\nmipipe_request_errors_total %llu\n"
             "# TYPE mipipe_prompt_tokens_total counter\nmipipe_prompt_tokens_total %llu\n"
             "# TYPE mipipe_generated_tokens_total counter\nmipipe_generated_tokens_total %llu\n",
             (unsigned long long)M.requests, (unsigned long long)M.completed, (unsigned long long)M.cancelled,
             (unsigned long long)M.errors, (unsigned long long)M.prompt_tokens, (unsigned long long)M.gen_tokens);
    m += b;
    snprintf(b, sizeof(b),
             "# TYPE mipipe_decode_tokens_per_second gauge\nmipipe_decode_tokens_per_second %.3f\n"
             "# TYPE mipipe_prefill_tokens_per_second gauge\nmipipe_prefill_tokens_per_second %.3f\n"
             "# TYPE mipipe_token_latency_ms summary\n"
             "mipipe_token_latency_ms{quantile=\"0.5\"} %.4f\nmipipe_token_latency_ms{quantile=\"0.9\"} %.4f\n"
             "mipipe_token_latency_ms{quantile=\"0.99\"} %.4f\n",
             M.last_decode_tok_s, M.last_prefill_tok_s, pctl(M.token_ms, 0.5), pctl(M.token_ms, 0.9),
             pctl(M.token_ms, 0.99));
    m += b;
  }
  {
    std::lock_guard<std::mutex> l(S.jobs_mu);
    snprintf(b, sizeof(b), "# TYPE mipipe_queue_depth gauge\nmipipe_queue_depth %zu\n", S.pending.size());
    m += b;
  }
  snprintf(b, sizeof(b), "# TYPE mipipe_open_connections gauge\nmipipe_open_connections %d\n", S.connections.load());
  m += b;
  std::unique_lock<std::mutex> el(S.eng_mu);
  if (S.eng) {
    Json h = S.eng->health();
    el.unlock();
    m += "# TYPE mipipe_stage_items_done counter\n";
    for (auto& st : h["stages"].arr()) {
      snprintf(b, sizeof(b), "mipipe_stage_items_done{stage=\"%d\"} %lld\n", (int)st["stage"].num(),
               (long long)st.get_num("items_done", 0));
      m += b;
    }
    m += "# TYPE mipipe_link_bytes_sent counter\n";
    for (auto& st : h["stages"].arr())
      if (st.has("bytes_sent")) {
        snprintf(b, sizeof(b), "mipipe_link_bytes_sent{stage=\"%d\",link=\"%s\"} %lld\n", (int)st["stage"].num(),
                 st.get_str("link", "").c_str(), (long long)st.get_num("bytes_sent", 0));
        m += b;
      }
    snprintf(b, sizeof(b), "# TYPE mipipe_engine_ok gauge\nmipipe_engine_ok %d\n", h.get_bool("ok", false) ? 1 : 0);
    m += b;
  }
  respond(fd, 200, "text/plain; version=0.0.4", m);
}

void handle_conn(Server& S, int fd, std::string peer) {
  S.connections++;
  Request r;
  r.peer = peer;
  const int rr = read_request(fd, r);
  if (rr < 0) respond_text(fd, 400, "Bad Request: invalid Content-Length");
  if (rr > 0) {
    try {
      if (r.method == "OPTIONS") {
        respond(fd, 204, "", "");
      } else if (r.path == "/chat") {
        if (r.method != "POST") respond(fd, 405, "text/plain; charset=utf-8", "Method Not Allowed", "Allow: POST\r\n");
        else if (authorized(S, fd, r)) handle_chat(S, fd, r);
      } else if (r.path == "/completion") {
        if (r.method != "POST") respond(fd, 405, "text/plain; charset=utf-8", "Method Not Allowed", "Allow: POST\r\n");
        else if (authorized(S, fd, r)) handle_completion(S, fd, r);
      } else if (r.path == "/metrics" && r.method == "GET") {
        handle_metrics(S, fd);
      } else if (r.path == "/health" && r.method == "GET") {
        Json h;
        {
          std::lock_guard<std::mutex> l(S.eng_mu);
          h = S.eng ? S.eng->health() : Json::object();
          if (!S.eng) h["ok"] = S.mock || !S.spawn_cli.empty();
          if (!S.spawn_cli.empty()) h["spawn_cli"] = S.spawn_cli;
          int restarts = 0;
          for (auto& mm : S.models) restarts += mm->restarts;
          h["engine_restarts"] = restarts;
        }
        h["mock"] = S.mock;
        respond(fd, 200, "application/json", h.dump());
      } else if (r.path == "/models" && r.method == "GET") {
        Json arr = Json::array();
        {
          std::lock_guard<std::mutex> l(S.eng_mu);
          for (auto& mm : S.models) {
            Json e = Json::object();
            e["id"] = mm->name;
            e["source"] = mm->source;
            e["loaded"] = (bool)mm->eng;
            e["restarts"] = mm->restarts;
            arr.push(e);
          }
        }
        Json o = Json::object();
        o["object"] = "list";
        o["data"] = arr;
        respond(fd, 200, "application/json", o.dump());
      } else if (r.method == "GET" || r.method == "HEAD") {
        serve_static(S, fd, r);
      } else {
        respond_text(fd, 405, "Method Not Allowed");
      }
    } catch (const std::exception& e) {
      respond_text(fd, 500, e.what());
    }
  }
  ::shutdown(fd, SHUT_RDWR);
  ::close(fd);
  S.connections--;
}

void usage() {
  fprintf(stderr, "usage: orchestrator (-m MODEL.gguf | --synthetic NAME | --mock) [--port 3005] [--host 0.0.0.0]\n"
                  "                    [--static DIR] [--api-key KEY] [--rate-limit N/min] [engine flags]\n"
                  "                    [--alias NAME] [--model-alias NAME=PATH.gguf|synthetic:NAME ...] [--max-models N]\n"
                  "                    [--spawn-cli mi-cli|PATH]  (a CLI child process per request, as the reference)\n");
  print_common_usage(stderr);
}

}  // namespace

int main(int argc, char** argv) {
  signal(SIGPIPE, SIG_IGN);
  Server S;
  g_srv = &S;
  int port = 3005;   // main.rs:107
  std::string host = "0.0.0.0";
  bool mock = false;
  std::string alias, synthetic_name = "model";
  std::vector<std::string> aliases;
  for (int i = 1; i + 1 < argc; ++i)
    if (!strcmp(argv[i], "--synthetic")) synthetic_name = argv[i + 1];
  CliOptions o;
  std::vector<char*> args(argv, argv + argc);
  for (int i = 1; i < argc; ++i)
    if (!strcmp(argv[i], "--mock")) mock = true;
  try {
    auto extra = [&](const std::string& a, const std::function<std::string()>& val) {
      if (a == "--port") port = std::atoi(val().c_str());
      else if (a == "--host") host = val();
      else if (a == "--static") S.static_dir = val();
      else if (a == "--api-key") S.api_key = val();
      else if (a == "--rate-limit") S.rate_limit = std::atoi(val().c_str());
      else if (a == "--mock") {}
      else if (a == "--mock-delay-ms") S.mock_delay_ms = std::atoi(val().c_str());
      else if (a == "--alias") alias = val();
      else if (a == "--model-alias") aliases.push_back(val());
      else if (a == "--max-models") S.max_models = std::max(1, std::atoi(val().c_str()));
      else if (a == "--no-continuous") S.continuous = false;
      else if (a == "--model-switch-ms") S.switch_after_ms = std::atof(val().c_str());
      else if (a == "--spawn-cli") S.spawn_cli = val();
      else if (a == "-h" || a == "--help") { usage(); exit(0); }
      else return false;
      return true;
    };
    if (mock) {
      // model flags optional in mock mode
      std::vector<char*> a2{argv[0], (char*)"--synthetic", (char*)"stories15m"};
      for (int i = 1; i < argc; ++i) a2.push_back(argv[i]);
      o = parse_cli((int)a2.size(), a2.data(), extra);
    } else {
      o = parse_cli(argc, argv, extra);
    }
  } catch (const std::exception& e) {
    fprintf(stderr, "orchestrator: %s\n", e.what());
    usage();
    return 2;
  }
  S.mock = mock;
  S.default_n = o.n_predict;
  if (!S.spawn_cli.empty()) {
    // forward the model / engine flags to every child; the server's own flags stay here
    static const char* own1[] = {"--port", "--host", "--static", "--api-key", "--rate-limit", "--mock-delay-ms",
                                 "--alias", "--model-alias", "--max-models", "--model-switch-ms", "--spawn-cli",
                                 "-p", "--prompt", "-n", "--n-predict"};
    static const char* own0[] = {"--mock", "--no-continuous", "--daemon"};
    for (int i = 1; i < argc; ++i) {
      bool skip = false;
      for (const char* f : own1)
        if (!strcmp(argv[i], f)) { skip = true; ++i; break; }
      for (const char* f : own0)
        if (!strcmp(argv[i], f)) skip = true;
      if (!skip) S.cli_args.push_back(argv[i]);
    }
    if (S.spawn_cli == "mi-cli" || S.spawn_cli == "default") {   // the mi-cli next to this binary
      char exe[4096];
      const ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
      if (n > 0) { exe[n] = 0; std::string d(exe); S.spawn_cli = d.substr(0, d.rfind('/')) + "/mi-cli"; }
    }
  }
  {
    struct stat stt;
    if (stat(S.static_dir.c_str(), &stt) != 0) {   // fall back to the package's static/ next to bin/
      char exe[4096];
      const ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
      if (n > 0) {
        exe[n] = 0;
        std::string d(exe);
        d = d.substr(0, d.rfind('/'));
        d = d.substr(0, d.rfind('/')) + "/static";
        if (stat(d.c_str(), &stt) == 0) S.static_dir = d;
      }
    }
  }
  // capture start-up logs (placement / offload lines) to replay to every request's log pane
  log_set_callback([&S](const std::string& line) {
    if (!S.ready && !S.mock) S.startup_logs.push_back(line);
    else broadcast_log(line);
  });
  try {
    if (!S.spawn_cli.empty()) {
      S.startup_logs.push_back("spawn-cli mode: every request runs " + S.spawn_cli + " (no engine in this process)\n");
      S.capacity = 1 << 20;
    } else if (!mock) {
      if (!o.eng.has("mb_size")) o.eng["mb_size"] = 4;
      std::unique_ptr<ModelSlot> d(new ModelSlot);
      d->cfg = o.eng;
      d->source = o.eng.has("gguf") ? o.eng.get_str("gguf", "") : "synthetic:" + synthetic_name;
      d->name = !alias.empty() ? alias : d->source.substr(d->source.rfind('/') + 1);
      S.models.push_back(std::move(d));
      for (const std::string& a : aliases) {
        const size_t eq = a.find('=');
        if (eq == std::string::npos || eq == 0) throw std::runtime_error("--model-alias expects NAME=PATH");
        std::unique_ptr<ModelSlot> m(new ModelSlot);
        m->name = a.substr(0, eq);
        m->source = a.substr(eq + 1);
        m->cfg = o.eng;
        if (m->source.rfind("synthetic:", 0) == 0) {
          m->cfg.erase("gguf");
          m->cfg["synthetic"] = synthetic_arch(m->source.substr(10));
        } else {
          m->cfg.erase("synthetic");
          m->cfg["gguf"] = m->source;
        }
        S.models.push_back(std::move(m));
      }
      load_slot(S, *S.models[0]);
      S.models[0]->last_used = now_ms();
      S.capacity = S.models[0]->sess->capacity();
    } else {
      S.startup_logs.push_back("mock engine: stage 0: layers 0-5 offloaded to GPU 0 (mock)\n");
      S.capacity = 4;
    }
  } catch (const std::exception& e) {
    MP_LOGE("orchestrator: engine init failed: %s", e.what());
    return 1;
  }
  S.ready = true;
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in addr{};
  addr.sin_family = AF_INET;
  addr.sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &addr.sin_addr) != 1) {
    MP_LOGE("bad --host %s", host.c_str());
    return 2;
  }
  if (bind(ls, (sockaddr*)&addr, sizeof(addr)) != 0 || listen(ls, 128) != 0) {
    MP_LOGE("cannot listen on %s:%d: %s", host.c_str(), port, strerror(errno));   // main.rs:109 panics; we exit 1
    return 1;
  }
  std::thread gen(generation_loop, std::ref(S));
  printf("orchestrator ready on http://%s:%d (static: %s, %s)\n", host.c_str(), port, S.static_dir.c_str(),
         mock ? "mock engine" : "engine loaded");
  fflush(stdout);
  while (!S.stop) {
    sockaddr_in peer{};
    socklen_t pl = sizeof(peer);
    int fd = accept(ls, (sockaddr*)&peer, &pl);
    if (fd < 0) continue;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    char ip[64];
    inet_ntop(AF_INET, &peer.sin_addr, ip, sizeof(ip));
    std::thread(handle_conn, std::ref(S), fd, std::string(ip)).detach();
  }
  gen.join();
  return 0;
}
