#include "session.h"

#include <algorithm>
#include <deque>
#include <chrono>
#include <cstdio>

#include "gguf.h"
#include "log.h"

namespace mp {

double session_now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
namespace {
double now_ms() { return session_now_ms(); }
}  // namespace

std::string Utf8Acc::push(const std::string& b) {
  buf += b;
  size_t cut = buf.size();
  for (size_t k = 1; k <= 4 && k <= buf.size(); ++k) {
    const unsigned char c = (unsigned char)buf[buf.size() - k];
    if ((c & 0xC0) == 0x80) continue;
    const int need = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : c >= 0xC0 ? 2 : 1;
    if (need > (int)k) cut = buf.size() - k;
    break;
  }
  std::string o = buf.substr(0, cut);
  buf.erase(0, cut);
  return o;
}

Session::Session(Engine& eng, const std::string& gguf_path) : eng_(&eng) {
  if (!gguf_path.empty()) {
    gguf_.reset(new GgufFile(gguf_path));
    if (gguf_->get("tokenizer.ggml.tokens")) tok_.reset(new Tokenizer(Tokenizer::from_gguf(*gguf_)));
  }
  if (!tok_) MP_LOGW("no tokenizer in the model: using a byte-level stand-in (synthetic model)");
}

Session::~Session() = default;

std::vector<int32_t> Session::encode(const std::string& text) const {
  if (tok_) return tok_->encode(text, tok_->add_bos_default(), true);
  std::vector<int32_t> o{1};
  const int V = eng_->model().vocab;
  for (unsigned char c : text) o.push_back((int32_t)((c + 3) % V));
  return o;
}

std::string Session::piece(int32_t id) const {
  if (tok_) return tok_->piece(id);
  return "[" + std::to_string(id) + "]";
}

bool Session::is_eog(int32_t id) const { return tok_ && tok_->is_eog(id); }

std::vector<GenResult> Session::run(std::vector<GenRequest>& reqs) {
  if ((int)reqs.size() > capacity()) throw std::runtime_error("more requests than sequence slots");
  std::vector<GenResult> res(reqs.size());
  std::vector<std::vector<int32_t>> prompts(reqs.size());
  const int max_ctx = eng_->max_ctx();
  int max_prompt = 0;
  for (size_t i = 0; i < reqs.size(); ++i) {
    prompts[i] = encode(reqs[i].prompt);
    if ((int)prompts[i].size() >= max_ctx) {   // keep the tail (most recent context)
      prompts[i].erase(prompts[i].begin(), prompts[i].end() - (max_ctx / 2));
      MP_LOGW("prompt of sequence %zu truncated to %d tokens (context %d)", i, max_ctx / 2, max_ctx);
    }
    res[i].n_prompt = (int)prompts[i].size();
    max_prompt = std::max(max_prompt, res[i].n_prompt);
  }
  int n_max = 0;
  for (auto& r : reqs) n_max = std::max(n_max, r.n_predict);
  n_max = std::max(0, std::min(n_max, max_ctx - max_prompt - 1));
  // all ranks of a multi-process pipeline must run the same number of rounds: early stop only
  // when this process owns the whole pipeline
  const bool early_stop = eng_->owns_first() && eng_->owns_last();
  const bool emit = eng_->owns_last();
  std::vector<Utf8Acc> acc(reqs.size());
  std::vector<bool> active(reqs.size(), true);
  auto consume = [&](size_t i, int32_t t, int step) {
    if (!active[i]) return;
    GenResult& r = res[i];
    if (step >= reqs[i].n_predict) { active[i] = false; r.stop = "length"; return; }
    if (is_eog(t)) { active[i] = false; r.stop = "eog"; return; }
    r.tokens.push_back(t);
    r.n_gen++;
    const std::string p = acc[i].push(piece(t));
    r.text += p;
    if (emit && !p.empty() && reqs[i].on_piece && !reqs[i].on_piece(p)) { active[i] = false; r.stop = "cancelled"; }
  };
  const double t0 = now_ms();
  const int draft_max = eng_->config().get_int("draft_max", 0);
  if (draft_max > 0 && early_stop) {
    // speculative decoding by prompt lookup (greedy): tokens arrive in accepted runs per round
    std::vector<int> steps(reqs.size(), 0);
    double t_first = 0;
    eng_->on_token = [&](int i, int32_t t) { consume((size_t)i, t, steps[i]++); };
    eng_->keep_going = [&](int i) { return (bool)active[i]; };
    auto cleanup = [&] { eng_->on_token = nullptr; eng_->keep_going = nullptr; };
    try {
      std::vector<std::vector<int32_t>> gen;
      const Json st = eng_->spec_generate(prompts, std::max(1, n_max), draft_max,
                                         eng_->config().get_int("lookup_ngram", 3), &gen);
      t_first = t0 + st.get_num("prefill_ms", 0.0);
      MP_LOGI("speculative lookup: %ld verify rounds, %ld/%ld drafted tokens accepted",
              (long)st.get_num("verify_rounds", 0), (long)st.get_num("accepted", 0), (long)st.get_num("drafted", 0));
    } catch (...) {
      cleanup();
      throw;
    }
    cleanup();
    const double t2 = now_ms();
    for (size_t i = 0; i < reqs.size(); ++i) {
      if (active[i]) res[i].stop = n_max < reqs[i].n_predict ? "context" : "length";
      const std::string tail = acc[i].buf;
      if (!tail.empty()) {
        res[i].text += tail;
        if (emit && active[i] && reqs[i].on_piece) reqs[i].on_piece(tail);
      }
      res[i].prefill_ms = t_first - t0;
      res[i].decode_ms = t2 - t_first;
    }
    return res;
  }
  eng_->start(prompts);
  const double t1 = now_ms();
  // a middle rank of a multi-process pipeline sees no tokens (they travel the ring from the last
  // stage to the first): nothing to consume there
  if (n_max > 0) {
    const auto toks = eng_->tokens();
    for (size_t i = 0; i < reqs.size(); ++i)
      if (i < toks.size() && !toks[i].empty()) consume(i, toks[i].back(), 0);
  }
  int step = 1;
  auto any_active = [&] { return std::any_of(active.begin(), active.end(), [](bool b) { return b; }); };
  while (step < n_max && (!early_stop || any_active())) {
    eng_->decode_steps(1);
    const auto toks = eng_->tokens();
    for (size_t i = 0; i < reqs.size(); ++i)
      if (i < toks.size() && !toks[i].empty()) consume(i, toks[i].back(), step);
    ++step;
  }
  const double t2 = now_ms();
  for (size_t i = 0; i < reqs.size(); ++i) {
    if (active[i]) res[i].stop = n_max < reqs[i].n_predict ? "context" : "length";
    const std::string tail = acc[i].buf;
    if (!tail.empty()) {
      res[i].text += tail;
      if (emit && active[i] && reqs[i].on_piece) reqs[i].on_piece(tail);
    }
    res[i].prefill_ms = t1 - t0;
    res[i].decode_ms = t2 - t1;
  }
  return res;
}

void Session::serve(const std::function<std::vector<Served>(int free)>& next) {
  if (!eng_->owns_first() || !eng_->owns_last()) throw std::runtime_error("serve: needs every stage in this process");
  struct Live {
    Served s;
    GenResult res;
    Utf8Acc acc;
    int step = 0;
    int pages = 0;   // KV pages reserved for prompt + n_predict (paged KV admission control)
    std::vector<int32_t> prompt;   // for re-admission into a replacement engine after a fault
    double t0 = 0, t1 = 0;
    bool resumed = false;          // requeued by a failover: keeps its timings and produced tokens
  };
  struct Pending {
    Served s;
    std::vector<int32_t> prompt;   // a resumed request: its prompt + the tokens it already produced
    int pages = 0;
    std::unique_ptr<Live> resume;  // a running request a failover could not re-admit at once
  };
  // engine geometry: re-read after a failover (the replacement runs on fewer GPUs, so its KV
  // pool, context and slot count can all be smaller)
  int cap = capacity(), max_ctx = eng_->max_ctx();
  // paged KV (kvpager.h): a request is admitted only when the pool can hold its prompt plus every
  // token it may generate on top of what the running requests may still grow into, so a decode
  // round never runs out of pages; requests that do not fit wait (FIFO) for pages to come back
  int pool = eng_->kv_pages();
  int reserved = 0;
  std::deque<Pending> waiting;
  std::vector<std::unique_ptr<Live>> live(cap);
  // pages a request can ever need (its context is capped at max_ctx), and that clamped to the pool
  auto pages_need = [&](long prompt_len, int n_predict) {
    const long want = prompt_len + std::max(0, n_predict) + 1;
    return (int)std::min<long>((want + 63) / 64, (long)max_ctx / 64);
  };
  auto pages_for = [&](long prompt_len, int n_predict) {
    return (int)std::min<long>(pages_need(prompt_len, n_predict), (long)pool);
  };
  auto consume = [&](int slot, int32_t t) -> bool {   // false: the request is finished
    Live& L = *live[slot];
    GenResult& r = L.res;
    if (L.step >= L.s.req.n_predict) { r.stop = "length"; return false; }
    if (is_eog(t)) { r.stop = "eog"; return false; }
    r.tokens.push_back(t);
    r.n_gen++;
    const std::string p = L.acc.push(piece(t));
    r.text += p;
    ++L.step;
    if (!p.empty() && L.s.req.on_piece && !L.s.req.on_piece(p)) { r.stop = "cancelled"; return false; }
    if (L.step >= L.s.req.n_predict) { r.stop = "length"; return false; }
    // the context or the request's share of the KV pool is full
    if (eng_->slot_position(slot) + 1 >= std::min(max_ctx, L.pages * 64)) { r.stop = "context"; return false; }
    return true;
  };
  auto finish = [&](int slot) {
    Live& L = *live[slot];
    if (!L.acc.buf.empty()) {
      L.res.text += L.acc.buf;
      if (L.s.req.on_piece && L.res.stop != "cancelled") L.s.req.on_piece(L.acc.buf);
    }
    L.res.decode_ms = now_ms() - L.t1;
    if (L.s.done) L.s.done(L.res);
    eng_->release(slot);
    reserved -= L.pages;
    live[slot].reset();
  };
  // runs an engine call; on a pipeline fault with a handler installed, swaps in the replacement
  // engine and re-admits every live request as prompt + the tokens it has produced (slots 0..n-1),
  // consuming the re-prefill's token like a normal admission.  false: failed over (skip the rest
  // of this round); rethrows when there is no handler, the handler gives up or the budget is spent.
  std::function<bool(const std::function<void()>&)> guarded = [&](const std::function<void()>& call) -> bool {
    try {
      call();
      return true;
    } catch (const std::exception& e) {
      if (!on_fault_ || failovers_ >= max_failovers_) throw;
      Engine* ne = on_fault_(e.what());
      if (!ne) throw;
      eng_ = ne;
      ++failovers_;
      MP_LOGW("serve: failed over after \"%s\" (%d); re-admitting the running requests", e.what(), failovers_);
    }
    cap = capacity();
    max_ctx = eng_->max_ctx();
    pool = eng_->kv_pages();
    std::vector<std::unique_ptr<Live>> moved;
    for (auto& l : live)
      if (l) moved.push_back(std::move(l));
    live.clear();
    live.resize(cap);
    reserved = 0;
    // the waiting queue under the new engine's limits: a resumed request (prompt + produced tokens)
    // that no longer fits the context ends with stop "context" (admit would reject it, and that
    // rejection would read as a pipeline fault); a new one is truncated like a fresh admission
    for (auto it = waiting.begin(); it != waiting.end();) {
      Pending& pd = *it;
      if ((int)pd.prompt.size() + 1 >= max_ctx) {
        if (pd.resume) {
          Live& L = *pd.resume;
          L.res.stop = "context";
          if (!L.acc.buf.empty()) {
            L.res.text += L.acc.buf;
            if (L.s.req.on_piece) L.s.req.on_piece(L.acc.buf);
          }
          L.res.decode_ms = now_ms() - L.t1;
          if (L.s.done) L.s.done(L.res);
          it = waiting.erase(it);
          continue;
        }
        pd.prompt.erase(pd.prompt.begin(), pd.prompt.end() - (max_ctx / 2));
      }
      pd.pages = pd.resume ? pages_for((long)pd.resume->prompt.size(), pd.resume->s.req.n_predict)
                           : pages_for((long)pd.prompt.size(), pd.s.req.n_predict);
      ++it;
    }
    // re-admit in order while the new engine has a slot, the context and the pages for the
    // request's prompt + produced tokens + what it may still generate.  A request that fits the new
    // engine but not right now (its slots or pages are taken) goes back to the FRONT of the queue,
    // prompt + produced tokens as its prompt, and resumes when pages come back; only one that can
    // never fit ends: stop "context" (its context exceeds the new max_ctx) or "failover" (its pages
    // exceed the smaller engine's whole pool)
    std::vector<std::vector<int32_t>> prompts;
    std::vector<Pending> requeue;
    for (auto& m : moved) {
      std::vector<int32_t> pr = m->prompt;
      pr.insert(pr.end(), m->res.tokens.begin(), m->res.tokens.end());
      const int pages = pages_for((long)m->prompt.size(), m->s.req.n_predict);
      // the pool test matches fresh admission (pages_for clamps to the pool and the request stops at
      // "context" once its share fills): what it holds now plus its next token must fit the pool
      const bool ctx_ok = (int)pr.size() + 1 < max_ctx,
                 pool_ok = ((long)pr.size() + 1 + 63) / 64 <= (long)pool;
      if ((int)prompts.size() < cap && ctx_ok && reserved + pages <= pool) {
        m->pages = pages;
        reserved += pages;
        live[prompts.size()] = std::move(m);
        prompts.push_back(std::move(pr));
        continue;
      }
      if (ctx_ok && pool_ok) {
        Pending pd;
        pd.prompt = std::move(pr);
        pd.pages = pages;
        m->resumed = true;
        pd.resume = std::move(m);
        requeue.push_back(std::move(pd));
        continue;
      }
      Live& L = *m;
      L.res.stop = ctx_ok ? "failover" : "context";
      if (!L.acc.buf.empty()) {
        L.res.text += L.acc.buf;
        if (L.s.req.on_piece) L.s.req.on_piece(L.acc.buf);
      }
      L.res.decode_ms = now_ms() - L.t1;
      if (L.s.done) L.s.done(L.res);
    }
    for (auto it = requeue.rbegin(); it != requeue.rend(); ++it) waiting.push_front(std::move(*it));
    if (prompts.empty()) return false;
    eng_->start(prompts);   // a replacement fault propagates (the handler already had its turn)
    for (size_t i = 0; i < prompts.size(); ++i)
      if (!consume((int)i, eng_->last_token((int)i))) finish((int)i);
    return false;
  };
  for (;;) {
    int free = 0;
    for (auto& l : live) free += l ? 0 : 1;
    // new requests only when nobody is waiting for pages (FIFO)
    if (free > (int)waiting.size() && waiting.empty())
      for (auto& f : next(free)) {
        Pending pd;
        pd.prompt = encode(f.req.prompt);
        if ((int)pd.prompt.size() >= max_ctx) pd.prompt.erase(pd.prompt.begin(), pd.prompt.end() - (max_ctx / 2));
        pd.pages = pages_for((long)pd.prompt.size(), f.req.n_predict);
        pd.s = std::move(f);
        waiting.push_back(std::move(pd));
      }
    std::vector<int> slots;
    std::vector<std::vector<int32_t>> prompts;
    const bool idle = free == cap;
    while (!waiting.empty() && (int)slots.size() < free && reserved + waiting.front().pages <= pool) {
      Pending pd = std::move(waiting.front());
      waiting.pop_front();
      int sl = 0;
      while (live[sl] || std::find(slots.begin(), slots.end(), sl) != slots.end()) ++sl;
      std::unique_ptr<Live> L = std::move(pd.resume);
      if (!L) {
        L = std::make_unique<Live>();
        L->res.n_prompt = (int)pd.prompt.size();
        L->prompt = pd.prompt;
        L->s = std::move(pd.s);
        L->t0 = now_ms();
      }
      L->pages = pd.pages;
      reserved += L->pages;
      live[sl] = std::move(L);
      slots.push_back(sl);
      prompts.push_back(std::move(pd.prompt));
    }
    if (!slots.empty()) {
      // nothing running: a plain start() of slots 0..n-1 (resets the engine's rounds)
      const bool ok = guarded([&] {
        if (idle && slots.back() == (int)slots.size() - 1) eng_->start(prompts);
        else eng_->admit(slots, prompts);
      });
      if (!ok) continue;   // failed over: every live request (these included) was re-admitted
      const double t = now_ms();
      for (int sl : slots) {
        Live& L = *live[sl];
        if (!L.resumed) {
          L.t1 = t;
          L.res.prefill_ms = t - L.t0;
        }
        if (L.s.req.n_predict <= 0 || !consume(sl, eng_->last_token(sl))) finish(sl);
      }
    }
    bool any = false;
    for (auto& l : live) any = any || (bool)l;
    if (!any) {
      if (waiting.empty() && slots.empty()) return;
      continue;
    }
    if (!guarded([&] { eng_->decode_steps(1); })) continue;
    for (int sl = 0; sl < cap; ++sl)
      if (live[sl] && !consume(sl, eng_->last_token(sl))) finish(sl);
  }
}

std::string Session::perf_summary(const GenResult& r, double load_ms) {
  char b[1024];
  const int ng = std::max(0, r.n_gen - 1);   // the first token comes out of the prefill
  snprintf(b, sizeof(b),
           "mi_perf_context_print:        load time = %10.2f ms\n"
           "mi_perf_context_print: prompt eval time = %10.2f ms / %5d tokens (%8.2f ms per token, %8.2f tokens per second)\n"
           "mi_perf_context_print:        eval time = %10.2f ms / %5d runs   (%8.2f ms per token, %8.2f tokens per second)\n"
           "mi_perf_context_print:       total time = %10.2f ms / %5d tokens\n",
           load_ms, r.prefill_ms, r.n_prompt, r.prefill_ms / std::max(1, r.n_prompt),
           1e3 * r.n_prompt / std::max(1e-9, r.prefill_ms), r.decode_ms, ng, r.decode_ms / std::max(1, ng),
           1e3 * ng / std::max(1e-9, r.decode_ms), r.prefill_ms + r.decode_ms, r.n_prompt + r.n_gen);
  return b;
}

}  // namespace mp
