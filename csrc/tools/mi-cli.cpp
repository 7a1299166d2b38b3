// mi-cli: the generation driver (the role of llama-cli in the reference; flags as
// spawned by `orchestrator/src/main.rs:38-53`).  stdout = prompt echo + generated text (streamed,
// UTF-8 safe), stderr = logs incl. the stage placement lines and the perf summary.
//
//   mi-cli -m model.gguf -p "Once upon a time" -n 200 -c 2048 -ngl 99 --stages 2 --verbose
//   mi-cli --synthetic llama3-70b --ftype Q4_K --bench --mb-size 16
//   mi-cli -m m.gguf --world 2 --rank 0 --next 10.0.0.2      (one process per stage, TCP ring)
//   mi-cli -m m.gguf --daemon      (JSON-lines server on stdin/stdout for the orchestrator)
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>

#include "cli_common.h"
#include "engine.h"
#include "log.h"
#include "session.h"

using namespace mp;

static void usage() {
  fprintf(stderr, "usage: mi-cli -m MODEL.gguf [-p PROMPT] [-n N] [-c CTX] [-ngl N] [options]\n");
  print_common_usage(stderr);
  fprintf(stderr,
          "mi-cli:\n"
          "  --bench [--bench-prompt L --bench-warmup W --bench-steps K]   decode throughput of full batches\n"
          "  --daemon                  read {\"prompt\":..,\"n_predict\":..} lines on stdin, answer with JSON lines\n"
          "  --no-display-prompt       do not echo the prompt\n"
          "  --state-save DIR          after generating, checkpoint the KV shards + sequences to DIR\n"
          "  --state-load DIR          resume a checkpoint: continue its sequence for -n more tokens\n");
}

static int run_daemon(Session& s) {
  // one JSON request per line -> {"piece": ...} lines then {"done": true, stats}
  std::string line;
  while (std::getline(std::cin, line)) {
    if (line.empty()) continue;
    Json rq;
    try {
      rq = Json::parse(line);
    } catch (const std::exception& e) {
      Json err = Json::object();
      err["error"] = e.what();
      printf("%s\n", err.dump().c_str());
      fflush(stdout);
      continue;
    }
    std::vector<GenRequest> reqs(1);
    reqs[0].prompt = rq.get_str("prompt", "");
    reqs[0].n_predict = rq.get_int("n_predict", 200);
    reqs[0].on_piece = [](const std::string& p) {
      Json o = Json::object();
      o["piece"] = p;
      printf("%s\n", o.dump().c_str());
      fflush(stdout);
      return true;
    };
    auto r = s.run(reqs)[0];
    Json d = Json::object();
    d["done"] = true;
    d["n_prompt"] = r.n_prompt;
    d["n_gen"] = r.n_gen;
    d["prefill_ms"] = r.prefill_ms;
    d["decode_ms"] = r.decode_ms;
    d["stop"] = r.stop;
    printf("%s\n", d.dump().c_str());
    fflush(stdout);
  }
  return 0;
}

int main(int argc, char** argv) {
  bool daemon = false;
  std::string state_save, state_load;
  CliOptions o;
  try {
    o = parse_cli(argc, argv, [&](const std::string& a, const std::function<std::string()>& val) {
      if (a == "--daemon") { daemon = true; return true; }
      if (a == "--state-save") { state_save = val(); return true; }
      if (a == "--state-load") { state_load = val(); return true; }
      if (a == "-h" || a == "--help") { usage(); exit(0); }
      return false;
    });
  } catch (const std::exception& e) {
    fprintf(stderr, "mi-cli: %s\n", e.what());
    usage();
    return 2;
  }
  try {
    if (o.bench) {
      if (!o.eng.has("mb_size")) o.eng["mb_size"] = 16;
      const int need = o.bench_prompt + o.bench_warmup + o.bench_steps + 8;
      if (o.eng.get_int("max_ctx", 2048) < need) o.eng["max_ctx"] = need;
    }
    Engine eng(o.eng);
    if (!o.trace.empty()) eng.enable_trace(true);
    if (o.bench) {
      Json r = eng.bench(o.bench_prompt, o.bench_warmup, o.bench_steps);
      r["info"] = eng.info();
      printf("%s\n", r.dump().c_str());
      if (!o.trace.empty()) eng.write_trace(o.trace);
      return 0;
    }
    Session s(eng, o.eng.get_str("gguf", ""));
    if (daemon) return run_daemon(s);
    if (!state_load.empty()) {
      // resume: continue sequence 0 of the checkpoint token by token
      eng.load_state(state_load);
      const bool solo = eng.owns_first() && eng.owns_last();
      Utf8Acc acc;
      int n = 0;
      const double t0 = session_now_ms();
      for (; n < o.n_predict; ++n) {
        eng.decode_steps(1);
        if (!eng.owns_last()) continue;
        const int32_t t = eng.tokens()[0].back();
        if (s.is_eog(t) && solo) break;
        const std::string p = acc.push(s.piece(t));
        fwrite(p.data(), 1, p.size(), stdout);
        fflush(stdout);
      }
      if (eng.owns_last()) {
        fputs((acc.buf + "\n").c_str(), stdout);
        MP_LOGI("resumed %s: %d tokens in %.1f ms", state_load.c_str(), n, session_now_ms() - t0);
      }
      if (!state_save.empty()) eng.save_state(state_save);
      return 0;
    }
    if (o.echo_prompt && eng.owns_last()) {
      fputs(o.prompt.c_str(), stdout);
      fflush(stdout);
    }
    std::vector<GenRequest> reqs(1);
    reqs[0].prompt = o.prompt;
    reqs[0].n_predict = o.n_predict;
    reqs[0].on_piece = [](const std::string& p) {
      fwrite(p.data(), 1, p.size(), stdout);
      fflush(stdout);
      return true;
    };
    auto r = s.run(reqs)[0];
    if (eng.owns_last()) {
      fputs("\n", stdout);
      fflush(stdout);
      MP_LOGI("\n%s", Session::perf_summary(r, eng.load_ms()).c_str());
    }
    if (!state_save.empty()) eng.save_state(state_save);
    if (!o.trace.empty()) eng.write_trace(o.trace);
  } catch (const std::exception& e) {
    MP_LOGE("mi-cli: error: %s", e.what());
    return 1;
  }
  return 0;
}
