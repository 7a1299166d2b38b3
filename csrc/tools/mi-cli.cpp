// mi-cli: the generation driver (the role of llama-cli in the reference; flags as
// spawned by `orchestrator/src/main.rs:38-53`).  stdout = prompt echo + generated text (streamed,
// UTF-8 safe), stderr = logs incl. the stage placement lines and the perf summary.
//
//   mi-cli -m model.gguf -p "Once upon a time" -n 200 -c 2048 -ngl 99 --stages 2 --verbose
//   mi-cli --synthetic llama3-70b --ftype Q4_K --bench --mb-size 16
//   mi-cli -m m.gguf --world 2 --rank 0 --next 10.0.0.2      (one process per stage, TCP ring)
//   mi-cli -m m.gguf --daemon      (JSON-lines server on stdin/stdout for the orchestrator)
//   mi-cli --rpc-server 50052      (long-lived stage worker; a client attaches with --rpc host:port,..)
#include <cstdio>
#include <cstring>
#include <iostream>
#include <string>

#include "cli_common.h"
#include "engine.h"
#include "log.h"
#include "rpc.h"
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
          "  --state-load DIR          resume a checkpoint: continue its sequence for -n more tokens\n"
          "  --rpc-server PORT [-m LOCAL.gguf] [--device D] [--rpc-jobs N]\n"
          "                            stage worker (llama.cpp rpc-server role): serve --rpc clients, N jobs (0 = forever)\n");
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

// mi-cli --rpc-server PORT [-m LOCAL.gguf] [--device D] [--rpc-jobs N] [--verbose]
static int rpc_server_main(int argc, char** argv) {
  int port = 0, device = -1, jobs = 0;
  std::string gguf;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto val = [&]() -> std::string {
      if (i + 1 >= argc) throw std::runtime_error("missing value for " + a);
      return argv[++i];
    };
    if (a == "--rpc-server") port = std::atoi(val().c_str());
    else if (a == "-m" || a == "--model") gguf = val();
    else if (a == "--device") device = std::atoi(val().c_str());
    else if (a == "--rpc-jobs") jobs = std::atoi(val().c_str());
    else if (a == "--verbose") log_set_level(LOG_DEBUG);
    else throw std::runtime_error("--rpc-server: unknown flag " + a);
  }
  if (port <= 0) throw std::runtime_error("--rpc-server needs a port");
  return run_rpc_server(port, gguf, device, jobs);
}

int main(int argc, char** argv) {
  for (int i = 1; i < argc; ++i)
    if (std::strcmp(argv[i], "--rpc-server") == 0) {
      try {
        return rpc_server_main(argc, argv);
      } catch (const std::exception& e) {
        MP_LOGE("mi-cli: %s", e.what());
        return 2;
      }
    }
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
    RpcClient rpc;
    const bool attached = !o.bench && !daemon && state_load.empty() && !o.rpc.empty() &&
                          rpc_attach(o.rpc, o.eng, o.prompt, o.n_predict, o.master.empty() ? "127.0.0.1" : o.master, rpc);
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
    if (attached) rpc_collect(rpc);
  } catch (const std::exception& e) {
    MP_LOGE("mi-cli: error: %s", e.what());
    return 1;
  }
  return 0;
}
