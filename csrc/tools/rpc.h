// Long-lived stage workers a client attaches to by host:port -- the role of llama.cpp's `rpc-server`
// in the reference (`orchestrator/src/main.rs:47-48`: `--rpc 127.0.0.1:50052,127.0.0.1:50053`).
//
//   worker:  mi-cli --rpc-server 50052 [-m LOCAL.gguf] [--device D]      (stays up across clients)
//   client:  mi-cli -m m.gguf --rpc 127.0.0.1:50052,127.0.0.1:50053 -p "..." -n 200
//
// The client is the LAST rank of a (#workers + 1)-stage pipeline -- the LM head and the sampler, so
// the text streams out where the user is (a Session emits on the stage that owns the head); worker
// i is rank i (worker 0: the embedding and the first layers).  Per generation the client opens one control connection per
// worker and sends one job: the engine config with the worker's rank, the ring's hosts and ports,
// the prompt and n_predict.  The data plane is the engine's TCP ring of the multi-process mode
// (`--world/--rank`, engine.cpp "tcp" links: the receiver of link l listens on base_port + l), so a
// worker is exactly a `--world/--rank` process whose arguments arrive over the socket.  The worker
// answers with one JSON result and waits for the next client.
//
// Unlike llama.cpp's rpc-server, weights are not shipped over the socket: each worker loads the
// GGUF from its own disk (the client's path, or the worker's -m), mmap'd and packed into its HBM.
// If the first worker does not answer, the client falls back to local stages, one per --rpc entry
// (the reference's command line then still runs on one box).
#pragma once
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "engine.h"
#include "json.h"
#include "log.h"
#include "session.h"

namespace mp {

// Control connections: plain POSIX sockets carrying length-prefixed JSON (8-byte length, then the
// text).  The worker keeps ONE listening socket for its whole life, so a client that arrives while
// the previous job is still answering waits in the accept backlog instead of being refused.
struct RpcConn {
  int fd = -1;
  RpcConn() = default;
  explicit RpcConn(int f) : fd(f) {}
  RpcConn(const RpcConn&) = delete;
  RpcConn& operator=(const RpcConn&) = delete;
  RpcConn(RpcConn&& o) noexcept : fd(o.fd) { o.fd = -1; }
  ~RpcConn() {
    if (fd >= 0) ::close(fd);
  }
  void write_all(const void* p, size_t n) const {
    const char* c = static_cast<const char*>(p);
    while (n) {
      const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
      if (w <= 0) throw std::runtime_error("rpc: connection lost (send)");
      c += w;
      n -= (size_t)w;
    }
  }
  void read_all(void* p, size_t n) const {
    char* c = static_cast<char*>(p);
    while (n) {
      const ssize_t r = ::recv(fd, c, n, 0);
      if (r <= 0) throw std::runtime_error("rpc: connection lost (recv)");
      c += r;
      n -= (size_t)r;
    }
  }
  void send_json(const Json& j) const {
    const std::string s = j.dump();
    const uint64_t n = s.size();
    write_all(&n, 8);
    write_all(s.data(), s.size());
  }
  Json recv_json() const {
    uint64_t n = 0;
    read_all(&n, 8);
    if (n > (64u << 20)) throw std::runtime_error("rpc: oversized control message");
    std::string s(n, '\0');
    read_all(&s[0], n);
    return Json::parse(s);
  }
};

inline int rpc_listen(int port) {
  const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons((uint16_t)port);
  if (ls < 0 || ::bind(ls, (sockaddr*)&a, sizeof(a)) != 0 || ::listen(ls, 16) != 0) {
    if (ls >= 0) ::close(ls);
    throw std::runtime_error("rpc: cannot listen on port " + std::to_string(port));
  }
  return ls;
}

// connect with retries until timeout_s (a worker may still be starting)
inline RpcConn rpc_connect(const std::string& host, int port, double timeout_s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
      const int fd = ::socket(res->ai_family, res->ai_socktype, 0);
      const bool ok = fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0;
      freeaddrinfo(res);
      if (ok) return RpcConn(fd);
      if (fd >= 0) ::close(fd);
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      throw std::runtime_error("rpc: no worker at " + host + ":" + std::to_string(port));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

// worker loop: one job per accepted control connection; max_jobs 0 = forever
inline int run_rpc_server(int port, const std::string& local_gguf, int device, int max_jobs) {
  const int ls = rpc_listen(port);
  MP_LOGI("rpc worker listening on port %d", port);
  for (int done = 0; max_jobs <= 0 || done < max_jobs; ++done) {
    const int fd = ::accept(ls, nullptr, nullptr);
    if (fd < 0) {
      ::close(ls);
      throw std::runtime_error("rpc: accept failed");
    }
    RpcConn ctl(fd);
    Json res = Json::object();
    try {
      Json job = ctl.recv_json();
      Json cfg = job["engine"];
      if (!local_gguf.empty()) cfg["gguf"] = local_gguf;
      cfg["device"] = device >= 0 ? device : 0;   // the worker's GPU (HIP_VISIBLE_DEVICES or --device)
      MP_LOGI("rpc job: rank %d of %d, %s", cfg.get_int("rank", -1), cfg.get_int("world", 0),
              cfg.get_str("gguf", cfg.has("synthetic") ? "synthetic" : "?").c_str());
      Engine eng(cfg);
      Session s(eng, cfg.get_str("gguf", ""));
      std::vector<GenRequest> reqs(1);
      reqs[0].prompt = job.get_str("prompt", "");
      reqs[0].n_predict = job.get_int("n_predict", 200);
      reqs[0].on_piece = [](const std::string&) { return true; };
      auto r = s.run(reqs)[0];
      res["ok"] = true;
      res["rank"] = cfg.get_int("rank", -1);
      res["stages"] = eng.info()["stages"];
      res["n_gen"] = r.n_gen;
    } catch (const std::exception& e) {
      MP_LOGE("rpc job failed: %s", e.what());
      res["ok"] = false;
      res["error"] = std::string(e.what());
    }
    try {
      ctl.send_json(res);
    } catch (const std::exception& e) {
      MP_LOGE("rpc: client gone before the result: %s", e.what());
    }
  }
  ::close(ls);
  return 0;
}

struct RpcClient {
  std::vector<RpcConn> ctl;   // one control connection per worker (rank i)
};

// Attach to the workers listed by --rpc (host:port,...): on success `eng_cfg` becomes the last rank
// of the ring and every worker has its job; false (nothing sent) when the first worker does not answer.
inline bool rpc_attach(const std::string& rpc, Json& eng_cfg, const std::string& prompt, int n_predict,
                       const std::string& self_host, RpcClient& cl, double connect_timeout = 0.5) {
  std::vector<std::string> ent;
  for (size_t a = 0; a <= rpc.size();) {
    const size_t b = rpc.find(',', a);
    const std::string e = rpc.substr(a, b == std::string::npos ? std::string::npos : b - a);
    if (!e.empty()) ent.push_back(e);
    if (b == std::string::npos) break;
    a = b + 1;
  }
  if (ent.empty()) return false;
  std::vector<std::string> hosts;
  std::vector<int> ports;
  for (auto& e : ent) {
    const auto c = e.rfind(':');
    if (c == std::string::npos) throw std::runtime_error("--rpc entries are host:port (got " + e + ")");
    hosts.push_back(e.substr(0, c));
    ports.push_back(std::atoi(e.c_str() + c + 1));
  }
  for (size_t i = 0; i < hosts.size(); ++i) {
    try {
      cl.ctl.push_back(rpc_connect(hosts[i], ports[i], i == 0 ? connect_timeout : 30.0));
    } catch (const std::exception& e) {
      if (i == 0) {
        MP_LOGI("rpc: no worker at %s:%d (%s): local stages, one per --rpc entry", hosts[0].c_str(), ports[0], e.what());
        return false;
      }
      throw;
    }
  }
  const int world = 1 + (int)hosts.size();
  Json h = Json::array();
  for (auto& x : hosts) h.push(x);
  h.push(self_host);
  eng_cfg["mode"] = "mp";
  eng_cfg["world"] = world;
  eng_cfg["link"] = "tcp";
  eng_cfg["hosts"] = h;
  eng_cfg.erase("stages");
  // this process's GPU: the first --devices entry, else 0 (the workers pick their own)
  int dev = 0;
  if (eng_cfg.has("devices") && eng_cfg["devices"].is_arr() && !eng_cfg["devices"].arr().empty())
    dev = (int)eng_cfg["devices"].arr()[0].num();
  eng_cfg.erase("devices");
  for (int r = 0; r + 1 < world; ++r) {
    Json job = Json::object();
    Json c = eng_cfg;
    c["rank"] = r;
    job["engine"] = c;
    job["prompt"] = prompt;
    job["n_predict"] = n_predict;
    cl.ctl[r].send_json(job);
  }
  eng_cfg["rank"] = world - 1;
  eng_cfg["device"] = dev;
  MP_LOGI("rpc: %d worker(s) attached, ring of %d stages", world - 1, world);
  return true;
}

// the workers' results (after the client's own generation)
inline void rpc_collect(RpcClient& cl) {
  for (size_t i = 0; i < cl.ctl.size(); ++i) {
    const Json r = cl.ctl[i].recv_json();
    if (!r.get_bool("ok", false)) throw std::runtime_error("rpc worker " + std::to_string(i) + ": " + r.get_str("error", "?"));
    MP_LOGI("rpc worker %zu done: %s", i, r.dump().c_str());
  }
}

}  // namespace mp
