#include "transport.h"

#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <thread>

#include <rccl/rccl.h>

#include "hip_stage.h"  // HIP_OK

namespace mp {

#define NCCL_OK(x)                                                                              \
  do {                                                                                          \
    ncclResult_t r_ = (x);                                                                      \
    if (r_ != ncclSuccess) throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(r_)); \
  } while (0)

// ---------------------------------------------------------------- LocalLink
LocalLink::LocalLink(int src_device, int dst_device) : src_dev_(src_device), dst_dev_(dst_device) {
  int cur = 0;
  HIP_OK(hipGetDevice(&cur));
  if (src_dev_ != dst_dev_) {
    // the receiver's copy reads the sender's HBM directly (xGMI peer read, one hop)
    (void)hipSetDevice(src_dev_);
    (void)hipDeviceEnablePeerAccess(dst_dev_, 0);
    (void)hipGetLastError();
    (void)hipSetDevice(dst_dev_);
    (void)hipDeviceEnablePeerAccess(src_dev_, 0);
    (void)hipGetLastError();
  }
  HIP_OK(hipSetDevice(src_dev_));
  for (auto& e : ready_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipSetDevice(dst_dev_));
  for (auto& e : done_) HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_OK(hipSetDevice(cur));
}

LocalLink::~LocalLink() {
  for (auto e : ready_) (void)hipEventDestroy(e);
  for (auto e : done_) (void)hipEventDestroy(e);
}

void LocalLink::abort() {
  std::lock_guard<std::mutex> l(mu_);
  aborted_ = true;
  cv_.notify_all();
}

void LocalLink::send(const void* buf, size_t bytes, hipStream_t st) {
  const auto to = std::chrono::milliseconds((long)(timeout_s * 1000));
  std::unique_lock<std::mutex> l(mu_);
  if (!cv_.wait_for(l, to, [&] { return aborted_ || posted_ - taken_ < (uint64_t)kDepth; }))
    throw std::runtime_error("LocalLink: send timed out (receiver stalled, queue full)");
  if (aborted_) throw std::runtime_error("LocalLink: aborted");
  const int slot = (int)(posted_ % kDepth);   // its previous message was taken: its events are free
  HIP_OK(hipEventRecord(ready_[slot], st));
  src_[slot] = buf;
  bytes_[slot] = bytes;
  ++posted_;
  cv_.notify_all();
  bytes_sent += bytes;
  ++msgs_sent;
}

void LocalLink::wait_consumed(uint64_t seq, hipStream_t st) {
  if (seq == 0) return;
  std::unique_lock<std::mutex> l(mu_);
  if (!cv_.wait_for(l, std::chrono::milliseconds((long)(timeout_s * 1000)), [&] { return aborted_ || taken_ >= seq; }))
    throw std::runtime_error("LocalLink: buffer reuse timed out (receiver stalled)");
  if (aborted_) throw std::runtime_error("LocalLink: aborted");
  HIP_OK(hipStreamWaitEvent(st, done_[(seq - 1) % kDepth], 0));
}

void LocalLink::recv(void* buf, size_t bytes, hipStream_t st) {
  std::unique_lock<std::mutex> l(mu_);
  if (!cv_.wait_for(l, std::chrono::milliseconds((long)(timeout_s * 1000)),
                    [&] { return aborted_ || posted_ > taken_; }))
    throw std::runtime_error("LocalLink: recv timed out (peer stalled)");
  if (aborted_) throw std::runtime_error("LocalLink: aborted");
  const int slot = (int)(taken_ % kDepth);
  if (bytes_[slot] != bytes) throw std::runtime_error("LocalLink: message size mismatch");
  HIP_OK(hipStreamWaitEvent(st, ready_[slot], 0));
  HIP_OK(hipMemcpyAsync(buf, src_[slot], bytes, hipMemcpyDefault, st));
  HIP_OK(hipEventRecord(done_[slot], st));
  ++taken_;
  cv_.notify_all();
}

// ---------------------------------------------------------------- RCCL
RcclLink::RcclLink(void* comm, int my_rank, int peer, int device, bool owns_comm)
    : comm_(comm), rank_(my_rank), peer_(peer), dev_(device), owns_(owns_comm) {}
RcclLink::~RcclLink() {
  if (comm_ && owns_) ncclCommDestroy((ncclComm_t)comm_);
}
void RcclLink::abort() {
  if (comm_ && owns_) ncclCommAbort((ncclComm_t)comm_);
  comm_ = nullptr;
}
int RcclLink::comm_nranks() const {
  int n = 0;
  if (comm_ && ncclCommCount((ncclComm_t)comm_, &n) != ncclSuccess) n = -1;
  return n;
}
void RcclLink::send(const void* buf, size_t bytes, hipStream_t st) {
  if (!comm_) throw std::runtime_error("RcclLink: aborted");
  NCCL_OK(ncclSend(buf, bytes, ncclUint8, peer_, (ncclComm_t)comm_, st));
  bytes_sent += bytes;
  ++msgs_sent;
}
void RcclLink::recv(void* buf, size_t bytes, hipStream_t st) {
  if (!comm_) throw std::runtime_error("RcclLink: aborted");
  NCCL_OK(ncclRecv(buf, bytes, ncclUint8, peer_, (ncclComm_t)comm_, st));
}

bool rccl_init_all(const std::vector<int>& devices, std::vector<void*>* comms, std::string* err) {
  std::vector<ncclComm_t> c(devices.size());
  std::vector<int> devs(devices);
  const ncclResult_t r = ncclCommInitAll(c.data(), (int)devs.size(), devs.data());
  if (r != ncclSuccess) {
    if (err) *err = ncclGetErrorString(r);
    return false;
  }
  comms->assign(c.begin(), c.end());
  return true;
}

void rccl_make_pair(int dev_a, int dev_b, void** comm_a, void** comm_b) {
  std::vector<void*> c;
  std::string err;
  if (!rccl_init_all({dev_a, dev_b}, &c, &err)) throw std::runtime_error("RCCL error: " + err);
  *comm_a = c[0];
  *comm_b = c[1];
}

void* rccl_init_rank(const uint8_t* id128, int nranks, int rank, int device) {
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::runtime_error("rccl_init_rank: bad rank / nranks");
  ncclUniqueId id;
  std::memcpy(&id, id128, 128);
  HIP_OK(hipSetDevice(device));
  ncclComm_t c;
  NCCL_OK(ncclCommInitRank(&c, nranks, id, rank));
  return c;
}

int rccl_unique_id(uint8_t* out128) {
  ncclUniqueId id;
  NCCL_OK(ncclGetUniqueId(&id));
  std::memcpy(out128, &id, 128);
  return 0;
}

void rccl_group_begin() { NCCL_OK(ncclGroupStart()); }
void rccl_group_end() { NCCL_OK(ncclGroupEnd()); }
void rccl_comm_destroy(void* comm) {
  if (comm) ncclCommDestroy((ncclComm_t)comm);
}
const char* rccl_version_string() {
  static char buf[32];
  int v = 0;
  ncclGetVersion(&v);
  snprintf(buf, sizeof buf, "%d.%d.%d", v / 10000, (v / 100) % 100, v % 100);
  return buf;
}

// ---------------------------------------------------------------- TCP
static void full_write(int fd, const void* p, size_t n) {
  const char* c = (const char*)p;
  while (n) {
    ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
    if (w <= 0) throw std::runtime_error("TcpLink: send failed");
    c += w;
    n -= (size_t)w;
  }
}
static void full_read(int fd, void* p, size_t n) {
  char* c = (char*)p;
  while (n) {
    ssize_t r = ::recv(fd, c, n, 0);
    if (r <= 0) throw std::runtime_error("TcpLink: peer closed");
    c += r;
    n -= (size_t)r;
  }
}
static void tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 16 << 20;   // PDF p.4-5 sysctl advice, applied per socket
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

std::unique_ptr<TcpLink> TcpLink::make_sender(const std::string& host, int port, double timeout_s) {
  auto l = std::unique_ptr<TcpLink>(new TcpLink());
  const auto t0 = std::chrono::steady_clock::now();
  while (true) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    if (getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0 && res) {
      int fd = socket(res->ai_family, res->ai_socktype, 0);
      if (fd >= 0 && connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
        freeaddrinfo(res);
        tune(fd);
        l->fd_ = fd;
        return l;
      }
      if (fd >= 0) ::close(fd);
      freeaddrinfo(res);
    }
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
      throw std::runtime_error("TcpLink: connect timeout to " + host + ":" + std::to_string(port));
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
}

std::unique_ptr<TcpLink> TcpLink::make_receiver(int port, double timeout_s) {
  auto l = std::unique_ptr<TcpLink>(new TcpLink());
  int ls = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons((uint16_t)port);
  if (bind(ls, (sockaddr*)&a, sizeof(a)) != 0 || listen(ls, 1) != 0) {
    ::close(ls);
    throw std::runtime_error("TcpLink: cannot listen on port " + std::to_string(port));
  }
  timeval tv{(long)timeout_s, 0};
  setsockopt(ls, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  int fd = accept(ls, nullptr, nullptr);
  ::close(ls);
  if (fd < 0) throw std::runtime_error("TcpLink: accept timeout");
  tune(fd);
  l->fd_ = fd;
  return l;
}

TcpLink::~TcpLink() {
  if (fd_ >= 0) ::close(fd_);
}
void TcpLink::abort() {
  if (fd_ >= 0) { shutdown(fd_, SHUT_RDWR); }
}

void TcpLink::set_timeout(double s) {
  timeout_s = s;
  timeval tv{(long)s, (long)((s - (long)s) * 1e6)};
  setsockopt(fd_, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd_, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
}

void TcpLink::send(const void* buf, size_t bytes, hipStream_t st) {
  const void* src = buf;
  if (st) {
    staging_.resize(bytes);
    HIP_OK(hipMemcpyAsync(staging_.data(), buf, bytes, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
    src = staging_.data();
  }
  const uint64_t n = bytes;
  full_write(fd_, &n, 8);
  full_write(fd_, src, bytes);
  bytes_sent += bytes;
  ++msgs_sent;
}

void TcpLink::recv(void* buf, size_t bytes, hipStream_t st) {
  uint64_t n = 0;
  full_read(fd_, &n, 8);
  if (n != bytes) throw std::runtime_error("TcpLink: message size mismatch");
  if (st) {
    staging_.resize(bytes);
    full_read(fd_, staging_.data(), bytes);
    HIP_OK(hipMemcpyAsync(buf, staging_.data(), bytes, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
  } else {
    full_read(fd_, buf, bytes);
  }
}

}  // namespace mp

namespace mp {

// ---------------------------------------------------------------- HostLink
// A stream means a GPU end (the hybrid CPU/GPU split): buf is device memory, copied through the
// host message on that stream (blocking the caller's host thread, like a CPU stage's transfers).
void HostLink::send(const void* buf, size_t bytes, hipStream_t st) {
  std::vector<uint8_t> m;
  if (st) {
    m.resize(bytes);
    HIP_OK(hipMemcpyAsync(m.data(), buf, bytes, hipMemcpyDeviceToHost, st));
    HIP_OK(hipStreamSynchronize(st));
  } else {
    m.assign((const uint8_t*)buf, (const uint8_t*)buf + bytes);
  }
  std::unique_lock<std::mutex> l(mu_);
  if (!cv_.wait_for(l, std::chrono::milliseconds((long)(timeout_s * 1000)), [&] { return aborted_ || q_.size() < max_q_; }))
    throw std::runtime_error("HostLink: send timed out (peer stalled)");
  if (aborted_) throw std::runtime_error("HostLink: aborted");
  q_.push_back(std::move(m));
  bytes_sent += bytes;
  ++msgs_sent;
  cv_.notify_all();
}

void HostLink::recv(void* buf, size_t bytes, hipStream_t st) {
  std::vector<uint8_t> m;
  {
    std::unique_lock<std::mutex> l(mu_);
    if (!cv_.wait_for(l, std::chrono::milliseconds((long)(timeout_s * 1000)), [&] { return aborted_ || !q_.empty(); }))
      throw std::runtime_error("HostLink: recv timed out (peer stalled)");
    if (aborted_) throw std::runtime_error("HostLink: aborted");
    if (q_.front().size() != bytes) throw std::runtime_error("HostLink: message size mismatch");
    m = std::move(q_.front());
    q_.pop_front();
    cv_.notify_all();
  }
  if (st) {
    HIP_OK(hipMemcpyAsync(buf, m.data(), bytes, hipMemcpyHostToDevice, st));
    HIP_OK(hipStreamSynchronize(st));
  } else {
    std::memcpy(buf, m.data(), bytes);
  }
}

void HostLink::abort() {
  std::lock_guard<std::mutex> l(mu_);
  aborted_ = true;
  cv_.notify_all();
}

}  // namespace mp
