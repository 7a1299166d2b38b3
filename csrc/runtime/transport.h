// Stage-to-stage transports (E8 of SURVEY.md §2.2): the reference ships activations between
// llama.cpp rpc-servers through the client over TCP (ggml-rpc, `main.rs:47-48`).  Here a Link is
// one DIRECTION between two stages; every op is stream-ordered (enqueued, not blocking the GPU
// of the caller), so comm overlaps the compute of other micro-batches.
//   - RcclLink:  ncclSend/ncclRecv on a 2-rank communicator per link (xGMI peer-to-peer).
//   - LocalLink: same-process hand-off, ONE device copy per message: the receiver's stream
//                copies straight out of the sender's buffer (peer read over xGMI when the two
//                stages sit on different GPUs; 1-GPU emulation of PP=S when they share one).
//   - TcpLink:   host sockets (cross-host parity with the reference's worker-over-TCP mode).
// One communicator per direction and one stream per side make every link FIFO-consistent, so
// the piped ring (activations forward, sampled tokens last -> first) is deadlock-free.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace mp {

class Link {
 public:
  virtual ~Link() = default;
  // host pointers allowed when stream == nullptr (CPU stages)
  virtual void send(const void* buf, size_t bytes, hipStream_t st) = 0;
  virtual void recv(void* buf, size_t bytes, hipStream_t st) = 0;
  virtual const char* kind() const = 0;
  // ranks of the communicator behind this link as the transport itself reports them (RCCL:
  // ncclCommCount); 0 for transports without one
  virtual int comm_nranks() const { return 0; }
  virtual void abort() {}
  // Buffer reuse for transports whose send() returns before the bytes have left the sender's buffer
  // (LocalLink's posted queue): last_seq() numbers the latest send; wait_consumed(seq, st) makes
  // stream st wait until message seq has been copied out, so st may overwrite its buffer.  For
  // stream-ordered transports (RCCL) and copying ones (TCP, host) the send stream's own order
  // already covers it: both are no-ops.
  virtual uint64_t last_seq() const { return 0; }
  virtual void wait_consumed(uint64_t seq, hipStream_t st) { (void)seq; (void)st; }
  // blocking waits give up after this long (a dead or stalled peer surfaces as an error)
  virtual void set_timeout(double s) { timeout_s = s; }
  double timeout_s = 600;
  uint64_t bytes_sent = 0, msgs_sent = 0;
};

// ---------------------------------------------------------------- LocalLink
// A posted queue of up to kDepth messages: send() records the message's ready event on the sender's
// stream, posts (buffer, bytes) and returns at once (it blocks only while kDepth messages are still
// untaken: back-pressure); recv() makes the receiver's stream wait for that ready event and copies
// straight out of the sender's buffer (ONE device copy, peer read over xGMI between GPUs), recording
// the message's done event.  The sender keeps its buffer until wait_consumed(seq, st) -- a host wait
// for the receiver to have enqueued message seq (normally long done: the engine reuses a micro-
// batch's buffer one round later) plus a stream wait on its done event.  Copies of one link run in
// order on the receiver's stream, so a done event re-recorded by a later message still covers the
// earlier copy.  Both ends may be on the same device (1-GPU rehearsal of PP = S).
class LocalLink : public Link {
 public:
  static constexpr int kDepth = 64;
  LocalLink(int src_device, int dst_device);
  ~LocalLink() override;
  void send(const void* buf, size_t bytes, hipStream_t st) override;
  void recv(void* buf, size_t bytes, hipStream_t st) override;
  const char* kind() const override { return "local"; }
  void abort() override;
  uint64_t last_seq() const override { return posted_; }
  void wait_consumed(uint64_t seq, hipStream_t st) override;
  bool peer() const { return src_dev_ != dst_dev_; }

 private:
  int src_dev_, dst_dev_;
  hipEvent_t ready_[kDepth] = {};   // sender's device: message bytes final
  hipEvent_t done_[kDepth] = {};    // receiver's device: message copied
  const void* src_[kDepth] = {};
  size_t bytes_[kDepth] = {};
  uint64_t posted_ = 0, taken_ = 0;   // message counters (1-based sequence numbers)
  std::mutex mu_;
  std::condition_variable cv_;
  bool aborted_ = false;
};

// ---------------------------------------------------------------- HostLink
// same-process hand-off between CPU stages (copying FIFO of host messages)
class HostLink : public Link {
 public:
  explicit HostLink(size_t max_queued = 64) : max_q_(max_queued) {}
  void send(const void* buf, size_t bytes, hipStream_t st) override;
  void recv(void* buf, size_t bytes, hipStream_t st) override;
  const char* kind() const override { return "host"; }
  void abort() override;

 private:
  std::deque<std::vector<uint8_t>> q_;
  size_t max_q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool aborted_ = false;
};

// ---------------------------------------------------------------- RcclLink
// One direction between this rank and `peer` of an RCCL communicator (ncclSend / ncclRecv on
// the caller's stream).  The communicator may be a 2-rank one per link (the default pipeline
// wiring: one FIFO per direction), or any larger communicator; peer == own rank is a self loop
// (ws = 1 tests), whose send and recv must be issued inside one rccl_group_begin/end pair.
class RcclLink : public Link {
 public:
  RcclLink(void* nccl_comm, int my_rank, int peer, int device, bool owns_comm = true);
  ~RcclLink() override;
  void send(const void* buf, size_t bytes, hipStream_t st) override;
  void recv(void* buf, size_t bytes, hipStream_t st) override;
  const char* kind() const override { return "rccl"; }
  int comm_nranks() const override;
  void abort() override;
  int rank() const { return rank_; }
  int peer() const { return peer_; }

 private:
  void* comm_;
  int rank_, peer_;
  [[maybe_unused]] int dev_;
  bool owns_;
};

// creates the communicator ends of `n` devices inside one process (ncclCommInitAll); returns false
// (and sets *err) when RCCL refuses the device list (e.g. the same GPU twice)
bool rccl_init_all(const std::vector<int>& devices, std::vector<void*>* comms, std::string* err);
// creates the two ends of a link between devices a -> b inside one process (ncclCommInitAll)
void rccl_make_pair(int dev_a, int dev_b, void** comm_a, void** comm_b);
// multi-process: init this rank's end of an `nranks` communicator from a 128-byte unique id
void* rccl_init_rank(const uint8_t* id128, int nranks, int rank, int device);
int rccl_unique_id(uint8_t* out128);
void rccl_group_begin();
void rccl_group_end();
void rccl_comm_destroy(void* comm);
const char* rccl_version_string();

// ---------------------------------------------------------------- TcpLink
class TcpLink : public Link {
 public:
  // sender connects to host:port; receiver listens on port (accepts one connection)
  static std::unique_ptr<TcpLink> make_sender(const std::string& host, int port, double timeout_s = 60);
  static std::unique_ptr<TcpLink> make_receiver(int port, double timeout_s = 60);
  ~TcpLink() override;
  void send(const void* buf, size_t bytes, hipStream_t st) override;
  void recv(void* buf, size_t bytes, hipStream_t st) override;
  const char* kind() const override { return "tcp"; }
  void abort() override;
  void set_timeout(double s) override;

 private:
  int fd_ = -1;
  std::vector<char> staging_;
};

}  // namespace mp
