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
  // blocking waits give up after this long (a dead or stalled peer surfaces as an error)
  virtual void set_timeout(double s) { timeout_s = s; }
  double timeout_s = 600;
  uint64_t bytes_sent = 0, msgs_sent = 0;
};

// ---------------------------------------------------------------- LocalLink
// A rendezvous: send() publishes (buffer, ready event) and blocks the sending HOST thread until
// the receiver has enqueued its copy; it then makes the sender's stream wait for that copy, so
// the engine's sent_ev (recorded after send) keeps the buffer alive exactly as long as needed.
// Host threads only meet at enqueue points (the GPU work stays asynchronous), and every stage
// issues its link operations in the global (round, micro-batch) order, so the ring cannot
// deadlock on the rendezvous.  Both ends may be on the same device.
class LocalLink : public Link {
 public:
  LocalLink(int src_device, int dst_device);
  ~LocalLink() override;
  void send(const void* buf, size_t bytes, hipStream_t st) override;
  void recv(void* buf, size_t bytes, hipStream_t st) override;
  const char* kind() const override { return "local"; }
  void abort() override;
  bool peer() const { return src_dev_ != dst_dev_; }

 private:
  int src_dev_, dst_dev_;
  hipEvent_t ready_ = nullptr;   // on the sender's device: the message's bytes are final
  hipEvent_t done_ = nullptr;    // on the receiver's device: the copy has completed
  const void* src_ = nullptr;
  size_t bytes_ = 0;
  uint64_t posted_ = 0, taken_ = 0;   // message counters (posted_ - taken_ <= 1)
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
