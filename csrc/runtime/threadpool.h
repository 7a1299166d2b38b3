// Persistent fork-join pool for the CPU backend: parallel_for(n, fn(begin, end)) splits [0, n) into
// one contiguous range per worker; the caller thread runs range 0.
//
// A decode step calls parallel_for ~8 times per layer with 30-300 us of work each, so the hand-off
// itself has to cost microseconds: the job is published through an atomic generation counter that
// idle workers spin on (with a pause) for a while before they sleep on the condition variable, and
// the caller spins on an atomic countdown.  (With a mutex + condition variable per call, a worker
// wake-up in this VM cost up to milliseconds: TinyLlama Q4_K_M decoded SLOWER on 8 threads than on
// one, 263 vs 193 ms per token.)
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#define MP_CPU_RELAX() _mm_pause()
#else
#define MP_CPU_RELAX() std::this_thread::yield()
#endif

namespace mp {

class ThreadPool {
 public:
  explicit ThreadPool(int n_threads) {
    n_ = std::max(1, std::min(n_threads, 255));
    for (int i = 1; i < n_; ++i) th_.emplace_back([this, i] { worker(i); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_.store(true);
      gen_.store(((gen_.load() >> 8) + 1) << 8);   // part count 0: nobody runs anything
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return n_; }

  void parallel_for(int64_t n, const std::function<void(int64_t, int64_t)>& fn, int64_t min_chunk = 1) {
    const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(n_, (n + min_chunk - 1) / std::max<int64_t>(1, min_chunk)));
    if (parts <= 1) {
      if (n > 0) fn(0, n);
      return;
    }
    fn_ = &fn;
    total_ = n;
    parts_ = parts;
    pending_.store(parts - 1, std::memory_order_relaxed);
    {
      // the generation word carries the job's part count (low 8 bits), so a worker that reads it
      // late -- after a job it takes no part in -- never acts on the next job's parameters (a
      // participant of job g holds the caller inside g until it counts down).  Bumped under the
      // mutex: a worker about to sleep re-checks it under the same mutex before waiting.
      std::lock_guard<std::mutex> g(mu_);
      gen_.store(((gen_.load(std::memory_order_relaxed) >> 8) + 1) << 8 | (uint64_t)parts, std::memory_order_release);
    }
    if (sleepers_.load(std::memory_order_acquire) > 0) cv_.notify_all();
    run_part(0);
    // spin for the stragglers, yielding once the wait gets long: on an oversubscribed host (several
    // engines, or test workers, sharing the cores) a pure spin starves the very workers it waits for
    for (int spins = 0; pending_.load(std::memory_order_acquire) != 0;) {
      if (++spins < 4096) MP_CPU_RELAX();
      else std::this_thread::yield();
    }
    fn_ = nullptr;
  }

 private:
  void run_part(int i) {
    const int64_t b = total_ * i / parts_, e = total_ * (i + 1) / parts_;
    if (b < e) (*fn_)(b, e);
  }
  void worker(int i) {
    uint64_t seen = 0;
    for (;;) {
      // spin ~2 ms for the next job, then sleep
      const auto t0 = std::chrono::steady_clock::now();
      int spins = 0;
      while (gen_.load(std::memory_order_acquire) == seen) {
        MP_CPU_RELAX();
        if (++spins == 1024) {
          spins = 0;
          if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
            std::unique_lock<std::mutex> lk(mu_);
            sleepers_.fetch_add(1);
            cv_.wait(lk, [&] { return gen_.load() != seen; });
            sleepers_.fetch_sub(1);
            break;
          }
          std::this_thread::yield();   // let a descheduled caller or sibling run (oversubscribed host)
        }
      }
      seen = gen_.load(std::memory_order_acquire);
      if (stop_.load()) return;
      if (i < (int)(seen & 0xFF)) {
        run_part(i);
        pending_.fetch_sub(1, std::memory_order_acq_rel);
      }
    }
  }

  int n_ = 1;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_;
  const std::function<void(int64_t, int64_t)>* fn_ = nullptr;
  int64_t total_ = 0;
  int parts_ = 0;
  std::atomic<int> pending_{0}, sleepers_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
};

}  // namespace mp
