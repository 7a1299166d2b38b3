// Minimal persistent fork-join pool for the CPU backend: parallel_for(n, fn(begin, end)) splits
// [0, n) into one contiguous range per worker; the caller thread runs range 0.
#pragma once
#include <algorithm>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mp {

class ThreadPool {
 public:
  explicit ThreadPool(int n_threads) {
    n_ = std::max(1, n_threads);
    for (int i = 1; i < n_; ++i) th_.emplace_back([this, i] { worker(i); });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      ++gen_;
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
    std::unique_lock<std::mutex> lk(mu_);
    fn_ = &fn;
    total_ = n;
    parts_ = parts;
    pending_ = parts - 1;
    ++gen_;
    lk.unlock();
    cv_.notify_all();
    run_part(0);
    lk.lock();
    done_cv_.wait(lk, [this] { return pending_ == 0; });
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
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return gen_ != seen; });
      seen = gen_;
      if (stop_) return;
      if (i >= parts_) continue;
      lk.unlock();
      run_part(i);
      lk.lock();
      if (--pending_ == 0) done_cv_.notify_one();
    }
  }

  int n_ = 1;
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t, int64_t)>* fn_ = nullptr;
  int64_t total_ = 0;
  int parts_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace mp
