// Persistent worker pool for the host runtime (request scanning, host-side
// conversion). Threads are created once; parallel_for() hands out task
// indices through an atomic counter and blocks until every task finished.
// Idle workers spin briefly (~kSpinIters pause loops, a few hundred us)
// before sleeping on the condition variable: the train path calls
// parallel_for every millisecond or so, and a futex wake-up per worker per
// call would add tens of microseconds to every batch.
#pragma once
#include <atomic>
#include <immintrin.h>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace jb {

class WorkerPool {
 public:
  explicit WorkerPool(int n) {
    if (n < 1) n = 1;
    for (int i = 0; i < n - 1; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~WorkerPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : threads_) t.join();
  }
  int size() const { return (int)threads_.size() + 1; }

  // run fn(i) for i in [0, n); the caller participates. Not reentrant.
  void parallel_for(int64_t n, const std::function<void(int64_t)>& fn) {
    std::lock_guard<std::mutex> call(call_mu_);
    if (n <= 0) return;
    if (threads_.empty() || n == 1) {
      for (int64_t i = 0; i < n; ++i) fn(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      pending_.store((int)threads_.size());
      ++gen_;
    }
    cv_.notify_all();
    work();
    // wait for the workers to leave this generation
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [this] { return pending_.load() == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      int64_t i = next_.fetch_add(1);
      if (i >= n_) break;
      (*fn_)(i);
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      for (int i = 0; i < kSpinIters && gen_.load(std::memory_order_acquire) == seen; ++i)
        _mm_pause();
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_.load() != seen; });
        seen = gen_.load();
        if (stop_) return;
      }
      work();
      if (pending_.fetch_sub(1) == 1) {
        std::lock_guard<std::mutex> g(mu_);
        done_cv_.notify_all();
      }
    }
  }

  std::vector<std::thread> threads_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t)>* fn_ = nullptr;
  int64_t n_ = 0;
  std::atomic<int64_t> next_{0};
  std::atomic<int> pending_{0};
  static constexpr int kSpinIters = 20000;
  std::atomic<uint64_t> gen_{0};
  bool stop_ = false;
};

// process-wide pool, sized on first use
WorkerPool& global_pool(int nthreads);

}  // namespace jb
