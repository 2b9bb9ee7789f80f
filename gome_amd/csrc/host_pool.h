// host_pool.h — one process-wide pool of host worker threads for the consumer's native work
// (consume.cpp: the OrderNode decode; host.cpp: the MatchResult render).  The batching consumer
// calls these once per drained batch (~32k messages at a few million messages/s: a batch every few
// milliseconds), and starting 8-16 std::threads per call cost more than some of the work they did.
// run(n, fn) runs fn(0) .. fn(n - 1) on the caller and the pool's workers and returns when all are
// done; callers from several threads take turns (one job at a time).  Workers are started on first
// use, up to the largest n asked for (at most MAX_WORKERS + the caller).
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace gome_host {

class Pool {
 public:
  static constexpr uint32_t MAX_WORKERS = 63;

  // Two pools: 0 for the decode and admission (consume.cpp), 1 for the render (host.cpp), so a
  // consumer can render batch k while it decodes batch k + 1 (BatchingConsumer.process_stream).
  static Pool& get(int which = 0) {
    static Pool p[2];  // (joined at exit: the destructors stop the workers)
    return p[which & 1];
  }

  void run(uint32_t n, const std::function<void(uint32_t)>& fn) {
    if (n == 0) return;
    if (n == 1) {
      fn(0);
      return;
    }
    std::lock_guard<std::mutex> one(job_mu_);  // (one job at a time)
    {
      std::unique_lock<std::mutex> lk(mu_);
      const uint32_t want = std::min<uint32_t>(n - 1, MAX_WORKERS);
      while (workers_.size() < want) workers_.emplace_back([this] { loop(); });
      fn_ = &fn;
      n_ = n;
      next_.store(0, std::memory_order_relaxed);
      done_ = 0;
      ++gen_;
    }
    cv_.notify_all();
    const uint32_t mine = drain();
    std::unique_lock<std::mutex> lk(mu_);
    done_ += mine;
    done_cv_.wait(lk, [&] { return done_ == n_; });
    fn_ = nullptr;
  }

  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  Pool() = default;

  // claim tasks of the current job until none is left; the number run
  uint32_t drain() {
    uint32_t c = 0;
    for (;;) {
      const uint32_t k = next_.fetch_add(1, std::memory_order_relaxed);
      if (k >= n_) return c;
      (*fn_)(k);
      ++c;
    }
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        if (!fn_) continue;
      }
      const uint32_t c = drain();
      if (c) {
        std::lock_guard<std::mutex> lk(mu_);
        done_ += c;
        if (done_ == n_) done_cv_.notify_all();
      }
    }
  }

  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const std::function<void(uint32_t)>* fn_ = nullptr;
  uint32_t n_ = 0, done_ = 0;
  std::atomic<uint32_t> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace gome_host
