// host_pool.h — one process-wide pool of host worker threads for the consumer's native work
// (consume.cpp: the OrderNode decode and the queue-order passes; host.cpp: the MatchResult render).
// The batching consumer calls these once per drained batch (~32k messages at a few million
// messages/s: a batch every few milliseconds), and starting 8-16 std::threads per call cost more
// than some of the work they did.  run(n, fn) runs fn(0) .. fn(n - 1) on the caller and the pool's
// workers and returns when all are done; callers from several threads take turns (one job at a
// time).  Workers are started on first use, up to the largest n asked for (at most MAX_WORKERS + the
// caller).
//
// A worker that finishes a job spins for the next one for a few tens of microseconds before it
// sleeps: gome_consume_order_nodes runs ~10 jobs back to back per batch, and waking sleeping
// threads through the condition variable cost ~0.2-0.3 ms a job on the GPU box's host (the symbol
// pass of a batch with no new symbol, nothing but that, measured 0.32 ms; gpurun_out/r06w).
#pragma once
#include <algorithm>
#include <atomic>
#include <chrono>
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
  static constexpr uint32_t MAX_TASKS = 0xFFFF;  // tasks of one job (the claim word's field)
  static constexpr int64_t SPIN_NS = 50000;  // a worker's spin for the next job, then it sleeps

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
    if (n > MAX_TASKS) {  // (a claim word holds 16-bit task indices: run larger jobs in rounds)
      for (uint32_t b = 0; b < n; b += MAX_TASKS) {
        const uint32_t m = std::min(MAX_TASKS, n - b);
        run(m, [&](uint32_t k) { fn(b + k); });
      }
      return;
    }
    std::lock_guard<std::mutex> one(job_mu_);  // (one job at a time)
    bool wake;
    {
      std::lock_guard<std::mutex> lk(mu_);
      const uint32_t want = std::min<uint32_t>(n - 1, MAX_WORKERS);
      while (workers_.size() < want) workers_.emplace_back([this] { loop(); });
      const uint64_t g = gen_.load(std::memory_order_relaxed) + 1;
      fn_.store(&fn, std::memory_order_relaxed);
      n_.store(n, std::memory_order_relaxed);
      done_.store(0, std::memory_order_relaxed);
      // (task claims carry the job's generation and task count: a claim checks both in one word)
      next_.store(g << 32 | static_cast<uint64_t>(n) << 16, std::memory_order_release);
      gen_.store(g, std::memory_order_release);  // (the job's fields visible with it)
      wake = sleepers_ > 0;
    }
    if (wake) cv_.notify_all();
    const uint32_t mine = drain(gen_.load(std::memory_order_relaxed));
    if (mine && done_.fetch_add(mine, std::memory_order_acq_rel) + mine == n) return;
    // the workers' share: spin a while, then sleep until the last of them reports
    const auto t0 = std::chrono::steady_clock::now();
    while (done_.load(std::memory_order_acquire) != n) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::nanoseconds(SPIN_NS)) {
        std::unique_lock<std::mutex> lk(mu_);
        done_cv_.wait(lk, [&] { return done_.load(std::memory_order_acquire) == n; });
        break;
      }
      std::this_thread::yield();
    }
  }

  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true, std::memory_order_release);
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  Pool() = default;

  // claim tasks of job g until none is left; the number run.  A claim is a compare-exchange on one
  // word holding the job's generation, its task count and the next task, so a worker that was
  // descheduled while the caller finished g and started g + 1 claims nothing (it would run g's
  // function, gone by then, or count a task of g + 1 twice).  The function is read after the claim:
  // job g cannot end while a claimed task of it has not run.
  uint32_t drain(uint64_t g) {
    uint32_t c = 0;
    uint64_t v = next_.load(std::memory_order_acquire);
    for (;;) {
      const uint32_t n = static_cast<uint32_t>(v >> 16) & 0xFFFFu, k = static_cast<uint32_t>(v) & 0xFFFFu;
      if ((v >> 32) != (g & 0xFFFFFFFFull) || k >= n) return c;
      if (!next_.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel, std::memory_order_acquire)) continue;
      (*fn_.load(std::memory_order_relaxed))(k);
      ++c;
      v = next_.load(std::memory_order_acquire);
    }
  }

  void loop() {
    uint64_t seen = gen_.load(std::memory_order_acquire);
    for (;;) {
      // the next job: spin for it a while, then sleep
      const auto t0 = std::chrono::steady_clock::now();
      while (gen_.load(std::memory_order_acquire) == seen &&
             std::chrono::steady_clock::now() - t0 < std::chrono::nanoseconds(SPIN_NS))
        std::this_thread::yield();
      if (gen_.load(std::memory_order_acquire) == seen) {
        std::unique_lock<std::mutex> lk(mu_);
        ++sleepers_;
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
        --sleepers_;
      }
      if (stop_.load(std::memory_order_acquire)) return;
      seen = gen_.load(std::memory_order_acquire);
      // (a job the caller finished alone leaves nothing to claim: drain returns 0)
      const uint32_t c = drain(seen);
      if (c && done_.fetch_add(c, std::memory_order_acq_rel) + c == n_.load(std::memory_order_relaxed)) {
        std::lock_guard<std::mutex> lk(mu_);
        done_cv_.notify_all();
      }
    }
  }

  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  std::atomic<const std::function<void(uint32_t)>*> fn_{nullptr};
  std::atomic<uint32_t> n_{0}, done_{0};
  std::atomic<uint64_t> next_{0};  // generation << 32 | tasks << 16 | the next task
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
  uint32_t sleepers_ = 0;  // (under mu_)
};

}  // namespace gome_host
