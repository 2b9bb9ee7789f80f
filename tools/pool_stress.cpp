// Stress test of gome_amd/csrc/host_pool.h: 300k small jobs back to back (2..16 tasks each), every
// task counted once; a watchdog prints the pool's state and exits 3 if no job finishes for 2 s.  The
// first spinning version double-counted a task when a worker read the next job's task count beside
// the previous job's claim counter (it hung with done > n); the claim word now holds both.
//   g++ -O2 -std=c++17 -pthread tools/pool_stress.cpp -o /tmp/pool_stress && /tmp/pool_stress
//   (and with -fsanitize=thread: no report)
#define private public
#include "../gome_amd/csrc/host_pool.h"
#undef private
#include <cstdio>
#include <atomic>
#include <vector>
#include <memory>
#include <thread>
#include <chrono>
std::atomic<long> prog{0};
int main() {
  auto& p = gome_host::Pool::get(0);
  std::thread wd([&] {
    long last = -1;
    for (;;) {
      std::this_thread::sleep_for(std::chrono::seconds(2));
      long cur = prog.load();
      if (cur == last) {
        printf("STUCK at job %ld: gen %lu next %lx (tag %lu k %lu) n %u done %u sleepers %u workers %zu\n", cur, p.gen_.load(), p.next_.load(), p.next_.load() >> 32, p.next_.load() & 0xffffffff, p.n_.load(), p.done_.load(), p.sleepers_, p.workers_.size());
        fflush(stdout);
        _Exit(3);
      }
      last = cur;
    }
  });
  wd.detach();
  for (int j = 0; j < 300000; ++j) {
    const uint32_t n = 2 + (j % 15);
    std::unique_ptr<std::atomic<int>[]> hit(new std::atomic<int>[n]);
    for (uint32_t t = 0; t < n; ++t) hit[t] = 0;
    std::atomic<int>* h = hit.get();
    p.run(n, [h](uint32_t t) { h[t].fetch_add(1); });
    prog = j;
  }
  printf("ok\n");
  fflush(stdout);
  _Exit(0);
}
