// Host pool stress: concurrent and nested ParallelFor calls from 8 threads;
// every item must run exactly once.
#include <atomic>
#include <cstdio>
#include <thread>
#include <cstdlib>
#include <vector>
#include "host/thread_pool.h"
int main() {
  std::atomic<long> total{0};
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t) th.emplace_back([&, t] {
    for (int r = 0; r < 2000; ++r) {
      std::vector<int> hit(37 + (r % 50), 0);
      gz::ParallelFor(static_cast<int>(hit.size()), [&](int i) { hit[i]++; if (i % 7 == 0) gz::ParallelFor(3, [&](int) { total++; }); });
      for (int v : hit) if (v != 1) { printf("BAD\n"); exit(1); }
      total += hit.size();
    }
  });
  for (auto& x : th) x.join();
  printf("ok %ld\n", total.load());
}
