#include "host/thread_pool.h"

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <mutex>
#include <thread>
#include <vector>

namespace gz {

namespace {

class Pool {
 public:
  explicit Pool(int workers) {
    for (int i = 0; i < workers; ++i) threads_.emplace_back([this] { Loop(); });
  }
  // Leaked at exit on purpose (workers may still be parked in wait()).

  // False (nothing run) if another caller holds the pool.
  bool TryRun(int n, const std::function<void(int)>& fn) {
    std::unique_lock<std::mutex> serial(run_mu_, std::try_to_lock);
    if (!serial.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      active_ = static_cast<int>(threads_.size());
      ++generation_;
    }
    cv_.notify_all();
    Work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return active_ == 0; });
    fn_ = nullptr;
    return true;
  }

 private:
  void Work() {
    for (;;) {
      const int i = next_.fetch_add(1);
      if (i >= n_) break;
      (*fn_)(i);
    }
  }
  void Loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return generation_ != seen; });
        seen = generation_;
      }
      Work();
      std::lock_guard<std::mutex> lk(mu_);
      if (--active_ == 0) done_cv_.notify_one();
    }
  }

  std::vector<std::thread> threads_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0;
  std::atomic<int> next_{0};
  int active_ = 0;
  uint64_t generation_ = 0;
};

Pool* GetPool() {
  static Pool* pool = new Pool(HostThreads() - 1);
  return pool;
}

}  // namespace

int HostThreads() {
  static const int n = [] {
    const char* e = std::getenv("GZ_HOST_THREADS");
    if (e && std::atoi(e) > 0) return std::min(256, std::atoi(e));
    const int hw = static_cast<int>(std::thread::hardware_concurrency());
    return std::max(1, std::min(16, hw));
  }();
  return n;
}

void ParallelFor(int n, const std::function<void(int)>& fn) {
  if (n <= 0) return;
  if (n == 1 || HostThreads() == 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  // Concurrent encodes (several frames per GPU) each run their passes inline
  // when another one holds the pool, instead of queueing behind it.
  if (!GetPool()->TryRun(n, fn))
    for (int i = 0; i < n; ++i) fn(i);
}

}  // namespace gz
