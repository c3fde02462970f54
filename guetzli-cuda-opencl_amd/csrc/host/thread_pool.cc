#include "host/thread_pool.h"

#include <algorithm>
#include <atomic>
#include <pthread.h>

#include <condition_variable>
#include <cstdlib>
#include <list>
#include <mutex>
#include <thread>
#include <vector>

namespace gz {

namespace {

// Several encodes (frames) run concurrently per process, each issuing its
// own data-parallel passes: every ParallelFor is a job on a shared list and
// idle workers take items from the oldest job that has some left, so
// concurrent callers share the workers instead of queueing behind each
// other.  The caller works on its own job too and returns when all its
// items are done.
struct Job {
  const std::function<void(int)>* fn;
  int n;
  std::atomic<int> next{0};
  std::atomic<int> done{0};
};

class Pool {
 public:
  explicit Pool(int workers) {
    for (int i = 0; i < workers; ++i) threads_.emplace_back([this] { Loop(); });
  }
  // Leaked at exit on purpose (workers may still be parked in wait()).

  void Run(int n, const std::function<void(int)>& fn) {
    Job job;
    job.fn = &fn;
    job.n = n;
    std::list<Job*>::iterator it;
    {
      std::lock_guard<std::mutex> lk(mu_);
      it = jobs_.insert(jobs_.end(), &job);
    }
    cv_.notify_all();
    Work(&job);
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.erase(it);  // no worker can pick it up any more
    }
    // items claimed by workers may still be running
    std::unique_lock<std::mutex> lk(done_mu_);
    done_cv_.wait(lk, [&] { return job.done.load() == n; });
  }

 private:
  // Runs claimed item i of `job` and then further items until none is left.
  // The next item is claimed BEFORE the current one is counted as done: the
  // owner (who waits for done == n) keeps the job alive while this thread
  // holds an uncounted item, and the job is not touched after the last count.
  void Drain(Job* job, int i) {
    const int n = job->n;
    const std::function<void(int)>* fn = job->fn;
    while (i < n) {
      (*fn)(i);
      const int next = job->next.fetch_add(1);
      if (job->done.fetch_add(1) + 1 == n) {
        std::lock_guard<std::mutex> lk(done_mu_);
        done_cv_.notify_all();
      }
      i = next;
    }
  }
  void Work(Job* job) { Drain(job, job->next.fetch_add(1)); }

  void Loop() {
    pthread_setname_np(pthread_self(), "gz_pool");  // per-thread CPU accounting
    for (;;) {
      Job* job = nullptr;
      int i;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          for (Job* j : jobs_)
            if (j->next.load() < j->n) {
              job = j;
              return true;
            }
          return false;
        });
        // claimed under mu_: the owner erases the job under mu_ first
        i = job->next.fetch_add(1);
        if (i >= job->n) continue;
      }
      Drain(job, i);
    }
  }

  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::list<Job*> jobs_;
  std::mutex done_mu_;
  std::condition_variable done_cv_;
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
  GetPool()->Run(n, fn);
}

}  // namespace gz
