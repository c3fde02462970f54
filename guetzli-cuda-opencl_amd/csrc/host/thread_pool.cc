#include "host/thread_pool.h"

#include <sched.h>

#include <pthread.h>
#include <stdio.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <list>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

namespace gz {

namespace {

std::atomic<int> g_active_encodes{0};

// Workers that may run items at once: the CPUs not taken by the encodes'
// own threads (at least one).
int WorkerCap() {
  return std::max(1, HostThreads() - std::max(1, g_active_encodes.load(std::memory_order_relaxed)));
}

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
  // the owner's wait: per job, so a finishing job wakes its owner only (not
  // every other frame's caller)
  std::mutex done_mu;
  std::condition_variable done_cv;
  bool finished = false;  // set under done_mu by the last item's thread
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
    int wake;
    {
      std::lock_guard<std::mutex> lk(mu_);
      it = jobs_.insert(jobs_.end(), &job);
      // wake as many workers as there are items for them (the caller takes
      // one), and no more than are asleep and not already being woken: with
      // several frames in flight most workers are busy on other frames'
      // jobs and take this one's items when they finish theirs, so waking
      // more only costs futex calls and futile wake-ups (the pool's system
      // time)
      wake = std::max(0, std::min(std::min(n - 1, idle_ - signaled_), WorkerCap() - busy_ - signaled_));
      signaled_ += wake;
    }
    for (int i = 0; i < wake; ++i) cv_.notify_one();
    Work(&job);
    {
      std::lock_guard<std::mutex> lk(mu_);
      jobs_.erase(it);  // no worker can pick it up any more
    }
    // items claimed by workers may still be running
    std::unique_lock<std::mutex> lk(job.done_mu);
    job.done_cv.wait(lk, [&] { return job.finished; });
  }

 private:
  // Runs claimed item i of `job` and then further items until none is left.
  // The next item is claimed BEFORE the current one is counted as done: the
  // owner (who waits for the last count) keeps the job alive while this thread
  // holds an uncounted item, and the job is not touched after the last count.
  void Drain(Job* job, int i) {
    const int n = job->n;
    const std::function<void(int)>* fn = job->fn;
    while (i < n) {
      (*fn)(i);
      const int next = job->next.fetch_add(1);
      if (job->done.fetch_add(1) + 1 == n) {
        // (the owner returns -- and destroys the job -- only after seeing
        // `finished` under the job's mutex, i.e. after this thread's last
        // touch of the job, the unlock)
        std::lock_guard<std::mutex> lk(job->done_mu);
        job->finished = true;
        job->done_cv.notify_one();
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
        for (;;) {
          if (busy_ < WorkerCap())
            for (Job* j : jobs_)
              if (j->next.load() < j->n) {
                job = j;
                break;
              }
          if (job) break;
          ++idle_;
          cv_.wait(lk);
          --idle_;
          if (signaled_ > 0) --signaled_;  // (a spurious wake-up may take another's: harmless)
        }
        // claimed under mu_: the owner erases the job under mu_ first
        i = job->next.fetch_add(1);
        if (i >= job->n) continue;
        ++busy_;
      }
      Drain(job, i);
      std::lock_guard<std::mutex> lk(mu_);
      --busy_;
    }
  }

  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::list<Job*> jobs_;
  int idle_ = 0;      // workers waiting on cv_ (under mu_)
  int busy_ = 0;      // workers running items (under mu_)
  int signaled_ = 0;  // of those, already notified and not yet awake
};

Pool* GetPool() {
  static Pool* pool = new Pool(HostThreads() - 1);
  return pool;
}

}  // namespace

namespace {
// CPUs this process may use: its affinity set (sched_getaffinity), capped by
// a cgroup v2 CPU quota (cpu.max "quota period"; a container's CPU share is
// often a quota, not an affinity mask).  *affinity: the affinity set's size,
// *online: the online CPUs.
int UsableCpus(int* affinity, int* online) {
  *online = std::max(1, static_cast<int>(std::thread::hardware_concurrency()));
  int n = *online;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0 && CPU_COUNT(&set) > 0) n = CPU_COUNT(&set);
  *affinity = n;
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char quota[32] = {0};
    long period = 0;
    if (fscanf(f, "%31s %ld", quota, &period) == 2 && period > 0 && std::strcmp(quota, "max") != 0) {
      const long q = std::atol(quota);
      if (q > 0) n = std::min<long>(n, std::max<long>(1, (q + period - 1) / period));
    }
    fclose(f);
  }
  return std::max(1, n);
}
}  // namespace

int ActiveEncodes() { return g_active_encodes.load(std::memory_order_relaxed); }
int PoolWorkerCap() { return WorkerCap(); }

ActiveEncode::ActiveEncode() { g_active_encodes.fetch_add(1, std::memory_order_relaxed); }
ActiveEncode::~ActiveEncode() { g_active_encodes.fetch_sub(1, std::memory_order_relaxed); }

int HostThreads() {
  static const int n = [] {
    const char* e = std::getenv("GZ_HOST_THREADS");
    if (e && std::atoi(e) > 0) return std::min(256, std::atoi(e));
    // the usable CPUs shared by the ranks on the node (torch.distributed.run
    // sets LOCAL_WORLD_SIZE), at most 16 per process -- unless this rank's
    // affinity set is already no larger than its share of the online CPUs
    // (a launcher pinned each rank to its own cpuset).  A container's cpuset
    // smaller than the host is not a per-rank pinning: the ranks share it.
    int affinity = 0, online = 0;
    int share = UsableCpus(&affinity, &online);
    const char* lw = std::getenv("LOCAL_WORLD_SIZE");
    const int local = lw ? std::max(1, std::atoi(lw)) : 1;
    const bool pinned = local > 1 && affinity <= online / local;
    if (!pinned && local > 1) share /= local;
    return std::max(1, std::min(16, share));
  }();
  return n;
}

namespace {
// GZ_POOL_PROFILE=1: CPU seconds of the items of every ParallelFor call
// site (all threads), printed to stderr at exit -- where the host cores go.
double ThreadCpuSeconds() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return static_cast<double>(ts.tv_sec) + 1e-9 * static_cast<double>(ts.tv_nsec);
}
struct SiteStats {
  double cpu = 0.0;
  long calls = 0, items = 0;
};
std::mutex g_prof_mu;
std::map<std::pair<const char*, int>, SiteStats>* g_prof = nullptr;
bool PoolProfiling() {
  static const bool on = [] {
    const char* e = std::getenv("GZ_POOL_PROFILE");
    if (!(e && std::atoi(e) > 0)) return false;
    g_prof = new std::map<std::pair<const char*, int>, SiteStats>();
    std::atexit([] {
      std::lock_guard<std::mutex> lk(g_prof_mu);
      for (const auto& kv : *g_prof)
        fprintf(stderr, "pool site %s:%d calls %ld items %ld cpu %.4f s\n", kv.first.first,
                kv.first.second, kv.second.calls, kv.second.items, kv.second.cpu);
    });
    return true;
  }();
  return on;
}
}  // namespace

void ParallelFor(int n, const std::function<void(int)>& fn, const char* file, int line) {
  if (n <= 0) return;
  if (PoolProfiling()) {
    std::atomic<long> ns{0};
    const std::function<void(int)> timed = [&](int i) {
      const double c0 = ThreadCpuSeconds();
      fn(i);
      ns += static_cast<long>(1e9 * (ThreadCpuSeconds() - c0));
    };
    if (n == 1 || HostThreads() == 1) {
      for (int i = 0; i < n; ++i) timed(i);
    } else {
      GetPool()->Run(n, timed);
    }
    std::lock_guard<std::mutex> lk(g_prof_mu);
    SiteStats& st = (*g_prof)[{file, line}];
    st.cpu += 1e-9 * static_cast<double>(ns.load());
    ++st.calls;
    st.items += n;
    return;
  }
  if (n == 1 || HostThreads() == 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  GetPool()->Run(n, fn);
}

}  // namespace gz
