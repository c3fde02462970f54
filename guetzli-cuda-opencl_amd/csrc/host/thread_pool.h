// Host worker pool for the data-parallel host passes of the search loop
// (back-end bulk changes, change order, block weights, scan encoding).  One
// pool per process, shared by every concurrent encode.  HostThreads() is
// GZ_HOST_THREADS, else min(16, the usable CPUs -- affinity and cgroup
// quota -- divided by LOCAL_WORLD_SIZE ranks) -- 16 being the CPU share a
// GPU gets on the target nodes.  The pool has HostThreads() - 1 workers, of
// which at most HostThreads() - (encodes in progress) run items at once:
// every encode's own thread is a CPU user too, so with many frames in flight
// the pool yields to them instead of oversubscribing the CPUs.
#pragma once

#include <stddef.h>

#include <functional>

namespace gz {

int HostThreads();
// Encodes in progress in this process, and the pool workers that may run
// items at once (HostThreads() - encodes in progress, at least 1).
int ActiveEncodes();
int PoolWorkerCap();

// An encode in progress (ProcessJpegData): counted while the object lives.
class ActiveEncode {
 public:
  ActiveEncode();
  ~ActiveEncode();
  ActiveEncode(const ActiveEncode&) = delete;
  ActiveEncode& operator=(const ActiveEncode&) = delete;
};

// Runs fn(i) for i in [0, n) on the pool (the caller takes part) and returns
// when all are done.  Items are handed out dynamically; concurrent callers'
// jobs share the workers.
// (file / line: the call site, for GZ_POOL_PROFILE)
void ParallelFor(int n, const std::function<void(int)>& fn, const char* file = __builtin_FILE(),
                 int line = __builtin_LINE());

}  // namespace gz
