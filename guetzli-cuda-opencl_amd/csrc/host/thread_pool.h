// Fixed-size host worker pool for the data-parallel host passes of the search
// loop (scan encoding, histograms).  One pool per process.  The worker count
// is GZ_HOST_THREADS, else min(16, the usable CPUs -- affinity and cgroup
// quota -- divided by LOCAL_WORLD_SIZE ranks) -- 16 being the CPU share a
// GPU gets on the target nodes.  The pool is not re-entrant; callers that
// find it busy run their items inline (ParallelFor).
#pragma once

#include <stddef.h>

#include <functional>

namespace gz {

int HostThreads();

// Runs fn(i) for i in [0, n) on the pool (the caller takes part) and returns
// when all are done.  Items are handed out dynamically.  If another thread
// is using the pool, the items run on the calling thread instead.
// (file / line: the call site, for GZ_POOL_PROFILE)
void ParallelFor(int n, const std::function<void(int)>& fn, const char* file = __builtin_FILE(),
                 int line = __builtin_LINE());

}  // namespace gz
