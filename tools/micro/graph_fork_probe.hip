// Do the parallel branches of a captured HIP graph (a fork onto a second
// stream by events during capture) run concurrently on gfx950 / ROCm 7?
// Two 1-workgroup kernels of ~N us each: serial graph ~2N, forked ~N if the
// branches overlap.  hipcc --offload-arch=gfx950 -O2 graph_fork_probe.hip
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void spin(long long cycles, int* out) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0) out[blockIdx.x] = 1;
}

static double run(hipGraphExec_t g, hipStream_t s) {
  hipGraphLaunch(g, s);
  hipStreamSynchronize(s);
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 20; ++i) hipGraphLaunch(g, s);
  hipStreamSynchronize(s);
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 20;
}

int main() {
  int* d = nullptr;
  hipMalloc(&d, 1024);
  hipStream_t s, s2;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  hipEvent_t fork, join;
  hipEventCreateWithFlags(&fork, hipEventDisableTiming);
  hipEventCreateWithFlags(&join, hipEventDisableTiming);
  const long long cyc = 100000;  // ~50 us at 2 GHz
  hipGraph_t g1, g2;
  hipGraphExec_t e1, e2;
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  spin<<<1, 64, 0, s>>>(cyc, d);
  spin<<<1, 64, 0, s>>>(cyc, d + 1);
  hipStreamEndCapture(s, &g1);
  hipGraphInstantiate(&e1, g1, nullptr, nullptr, 0);
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  hipEventRecord(fork, s);
  hipStreamWaitEvent(s2, fork, 0);
  spin<<<1, 64, 0, s2>>>(cyc, d);
  hipEventRecord(join, s2);
  spin<<<1, 64, 0, s>>>(cyc, d + 1);
  hipStreamWaitEvent(s, join, 0);
  hipStreamEndCapture(s, &g2);
  hipGraphInstantiate(&e2, g2, nullptr, nullptr, 0);
  printf("serial graph %.1f us, forked graph %.1f us\n", run(e1, s), run(e2, s));
  return 0;
}
