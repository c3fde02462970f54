// D2H copy of one 1080p coefficient set (12.4 MB) into pinned host memory
// allocated three ways: which engine the runtime picks (a blit kernel shows
// up as __amd_rocclr_copyBuffer in a kernel trace) and the time it takes.
//   hipcc --offload-arch=gfx950 -O2 d2h_probe.hip -o d2h_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

int main() {
  const size_t bytes = 32400ull * 64 * 3 * 2;
  void* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return 1;
  hipMemset(d, 1, bytes);
  hipStream_t s;
  hipStreamCreate(&s);
  const unsigned flags[3] = {hipHostMallocCoherent, hipHostMallocNonCoherent, hipHostMallocDefault};
  const char* names[3] = {"coherent", "noncoherent", "default"};
  for (int f = 0; f < 3; ++f) {
    void* h = nullptr;
    if (hipHostMalloc(&h, bytes, flags[f]) != hipSuccess) return 2;
    for (int rep = 0; rep < 4; ++rep) {
      hipDeviceSynchronize();
      const auto t0 = std::chrono::steady_clock::now();
      hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s);
      hipStreamSynchronize(s);
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (rep == 3) printf("%-12s %8.1f us  %6.1f GB/s\n", names[f], us, bytes / us / 1e3);
    }
    hipHostFree(h);
  }
  hipFree(d);
  return 0;
}
