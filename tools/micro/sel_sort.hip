// The selection's last-workgroup sort (order_kernels.inc: sel_order, the
// bucket counting sort) against the all-LDS bitonic network it replaced,
// one 1024-thread workgroup, n keys (random, or clustered in few buckets):
// time per launch (profiles/round5_sel_sort.txt).
//   hipcc -O3 --offload-arch=gfx950 -I guetzli-cuda-opencl_amd/csrc tools/micro/sel_sort.hip -o /tmp/sel_sort
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "kernels/gz_math.h"
#include "kernels/scan_kernels.inc"
#include "kernels/order_kernels.inc"

using gz::kSelThreads;

template <int E>
__global__ __launch_bounds__(kSelThreads) void k_reg(const unsigned long long* cand, int nc, int cap, uint32_t lo24,
                                                     uint32_t hi24, unsigned long long* out) {
  extern __shared__ unsigned long long sk[];
  gz::sel_order<E>(sk, sk + cap, reinterpret_cast<uint32_t*>(sk + 2 * cap), cand, nc, lo24, hi24);
  for (int i = threadIdx.x; i < nc; i += kSelThreads) out[i] = sk[i];
}

__global__ __launch_bounds__(kSelThreads) void k_lds(const unsigned long long* cand, int nc, int n2,
                                                     unsigned long long* out) {
  extern __shared__ unsigned long long sk[];
  const int t = threadIdx.x;
  for (int i = t; i < n2; i += kSelThreads) sk[i] = i < nc ? cand[i] : ~0ull;
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int q = t; q < n2 / 2; q += kSelThreads) {
        const int i = 2 * q - (q & (stride - 1));
        const int j = i + stride;
        const bool up = (i & size) == 0;
        const unsigned long long x = sk[i], y = sk[j];
        if ((x > y) == up) {
          sk[i] = y;
          sk[j] = x;
        }
      }
      __syncthreads();
    }
  for (int i = t; i < nc; i += kSelThreads) out[i] = sk[i];
}

int main() {
  const int maxn = 16384;
  std::vector<unsigned long long> h(maxn);
  srand(1);
  unsigned long long *d, *o;
  (void)hipMalloc(&d, maxn * 8);
  (void)hipMalloc(&o, maxn * 8);
  (void)hipMemcpy(d, h.data(), maxn * 8, hipMemcpyHostToDevice);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_lds), hipFuncAttributeMaxDynamicSharedMemorySize, maxn * 8);
  const int lds = 2 * 8192 * 8 + (gz::kSelSortBins + 1) * 4;
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_reg<1>), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_reg<2>), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_reg<4>), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_reg<8>), hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int clustered = 0; clustered < 2; ++clustered)
  for (int nc : {300, 1500, 2048, 3000, 4096, 8192}) {
    // clustered: keys in 40 distinct 24-bit bins (ties of bits across blocks)
    for (int i = 0; i < maxn; ++i) {
      const unsigned long long bits = clustered ? 0x40000000ull + (static_cast<unsigned>(rand()) % 40) * 256 + rand() % 3
                                                : static_cast<unsigned>(rand());
      h[i] = (bits << 32) | static_cast<unsigned>(rand() % 30000);
    }
    (void)hipMemcpy(d, h.data(), maxn * 8, hipMemcpyHostToDevice);
    uint32_t lo24 = ~0u, hi24 = 0;
    for (int i = 0; i < nc; ++i) {
      lo24 = std::min<uint32_t>(lo24, h[i] >> 40);
      hi24 = std::max<uint32_t>(hi24, h[i] >> 40);
    }
    int n2 = 2;
    while (n2 < nc) n2 <<= 1;
    const int cap = 8192;
    for (int form = 0; form < 2; ++form) {
      auto launch = [&]() {
        if (form == 0) {
          k_lds<<<1, kSelThreads, n2 * 8>>>(d, nc, n2, o);
        } else {
          if (nc <= 1024) k_reg<1><<<1, kSelThreads, lds>>>(d, nc, cap, lo24, hi24, o);
          else if (nc <= 2048) k_reg<2><<<1, kSelThreads, lds>>>(d, nc, cap, lo24, hi24, o);
          else if (nc <= 4096) k_reg<4><<<1, kSelThreads, lds>>>(d, nc, cap, lo24, hi24, o);
          else k_reg<8><<<1, kSelThreads, lds>>>(d, nc, cap, lo24, hi24, o);
        }
      };
      for (int i = 0; i < 3; ++i) launch();
      (void)hipEventRecord(e0);
      const int reps = 50;
      for (int i = 0; i < reps; ++i) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      std::vector<unsigned long long> r(nc);
      (void)hipMemcpy(r.data(), o, nc * 8, hipMemcpyDeviceToHost);
      std::vector<unsigned long long> ref(h.begin(), h.begin() + nc);
      std::sort(ref.begin(), ref.end());
      printf("%s n %5d %s  %7.2f us per launch  %s\n", clustered ? "clustered" : "random   ", nc,
             form ? "buckets " : "bitonic ", ms * 1e3 / reps,
             r == ref ? "sorted" : "WRONG");
    }
  }
  return 0;
}
