// Copy bandwidth by access width (dword vs dwordx2 vs dwordx4 per lane) at
// the plane sizes of the Compare pass.  Calibration for kernel design.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <typename T>
__global__ void k_copy(const T* __restrict__ a, T* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// 2-D stencil-like read pattern: each lane reads its column for 8 rows (dword), writes 1
__global__ void k_col8(const float* __restrict__ a, float* __restrict__ b, int w, int h) {
  int x = blockIdx.x * 256 + threadIdx.x, y0 = blockIdx.y * 8;
  if (x >= w) return;
  float s = 0;
  for (int k = 0; k < 8; ++k) if (y0 + k < h) { s += a[(size_t)(y0 + k) * w + x]; }
  for (int k = 0; k < 8; ++k) if (y0 + k < h) b[(size_t)(y0 + k) * w + x] = s + k;
}

template <typename T>
float run(const void* a, void* b, size_t bytes, int grid) {
  size_t n = bytes / sizeof(T);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) k_copy<T><<<grid, 256>>>((const T*)a, (T*)b, n);
  hipEventRecord(e0);
  const int reps = 50;
  for (int i = 0; i < reps; ++i) k_copy<T><<<grid, 256>>>((const T*)a, (T*)b, n);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  size_t maxb = 400u << 20;
  void *a, *b;
  hipMalloc(&a, maxb); hipMalloc(&b, maxb);
  hipMemset(a, 1, maxb);
  for (size_t mb : {8, 25, 50, 100, 400}) {
    size_t bytes = mb << 20;
    for (int grid : {1024, 4096, 16384}) {
      float t1 = run<float>(a, b, bytes, grid), t2 = run<float2>(a, b, bytes, grid), t4 = run<float4>(a, b, bytes, grid);
      printf("%4zu MB grid %5d: dword %6.1f us %5.0f GB/s | x2 %6.1f us %5.0f GB/s | x4 %6.1f us %5.0f GB/s\n", mb, grid,
             t1 * 1e3, 2 * bytes / t1 / 1e6, t2 * 1e3, 2 * bytes / t2 / 1e6, t4 * 1e3, 2 * bytes / t4 / 1e6);
    }
  }
  // 6 planes of 1080p, column pattern
  int w = 1920, h = 1080;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  dim3 g((w + 255) / 256, (h + 7) / 8);
  for (int i = 0; i < 3; ++i) k_col8<<<g, 256>>>((float*)a, (float*)b, w, h);
  hipEventRecord(e0);
  for (int i = 0; i < 50; ++i) k_col8<<<g, 256>>>((float*)a, (float*)b, w, h);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("col8 1080p plane: %.1f us, %.0f GB/s\n", ms / 50 * 1e3, 2.0 * w * h * 4 / (ms / 50) / 1e6);
  return 0;
}
