// FETCH_SIZE / WRITE_SIZE calibration on gfx950 by access width.
//
// Each kernel moves a known number of bytes (1 GiB buffers: past the 256 MiB
// Infinity Cache, so reads reach HBM) with 4, 8 or 16 bytes per lane, fully
// coalesced, or as 64-byte pieces of every other 128-byte line (partial-line
// reads).  Run under `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE`;
// tools/traffic_summary.py --calibrate turns the counts into bytes-per-count
// factors per width.  Prints the kernel name -> algorithmic bytes table.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <typename T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ a, size_t n, float* sink) {
  float s = 0.0f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    const T v = a[i];
    s += reinterpret_cast<const float*>(&v)[0];
  }
  if (s == 12345.0f) sink[0] = s;  // keeps the loads; never true for the fill
}

// 64-byte pieces of every other 128-byte line: 4 lanes x 16 B per piece.
__global__ __launch_bounds__(256) void k_read_half_lines(const float4* __restrict__ a, size_t lines,
                                                        float* sink) {
  float s = 0.0f;
  const size_t t = blockIdx.x * 256ull + threadIdx.x;
  for (size_t q = t; q < lines * 4; q += gridDim.x * 256ull) {
    const size_t line = (q / 4) * 2, part = q % 4;  // even lines only
    s += a[line * 8 + part].x;
  }
  if (s == 12345.0f) sink[0] = s;
}

template <typename T>
__global__ __launch_bounds__(256) void k_write(T* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) {
    T v;
    reinterpret_cast<float*>(&v)[0] = static_cast<float>(i & 7);
    for (int k = 1; k < static_cast<int>(sizeof(T) / 4); ++k) reinterpret_cast<float*>(&v)[k] = 0.0f;
    b[i] = v;
  }
}

int main() {
  const size_t bytes = 1ull << 30;
  void *a, *b;
  float* sink;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess ||
      hipMalloc(&sink, 64) != hipSuccess)
    return 1;
  hipMemset(a, 0, bytes);
  const int grid = 8192;
  k_read<float><<<grid, 256>>>((const float*)a, bytes / 4, sink);
  k_read<float2><<<grid, 256>>>((const float2*)a, bytes / 8, sink);
  k_read<float4><<<grid, 256>>>((const float4*)a, bytes / 16, sink);
  k_read_half_lines<<<grid, 256>>>((const float4*)a, bytes / 256, sink);
  k_write<float><<<grid, 256>>>((float*)b, bytes / 4);
  k_write<float2><<<grid, 256>>>((float2*)b, bytes / 8);
  k_write<float4><<<grid, 256>>>((float4*)b, bytes / 16);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"k_read<float>\": %zu, \"k_read<float2>\": %zu, \"k_read<float4>\": %zu, "
         "\"k_read_half_lines\": %zu, \"k_write<float>\": %zu, \"k_write<float2>\": %zu, "
         "\"k_write<float4>\": %zu}\n",
         bytes, bytes, bytes, bytes / 2, bytes, bytes, bytes);
  return 0;
}
