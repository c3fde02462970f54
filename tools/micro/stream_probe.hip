// Bandwidth ceilings for the access shapes of the blur passes at 4K
// (6 planes of 3840x2160 f32 = 199 MB in): plain copy, read-4/write-1 row
// decimation (the horizontal step-4 pass's HBM shape), and column segments
// (the vertical pass's shape), each HIP-event timed over back-to-back
// launches.  Calibration only; not part of the product.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CK(x) do { if ((x) != hipSuccess) { printf("hip error %s\n", #x); return 1; } } while (0)

__global__ void k_copy4(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

// read 4 consecutive floats per thread (float4), write their sum: in n4 float4, out n4 floats
__global__ void k_dec4(const float4* __restrict__ a, float* __restrict__ b, size_t n4) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i < n4) { float4 v = a[i]; b[i] = v.x + v.y + v.z + v.w; }
}

// dword version: each thread reads 4 dwords strided by 64 lanes (a wave reads 1 KB contiguous), writes 1
__global__ void k_dec4w(const float* __restrict__ a, float* __restrict__ b, size_t nout) {
  size_t wv = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6; int lane = threadIdx.x & 63;
  size_t base = wv * 256;
  if (base >= nout * 4) return;
  float s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) s += a[base + lane + 64 * k];
  b[wv * 64 + lane] = s;
}

// column segments: lane = column, reads SEG rows, writes SEG/4 rows
template <int SEG>
__global__ void k_col(const float* __restrict__ a, float* __restrict__ b, int w, int h) {
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int y0 = (blockIdx.y * 4 + (threadIdx.x >> 6)) * SEG;
  if (x >= w || y0 >= h) return;
  float v[SEG];
#pragma unroll
  for (int k = 0; k < SEG; ++k) v[k] = a[(size_t)min(y0 + k, h - 1) * w + x];
#pragma unroll
  for (int k = 0; k < SEG / 4; ++k) b[(size_t)(y0 / 4 + k) * w + x] = v[4 * k] + v[4 * k + 1] + v[4 * k + 2] + v[4 * k + 3];
}

__constant__ float c_taps[80];

// vertical blur replica: lane = column, NO outputs per lane, NIN = (NO-1)*S + 2R+1 rows
// loaded at once; taps from constant memory; seg-major order within a WG
template <int NO, int S, int R>
__global__ __launch_bounds__(256) void k_vc(const float* __restrict__ a, float* __restrict__ b, int w, int h, int dy) {
  constexpr int NT = 2 * R + 1, NIN = (NO - 1) * S + NT;
  const int x = blockIdx.x * 64 + (threadIdx.x & 63);
  const int seg = blockIdx.y * 4 + (threadIdx.x >> 6);
  const int oy0 = seg * NO;
  if (x >= w || oy0 >= dy) return;
  const int y0 = oy0 * S - R;
  float v[NIN];
#pragma unroll
  for (int k = 0; k < NIN; ++k) {
    const int y = y0 + k;
    const int yc = y < 0 ? 0 : (y < h ? y : h - 1);
    const float t = a[(size_t)yc * w + x];
    v[k] = (y >= 0 && y < h) ? t : 0.0f;
  }
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    if (oy0 + o >= dy) break;
    float sum = 0.0f;
#pragma unroll
    for (int t = 0; t < NT; ++t) sum += v[o * S + t] * c_taps[t];
    b[(size_t)(oy0 + o) * w + x] = sum;
  }
}

// mask_front's HBM shape: a wave walks ROWS rows of a 64-column strip of two
// planes, writing one; PF rows of loads kept in flight (register queue)
template <int PF, int ROWS>
__global__ __launch_bounds__(256) void k_strm(const float* __restrict__ a, const float* __restrict__ b,
                                              float* __restrict__ o, int w, int h, int strips) {
  const int lane = threadIdx.x & 63;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int x = (item % strips) * 64 + lane, y0 = (item / strips) * ROWS;
  if (y0 >= h) return;
  const int xc = min(x, w - 1);
  float qa[PF], qb[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int y = min(y0 + k, h - 1);
    qa[k] = a[(size_t)y * w + xc];
    qb[k] = b[(size_t)y * w + xc];
  }
  float acc = 0.0f;
  for (int r = 0; r < ROWS; ++r) {
    const float va = qa[0], vb = qb[0];
#pragma unroll
    for (int k = 0; k + 1 < PF; ++k) { qa[k] = qa[k + 1]; qb[k] = qb[k + 1]; }
    const int yn = min(y0 + r + PF, h - 1);
    qa[PF - 1] = a[(size_t)yn * w + xc];
    qb[PF - 1] = b[(size_t)yn * w + xc];
    acc = acc * 0.5f + (va - vb);
    if (y0 + r < h && x < w) o[(size_t)(y0 + r) * w + x] = acc;
  }
}

template <class F>
float timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  for (int i = 0; i < 3; ++i) f();
  hipEventRecord(e0);
  const int reps = 20;
  for (int i = 0; i < reps; ++i) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  return ms / reps * 1e3f;  // us
}

int main() {
  const int W = 3840, H = 2160, P = 6;
  const size_t n = (size_t)W * H * P;
  float *a, *b;
  CK(hipMalloc(&a, n * 4));
  CK(hipMalloc(&b, n * 4));
  CK(hipMemset(a, 0, n * 4));
  CK(hipMemset(b, 0, n * 4));
  double mb = n * 4 / 1e6;
  float t = timeit([&] { k_copy4<<<16384, 256>>>((const float4*)a, (float4*)b, n / 4); });
  printf("copy     %7.1f us  %6.0f GB/s (r+w %.0f MB)\n", t, 2 * mb / t * 1e3, 2 * mb);
  t = timeit([&] { k_dec4<<<(n / 4 + 255) / 256, 256>>>((const float4*)a, b, n / 4); });
  printf("dec4 x4  %7.1f us  %6.0f GB/s (r+w %.0f MB)\n", t, 1.25 * mb / t * 1e3, 1.25 * mb);
  t = timeit([&] { k_dec4w<<<(n / 4 / 64 * 64 + 255) / 256, 256>>>(a, b, n / 4); });
  printf("dec4 dw  %7.1f us  %6.0f GB/s\n", t, 1.25 * mb / t * 1e3);
  const int Wd = W / 4;  // the decimated planes of the vertical pass: 6 x 2160 x 960
  const int hh = H * P;
  double mbv = (double)Wd * hh * 4 / 1e6;
  t = timeit([&] { k_col<16><<<dim3(Wd / 64, (hh / 16 + 3) / 4), 256>>>(a, b, Wd, hh); });
  printf("col16    %7.1f us  %6.0f GB/s\n", t, 1.25 * mbv / t * 1e3);
  t = timeit([&] { k_col<64><<<dim3(Wd / 64, (hh / 64 + 3) / 4), 256>>>(a, b, Wd, hh); });
  printf("col64    %7.1f us  %6.0f GB/s\n", t, 1.25 * mbv / t * 1e3);
  t = timeit([&] { k_col<16><<<dim3(W / 64, (hh / 16 + 3) / 4), 256>>>(a, b, W, hh); });
  printf("col16 W  %7.1f us  %6.0f GB/s (full-width planes)\n", t, 1.25 * mb / t * 1e3);
  {
    float taps[80];
    for (int i = 0; i < 80; ++i) taps[i] = 1.0f / (1 + i);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(c_taps), taps, sizeof(taps)));
    // one plane-stack: 6 planes x 2160 rows treated as 6 separate images of h=2160
    const int h = H, dy = H / 4;
    for (int rep = 0; rep < 1; ++rep) {
      t = timeit([&] { for (int p = 0; p < P; ++p) k_vc<8, 4, 31><<<dim3(Wd / 64, (dy / 8 + 3) / 4), 256>>>(a + (size_t)p * Wd * h, b + (size_t)p * Wd * dy, Wd, h, dy); });
      printf("vc NO8 S4 R31 (6 launches)  %7.1f us\n", t);
      t = timeit([&] { for (int p = 0; p < P; ++p) k_vc<16, 4, 31><<<dim3(Wd / 64, (dy / 16 + 3) / 4), 256>>>(a + (size_t)p * Wd * h, b + (size_t)p * Wd * dy, Wd, h, dy); });
      printf("vc NO16 S4 R31 (6 launches) %7.1f us\n", t);
      t = timeit([&] { for (int p = 0; p < P; ++p) k_vc<4, 4, 31><<<dim3(Wd / 64, (dy / 4 + 3) / 4), 256>>>(a + (size_t)p * Wd * h, b + (size_t)p * Wd * dy, Wd, h, dy); });
      printf("vc NO4 S4 R31 (6 launches)  %7.1f us\n", t);
      t = timeit([&] { k_vc<8, 4, 31><<<dim3(Wd / 64, (dy * P / 8 + 3) / 4), 256>>>(a, b, Wd, h * P, dy * P); });
      printf("vc NO8 S4 R31 (1 launch, stacked) %7.1f us\n", t);
    }
  }
  {
    // 3 planes pairs of 4K: a = plane set 0, b = plane set 1 (each 3 x 33 MB), out 3 planes
    const int h = H * 3;
    const int strips = W / 64;
    const float* pa = a; const float* pb = a + (size_t)W * h; float* po = b;
    double mbm = 3.0 * 3 * W * H * 4 / 1e6;
#define STRM(PF, ROWS) t = timeit([&] { const int items = strips * ((h + ROWS - 1) / ROWS); k_strm<PF, ROWS><<<(items + 3) / 4, 256>>>(pa, pb, po, W, h, strips); }); \
    printf("strm PF%2d ROWS%3d  %7.1f us  %6.0f GB/s\n", PF, ROWS, t, mbm / t * 1e3);
    STRM(1, 16) STRM(2, 16) STRM(4, 16) STRM(8, 16) STRM(1, 64) STRM(4, 64) STRM(8, 64) STRM(16, 64) STRM(8, 256) STRM(16, 256)
  }
  return 0;
}
