// Where does the one-residual-step division by the gamma range constant
// differ from IEEE division?  Histogram of mismatches by biased exponent of
// the numerator (calibration only).
#include <hip/hip_runtime.h>
#include <stdio.h>
constexpr float kDen = 274.579999999999984f - 0.770000000000000f;
__global__ void k(float r, unsigned long long* hist) {
  for (unsigned long long u = blockIdx.x * 256ull + threadIdx.x; u < (1ull << 32); u += gridDim.x * 256ull) {
    const float n = __uint_as_float(static_cast<uint32_t>(u));
    if (n != n || isinf(n)) continue;
    const float q = n * r;
    const float e = fmaf(-q, kDen, n);
    const float f = fmaf(e, r, q);
    const float g = n / kDen;
    if (__float_as_uint(f) != __float_as_uint(g)) {
      atomicAdd(&hist[(u >> 23) & 255], 1ull);
      if (fabsf(n) >= 0x1p-100f) printf("fail n=%a (%08x) fast=%a ieee=%a\n", n, (unsigned)u, f, g);
    }
  }
}
int main() {
  unsigned long long* d; unsigned long long h[256];
  (void)hipMalloc(&d, sizeof(h)); (void)hipMemset(d, 0, sizeof(h));
  const float r = 1.0f / kDen;
  k<<<8192, 256>>>(r, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  printf("r bits %08x den %.9g\n", *(const unsigned*)&r, kDen);
  for (int i = 0; i < 256; ++i) if (h[i]) printf("exp %3d (2^%d): %llu\n", i, i - 127, h[i]);
}
