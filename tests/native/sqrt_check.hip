// Test helper (not product code): exhaustive checks of two device helpers of
// k_block_diff2 against the forms they replace (tests/test_gpu.py::
// test_block_diff_sqrt_and_interp_exhaustive).
//
//  * k_block_diff2's square root -- the hardware root corrected by its neighbours'
//    residuals, on inputs pre-scaled by 2^32 -- against the compiler's
//    correctly rounded sqrtf, bit for bit, for every float in [0, 2^96).
//  * interp_pair_f over a paired table against interp_f over the plain table
//    (InterpolateOpt), bit for bit, for every finite float argument.
// Mismatches are counted with vector atomics (one per workgroup) and the
// smallest mismatching bit pattern is kept.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "kernels/gz_math.h"

namespace {

constexpr unsigned kSqrtEnd = (127u + 96u) << 23;  // bit pattern of 2^96

__device__ __forceinline__ float sqrt_scaled(float x) {  // (the kernel keeps the result scaled by 2^16)
  return gz::sqrt_cr_big(x * 0x1p32f) * 0x1p-16f;
}

__global__ __launch_bounds__(256) void k_sqrt_check(unsigned long long* bad, unsigned* first) {
  __shared__ unsigned s_bad;
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  const unsigned stride = gridDim.x * 256u;
  unsigned n = 0, lo = 0xffffffffu;
  for (unsigned u = blockIdx.x * 256u + threadIdx.x; u < kSqrtEnd; u += stride) {
    const float x = __uint_as_float(u);
    if (__float_as_uint(sqrt_scaled(x)) != __float_as_uint(sqrtf(x))) {
      ++n;
      lo = min(lo, u);
    }
  }
  if (n) {
    atomicAdd(&s_bad, n);
    atomicMin(first, lo);
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_bad) atomicAdd(bad, static_cast<unsigned long long>(s_bad));
}

__global__ __launch_bounds__(256) void k_interp_check(const float* __restrict__ tab, unsigned long long* bad,
                                                      unsigned* first) {
  __shared__ float a[21];
  __shared__ float2 t[21];
  __shared__ unsigned s_bad;
  if (threadIdx.x < 21) {
    const int i = threadIdx.x;
    a[i] = tab[i];
    t[i] = float2{tab[i], i < 20 ? tab[i + 1] - tab[i] : 0.0f};
  }
  if (threadIdx.x == 0) s_bad = 0;
  __syncthreads();
  const unsigned stride = gridDim.x * 256u;
  unsigned n = 0, lo = 0xffffffffu;
  // every bit pattern whose exponent is not all ones (finite values, both signs)
  for (unsigned long long v = blockIdx.x * 256u + threadIdx.x; v < (1ull << 32); v += stride) {
    const unsigned u = static_cast<unsigned>(v);
    if ((u & 0x7f800000u) == 0x7f800000u) continue;
    const float sx = __uint_as_float(u);
    if (__float_as_uint(gz::interp_f(a, 21, sx)) != __float_as_uint(gz::interp_pair_f(t, 21, sx))) {
      ++n;
      lo = min(lo, u);
    }
  }
  if (n) {
    atomicAdd(&s_bad, n);
    atomicMin(first, lo);
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_bad) atomicAdd(bad, static_cast<unsigned long long>(s_bad));
}

}  // namespace

// which: 0 the square root, 1 the interpolation over `tab` (21 floats, host
// memory).  Returns 0 on success (out[0] mismatches, out[1] the smallest
// mismatching bit pattern or 0xffffffff), -1 on a HIP error.
extern "C" int gz_helper_check(int which, const float* tab, unsigned long long* out) {
  unsigned long long* d_bad = nullptr;
  unsigned* d_first = nullptr;
  float* d_tab = nullptr;
  int rc = -1;
  const unsigned init = 0xffffffffu;
  if (hipMalloc(&d_bad, 8) != hipSuccess || hipMalloc(&d_first, 4) != hipSuccess ||
      hipMalloc(&d_tab, 21 * 4) != hipSuccess)
    goto done;
  if (hipMemset(d_bad, 0, 8) != hipSuccess || hipMemcpy(d_first, &init, 4, hipMemcpyHostToDevice) != hipSuccess)
    goto done;
  if (which == 0) {
    k_sqrt_check<<<4096, 256>>>(d_bad, d_first);
  } else {
    if (hipMemcpy(d_tab, tab, 21 * 4, hipMemcpyHostToDevice) != hipSuccess) goto done;
    k_interp_check<<<4096, 256>>>(d_tab, d_bad, d_first);
  }
  if (hipDeviceSynchronize() != hipSuccess) goto done;
  {
    unsigned first = 0;
    if (hipMemcpy(out, d_bad, 8, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&first, d_first, 4, hipMemcpyDeviceToHost) != hipSuccess)
      goto done;
    out[1] = first;
  }
  rc = 0;
done:
  if (d_bad) (void)hipFree(d_bad);
  if (d_first) (void)hipFree(d_first);
  if (d_tab) (void)hipFree(d_tab);
  return rc;
}
