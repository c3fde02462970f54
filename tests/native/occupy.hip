// Test helper (not product code): a kernel that holds most of the device's
// CU slots until the host releases it, so a GPU test can run the entropy
// coder while another stream's workgroups sit on the slots its predecessors
// would need (tests/test_gpu.py::test_coder_forward_progress_under_occupancy).
//
// One 64-thread workgroup per CU (each declares all 160 KiB of LDS, so no
// other workgroup fits beside it); workgroups that land on `spare_xcd` exit
// at once, so that XCD alone stays free.  Every holding workgroup spins on a
// host-mapped release word with a bounded wall-clock limit, so the grid
// always drains.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kLdsBytes = 160 * 1024;

__global__ __launch_bounds__(64) void k_occupy(const uint32_t* release, uint32_t* held, int spare_xcd,
                                               uint64_t limit_ticks) {
  __shared__ uint32_t lds[kLdsBytes / 4];
  uint32_t xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (static_cast<int>(xcc & 0xf) == spare_xcd) return;
  if (threadIdx.x == 0) {
    lds[0] = 1u;
    __hip_atomic_fetch_add(held, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0u) {
      if (wall_clock64() - t0 > limit_ticks) break;
      __builtin_amdgcn_s_sleep(127);
    }
    __hip_atomic_fetch_sub(held, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (threadIdx.x == 1) lds[1] = lds[0];
}

struct Occupy {
  hipStream_t stream = nullptr;
  uint32_t* release = nullptr;  // host-mapped
  uint32_t* held = nullptr;     // device
};

}  // namespace

extern "C" {

// Starts the holding kernel on its own stream; returns an opaque handle (null
// on failure).  limit_ms bounds the hold whatever the host does.
void* occupy_start(int device, int spare_xcd, int limit_ms) {
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return nullptr;
  Occupy* o = new Occupy;
  if (hipStreamCreateWithFlags(&o->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc(reinterpret_cast<void**>(&o->release), 64, hipHostMallocCoherent | hipHostMallocMapped) !=
          hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&o->held), 64) != hipSuccess ||
      hipMemsetAsync(o->held, 0, 64, o->stream) != hipSuccess) {
    delete o;
    return nullptr;
  }
  *o->release = 0u;
  uint32_t* rel_dev = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&rel_dev), o->release, 0) != hipSuccess) return nullptr;
  const uint64_t ticks = static_cast<uint64_t>(limit_ms) * 100000ull;  // wall clock: 100 MHz
  k_occupy<<<prop.multiProcessorCount, 64, 0, o->stream>>>(rel_dev, o->held, spare_xcd, ticks);
  if (hipGetLastError() != hipSuccess) return nullptr;
  return o;
}

// Workgroups holding a CU right now -- started and not yet released or
// timed out (read on a stream of its own).
int occupy_held(void* h) {
  Occupy* o = static_cast<Occupy*>(h);
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -1;
  uint32_t v = 0;
  const bool ok = hipMemcpyAsync(&v, o->held, 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
                  hipStreamSynchronize(s) == hipSuccess;
  (void)hipStreamDestroy(s);
  return ok ? static_cast<int>(v) : -1;
}

// Releases the holders, waits for the grid to drain and frees everything.
int occupy_release(void* h) {
  Occupy* o = static_cast<Occupy*>(h);
  __atomic_store_n(o->release, 1u, __ATOMIC_SEQ_CST);
  const bool ok = hipStreamSynchronize(o->stream) == hipSuccess;
  (void)hipFree(o->held);
  (void)hipHostFree(o->release);
  (void)hipStreamDestroy(o->stream);
  delete o;
  return ok ? 0 : -1;
}

}  // extern "C"
