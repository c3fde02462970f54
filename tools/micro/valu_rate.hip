// VALU issue cost per wave64 instruction on gfx950, by type: the ceiling
// bench.py's valu_issue weights k_block_zeroing's instruction mix with
// (FP64 adds / multiplies / FMAs / square roots next to FP32 and integer
// ops; cvt_f64_f32_pair is a v_cvt_f32_f64 + v_cvt_f64_f32 pair, two
// instructions per step).  Each kernel runs 8 independent dependency chains per lane (enough
// to hide the pipeline latency) over enough waves to fill every SIMD several
// times; cycles per instruction per SIMD = SIMDs x clock x seconds /
// (wave instructions).  Prints one JSON object.
//
//   hipcc -O3 --offload-arch=gfx950 tools/micro/valu_rate.hip -o tools/micro/valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>

constexpr int kIters = 4096;
constexpr int kChains = 8;

template <int kOp>
__global__ __launch_bounds__(256) void k_rate(double* out, float* outf, int* outi, double s) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  double a[kChains];
  float f[kChains];
  int n[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    a[c] = 1.0 + 1e-3 * (t + c);
    f[c] = 1.0f + 1e-3f * (t + c);
    n[c] = t + c;
  }
  const double m = 0.999999 + 1e-12 * s;
  const float mf = static_cast<float>(m);
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if constexpr (kOp == 0) a[c] = fma(a[c], m, s);            // v_fma_f64
      else if constexpr (kOp == 1) a[c] = a[c] * m;             // v_mul_f64
      else if constexpr (kOp == 2) a[c] = a[c] + s;             // v_add_f64
      else if constexpr (kOp == 3) a[c] = sqrt(a[c] + s);       // v_sqrt_f64 (+ fix-up)
      else if constexpr (kOp == 4) f[c] = fmaf(f[c], mf, 1e-7f);  // v_fma_f32
      else if constexpr (kOp == 5) n[c] = n[c] * 747796405 + 1;   // v_mad_u32_u24 / v_mul_lo
      else if constexpr (kOp == 6) a[c] = __builtin_amdgcn_rsq(a[c]);  // v_rsq_f64 (transcendental)
      else if constexpr (kOp == 7) f[c] = __builtin_amdgcn_rsqf(f[c]);  // v_rsq_f32 (transcendental)
      else if constexpr (kOp == 8) f[c] = f[c] + mf;                    // v_add_f32
      else if constexpr (kOp == 9) a[c] = static_cast<double>(static_cast<float>(a[c]));  // cvt f64<->f32
    }
  }
  double r = 0.0;
  float rf = 0.0f;
  int ri = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    r += a[c];
    rf += f[c];
    ri ^= n[c];
  }
  out[t] = r;
  outf[t] = rf;
  outi[t] = ri;
}

int main() {
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const double clock_hz = prop.clockRate * 1e3;
  const int blocks = cus * 4 * 8;  // 8 waves per SIMD
  const size_t n = static_cast<size_t>(blocks) * 256;
  double* d;
  float* df;
  int* di;
  (void)hipMalloc(&d, n * 8);
  (void)hipMalloc(&df, n * 4);
  (void)hipMalloc(&di, n * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"fma_f64", "mul_f64", "add_f64", "sqrt_f64", "fma_f32", "mul_u32", "rsq_f64",
                         "rsq_f32", "add_f32", "cvt_f64_f32_pair"};
  printf("{\"cus\": %d, \"clock_mhz\": %.0f", cus, clock_hz / 1e6);
  for (int op = 0; op < 10; ++op) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      switch (op) {
        case 0: k_rate<0><<<blocks, 256>>>(d, df, di, 1e-9); break;
        case 1: k_rate<1><<<blocks, 256>>>(d, df, di, 1e-9); break;
        case 2: k_rate<2><<<blocks, 256>>>(d, df, di, 1e-9); break;
        case 3: k_rate<3><<<blocks, 256>>>(d, df, di, 1e-9); break;
        case 4: k_rate<4><<<blocks, 256>>>(d, df, di, 1e-9); break;
        case 5: k_rate<5><<<blocks, 256>>>(d, df, di, 1e-9); break;
        case 6: k_rate<6><<<blocks, 256>>>(d, df, di, 1e-9); break;
        case 7: k_rate<7><<<blocks, 256>>>(d, df, di, 1e-9); break;
        case 8: k_rate<8><<<blocks, 256>>>(d, df, di, 1e-9); break;
        default: k_rate<9><<<blocks, 256>>>(d, df, di, 1e-9); break;
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0.0f;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    // wave instructions of the timed op (the chains' op only; the loop
    // overhead is amortised over 8 chains)
    const double waves = static_cast<double>(blocks) * 4;
    const double insts = waves * kIters * kChains;
    const double cyc = (cus * 4.0) * clock_hz * (best * 1e-3) / insts;
    printf(", \"%s\": {\"ms\": %.4f, \"cycles_per_wave_inst\": %.3f}", names[op], best, cyc);
  }
  printf("}\n");
  return 0;
}
