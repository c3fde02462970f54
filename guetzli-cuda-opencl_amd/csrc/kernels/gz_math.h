// Device-side scalar math of the Butteraugli `--c` path, shared by the
// full-image Compare kernels and the per-block zeroing kernel.
//
// Numerics contract: every function reproduces the
// float/double promotion of the reference source it cites.  The library is
// built with -ffp-contract=off, IEEE f32 denormals and correctly rounded f32
// div/sqrt, so each scalar op rounds exactly like the x86 SSE oracle.
// Transcendental tables (blur taps, sRGB, mask LUTs) are computed on the host
// with glibc and live in GzTables (constant memory).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gz {

constexpr int kMaxTaps = 72;   // largest blur: sigma 14.26 -> 65 taps
constexpr int kNumSigmas = 10;

// Blur kernels used by the path (clbutter_comparator.cpp:57-94 callers).
enum SigmaId : int {
  kSigOpsin = 0,   // 1.1      OpsinDynamicsImageOpt           :885
  kSigEdgeX = 1,   // 1.5      EdgeDetectorMapOpt              :1460
  kSigEdgeY = 2,   // 0.586
  kSigEdgeB = 3,   // 0.4
  kSigLowFreq = 4, // 14       EdgeDetectorLowFreqOpt          :1491
  kSigMaskX = 5,   // 9.65781083553   MaskOpt                  :1227
  kSigMaskY = 6,   // 14.2644604355
  kSigMaskB = 7,   // 4.53358927369
  kSigDiffmap = 8, // 8.8510880283 (border_ratio 0.03027655136) CalculateDiffmapOpt :958
  // kSigMaskB evaluated on every 3rd row and column only: per Compare the B
  // activity mask is read at (3j + 3, 3i + 3) alone (CombineChannelsOpt
  // :1542-1565), so its blur is run as a step-3 blur with the sigma-4.53
  // taps -- the same sums at the sampled positions, a ninth of the outputs
  kSigMaskBSub = 9,
};

// Compile-time geometry of the nine blurs (BlurOpt, clbutter_comparator.cpp:
// 60-69: radius = max(1, int(2.25f * sigma)), step = max(1, int(sigma / 3))),
// so that tap loops unroll with the taps in scalar registers.  Checked
// against the host-built table when an engine is created.
// Two f32 lanes in one register pair: arithmetic on it compiles to the
// packed v_pk_mul_f32 / v_pk_add_f32 (two correctly rounded f32 results per
// instruction; -ffp-contract=off keeps them separate, as the scalar code).
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int kSig> struct BlurGeom;
template <> struct BlurGeom<kSigOpsin> { static constexpr int R = 2, STEP = 1; };
template <> struct BlurGeom<kSigEdgeX> { static constexpr int R = 3, STEP = 1; };
template <> struct BlurGeom<kSigEdgeY> { static constexpr int R = 1, STEP = 1; };
template <> struct BlurGeom<kSigEdgeB> { static constexpr int R = 1, STEP = 1; };
template <> struct BlurGeom<kSigLowFreq> { static constexpr int R = 31, STEP = 4; };
template <> struct BlurGeom<kSigMaskX> { static constexpr int R = 21, STEP = 3; };
template <> struct BlurGeom<kSigMaskY> { static constexpr int R = 32, STEP = 4; };
template <> struct BlurGeom<kSigMaskB> { static constexpr int R = 10, STEP = 1; };
template <> struct BlurGeom<kSigDiffmap> { static constexpr int R = 19, STEP = 2; };
template <> struct BlurGeom<kSigMaskBSub> { static constexpr int R = 10, STEP = 3; };
constexpr int kBlurGeomR[kNumSigmas] = {2, 3, 1, 1, 31, 21, 32, 10, 19, 10};
constexpr int kBlurGeomStep[kNumSigmas] = {1, 1, 1, 1, 4, 3, 4, 1, 2, 3};

// Calls F(kSig) for the (uniform) runtime sigma id.
#define GZ_BLUR_SWITCH(sig, F)            \
  switch (sig) {                          \
    case kSigOpsin: F(kSigOpsin); break;  \
    case kSigEdgeX: F(kSigEdgeX); break;  \
    case kSigEdgeY: F(kSigEdgeY); break;  \
    case kSigEdgeB: F(kSigEdgeB); break;  \
    case kSigLowFreq: F(kSigLowFreq); break; \
    case kSigMaskX: F(kSigMaskX); break;  \
    case kSigMaskY: F(kSigMaskY); break;  \
    case kSigMaskB: F(kSigMaskB); break;  \
    case kSigMaskBSub: F(kSigMaskBSub); break; \
    default: F(kSigDiffmap); break;       \
  }

struct BlurSpec {
  int radius;          // "diff" in BlurOpt
  int step;            // xstep == ystep
  float border_ratio;
  float weight_no_border;
  float taps[kMaxTaps];  // expn[0 .. 2*radius]
};

struct GzTables {
  float srgb[256];          // (float)Srgb8ToLinearTable()[i]   gamma_correct.cc:23-38
  int cr_r[256], cb_b[256], cr_g[256], cb_g[256];  // color_transform.h
  float hf_dx[21], hf_dy[21], lf_dy[21];           // clbutter_comparator.cpp:146-193
  double hf_dy_d[21], lf_dy_d[21];                 // butteraugli.cc:217-247
  float mask_lut[6][512];                          // clbutter_comparator.cpp:980-1064
  float block_csf[37];                             // :103-144
  double block_csf_d[37];                          // butteraugli.cc:157-198
  double ac_w_d[3][33];  // block_csf_d[k] * 64.8, 1.0, block_csf_d[k] * 2.4 (k = 4..36): the AC sums' factors
  float csf_xb[2][37];   // block_csf[k] * 64.8f, block_csf[k] * 2.4f: the X / B terms' first product (f32)
  float zeroing_csf[192];                          // order.inc:3
  uint8_t zigzag[64];                              // kJPEGZigZagOrder, jpeg_data.h:73-82
  uint8_t old_csf[64];                             // oldCsf, processor.cc:381-390
  int idct[64];                                    // idct.cc:29-38
  float opsin8_scale[8];  // border scales of the sigma-1.1 blur on an 8-wide axis (8x8 opsin)
  BlurSpec blur[kNumSigmas];
};

// Planes handled by one launch of the separable blur (blockIdx.z = plane).
constexpr int kMaxBlurPlanes = 9;  // the merged sigma-14 + mask launches
struct BlurPlanes {
  const float* in[kMaxBlurPlanes];
  float* out[kMaxBlurPlanes];
  // mask planes of a vertical pass: when set, out gets MaskOpt's LUT value
  // MaskX/Y/B (the mask) of each blurred sample and out2 MaskDcX/Y/B (the
  // DC mask), both times kGlobalScale^-2 (the S13 tail, once per sample)
  float* out2[kMaxBlurPlanes];
  int sig[kMaxBlurPlanes];
  // packed 1-D grid over the planes' (tile, row) work items: plane p owns
  // workgroups [start[p], start[p+1]), tiles[p] 256-wide tiles per row
  int nplanes;
  int tiles[kMaxBlurPlanes];
  int start[kMaxBlurPlanes + 1];
};

// Defined once in gz_device.hip (the single device translation unit).
extern __constant__ GzTables c_tab;

// ---------------------------------------------------------------------------
// XCD-aware workgroup numbering.  Workgroups are dealt round-robin over the
// 8 XCDs, each with its own 4 MiB L2; renumbering them so that every XCD
// owns one contiguous range of the (x fastest, then y, then z) grid puts the
// neighbouring rows a stencil re-reads on the same L2.  Bijective for any
// grid size (MI355X guide, T1).  A speed choice only: results do not depend
// on placement.
// ---------------------------------------------------------------------------
struct BlockId {
  int x, y, z;
};
__device__ __forceinline__ BlockId xcd_block_id() {
  const unsigned gx = gridDim.x, gy = gridDim.y;
  const unsigned n = gx * gy * gridDim.z;
  const unsigned lin = (blockIdx.z * gy + blockIdx.y) * gx + blockIdx.x;
  const unsigned q = n / 8, r = n % 8, xcd = lin % 8, k = lin / 8;
  const unsigned id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + k;
  return BlockId{static_cast<int>(id % gx), static_cast<int>((id / gx) % gy),
                 static_cast<int>(id / (gx * gy))};
}

// ---------------------------------------------------------------------------
// Small helpers
// ---------------------------------------------------------------------------

// Index of this thread's wave in a 256-thread workgroup, as a wave-uniform
// (scalar) value: lets the compiler keep per-wave work items, loop bounds
// and branches in SGPRs instead of treating them as lane-divergent.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// Row y of a plane of width w: with y wave-uniform the pointer is formed in
// scalar registers and a lane's access is a 32-bit offset from it (saddr +
// voffset addressing: no 64-bit address arithmetic per lane).
template <class T>
__device__ __forceinline__ T* row_ptr(T* base, int y, int w) {
  return base + static_cast<size_t>(y) * w;
}

// v where keep, else +0, by a bit mask: loads stay unconditional (a select
// on a loaded value may otherwise become a branch around the load that
// waits for it on the spot).
__device__ __forceinline__ float masked(float v, bool keep) {
  return __int_as_float(__float_as_int(v) & (keep ? -1 : 0));
}

// Lane shifts by DPP (a VALU modifier, no LDS round trip): wave_next(v) is
// lane i+1's value in lane i, wave_prev(v) lane i-1's; the edge lane gets 0.
// Call them with the whole wave active (outside lane-divergent branches).
// bound_ctrl gives the edge lane its 0 (all rows and banks enabled, the old
// value is never read): no zeroing move per shift, and the compiler can fold
// the shift into the instruction that consumes it.
__device__ __forceinline__ float wave_next(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x130, 0xf, 0xf, true));
}
__device__ __forceinline__ float wave_prev(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), 0x138, 0xf, 0xf, true));
}


__device__ __forceinline__ float interp_f(const float* a, int size, float sx) {
  // InterpolateOpt, clbutter_comparator.cpp:195-210
  const float ix = fabsf(sx);
  const int base = static_cast<int>(ix);
  float res;
  if (base >= size - 1) {
    res = a[size - 1];
  } else {
    const float mix = ix - base;
    res = a[base] + mix * (a[base + 1] - a[base]);
  }
  return sx < 0 ? -res : res;
}

// interp_f over a paired table t[i] = (a[i], a[i + 1] - a[i]) for i < size - 1
// and t[size - 1] = (a[size - 1], 0): one 8-byte read, no branch.  The same
// operations on the same values: the difference is the same f32 subtraction,
// mix = ix - trunc(ix) is exact (v_fract; for ix >= 2^23 both are 0), and an
// index at or past size - 1 takes a[size - 1] + mix * 0 == a[size - 1] (mix is
// finite and >= 0, so the product is +0).
__device__ __forceinline__ float interp_pair_f(const float2* t, int size, float sx) {
  const float ix = fabsf(sx);
  const int base = static_cast<int>(ix);
  const float mix = __builtin_amdgcn_fractf(ix);
  const float2 p = t[base < size - 1 ? base : size - 1];
  const float res = p.x + mix * p.y;
  return sx < 0 ? -res : res;
}

// sqrtf of x >= 0 (finite) where x == 0 or x >= 2^-96: the hardware square
// root (within 1 ulp) corrected by the signs of its two neighbours' residuals
// -- the compiler's own correctly rounded sequence without its scaling of
// inputs below 2^-96 and its class test (x == 0: the lower neighbour is a NaN,
// the upper one's residual +0, so 0 stays).  sqrt_needs_scale() flags the
// inputs it does not cover; a wave with any takes sqrtf.
__device__ __forceinline__ float sqrt_cr_big(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float dn = __uint_as_float(__float_as_uint(s) - 1u);
  const float up = __uint_as_float(__float_as_uint(s) + 1u);
  const float r = fmaf(-dn, s, x) <= 0.0f ? dn : s;
  return fmaf(-up, s, x) > 0.0f ? up : r;
}
__device__ __forceinline__ bool sqrt_needs_scale(float x) {  // 0 < x < 2^-96
  return __float_as_uint(x) - 1u < 0x0f7fffffu;
}

__device__ __forceinline__ float interp_clamp_neg_f(const float* a, int size, float sx) {
  // InterpolateClampNegativeOpt, :212-229
  if (sx < 0) sx = 0;
  const float ix = fabsf(sx);
  const int base = static_cast<int>(ix);
  if (base >= size - 1) return a[size - 1];
  const float mix = ix - base;
  return a[base] + mix * (a[base + 1] - a[base]);
}

__device__ __forceinline__ double interp_d(const double* a, int size, double sx) {
  // Interpolate, butteraugli.cc:249-263
  const double ix = fabs(sx);
  const int base = static_cast<int>(ix);
  double res;
  if (base >= size - 1) {
    res = a[size - 1];
  } else {
    const double mix = ix - base;
    res = a[base] + mix * (a[base + 1] - a[base]);
  }
  return sx < 0 ? -res : res;
}

// XybLowFreqToValsOpt + XybDiffLowFreqSquaredAccumulateOpt with the second
// colour == 0 (the only form used on the path), :253-299.
__device__ __forceinline__ void lowfreq_sq_zero_f(float x, float y, float z, float factor,
                                                  float res[3], const float* lf_dy = c_tab.lf_dy) {
  z += 0.0812519812628f * y;
  const float vz = z * 7.34905756986f;
  const float vx = x * 6.64482198135f;
  const float vy = interp_f(lf_dy, 21, y * 0.837846224276f);
  res[0] += factor * vx * vx;
  res[1] += factor * vy * vy;
  res[2] += factor * vz * vz;
}

// interp_f over lf_dy as a plain table or as interp_pair_f's paired one
__device__ __forceinline__ float interp_tab(const float* a, int size, float sx) { return interp_f(a, size, sx); }
__device__ __forceinline__ float interp_tab(const float2* t, int size, float sx) {
  return interp_pair_f(t, size, sx);
}

// (lf_dy: c_tab.lf_dy or an LDS copy of it, plain or paired)
template <class Tab = float>
__device__ __forceinline__ void lowfreq_vals_f(float x, float y, float z, float v[3],
                                               const Tab* lf_dy = c_tab.lf_dy) {
  z += 0.0812519812628f * y;
  v[2] = z * 7.34905756986f;
  v[0] = x * 6.64482198135f;
  v[1] = interp_tab(lf_dy, 21, y * 0.837846224276f);
}

// General two-colour form (used by the corner edge detector).
template <class Tab = float>
__device__ __forceinline__ void lowfreq_sq_f(const float a[3], const float b[3], float factor,
                                             float res[3], const Tab* lf_dy = c_tab.lf_dy) {
  float v0[3];
  lowfreq_vals_f(a[0], a[1], a[2], v0, lf_dy);
  if (b[0] == 0.0f && b[1] == 0.0f && b[2] == 0.0f) {
    res[0] += factor * v0[0] * v0[0];
    res[1] += factor * v0[1] * v0[1];
    res[2] += factor * v0[2] * v0[2];
    return;
  }
  float v1[3];
  lowfreq_vals_f(b[0], b[1], b[2], v1, lf_dy);
  const float dx = v0[0] - v1[0], dy = v0[1] - v1[1], dz = v0[2] - v1[2];
  res[0] += factor * dx * dx;
  res[1] += factor * dy * dy;
  res[2] += factor * dz * dz;
}

__device__ __forceinline__ void lowfreq_sq_zero_d(double x, double y, double z, double factor,
                                                  double res[3],
                                                  const double* lf_dy = c_tab.lf_dy_d) {
  // butteraugli.cc:305-340 (double)
  z += 0.0812519812628 * y;
  const double vz = z * 7.34905756986;
  const double vx = x * 6.64482198135;
  const double vy = interp_d(lf_dy, 21, y * 0.837846224276);
  res[0] += factor * vx * vx;
  res[1] += factor * vy * vy;
  res[2] += factor * vz * vz;
}

template <typename T>
__device__ __forceinline__ T remove_range(T v, T range) {
  if (v >= -range && v < range) return 0;
  return v < 0 ? v + range : v - range;
}

// ---------------------------------------------------------------------------
// Opsin dynamics per pixel (clbutter_comparator.cpp:708-912)
// ---------------------------------------------------------------------------

__device__ __forceinline__ void opsin_absorbance(float r, float g, float b, float out[3]) {
  out[0] = 0.348036746003f * r + 0.577814843137f * g + 0.0544556093735f * b + 0.774145581713f;
  out[1] = 0.26922717275f * r + 0.767247733938f * g + 0.0366922708552f * b + 0.920130265014f;
  out[2] = 0.0882062883536f * r + 0.158581714673f * g + 0.712857943858f * b + 10.6524069248f;
}

#ifndef GZ_CLENSHAW_2X
#define GZ_CLENSHAW_2X 1
#endif
__device__ __forceinline__ f32x2 clenshaw6x2(float x, f32x2 c0, f32x2 c1, f32x2 c2, f32x2 c3,
                                             f32x2 c4, f32x2 c5) {
  const f32x2 xx = {x, x};
  // the first step from b1 = b2 = 0 gives exactly c5 for finite x
  // ((x * 0 + x * 0) - 0 is a zero, and a zero plus c5 != 0 is c5)
  f32x2 b1 = c5, b2 = {0.0f, 0.0f}, xb, t;
#if GZ_CLENSHAW_2X
  // xb + xb of the reference's step as (2 x) * b1: doubling is exact and
  // commutes with the product's rounding (nothing here comes near the
  // subnormal range or overflow), one operation fewer per step
  const f32x2 x2 = xx + xx;
  xb = x2 * b1; t = xb - b2 + c4; b2 = b1; b1 = t;
  xb = x2 * b1; t = xb - b2 + c3; b2 = b1; b1 = t;
  xb = x2 * b1; t = xb - b2 + c2; b2 = b1; b1 = t;
  xb = x2 * b1; t = xb - b2 + c1; b2 = b1; b1 = t;
#else
  xb = xx * b1; t = (xb + xb) - b2 + c4; b2 = b1; b1 = t;
  xb = xx * b1; t = (xb + xb) - b2 + c3; b2 = b1; b1 = t;
  xb = xx * b1; t = (xb + xb) - b2 + c2; b2 = b1; b1 = t;
  xb = xx * b1; t = (xb + xb) - b2 + c1; b2 = b1; b1 = t;
#endif
  xb = xx * b1;
  return xb - b2 + c0;
}

// Correctly rounded f32 division for operands in the normal range whose
// quotient is normal (|a|, |b|, |a/b| within 2^-100 .. 2^100): the
// compiler's IEEE sequence (v_div_scale, reciprocal + one Newton step, two
// residual corrections, v_div_fmas, v_div_fixup) with the scale / fix-up
// steps dropped -- they are the identity in that range (no operand or
// quotient near the exponent limits, no zero, inf or NaN), so every value
// is the one a / b gives.  Used where the operands are bounded by
// construction (opsin absorbance >= 0.77, gamma values, MHIC mixing
// denominators >= 106).
__device__ __forceinline__ float fdiv_normal(float a, float b) {
  float y = __builtin_amdgcn_rcpf(b);
  const float e = __builtin_fmaf(-b, y, 1.0f);
  y = __builtin_fmaf(e, y, y);
  float q = a * y;
  float r = __builtin_fmaf(-b, q, a);
  q = __builtin_fmaf(r, y, q);
  r = __builtin_fmaf(-b, q, a);
  return __builtin_fmaf(r, y, q);
}

// (x - lo) / (hi - lo) of GammaPolynomialOpt as q = n * RN(1/d) plus one
// residual correction: equal to the IEEE quotient for every numerator in
// [2^-30, 2^10) (checked exhaustively over all floats of that range against
// n / d on the host; tools/micro/div_probe.hip is the device form of the
// check); here n = x - 0.77 with x the opsin absorbance, >= 0.774 and <= 256,
// so n is 0 (exact either way) or >= 2^-24.
__device__ __forceinline__ float fdiv_gamma_range(float n) {
  constexpr float d = 274.579999999999984f - 0.770000000000000f;
  constexpr float r = 1.0f / d;
  const float q = n * r;
  const float e = __builtin_fmaf(-q, d, n);
  return __builtin_fmaf(e, r, q);
}

__device__ __forceinline__ float gamma_poly(float x) {
  // GammaPolynomialOpt, :861-874 (RationalPolynomialOpt :828-859)
  const float lo = 0.770000000000000f;
  const float x01 = fdiv_gamma_range(x - lo);
  // float(2.0 * double(x01) - 1.0) == 2.0f * x01 - 1.0f: the doubled value is
  // exact, and the difference is exact in double unless |2 x01| < 2^-29,
  // where both forms give -1.0f
  const float xc = 2.0f * x01 - 1.0f;
  // numerator and denominator recursions side by side in packed f32 (each
  // half is ClenshawRecursionOpt's exact operation sequence, :806-824)
  const f32x2 r = clenshaw6x2(xc, f32x2{881.979476556478289f, 12.262350348616792f},
                              f32x2{1496.058452015812463f, 20.557285797683576f},
                              f32x2{908.662212739659481f, 12.161463238367844f},
                              f32x2{373.566100223287378f, 4.711532733641639f},
                              f32x2{85.840860336314364f, 0.899112889751053f},
                              f32x2{6.683258861509244f, 0.035662329617191f});
  const float yp = r.x, yq = r.y;
  // (the denominator polynomial is >= 1.3 on [-1, 1]; the select keeps the
  // reference's guard without a branch)
  const float g = fdiv_normal(yp, yq);
  return yq == 0.0f ? 0.0f : g;
}

// blurred: sigma-1.1 blur of the linear pixel; lin: the linear pixel.
__device__ __forceinline__ void opsin_pixel(const float blurred[3], const float lin[3],
                                            float xyb[3]) {
  float pm[3], sens[3], cm[3];
  opsin_absorbance(blurred[0], blurred[1], blurred[2], pm);
#pragma unroll
  for (int c = 0; c < 3; ++c) sens[c] = fdiv_normal(gamma_poly(pm[c]), pm[c]);
  opsin_absorbance(lin[0], lin[1], lin[2], cm);
#pragma unroll
  for (int c = 0; c < 3; ++c) cm[c] *= sens[c];
  xyb[0] = 1.01611726948f * cm[0] - 0.982482243696f * cm[1];
  xyb[1] = 1.43571362627f * cm[0] + 0.896039849412f * cm[1];
  xyb[2] = cm[2];
}

// MaskHighIntensityChangeOpt mixing for one pixel, :739-778.
// sqr_max_diff is the max over valid 4-neighbours of
// float(0.5*(c0y[n]+c1y[n]) - ave_y)^2, or -1 when none.
// The reference promotes these to double; in float they are bit-identical:
// (a + b) * 0.5 is one rounding of the exact half in both, and h - ave with
// h = 0.5 * (n0 + n1) (exact: the Y sums here are far from subnormal) is the
// correctly rounded exact difference either way (exact in double when the
// exponents are within 29 bits of each other; otherwise both round to the
// larger operand).
__device__ __forceinline__ float mhic_ave(float a, float b) { return (a + b) * 0.5f; }
__device__ __forceinline__ float mhic_sqdiff(float n0, float n1, float ave_y) {
  const float d = (n0 + n1) * 0.5f - ave_y;
  return d * d;
}
__device__ __forceinline__ void mhic_mix(const float c0[3], const float c1[3], const float ave[3],
                                         float sqr_max_diff, float x0[3], float x1[3]) {
  const float kRX = 275.19165240059317f, kRY = 18599.41286306991f;
  const float kRZ = 410.8995306951065f, kChroma = 106.95800948271017f;
  const float chroma_scale = fdiv_normal(kChroma, ave[1] + kChroma);
  const float mix[3] = {fdiv_normal(chroma_scale * kRX, sqr_max_diff + kRX),
                        fdiv_normal(kRY, sqr_max_diff + kRY),
                        fdiv_normal(chroma_scale * kRZ, sqr_max_diff + kRZ)};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    x0[c] = mix[c] * c0[c] + (1 - mix[c]) * ave[c];
    x1[c] = mix[c] * c1[c] + (1 - mix[c]) * ave[c];
  }
}

// ---------------------------------------------------------------------------
// Two pixels at once (f32x2: v_pk_* instructions, two IEEE operations each):
// every function below applies to each half exactly the operation sequence
// of its scalar form above, so each half's value is bit-identical to the
// scalar result for that pixel.  (Packed f32 halves the issue slots of the
// VALU-bound streams: round 6, profiles/round6_opsin_pair_ab.txt.)
// ---------------------------------------------------------------------------
__device__ __forceinline__ f32x2 splat2(float v) { return f32x2{v, v}; }
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 sel2(bool kx, bool ky, f32x2 a, f32x2 b) {
  return f32x2{kx ? a.x : b.x, ky ? a.y : b.y};
}

__device__ __forceinline__ void opsin_absorbance2(f32x2 r, f32x2 g, f32x2 b, f32x2 out[3]) {
  out[0] = splat2(0.348036746003f) * r + splat2(0.577814843137f) * g + splat2(0.0544556093735f) * b +
           splat2(0.774145581713f);
  out[1] = splat2(0.26922717275f) * r + splat2(0.767247733938f) * g + splat2(0.0366922708552f) * b +
           splat2(0.920130265014f);
  out[2] = splat2(0.0882062883536f) * r + splat2(0.158581714673f) * g + splat2(0.712857943858f) * b +
           splat2(10.6524069248f);
}

// fdiv_normal per half (the reciprocal per half, the corrections packed)
__device__ __forceinline__ f32x2 fdiv_normal2(f32x2 a, f32x2 b) {
  f32x2 y = {__builtin_amdgcn_rcpf(b.x), __builtin_amdgcn_rcpf(b.y)};
  const f32x2 e = fma2(-b, y, splat2(1.0f));
  y = fma2(e, y, y);
  f32x2 q = a * y;
  f32x2 r = fma2(-b, q, a);
  q = fma2(r, y, q);
  r = fma2(-b, q, a);
  return fma2(r, y, q);
}

__device__ __forceinline__ f32x2 fdiv_gamma_range2(f32x2 n) {
  constexpr float d = 274.579999999999984f - 0.770000000000000f;
  constexpr float r = 1.0f / d;
  const f32x2 q = n * splat2(r);
  const f32x2 e = fma2(-q, splat2(d), n);
  return fma2(e, splat2(r), q);
}

// clenshaw6x2's recursion for one polynomial at two points
__device__ __forceinline__ f32x2 clenshaw6_at2(f32x2 xx, float c0, float c1, float c2, float c3, float c4,
                                               float c5) {
  f32x2 b1 = splat2(c5), b2 = {0.0f, 0.0f}, xb, t;
#if GZ_CLENSHAW_2X
  const f32x2 x2 = xx + xx;  // (clenshaw6x2's doubling)
  xb = x2 * b1; t = xb - b2 + splat2(c4); b2 = b1; b1 = t;
  xb = x2 * b1; t = xb - b2 + splat2(c3); b2 = b1; b1 = t;
  xb = x2 * b1; t = xb - b2 + splat2(c2); b2 = b1; b1 = t;
  xb = x2 * b1; t = xb - b2 + splat2(c1); b2 = b1; b1 = t;
#else
  xb = xx * b1; t = (xb + xb) - b2 + splat2(c4); b2 = b1; b1 = t;
  xb = xx * b1; t = (xb + xb) - b2 + splat2(c3); b2 = b1; b1 = t;
  xb = xx * b1; t = (xb + xb) - b2 + splat2(c2); b2 = b1; b1 = t;
  xb = xx * b1; t = (xb + xb) - b2 + splat2(c1); b2 = b1; b1 = t;
#endif
  xb = xx * b1;
  return xb - b2 + splat2(c0);
}

__device__ __forceinline__ f32x2 gamma_poly2(f32x2 x) {
  const f32x2 x01 = fdiv_gamma_range2(x - splat2(0.770000000000000f));
  const f32x2 xc = splat2(2.0f) * x01 - splat2(1.0f);
  const f32x2 yp = clenshaw6_at2(xc, 881.979476556478289f, 1496.058452015812463f, 908.662212739659481f,
                                 373.566100223287378f, 85.840860336314364f, 6.683258861509244f);
  const f32x2 yq = clenshaw6_at2(xc, 12.262350348616792f, 20.557285797683576f, 12.161463238367844f,
                                 4.711532733641639f, 0.899112889751053f, 0.035662329617191f);
  const f32x2 g = fdiv_normal2(yp, yq);
  return sel2(yq.x == 0.0f, yq.y == 0.0f, splat2(0.0f), g);
}

__device__ __forceinline__ void opsin_pixel2(const f32x2 blurred[3], const f32x2 lin[3], f32x2 xyb[3]) {
  f32x2 pm[3], sens[3], cm[3];
  opsin_absorbance2(blurred[0], blurred[1], blurred[2], pm);
#pragma unroll
  for (int c = 0; c < 3; ++c) sens[c] = fdiv_normal2(gamma_poly2(pm[c]), pm[c]);
  opsin_absorbance2(lin[0], lin[1], lin[2], cm);
#pragma unroll
  for (int c = 0; c < 3; ++c) cm[c] *= sens[c];
  xyb[0] = splat2(1.01611726948f) * cm[0] - splat2(0.982482243696f) * cm[1];
  xyb[1] = splat2(1.43571362627f) * cm[0] + splat2(0.896039849412f) * cm[1];
  xyb[2] = cm[2];
}

__device__ __forceinline__ f32x2 mhic_ave2(f32x2 a, f32x2 b) { return (a + b) * splat2(0.5f); }
__device__ __forceinline__ f32x2 mhic_sqdiff2(f32x2 n0, f32x2 n1, f32x2 ave_y) {
  const f32x2 d = (n0 + n1) * splat2(0.5f) - ave_y;
  return d * d;
}
__device__ __forceinline__ void mhic_mix2(const f32x2 c0[3], const f32x2 c1[3], const f32x2 ave[3],
                                          f32x2 sqr_max_diff, f32x2 x0[3], f32x2 x1[3]) {
  const float kRX = 275.19165240059317f, kRY = 18599.41286306991f;
  const float kRZ = 410.8995306951065f, kChroma = 106.95800948271017f;
  const f32x2 chroma_scale = fdiv_normal2(splat2(kChroma), ave[1] + splat2(kChroma));
  const f32x2 mix[3] = {fdiv_normal2(chroma_scale * splat2(kRX), sqr_max_diff + splat2(kRX)),
                        fdiv_normal2(splat2(kRY), sqr_max_diff + splat2(kRY)),
                        fdiv_normal2(chroma_scale * splat2(kRZ), sqr_max_diff + splat2(kRZ))};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    x0[c] = mix[c] * c0[c] + (splat2(1.0f) - mix[c]) * ave[c];
    x1[c] = mix[c] * c1[c] + (splat2(1.0f) - mix[c]) * ave[c];
  }
}


// ---------------------------------------------------------------------------
// Colour conversion (color_transform.h:211-218) and sRGB -> linear
// ---------------------------------------------------------------------------

__device__ __forceinline__ int clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
// ToPixels' byte of a 16-bit pixel value at column x (output_image.cc:83:
// (p + 8 - (x & 1)) >> 4, stored as uint8_t)
__device__ __forceinline__ int pixel_byte(unsigned p, int x) { return ((p + 8 - (x & 1)) >> 4) & 0xff; }

// libjpeg build_ycc_rgb_table fixed-point factors FIX(x) = int(x * 2^16 + 0.5)
// (color_transform.h tables): 1.40200, 1.77200, 0.71414, 0.34414.
constexpr int kFixCrR = 91881, kFixCbB = 116130, kFixCrG = 46802, kFixCbG = 22554;

// ---------------------------------------------------------------------------
// Mask LUT stage at one pixel (MaskOpt tail, :1234-1263)
// ---------------------------------------------------------------------------

// MaskOpt's tail for one channel c of a blurred mask sample s:
// (MaskX/Y/B, MaskDcX/Y/B) * kGlobalScale^-2 -- mask_luts' operations.
__device__ __forceinline__ void mask_lut_pair(int c, float sv, float* m, float* mdc) {
  const float p = (c == 0 ? 232.206464018f : (c == 1 ? 22.9455222245f : 503.962310606f)) * sv;
  const float gs = static_cast<float>(1.0 / static_cast<double>(14.921561160295326f));
  const float gs2 = gs * gs;
  *m = interp_clamp_neg_f(c_tab.mask_lut[c], 512, p) * gs2;
  *mdc = interp_clamp_neg_f(c_tab.mask_lut[3 + c], 512, p) * gs2;
}

__device__ __forceinline__ void mask_luts(float s0, float s1, float s2, float mask[3],
                                          float mask_dc[3]) {
  const float p0 = 232.206464018f * s0, p1 = 22.9455222245f * s1, p2 = 503.962310606f * s2;
  const float gs = static_cast<float>(1.0 / static_cast<double>(14.921561160295326f));
  const float gs2 = gs * gs;
  mask[0] = interp_clamp_neg_f(c_tab.mask_lut[0], 512, p0) * gs2;
  mask[1] = interp_clamp_neg_f(c_tab.mask_lut[1], 512, p1) * gs2;
  mask[2] = interp_clamp_neg_f(c_tab.mask_lut[2], 512, p2) * gs2;
  mask_dc[0] = interp_clamp_neg_f(c_tab.mask_lut[3], 512, p0) * gs2;
  mask_dc[1] = interp_clamp_neg_f(c_tab.mask_lut[4], 512, p1) * gs2;
  mask_dc[2] = interp_clamp_neg_f(c_tab.mask_lut[5], 512, p2) * gs2;
}

// ---------------------------------------------------------------------------
// 8-point FFTs (DJB in-place FFT used by butteraugli; the exact butterfly
// sequence of clbutter_comparator.cpp:320-519 / butteraugli.cc:371-570).
// Operates on split re/im arrays of 8.
// ---------------------------------------------------------------------------

template <typename T>
__device__ __forceinline__ void fft_reorder8(T* re, T* im) {
  const T tr = re[2], ti = im[2];
  re[2] = re[3]; im[2] = im[3];
  re[3] = re[5]; im[3] = im[5];
  re[5] = re[7]; im[5] = im[7];
  re[7] = re[4]; im[7] = im[4];
  re[4] = re[1]; im[4] = im[1];
  re[1] = re[6]; im[1] = im[6];
  re[6] = tr; im[6] = ti;
}

template <typename T>
__device__ __forceinline__ void fft4_inplace(T* re, T* im) {
  T t1, t2, t3, t4, t5, t6, t7, t8;
  t5 = re[2]; t1 = re[0] - t5; t7 = re[3]; t5 += re[0]; t3 = re[1] - t7; t7 += re[1];
  t8 = t5 + t7; re[0] = t8; t5 -= t7; re[1] = t5;
  t6 = im[2]; t2 = im[0] - t6; t6 += im[0]; t5 = im[3];
  im[2] = t2 + t3; t2 -= t3; im[3] = t2;
  t4 = im[1] - t5; re[3] = t1 + t4; t1 -= t4; re[2] = t1;
  t5 += im[1]; im[0] = t6 + t5; t6 -= t5; im[1] = t6;
}

template <typename T>
__device__ __forceinline__ void fft8_inplace(T* re, T* im, T sqrt_half) {
  T t1, t2, t3, t4, t5, t6, t7, t8;
  t7 = im[4]; t4 = im[0] - t7; t7 += im[0]; im[0] = t7;
  t8 = re[6]; t5 = re[2] - t8; t8 += re[2]; re[2] = t8;
  t7 = im[6]; im[6] = t4 - t5; t4 += t5; im[4] = t4;
  t6 = im[2] - t7; t7 += im[2]; im[2] = t7;
  t8 = re[4]; t3 = re[0] - t8; t8 += re[0]; re[0] = t8;
  re[4] = t3 - t6; t3 += t6; re[6] = t3;
  t7 = re[5]; t3 = re[1] - t7; t7 += re[1]; re[1] = t7;
  t8 = im[7]; t6 = im[3] - t8; t8 += im[3]; im[3] = t8;
  t1 = t3 - t6; t3 += t6;
  t7 = im[5]; t4 = im[1] - t7; t7 += im[1]; im[1] = t7;
  t8 = re[7]; t5 = re[3] - t8; t8 += re[3]; re[3] = t8;
  t2 = t4 - t5; t4 += t5;
  t6 = t1 - t4; t8 = sqrt_half; t6 *= t8; re[5] = re[4] - t6;
  t1 += t4; t1 *= t8; im[5] = im[4] - t1;
  t6 += re[4]; re[4] = t6; t1 += im[4]; im[4] = t1;
  t5 = t2 - t3; t5 *= t8; im[7] = im[6] - t5;
  t2 += t3; t2 *= t8; re[7] = re[6] - t2;
  t2 += re[6]; re[6] = t2; t5 += im[6]; im[6] = t5;
  fft4_inplace(re, im);
  fft_reorder8(re, im);
}

template <typename T>
__device__ __forceinline__ void real_fft8(const T* in, T* re, T* im, T sqrt_half) {
  T t1, t2, t3, t5, t6, t7, t8;
  t8 = in[6]; t5 = in[2] - t8; t8 += in[2]; re[2] = t8; im[6] = -t5; im[4] = t5;
  t8 = in[4]; t3 = in[0] - t8; t8 += in[0]; re[0] = t8; re[4] = t3; re[6] = t3;
  t7 = in[5]; t3 = in[1] - t7; t7 += in[1]; re[1] = t7;
  t8 = in[7]; t5 = in[3] - t8; t8 += in[3]; re[3] = t8;
  t2 = -t5; t6 = t3 - t5; t8 = sqrt_half; t6 *= t8; re[5] = re[4] - t6;
  t1 = t3 + t5; t1 *= t8; im[5] = im[4] - t1;
  t6 += re[4]; re[4] = t6; t1 += im[4]; im[4] = t1;
  t5 = t2 - t3; t5 *= t8; im[7] = im[6] - t5;
  t2 += t3; t2 *= t8; re[7] = re[6] - t2;
  t2 += re[6]; re[6] = t2; t5 += im[6]; im[6] = t5;
  t5 = re[2]; t1 = re[0] - t5; t7 = re[3]; t5 += re[0]; t3 = re[1] - t7; t7 += re[1];
  t8 = t5 + t7; re[0] = t8; t5 -= t7; re[1] = t5;
  im[2] = t3; im[3] = -t3; re[3] = t1; re[2] = t1; im[0] = 0; im[1] = 0;
  fft_reorder8(re, im);
}

// True in every thread of the last workgroup of the launch to reach this
// point (every thread of every workgroup must call it).  Arrivals count in
// two levels -- workgroup t into arr[1 + t / 64], the last of each 64 into
// arr[0] -- and every counter is reset by its last arrival: same-address
// device atomics serialise, so one counter would take one atomic per
// workgroup in turn.  arr: 1 + ceil(groups / 64) counters, zero on entry.
// Only for data that every workgroup updates and the last one reads with
// device-scope atomics (coherent across the XCDs' L2s): the barrier waits
// for this workgroup's atomics to complete before the arrival is counted.
// No device-scope fence -- on gfx950 that writes back the XCD's L2, which
// costs more than the whole kernel.
__device__ __forceinline__ bool last_arrival(uint32_t* arr, int t, int groups) {
  __shared__ int s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's atomics acknowledged
  __syncthreads();
  if (threadIdx.x == 0) {
    const int grp = t >> 6, ngrp = (groups + 63) >> 6;
    const uint32_t gsize = static_cast<uint32_t>(min(64, groups - (grp << 6)));
    int last = 0;
    if (atomicAdd(&arr[1 + grp], 1u) == gsize - 1) {
      atomicExch(&arr[1 + grp], 0u);
      if (atomicAdd(&arr[0], 1u) == static_cast<uint32_t>(ngrp - 1)) {
        atomicExch(&arr[0], 0u);
        last = 1;
      }
    }
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

}  // namespace gz
