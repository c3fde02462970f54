// The single device translation unit of libguetzli_hip: constant tables,
// all kernels (included .inc files) and the Engine that sequences them.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off
//        -fno-gpu-flush-denormals-to-zero (see csrc/Makefile).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <list>
#include <map>
#include <condition_variable>
#include <mutex>
#include <tuple>
#include <string>
#include <vector>

#include "../runtime/engine.h"
#include "../host/thread_pool.h"
#include "gz_math.h"

namespace gz {
__constant__ GzTables c_tab;
}

#include "butteraugli_kernels.inc"
#include "scan_kernels.inc"
#include "block_zeroing.inc"
#include "block_zeroing420.inc"
#include "coeff_kernels.inc"
#include "order_kernels.inc"
#include "jpeg_kernels.inc"

namespace gz {

namespace {

// ---------------------------------------------------------------------------
// Host-side table construction (glibc exp/pow in double, as the reference).
// ---------------------------------------------------------------------------

const float kZeroingCsf[192] = {
#include "../host/zeroing_csf.inc"
};

const double kBlockCsfD[37] = {
    5.28270670524, 0.0, 0.0, 0.0, 0.3831134973, 0.676303603859, 3.58927792424, 18.6104367002,
    18.6104367002, 3.09093131948, 1.0, 0.498250875965, 0.36198671102, 0.308982169883,
    0.1312701920435, 2.37370549629, 3.58927792424, 1.0, 2.37370549629, 0.991205724152,
    1.05178802919, 0.627264168628, 0.4, 0.1312701920435, 0.676303603859, 0.498250875965,
    0.991205724152, 0.5, 0.3831134973, 0.349686450518, 0.627264168628, 0.308982169883,
    0.3831134973, 0.36198671102, 1.05178802919, 0.3831134973, 0.12,
};


// (extmul, extoff, offset, scaler, mul) of MaskX..MaskDcB, clbutter_comparator.cpp:994-1064
const float kMaskParams[6][5] = {
    {0.975741017749f, -4.25328244168f, 0.454909521427f, 0.0738288224836f, 20.8029176447f},
    {0.373995618954f, 1.5307267433f, 0.911952641929f, 1.1731667845f, 16.2447033988f},
    {0.61582234137f, -4.25376118646f, 1.05105070921f, 0.47434643535f, 31.1444967089f},
    {1.79116943438f, -3.86797479189f, 0.670960225853f, 0.486575865525f, 20.4563479139f},
    {0.212223514236f, -3.65647120524f, 1.73396799447f, 0.170392660501f, 21.6566724788f},
    {0.349376011816f, -0.894711072781f, 0.901647926679f, 0.380086095024f, 18.0373825149f},
};

int Fix16(double x) { return static_cast<int>(x * 65536.0 + 0.5); }

void BuildBlur(float sigma, float border_ratio, BlurSpec* b) {
  // BlurOpt tap construction, clbutter_comparator.cpp:60-69
  const float m = 2.25f;
  const float scaler = static_cast<float>(-1.0 / (2 * sigma * sigma));
  int diff = static_cast<int>(m * fabsf(sigma));
  if (diff < 1) diff = 1;
  b->radius = diff;
  for (int i = -diff; i <= diff; ++i)
    b->taps[i + diff] = static_cast<float>(exp(static_cast<double>(scaler * i * i)));
  int step = static_cast<int>(sigma / 3);
  b->step = step < 1 ? 1 : step;
  b->border_ratio = border_ratio;
  float wnb = 0.0f;
  for (int j = 0; j <= 2 * diff; ++j) wnb += b->taps[j];
  b->weight_no_border = wnb;
}

static_assert(kFixCrR == 91881 && kFixCbB == 116130 && kFixCrG == 46802 && kFixCbG == 22554,
              "libjpeg YCbCr->RGB fixed-point constants");

void BuildTables(GzTables* t) {
  if (Fix16(1.40200) != kFixCrR || Fix16(1.77200) != kFixCbB || Fix16(0.71414) != kFixCrG ||
      Fix16(0.34414) != kFixCbG)
    abort();  // the device forms the YCbCr tables from these constants
  memset(t, 0, sizeof(*t));
  for (int i = 0; i < 256; ++i) {
    const double lin =
        i < 11 ? i / 12.92 : 255.0 * pow(((i / 255.0) + 0.055) / 1.055, 2.4);  // gamma_correct.cc:27-33
    t->srgb[i] = static_cast<float>(lin);
    const int x = i - 128;  // libjpeg build_ycc_rgb_table (color_transform.h tables)
    t->cr_r[i] = (Fix16(1.40200) * x + 32768) >> 16;  // == (kFixCrR * x + 32768) >> 16 on the device
    t->cb_b[i] = (Fix16(1.77200) * x + 32768) >> 16;
    t->cr_g[i] = -Fix16(0.71414) * x;
    t->cb_g[i] = -Fix16(0.34414) * x + 32768;
  }
  t->hf_dx[0] = 0.0f; t->hf_dx[1] = 11.38708334481672f;
  t->hf_dy[0] = 0.0f; t->hf_dy[1] = 1.4103373714040413f;
  t->lf_dy[0] = 0.0f;
  for (int i = 2; i < 21; ++i) {
    t->hf_dx[i] = t->hf_dx[i - 1] + 14.550189611520716f;
    t->hf_dy[i] = t->hf_dy[i - 1] + 0.7084088867024f;
  }
  for (int i = 1; i < 21; ++i) t->lf_dy[i] = t->lf_dy[i - 1] + 5.2511644570349185f;
  t->hf_dy_d[0] = 0.0; t->hf_dy_d[1] = 1.4103373714040413;
  for (int i = 2; i < 21; ++i) t->hf_dy_d[i] = t->hf_dy_d[i - 1] + 0.7084088867024;
  t->lf_dy_d[0] = 0.0;
  for (int i = 1; i < 21; ++i) t->lf_dy_d[i] = t->lf_dy_d[i - 1] + 5.2511644570349185;
  for (int m = 0; m < 6; ++m) {
    const float extmul = kMaskParams[m][0], extoff = kMaskParams[m][1];
    const float offset = kMaskParams[m][2], scaler = kMaskParams[m][3], mul = kMaskParams[m][4];
    for (size_t i = 0; i < 512; ++i) {
      const float c = static_cast<float>(mul / ((0.01 * scaler * i) + offset));
      const float v = static_cast<float>(1.0 + extmul * (c + extoff));
      t->mask_lut[m][i] = v * v;
    }
  }
  for (int i = 0; i < 37; ++i) {
    t->block_csf[i] = static_cast<float>(kBlockCsfD[i]);
    t->block_csf_d[i] = kBlockCsfD[i];
    // k_block_diff2's X / B term csf[k] * 64.8f * v is (csf[k] * 64.8f) * v:
    // its first product, the same f32 multiply
    t->csf_xb[0][i] = t->block_csf[i] * 64.8f;
    t->csf_xb[1][i] = t->block_csf[i] * 2.4f;
  }
  // the AC sums' term csf_d[k] * 64.8 * sq[k] is (csf_d[k] * 64.8) * sq[k]:
  // its first product per k, formed here with the same double multiply
  for (int k = 4; k < 37; ++k) {
    t->ac_w_d[0][k - 4] = kBlockCsfD[k] * 64.8;
    t->ac_w_d[1][k - 4] = 1.0;  // Y: acc += t1[k] == acc += 1.0 * t1[k]
    t->ac_w_d[2][k - 4] = kBlockCsfD[k] * 2.4;
  }
  memcpy(t->zeroing_csf, kZeroingCsf, sizeof(kZeroingCsf));
  {
    static const uint8_t kZigZag[64] = {
        0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
        3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
        10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
        21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
    static const uint8_t kOldCsf[64] = {
        10, 10, 20, 40, 60, 70, 80, 90, 10, 20, 30, 60, 70, 80, 90, 90,
        20, 30, 60, 70, 80, 90, 90, 90, 40, 60, 70, 80, 90, 90, 90, 90,
        60, 70, 80, 90, 90, 90, 90, 90, 70, 80, 90, 90, 90, 90, 90, 90,
        80, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90};
    memcpy(t->zigzag, kZigZag, sizeof(kZigZag));
    memcpy(t->old_csf, kOldCsf, sizeof(kOldCsf));
  }
  memcpy(t->idct, kIdctM, sizeof(kIdctM));
  BuildBlur(1.1f, 0.0f, &t->blur[kSigOpsin]);
  BuildBlur(1.5f, 0.0f, &t->blur[kSigEdgeX]);
  BuildBlur(0.586f, 0.0f, &t->blur[kSigEdgeY]);
  BuildBlur(0.4f, 0.0f, &t->blur[kSigEdgeB]);
  BuildBlur(14.0f, 0.0f, &t->blur[kSigLowFreq]);
  BuildBlur(9.65781083553f, 0.0f, &t->blur[kSigMaskX]);
  BuildBlur(14.2644604355f, 0.0f, &t->blur[kSigMaskY]);
  BuildBlur(4.53358927369f, 0.0f, &t->blur[kSigMaskB]);
  BuildBlur(8.8510880283f, 0.03027655136f, &t->blur[kSigDiffmap]);
  t->blur[kSigMaskBSub] = t->blur[kSigMaskB];
  t->blur[kSigMaskBSub].step = 3;
  // blur_scale() of the sigma-1.1 blur at each position of an 8-pixel axis
  // (the 8x8-local opsin of SwitchBlock / CompareBlock); same float sum and
  // double normalisation as the device function
  {
    const BlurSpec& b = t->blur[kSigOpsin];
    for (int pos = 0; pos < 8; ++pos) {
      const int minx = pos < b.radius ? 0 : pos - b.radius;
      const int maxx = (8 < pos + b.radius + 1 ? 8 : pos + b.radius + 1) - 1;
      float weight = 0.0f;
      for (int j = minx; j <= maxx; ++j) weight += b.taps[j - pos + b.radius];
      weight = static_cast<float>((1.0 - static_cast<double>(b.border_ratio)) * weight +
                                  static_cast<double>(b.border_ratio * b.weight_no_border));
      t->opsin8_scale[pos] = static_cast<float>(1.0 / static_cast<double>(weight));
    }
  }
}

std::mutex g_tab_mu;
bool g_tab_uploaded[64] = {false};
GzTables* g_host_tab = nullptr;

const GzTables& HostTables() {
  // called under g_tab_mu
  if (!g_host_tab) {
    g_host_tab = new GzTables;
    BuildTables(g_host_tab);
  }
  return *g_host_tab;
}

inline dim3 PixGrid(int w, int h, int planes = 1) {
  return dim3((w + 255) / 256, h, planes);
}

// The blurred mask planes (in down-sampled form) at base + c * n.
inline MaskPlanes MaskPlanesOf(const float* base, size_t n, bool sub_b) {
  MaskPlanes mk{};
  for (int c = 0; c < 3; ++c) {
    mk.p[c] = base + c * n;
    mk.step[c] = HostTables().blur[c == 2 && sub_b ? kSigMaskBSub : kSigMaskX + c].step;
  }
  return mk;
}
// Wave items of k_blur_vstream: per plane (64-column group, VsRows segment).
inline int VStreamSegments(int sig, int h) {
  switch (sig) {
    case kSigLowFreq: return vstream_segments<kSigLowFreq>(h);
    case kSigMaskX: return vstream_segments<kSigMaskX>(h);
    case kSigMaskY: return vstream_segments<kSigMaskY>(h);
    case kSigMaskB: return vstream_segments<kSigMaskB>(h);
    case kSigMaskBSub: return vstream_segments<kSigMaskBSub>(h);
    default: return vstream_segments<kSigDiffmap>(h);
  }
}
inline dim3 BlurVStreamGrid(int w, int h, int planes, BlurPlanes& bp) {
  bp.nplanes = planes;
  bp.start[0] = 0;
  for (int p = 0; p < planes; ++p) {
    const int st = HostTables().blur[bp.sig[p]].step;
    const int dx = (w + st - 1) / st;
    bp.tiles[p] = (dx + kVsCols - 1) / kVsCols;
    bp.start[p + 1] = bp.start[p] + bp.tiles[p] * VStreamSegments(bp.sig[p], h);
  }
  return dim3((bp.start[planes] + 3) / 4);
}
// Outputs of one k_blur_h4 wave for a sigma.
inline int H4Outputs(int sig) {
  switch (sig) {
    case kSigLowFreq: return H4Geom<kSigLowFreq, H4K<kSigLowFreq>::K>::OUT;
    case kSigMaskX: return H4Geom<kSigMaskX, H4K<kSigMaskX>::K>::OUT;
    case kSigMaskY: return H4Geom<kSigMaskY, H4K<kSigMaskY>::K>::OUT;
    case kSigMaskB: return H4Geom<kSigMaskB, H4K<kSigMaskB>::K>::OUT;
    case kSigMaskBSub: return H4Geom<kSigMaskBSub, H4K<kSigMaskBSub>::K>::OUT;
    default: return H4Geom<kSigDiffmap, H4K<kSigDiffmap>::K>::OUT;
  }
}
// Wave items of k_blur_h4: per plane (band of H4Outputs, row).
inline dim3 BlurH4Grid(int w, int h, int planes, BlurPlanes& bp) {
  bp.nplanes = planes;
  bp.start[0] = 0;
  for (int p = 0; p < planes; ++p) {
    const int st = HostTables().blur[bp.sig[p]].step;
    const int dx = (w + st - 1) / st;
    bp.tiles[p] = (dx + H4Outputs(bp.sig[p]) - 1) / H4Outputs(bp.sig[p]);
    const int rep = bp.sig[p] == kSigDiffmap ? HRowRep<kSigDiffmap>::N : 1;
    bp.start[p + 1] = bp.start[p] + bp.tiles[p] * ((h + rep - 1) / rep);
  }
  return dim3((bp.start[planes] + 3) / 4);
}
inline RowsPlain Rows(const BlurPlanes& bp, int w) {
  RowsPlain r{};
  for (int p = 0; p < kMaxBlurPlanes; ++p) r.in[p] = bp.in[p];
  r.w = w;
  return r;
}

}  // namespace

#define GZ_HIP(call)                                   \
  do {                                                 \
    hipError_t e_ = (call);                            \
    if (e_ != hipSuccess) return Fail(#call, (int)e_); \
  } while (0)
#define GZ_LAUNCH()                                               \
  do {                                                            \
    hipError_t e_ = hipGetLastError();                            \
    if (e_ != hipSuccess) return Fail("kernel launch", (int)e_);  \
  } while (0)

// ---------------------------------------------------------------------------
// Optional per-launch timing with HIP events on the engine's stream
// (gz_profile_* in the C ABI).  Off by default; when on, every launch is
// bracketed by two events and the elapsed times are folded into a
// process-wide table after the call's final stream synchronisation.
// ---------------------------------------------------------------------------
namespace {
std::atomic<int> g_prof_on{0};
std::mutex g_prof_mu;
std::map<std::string, std::pair<long, double>> g_prof;
}  // namespace

void ProfileEnable(bool on) { g_prof_on.store(on ? 1 : 0); }
void ProfileReset() {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  g_prof.clear();
}
bool ProfileGet(const char* name, long* count, double* total_ms) {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  auto it = g_prof.find(name);
  if (it == g_prof.end()) return false;
  *count = it->second.first;
  *total_ms = it->second.second;
  return true;
}
std::string ProfileNames() {
  std::lock_guard<std::mutex> lk(g_prof_mu);
  std::string out;
  for (auto& kv : g_prof) {
    if (!out.empty()) out += ",";
    out += kv.first;
  }
  return out;
}

void Engine::ProfBegin(const char* name) {
  if (!g_prof_on.load()) return;
  hipEvent_t a = nullptr, b = nullptr;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
  hipEventRecord(a, static_cast<hipStream_t>(stream_));
  pending_.push_back({name, a, b});
}
void Engine::ProfEnd() {
  if (pending_.empty() || !g_prof_on.load()) return;
  hipEventRecord(static_cast<hipEvent_t>(pending_.back().stop), static_cast<hipStream_t>(stream_));
}
// Closes the open region `name` (begun with ProfBegin, possibly with other
// regions recorded in between).
void Engine::ProfMark(const char* name) {
  if (!g_prof_on.load()) return;
  for (auto it = pending_.rbegin(); it != pending_.rend(); ++it)
    if (it->name == name) {
      hipEventRecord(static_cast<hipEvent_t>(it->stop), static_cast<hipStream_t>(stream_));
      return;
    }
}

void Engine::ProfFlush() {
  if (pending_.empty()) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto& p : pending_) {
    float ms = 0.0f;
    if (hipEventSynchronize(static_cast<hipEvent_t>(p.stop)) == hipSuccess &&
        hipEventElapsedTime(&ms, static_cast<hipEvent_t>(p.start), static_cast<hipEvent_t>(p.stop)) == hipSuccess) {
      auto& e = g_prof[p.name];
      e.first += 1;
      e.second += ms;
    }
    hipEventDestroy(static_cast<hipEvent_t>(p.start));
    hipEventDestroy(static_cast<hipEvent_t>(p.stop));
  }
  pending_.clear();
}

#define GZ_TIMED(name, ...) \
  do {                      \
    ProfBegin(name);        \
    __VA_ARGS__;            \
    ProfEnd();              \
    GZ_LAUNCH();            \
  } while (0)

bool Engine::Fail(const char* what, int code) {
  char buf[256];
  snprintf(buf, sizeof(buf), "%s failed: %s (%d)", what,
           hipGetErrorString(static_cast<hipError_t>(code)), code);
  err_ = buf;
  failed_ = true;
  return false;
}

std::unique_ptr<Engine> Engine::Create(int device, int w, int h, std::string* err) {
  std::unique_ptr<Engine> e(new Engine);
  auto fail = [&](const std::string& m) {
    if (err) *err = m;
    return std::unique_ptr<Engine>();
  };
  if (w < 8 || h < 8 || w >= (1 << 16) || h >= (1 << 16)) return fail("unsupported image size");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail("no HIP device available");
  if (device < 0 || device >= ndev || device >= 64) return fail("bad device index");
  if (hipSetDevice(device) != hipSuccess) return fail("hipSetDevice failed");
  {
    std::lock_guard<std::mutex> lk(g_tab_mu);
    if (!g_tab_uploaded[device]) {
      const GzTables& t = HostTables();
      for (const BlurSpec& b : t.blur)
        if ((kBlurTile - 1) * b.step + 2 * b.radius + 1 + b.step > kBlurLds || 2 * b.radius + 1 > kMaxTaps ||
            b.step < 1 || b.step > 4)
          return fail("blur spec exceeds the tiled kernel's LDS span");
      for (int sig = 0; sig < kNumSigmas; ++sig)
        if (t.blur[sig].step != kBlurGeomStep[sig] || t.blur[sig].radius != kBlurGeomR[sig])
          return fail("blur geometry differs from the compiled BlurGeom table");
      for (int sig = kSigEdgeX; sig <= kSigEdgeB; ++sig)
        if (t.blur[sig].step != 1 || t.blur[sig].radius > kB2MaxR)
          return fail("edge blur spec does not fit the fused 2-D kernel");
      if (hipMemcpyToSymbol(HIP_SYMBOL(c_tab), &t, sizeof(t)) != hipSuccess)
        return fail("table upload failed");
      g_tab_uploaded[device] = true;
    }
  }
  e->device_ = device;
  e->w_ = w;
  e->h_ = h;
  e->bw_ = (w + 7) / 8;
  e->bh_ = (h + 7) / 8;
  e->nb_ = e->bw_ * e->bh_;
  e->rw_ = (w + 2) / 3;
  e->rh_ = (h + 2) / 3;
  e->n_ = static_cast<size_t>(w) * h;
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return fail("stream");
  e->stream_ = s;
  const size_t n = e->n_, rn = static_cast<size_t>(e->rw_) * e->rh_;
  const size_t nc = static_cast<size_t>(e->nb_) * 64 * 3;
  bool ok = true;
  auto alloc = [&](void** p, size_t bytes) {
    if (ok && hipMalloc(p, bytes) != hipSuccess) ok = false;
    e->bytes_ += bytes;
  };
  alloc(reinterpret_cast<void**>(&e->d_rgb_), 3 * n);
  alloc(reinterpret_cast<void**>(&e->d_orig_), nc * sizeof(int16_t));
  alloc(reinterpret_cast<void**>(&e->d_cur_), nc * sizeof(int16_t));
  alloc(reinterpret_cast<void**>(&e->d_ref_xyb_), 3 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_lin_), 3 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_px8_), n * 4);
  alloc(reinterpret_cast<void**>(&e->d_xyb_), 3 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_m0_), 3 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_m1_), 3 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_tmp_), 6 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_bl_), 6 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_ma_), 3 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_mb_), 3 * n * 4);
  alloc(reinterpret_cast<void**>(&e->d_edge_), 3 * rn * 4);
  alloc(reinterpret_cast<void**>(&e->d_dc_), 3 * rn * 4);
  alloc(reinterpret_cast<void**>(&e->d_ac_), 3 * rn * 4);
  alloc(reinterpret_cast<void**>(&e->d_resval_), rn * 4);
  alloc(reinterpret_cast<void**>(&e->d_block_max_), e->nb_ * 4);
  alloc(reinterpret_cast<void**>(&e->d_mask_scale_), 3 * e->nb_ * 4);
  alloc(&e->d_zero_out_, static_cast<size_t>(e->nb_) * 192 * sizeof(CoeffData));
  alloc(reinterpret_cast<void**>(&e->d_zero_count_), static_cast<size_t>(e->nb_) * 4);
  alloc(reinterpret_cast<void**>(&e->d_zero_order_), static_cast<size_t>(e->nb_) * 4);
  alloc(reinterpret_cast<void**>(&e->d_zero_off_), static_cast<size_t>(e->nb_ + 1) * 4);
  alloc(reinterpret_cast<void**>(&e->d_zero_nnz_), static_cast<size_t>(e->nb_) * 4);
  alloc(reinterpret_cast<void**>(&e->d_zero_bins_), 2 * kOrderBins * 4);
  alloc(reinterpret_cast<void**>(&e->d_scan_sums_), (static_cast<size_t>(e->nb_) / 4 + 2) * 4);
  alloc(reinterpret_cast<void**>(&e->d_cand_idx_), static_cast<size_t>(e->nb_) * 192);
  alloc(reinterpret_cast<void**>(&e->d_cand_err_), static_cast<size_t>(e->nb_) * 192 * 4);
  if (ok && hipHostMalloc(reinterpret_cast<void**>(&e->h_zero_off_), static_cast<size_t>(e->nb_ + 1) * 4) != hipSuccess)
    ok = false;
  if (ok && hipHostMalloc(reinterpret_cast<void**>(&e->h_coeffs_), nc * sizeof(int16_t)) != hipSuccess)
    ok = false;
  const size_t stage_groups = (3 * static_cast<size_t>(e->nb_) + kStageBlocks - 1) / kStageBlocks;
  alloc(reinterpret_cast<void**>(&e->d_jhist_), jhist_device_bytes(stage_groups));
  // worst case per MCU: 3 x (DC 16 + 11 bits, 63 x (16 + 10) bits, EOB 16) < 160 words
  e->jwords_cap_ = static_cast<size_t>(e->nb_) * 160 + 16;
  alloc(reinterpret_cast<void**>(&e->d_jwords_[0]), e->jwords_cap_ * 4);
  alloc(reinterpret_cast<void**>(&e->d_jwords_[1]), e->jwords_cap_ * 4);
  const size_t code_groups = (static_cast<size_t>(e->nb_) + kCodeMcus - 1) / kCodeMcus;
  // 0xff counters | arrival counters | status words | shared words | seam counters
  const size_t jctl_bytes = kCodeFfCopies * 8 + (1 + code_groups / 64 + 2) * 8 + code_groups * 8 +
                            code_groups * 16 + (code_groups + 1) * 4;
  alloc(reinterpret_cast<void**>(&e->d_jctl_), jctl_bytes);
  // (stage counts, chroma count, then the coder's words: kJCodeHost ..)
  const size_t jhost_bytes = 4 * (kJCodeHost + kCodeHostFf + (static_cast<size_t>(e->nb_) + kCodeMcus - 1) / kCodeMcus + 16);
  if (ok && hipHostMalloc(reinterpret_cast<void**>(&e->h_jhist_), jhost_bytes, hipHostMallocCoherent) != hipSuccess)
    ok = false;
  if (ok && hipHostGetDevicePointer(reinterpret_cast<void**>(&e->m_jhist_), e->h_jhist_, 0) != hipSuccess)
    ok = false;
  if (ok && (hipMemsetAsync(e->d_jhist_, 0, jhist_device_bytes(stage_groups), s) != hipSuccess ||
             hipMemsetAsync(e->d_jctl_, 0, jctl_bytes, s) != hipSuccess))
    ok = false;
  e->scale_stride_ = (std::max(w, h) + 63) / 64 * 64;
  alloc(reinterpret_cast<void**>(&e->d_scales_), static_cast<size_t>(kNumSigmas) * 2 * e->scale_stride_ * 4);
  // (block maxima [nb_], 4 spare words, k_diffmap's tile maxima)
  const size_t dm_groups = static_cast<size_t>((w + kDmTile - 1) / kDmTile) * ((h + kDmTile - 1) / kDmTile);
  if (ok && hipHostMalloc(reinterpret_cast<void**>(&e->h_block_max_), (e->nb_ + 4 + dm_groups) * 4,
                          hipHostMallocCoherent) != hipSuccess)
    ok = false;
  if (ok && hipHostGetDevicePointer(reinterpret_cast<void**>(&e->m_block_max_), e->h_block_max_, 0) != hipSuccess)
    ok = false;
  // k_diffmap's maxima words (the coder's skip test)
  const size_t dm_bytes = 4 * kDmMaxWords;
  alloc(reinterpret_cast<void**>(&e->d_dmax_), dm_bytes);
  if (ok && hipMemsetAsync(e->d_dmax_, 0, dm_bytes, s) != hipSuccess) ok = false;

  if (!ok) return fail("device allocation failed");
  // pinned staging (coefficients, offsets, histograms, block maxima)
  e->bytes_ += nc * sizeof(int16_t) + static_cast<size_t>(e->nb_) * 12 + 8192;
  k_blur_scales<<<dim3((e->scale_stride_ + 255) / 256, kNumSigmas * 2), 256, 0, s>>>(
      w, h, e->scale_stride_, e->d_scales_);
  if (hipGetLastError() != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return fail("blur scale precompute failed");
  return e;
}

namespace {
std::mutex g_pool_mu;
// Idle engines, most recently released first.  Intentionally leaked: idle
// engines must not be freed from a static destructor after the HIP runtime
// has shut down.
auto* g_idle = new std::list<std::unique_ptr<Engine>>;
size_t g_idle_bytes = 0;
constexpr size_t kMaxIdlePerKey = 8;

size_t PoolCapBytes() {
  static const size_t cap = [] {
    const char* v = getenv("GZ_ENGINE_POOL_BYTES");
    return v ? static_cast<size_t>(strtoull(v, nullptr, 10)) : (static_cast<size_t>(16) << 30);
  }();
  return cap;
}

// Unlinks least recently used engines until the idle set is within
// keep_bytes and every size has at most kMaxIdlePerKey; the caller destroys
// them outside the lock.  g_pool_mu held.
void EvictLocked(size_t keep_bytes, std::vector<std::unique_ptr<Engine>>* out) {
  std::map<std::tuple<int, int, int>, size_t> per_key;
  for (auto it = g_idle->begin(); it != g_idle->end();) {
    size_t& n = per_key[std::make_tuple((*it)->device(), (*it)->width(), (*it)->height())];
    if (++n > kMaxIdlePerKey) {
      g_idle_bytes -= (*it)->bytes();
      out->push_back(std::move(*it));
      it = g_idle->erase(it);
    } else {
      ++it;
    }
  }
  while (g_idle_bytes > keep_bytes && !g_idle->empty()) {
    g_idle_bytes -= g_idle->back()->bytes();
    out->push_back(std::move(g_idle->back()));
    g_idle->pop_back();
  }
}
}  // namespace

std::unique_ptr<Engine> AcquireEngine(int device, int w, int h, std::string* err) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto it = g_idle->begin(); it != g_idle->end(); ++it) {
      if ((*it)->device() == device && (*it)->width() == w && (*it)->height() == h) {
        std::unique_ptr<Engine> e = std::move(*it);
        g_idle->erase(it);
        g_idle_bytes -= e->bytes();
        return e;
      }
    }
  }
  return Engine::Create(device, w, h, err);
}

void ReleaseEngine(std::unique_ptr<Engine> e) {
  if (!e || e->failed()) return;  // a failed engine is destroyed, never reused
  std::vector<std::unique_ptr<Engine>> evicted;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_idle_bytes += e->bytes();
    g_idle->push_front(std::move(e));
    EvictLocked(PoolCapBytes(), &evicted);
  }
}

size_t TrimEnginePool(size_t keep_bytes) {
  std::vector<std::unique_ptr<Engine>> evicted;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    EvictLocked(keep_bytes, &evicted);
  }
  size_t freed = 0;
  for (const auto& e : evicted) freed += e->bytes();
  return freed;
}

size_t EnginePoolIdleBytes() {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  return g_idle_bytes;
}

// The search's end-of-candidate wait (Sync).  The runtime's event and
// stream waits poll a host core for as long as they last (measured: wait CPU
// = wait wall time, hipEventBlockingSync or not), and with several frames
// sharing a GPU a wait lasts as long as the other frames' kernels ahead of
// it.  So the stream signals the waiting thread itself: a host function
// enqueued behind the awaited work (run by the runtime's completion thread)
// sets a flag and wakes the thread, which sleeps on a condition variable.
// (Only where nothing follows in the stream: a host function holds the
// stream until it has run.  The short histogram-stage wait, which the
// Compare pass follows, stays an event wait.)  Measured at 1080p x 8 frames
// in flight: host CPU per frame -11 %, throughput within the run-to-run
// spread (profiles/round3_wait_ab.txt).
namespace {
struct StreamWaiter {
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  static void Signal(void* p) {
    StreamWaiter* w = static_cast<StreamWaiter*>(p);
    std::lock_guard<std::mutex> lk(w->mu);
    w->done = true;
    w->cv.notify_one();
  }
};
}  // namespace

static hipError_t WaitOnStream(hipStream_t s) {
  // GZ_SPIN_US > 0: poll the stream for up to that long before sleeping.
  // Most waits of the search (a Compare pass, the bulk prefix, the change
  // order) end within a few hundred us, and a polled wake-up hands the
  // frame's next work to the device sooner than the host function's.
  // Measured at 10 frames in flight (interleaved rounds,
  // profiles/round4_spin_wait_ab.txt): 235-237 MP/s sleeping at once, 239 with
  // 200-500 us of polling, 241-246 with 700-1000 us, at 0.046 / 0.056-0.066 /
  // 0.068-0.071 s of host CPU per frame -- +1-4 % for up to +55 % host CPU,
  // so the default stays the sleeping wait (0).
  //
  // Adaptive (round 5): with at most two encodes in progress in the process
  // and CPUs to spare -- one frame alone, a strip rank -- nothing competes
  // for the host cores and the wait polls for up to kSpinIdleUs first, so a
  // lone frame's many short waits (the change order, the bulk prefix, each
  // candidate) end when the work does; with more encodes in flight it
  // sleeps at once as before (the concurrent bench's CPU per frame is
  // unchanged).  GZ_SPIN_US >= 0 fixes the polling time for every wait.
  constexpr int kSpinIdleUs = 5000;
  static const int env_spin = getenv("GZ_SPIN_US") ? atoi(getenv("GZ_SPIN_US")) : -1;
  int spin_us = env_spin;
  if (spin_us < 0) {
    const int active = ActiveEncodes();
    spin_us = active <= 2 && HostThreads() - active >= 2 ? kSpinIdleUs : 0;
  }
  if (spin_us > 0) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      const hipError_t q = hipStreamQuery(s);
      if (q == hipSuccess) return hipSuccess;
      if (q != hipErrorNotReady) return q;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(spin_us)) break;
    }
  }
  StreamWaiter w;
  const hipError_t r = hipLaunchHostFunc(s, &StreamWaiter::Signal, &w);
  if (r != hipSuccess) return r;
  std::unique_lock<std::mutex> lk(w.mu);
  w.cv.wait(lk, [&] { return w.done; });
  return hipSuccess;
}

// A wait for work of unknown length (a copy or kernels that may sit behind
// other streams' work on a shared device): none if the stream is already
// idle, else the sleeping wait (the runtime's synchronisation polls a core
// for as long as it waits).
static hipError_t WaitIdle(hipStream_t s) {
  const hipError_t q = hipStreamQuery(s);
  if (q == hipSuccess) return hipSuccess;
  if (q != hipErrorNotReady) return q;
  return WaitOnStream(s);
}

Engine::~Engine() {
  if (device_ >= 0) hipSetDevice(device_);
  void* bufs[] = {d_rgb_, d_orig_, d_cur_, d_ref_xyb_, d_lin_, d_xyb_, d_m0_, d_m1_,
                  d_tmp_, d_bl_, d_ma_, d_mb_, d_edge_, d_dc_, d_ac_, d_resval_,
                  d_block_max_, d_mask_scale_, d_zero_out_, d_scales_,
                  d_zero_count_, d_zero_order_, d_zero_off_, d_cand_idx_, d_cand_err_,
                  d_jhist_, d_jwords_[0], d_jwords_[1], d_jctl_, d_zero_nnz_,
                  d_zero_bins_, d_scan_sums_, d_planes_, d_cand_rgb_, d_ord_, d_dmax_, d_px8_};
  for (void* p : bufs)
    if (p) hipFree(p);
  for (void* g : compare_graph_)
    if (g) hipGraphExecDestroy(static_cast<hipGraphExec_t>(g));
  if (stage_event_) hipEventDestroy(static_cast<hipEvent_t>(stage_event_));
  if (h_block_max_) hipHostFree(h_block_max_);
  if (h_delta_idx_) hipHostFree(h_delta_idx_);
  if (h_zero_off_) hipHostFree(h_zero_off_);
  if (h_coeffs_) hipHostFree(h_coeffs_);
  if (h_jhist_) hipHostFree(h_jhist_);
  if (h_bulk_) (void)hipHostFree(h_bulk_);
  if (h_jbytes_) hipHostFree(h_jbytes_);
  if (h_cand_idx_) hipHostFree(h_cand_idx_);
  if (h_cand_err_) hipHostFree(h_cand_err_);
  if (h_delta_val_) hipHostFree(h_delta_val_);
  if (h_ord_) hipHostFree(h_ord_);
  if (h_ord_entries_) hipHostFree(h_ord_entries_);
  if (h_win_) hipHostFree(h_win_);
  if (d_win_) hipFree(d_win_);
  if (d_ord_entries_) hipFree(d_ord_entries_);
  if (h_cbreq_) (void)hipHostFree(h_cbreq_);
  if (stream_) hipStreamDestroy(static_cast<hipStream_t>(stream_));
}

bool Engine::SetReference(const uint8_t* rgb, bool device_ptr) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  GZ_HIP(hipMemcpyAsync(d_rgb_, rgb, 3 * n_, device_ptr ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
  GZ_TIMED("ref_linear", k_rgb_to_linear<<<(n_ + 255) / 256, 256, 0, s>>>(d_rgb_, n_, d_lin_));
  {
    const int tx = (w_ + kOpTX - 1) / kOpTX, ty = (h_ + kOpTY - 1) / kOpTY;
    GZ_TIMED("ref_opsin", k_opsin2d<<<tx * ty, 256, 0, s>>>(d_lin_, w_, h_, tx, d_ref_xyb_, d_scales_,
                                                              scale_stride_));
  }
  GZ_HIP(WaitIdle(s));
  ProfFlush();
  have_mask_scale_ = false;
  return true;
}

bool Engine::SetOriginalCoeffs(const int16_t* coeffs, bool device_ptr) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  GZ_HIP(hipMemcpyAsync(d_orig_, coeffs, static_cast<size_t>(nb_) * 64 * 3 * sizeof(int16_t),
                        device_ptr ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
  GZ_HIP(WaitIdle(s));
  ProfFlush();
  return true;
}

bool Engine::ComputeOriginalCoeffs(int16_t* host_out) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  const size_t nc = static_cast<size_t>(nb_) * 64 * 3;
  GZ_TIMED("rgb_to_coeffs", k_rgb_to_coeffs<<<(3 * nb_ + 63) / 64, 64, 0, s>>>(d_rgb_, w_, h_, bw_, nb_, d_orig_));
  GZ_HIP(hipMemcpyAsync(h_coeffs_, d_orig_, nc * sizeof(int16_t), hipMemcpyDeviceToHost, s));
  GZ_HIP(WaitIdle(s));
  ProfFlush();
  memcpy(host_out, h_coeffs_, nc * sizeof(int16_t));
  return true;
}

bool Engine::UploadCoeffs(const int16_t* coeffs) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  cand_src_ = kCandCoeffs;
  GZ_HIP(hipMemcpyAsync(d_cur_, coeffs, static_cast<size_t>(nb_) * 64 * 3 * sizeof(int16_t),
                        hipMemcpyHostToDevice, s));
  return true;
}

bool Engine::CurrentFromOriginal() {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  cand_src_ = kCandCoeffs;
  GZ_HIP(hipMemcpyAsync(d_cur_, d_orig_, static_cast<size_t>(nb_) * 64 * 3 * sizeof(int16_t),
                        hipMemcpyDeviceToDevice, s));
  return true;
}

bool Engine::UploadCoeffDelta(const uint32_t* idx, const int16_t* val, size_t n) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  cand_src_ = kCandCoeffs;
  if (n == 0) return true;
  // the previous delta's kernel may still read the pinned staging
  GZ_HIP(WaitIdle(s));
  if (n > delta_cap_) {
    if (h_delta_idx_) GZ_HIP(hipHostFree(h_delta_idx_));
    if (h_delta_val_) GZ_HIP(hipHostFree(h_delta_val_));
    h_delta_idx_ = nullptr;
    h_delta_val_ = nullptr;
    delta_cap_ = 0;
    const size_t cap = std::max<size_t>(n + n / 2, 1 << 16);
    GZ_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_delta_idx_), cap * 4, hipHostMallocCoherent));
    GZ_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_delta_val_), cap * 2, hipHostMallocCoherent));
    GZ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&m_delta_idx_), h_delta_idx_, 0));
    GZ_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&m_delta_val_), h_delta_val_, 0));
    delta_cap_ = cap;
  }
  memcpy(h_delta_idx_, idx, n * 4);
  memcpy(h_delta_val_, val, n * 2);
  // the kernel reads the (index, value) pairs straight from pinned host
  // memory: no staging copies in the stream
  GZ_TIMED("scatter_coeffs", k_scatter_coeffs<<<(n + 255) / 256, 256, 0, s>>>(m_delta_idx_, m_delta_val_, n, d_cur_));
  return true;
}

bool Engine::QuantizeFromOriginal(const int q[3][64], int16_t* host_out) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  cand_src_ = kCandCoeffs;
  QuantMatrix qm;
  memcpy(qm.q, q, sizeof(qm.q));
  const size_t per = static_cast<size_t>(nb_) * 64;
  GZ_TIMED("quantize", k_quantize<<<dim3((per + 255) / 256, 3), 256, 0, s>>>(d_orig_, qm, per, d_cur_));
  if (host_out) {  // through the pinned staging: a DMA, no pageable bounce
    GZ_HIP(hipMemcpyAsync(h_coeffs_, d_cur_, 3 * per * sizeof(int16_t), hipMemcpyDeviceToHost, s));
    GZ_HIP(WaitIdle(s));
    memcpy(host_out, h_coeffs_, 3 * per * sizeof(int16_t));
  }
  ProfFlush();
  return true;
}

bool Engine::MaskPipeline(const float* xyb0, const float* xyb1, bool sub_b, bool front) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  if (front) {
    const int strips = (w_ + kMsCols - 1) / kMsCols, segs = (h_ + kMsRows - 1) / kMsRows;
    const int waves = 3 * strips * segs;
    GZ_TIMED("mask_front", k_mask_stream<<<(waves + 3) / 4, 256, 0, s>>>(xyb0, xyb1, w_, h_, strips, segs,
                                                                          kMsRows, d_mb_));
  }
  BlurPlanes bp{};
  for (int c = 0; c < 3; ++c) {
    bp.in[c] = d_mb_ + c * n_;
    bp.out[c] = d_tmp_ + c * n_;
    bp.sig[c] = c == 2 && sub_b ? kSigMaskBSub : kSigMaskX + c;
  }
  const dim3 grid2 = BlurH4Grid(w_, h_, 3, bp);  // fills bp's packed-grid fields
  GZ_TIMED("mask_blur_h", k_blur_h4<kBlurMask><<<grid2, 256, 0, s>>>(
      Rows(bp, w_), bp, w_, h_, d_scales_, scale_stride_));
  for (int c = 0; c < 3; ++c) {
    bp.in[c] = d_tmp_ + c * n_;
    bp.out[c] = d_ma_ + c * n_;
  }
  const dim3 grid3 = BlurVStreamGrid(w_, h_, 3, bp);  // fills bp's packed-grid fields
  GZ_TIMED("mask_blur_v", k_blur_vstream<kBlurMask><<<grid3, 256, 0, s>>>(bp, w_, h_, d_scales_, scale_stride_));
  return true;
}

// The kernel sequence of one Compare pass (no host synchronisation);
// captured once into a hipGraph for the plain (no debug, no profiling) case.
bool Engine::EnqueueCompare(CompareDebug* dbg) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const size_t n = n_, rn = static_cast<size_t>(rw_) * rh_;
  auto d2h = [&](float* dst, const float* src, size_t count) -> bool {
    if (!dst) return true;
    GZ_HIP(hipMemcpyAsync(dst, src, count * 4, hipMemcpyDeviceToHost, s));
    return true;
  };
  ProfBegin("compare_pass");
  // Res points that k_edge_map / k_block_diff2 skip are never read by
  // k_combine (it reads only ry + 5 < h, rx + 5 < w, all written this pass),
  // so the zeroing is only for the stage dumps, which compare whole arrays.
  if (dbg) {
    GZ_HIP(hipMemsetAsync(d_edge_, 0, 3 * rn * 4, s));
    GZ_HIP(hipMemsetAsync(d_dc_, 0, 3 * rn * 4, s));
    GZ_HIP(hipMemsetAsync(d_ac_, 0, 3 * rn * 4, s));
  }
  // S0: candidate coefficients -> sRGB pixels (packed)
  if (cand_src_ == kCandRgb) {
    GZ_TIMED("rgb_to_linear", k_rgb_to_srgb8<<<(n_ + 255) / 256, 256, 0, s>>>(d_cand_rgb_, n_, d_px8_));
  } else {
    GZ_TIMED("coeffs_to_linear", k_coeffs_to_srgb8<<<dim3((bw_ + kC2lBlocks - 1) / kC2lBlocks, bh_), 256, 0, s>>>(
        d_cur_, w_, h_, bw_, nb_, d_px8_, cand_src_ == kCand420 ? d_planes_ : nullptr));
  }
  if (dbg && dbg->cand_linear) {
    GZ_TIMED("srgb8_to_linear", k_srgb8_to_linear<<<(n_ + 255) / 256, 256, 0, s>>>(d_px8_, n_, d_lin_));
    if (!d2h(dbg->cand_linear, d_lin_, 3 * n)) return false;
  }
  // S1-S3: opsin dynamics (blur + transform) and high intensity change
  // masking, fused
  {
    static const int env_rows = getenv("GZ_OPSIN_ROWS") ? atoi(getenv("GZ_OPSIN_ROWS")) : 0;
    const int rows = env_rows > 0 ? env_rows : OpsinStreamRows(w_, h_);
    const int strips = (w_ + kOsCols - 1) / kOsCols, segs = (h_ + rows - 1) / rows;
    float* xyb_dbg = dbg && dbg->cand_xyb ? d_xyb_ : nullptr;
    GZ_TIMED("opsin_mhic", (GZ_OS_PAIR ? k_opsin_mhic_stream2 : k_opsin_mhic_stream)<<<(strips * segs + 3) / 4, 256, 0, s>>>(
        d_px8_, d_ref_xyb_, w_, h_, strips, segs, rows, d_m0_, d_m1_, xyb_dbg, d_scales_,
        scale_stride_, d_dmax_));
    if (xyb_dbg && !d2h(dbg->cand_xyb, d_xyb_, 3 * n)) return false;
  }
  if (dbg && !d2h(dbg->mhic0, d_m0_, 3 * n)) return false;
  if (dbg && !d2h(dbg->mhic1, d_m1_, 3 * n)) return false;
  // S4 + S9-S11: the edge detector's 6 step-1 blurs (radius <= 3) and the
  // mask front, fused (one read of m0 / m1): blurred planes -> d_bl_, mask
  // front -> d_mb_ (consumed by the mask blurs below)
  {
    static const int env_rows = getenv("GZ_EDGE_ROWS") ? atoi(getenv("GZ_EDGE_ROWS")) : 0;
    const int rows = env_rows > 0 ? env_rows : EdgeMaskRows(w_, h_);
    const int strips = (w_ + kEmCols - 1) / kEmCols, segs = (h_ + rows - 1) / rows;
    const int waves = 3 * strips * segs;
    GZ_TIMED("edge_mask", k_edge_mask_stream<<<(waves + 3) / 4, 256, 0, s>>>(
        d_m0_, d_m1_, w_, h_, strips, segs, rows, d_bl_, d_mb_, d_scales_, scale_stride_));
  }
  // (the search's passes compute the edge term in k_block_diff2; the stage
  // dumps keep k_edge_map, whose output they read before block_diff runs)
  static const bool fuse_env = !getenv("GZ_FUSE_EDGE") || atoi(getenv("GZ_FUSE_EDGE")) != 0;
  const bool prod = dbg && dbg->production;
  const bool fuse_edge = fuse_env && !(dbg && dbg->edge && !prod);
  if (!fuse_edge)
    GZ_TIMED("edge_map", k_edge_map<<<PixGrid(rw_, rh_), 256, 0, s>>>(d_bl_, d_bl_ + 3 * n, w_, h_, rw_, rh_, d_edge_));
  if (dbg && !fuse_edge && !d2h(dbg->edge, d_edge_, 3 * rn)) return false;
  // S6: block diff
  GZ_TIMED("block_diff", k_block_diff2<<<dim3((rw_ + kBdT - 1) / kBdT, (rh_ + kBdT - 1) / kBdT), kBd2Threads, 0, s>>>(
      d_m0_, d_m1_, w_, h_, rw_, rh_, d_dc_, d_ac_, fuse_edge ? d_bl_ : nullptr,
      fuse_edge ? d_bl_ + 3 * n : nullptr, d_edge_));
  // (the fused edge term is in d_edge_ once k_block_diff2 has run)
  if (dbg && fuse_edge && !d2h(dbg->edge, d_edge_, 3 * rn)) return false;
  if (dbg && !d2h(dbg->block_dc, d_dc_, 3 * rn)) return false;
  if (dbg && !d2h(dbg->block_ac, d_ac_, 3 * rn)) return false;
  // S7 + S12: the six sigma-14 blurs (low-frequency edge term, m0 / m1) and
  // the three mask blurs (of the mask front in d_mb_) as one horizontal and
  // one vertical launch over nine planes; then S8.  The full B mask only for
  // the stage dumps: Compare itself samples it at (3j + 3, 3i + 3) alone.
  // (raw blurred mask planes for the stage dumps of the masks and of the
  // combined value; the search's passes apply the mask LUTs per sample in
  // the vertical pass and combine without them)
  const bool full_mask = dbg && !prod && (dbg->mask || dbg->mask_dc || dbg->combined);
  // EdgeDetectorLowFreq's term is fused into k_combine_channels unless a
  // stage dump wants the AC values with it, or k_combine runs
  const bool fuse_lf = !full_mask && !(dbg && dbg->block_ac_lf && !prod);
  {
    const int st = HostTables().blur[kSigLowFreq].step;
    const size_t dn = static_cast<size_t>((w_ + st - 1) / st) * ((h_ + st - 1) / st);
    BlurPlanes bp{};
    for (int c = 0; c < 3; ++c) {
      bp.in[c] = d_m0_ + c * n;
      bp.in[3 + c] = d_m1_ + c * n;
      bp.in[6 + c] = d_mb_ + c * n;
      bp.sig[c] = bp.sig[3 + c] = kSigLowFreq;
      bp.sig[6 + c] = c == 2 && !full_mask ? kSigMaskBSub : kSigMaskX + c;
    }
    // horizontal outputs: sigma-14 planes in d_tmp_, mask planes in d_xyb_
    // (free after the opsin stage)
    for (int p = 0; p < 6; ++p) bp.out[p] = d_tmp_ + p * n;
    for (int c = 0; c < 3; ++c) bp.out[6 + c] = d_xyb_ + c * n;
    const dim3 gh = BlurH4Grid(w_, h_, 9, bp);  // fills bp's packed-grid fields
    GZ_TIMED("blur_h", k_blur_h4<kBlurLfMask><<<gh, 256, 0, s>>>(Rows(bp, w_), bp, w_, h_, d_scales_,
                                                                   scale_stride_));
    for (int p = 0; p < 9; ++p) bp.in[p] = bp.out[p];
    for (int p = 0; p < 6; ++p) bp.out[p] = d_bl_ + p * dn;
    // mask samples: the LUT pairs (masks -> d_ma_, DC masks -> d_mb_, free
    // after the h pass) -- except for the stage dumps, which want the raw
    // blurred planes (k_mask_full, k_combine)
    for (int c = 0; c < 3; ++c) {
      bp.out[6 + c] = d_ma_ + c * n;
      bp.out2[6 + c] = full_mask ? nullptr : d_mb_ + c * n;
    }
    const dim3 gv = BlurVStreamGrid(w_, h_, 9, bp);  // fills bp's packed-grid fields
    GZ_TIMED("blur_v", k_blur_vstream<kBlurLfMask><<<gv, 256, 0, s>>>(bp, w_, h_, d_scales_, scale_stride_));
    // (the search's passes add the low-frequency term in k_combine_channels)
    if (!fuse_lf)
      GZ_TIMED("low_freq", k_low_freq<<<PixGrid(rw_, rh_), 256, 0, s>>>(d_bl_, d_bl_ + 3 * dn, w_, h_, rw_, d_ac_));
  }
  if (dbg && !prod && !d2h(dbg->block_ac_lf, d_ac_, 3 * rn)) return false;
  MaskPlanes mk = MaskPlanesOf(d_ma_, n, !full_mask);
  if (dbg && full_mask && (dbg->mask || dbg->mask_dc)) {
    GZ_TIMED("mask_full_dbg", k_mask_full<<<PixGrid(w_, h_), 256, 0, s>>>(mk, w_, h_, d_mb_, d_tmp_));
    if (!d2h(dbg->mask, d_mb_, 3 * n)) return false;
    if (!d2h(dbg->mask_dc, d_tmp_, 3 * n)) return false;
  }
  // S14/S15: combine channels (+ sqrt; + the mask LUTs for the stage dumps)
  if (full_mask) {
    float* dbg_comb = nullptr;
    if (dbg->combined) dbg_comb = d_bl_;  // scratch, consumed below
    GZ_TIMED("combine", k_combine<<<PixGrid(rw_, rh_), 256, 0, s>>>(mk, d_dc_, d_ac_, d_edge_, w_, h_, rw_, rh_,
                                                 d_resval_, dbg_comb));
    if (dbg_comb && !d2h(dbg->combined, dbg_comb, rn)) return false;
  } else {
    const MaskPlanes mkdc = MaskPlanesOf(d_mb_, n, true);
    for (int c = 0; c < 3; ++c)  // (k_combine_channels indexes with compile-time steps)
      if (mk.step[c] != kMaskStepSub[c] || mkdc.step[c] != kMaskStepSub[c])
        return Fail("combine_channels: mask plane steps", hipErrorInvalidValue);
    const size_t ldn = static_cast<size_t>((w_ + kBlurGeomStep[kSigLowFreq] - 1) / kBlurGeomStep[kSigLowFreq]) *
                       ((h_ + kBlurGeomStep[kSigLowFreq] - 1) / kBlurGeomStep[kSigLowFreq]);
    GZ_TIMED("combine_channels", k_combine_channels<<<PixGrid(rw_, rh_), 256, 0, s>>>(
        mk, mkdc, d_dc_, d_ac_, d_edge_, w_, h_, rw_, rh_, d_resval_, fuse_lf ? d_bl_ : nullptr,
        fuse_lf ? d_bl_ + 3 * ldn : nullptr));
  }
  // S16/S17: diffmap blur on the (w-5)x(h-5) crop, final map, block maxima
  // and the distance, one launch
  {
    float* dm = nullptr;
    if (dbg && dbg->distmap) dm = d_bl_;
    GZ_TIMED("diffmap", k_diffmap<<<dim3((w_ + kDmTile - 1) / kDmTile, (h_ + kDmTile - 1) / kDmTile), kDmThreads, 0, s>>>(
                            d_resval_, rw_, rh_, w_, h_, bw_, bh_, d_scales_, scale_stride_, dm, d_block_max_,
                            m_block_max_ + nb_ + 4, d_dmax_));
    if (dm && !d2h(dbg->distmap, dm, n)) return false;
  }
  ProfMark("compare_pass");
  return true;
}

bool Engine::Compare(float* distance, float* block_max, CompareDebug* dbg) {
  GZ_HIP(hipSetDevice(device_));
  if (dbg) {
    if (!EnqueueCompare(dbg)) return false;
  } else if (!CompareEnqueue()) {
    return false;
  }
  if (!Sync()) return false;
  return CompareFinish(distance, block_max);
}

bool Engine::CompareEnqueue() {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (g_prof_on.load()) {
    if (!EnqueueCompare(nullptr)) return false;
  } else {
    void*& graph = compare_graph_[cand_src_];
    if (!graph) {
      hipGraph_t g = nullptr;
      GZ_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      const bool ok = EnqueueCompare(nullptr);
      const hipError_t end = hipStreamEndCapture(s, &g);
      if (!ok) {
        if (g) hipGraphDestroy(g);
        return false;
      }
      GZ_HIP(end);
      hipGraphExec_t exec = nullptr;
      const hipError_t inst = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
      hipGraphDestroy(g);
      GZ_HIP(inst);
      graph = exec;
    }
    GZ_HIP(hipGraphLaunch(static_cast<hipGraphExec_t>(graph), s));
  }
  // (k_diffmap's tile maxima reach h_block_max_ + nb_ + 4 themselves)
  return true;
}

bool Engine::Sync() {
  GZ_HIP(WaitOnStream(static_cast<hipStream_t>(stream_)));
  ProfFlush();
  return true;
}

bool Engine::CompareFinish(float* distance, float* block_max) {
  // ButteraugliScoreFromDiffmap's maximum from the tiles' (k_diffmap, mapped
  // memory), folded as the device did: fmax from +0
  const int groups = ((w_ + kDmTile - 1) / kDmTile) * ((h_ + kDmTile - 1) / kDmTile);
  const float* wg = h_block_max_ + nb_ + 4;
  float d = 0.0f;
  for (int g = 0; g < groups; ++g) d = std::fmax(d, wg[g]);
  *distance = d;
  if (block_max) {
    hipStream_t s = static_cast<hipStream_t>(stream_);
    GZ_HIP(hipSetDevice(device_));
    GZ_HIP(hipMemcpyAsync(h_block_max_, d_block_max_, static_cast<size_t>(nb_) * 4, hipMemcpyDeviceToHost, s));
    GZ_HIP(WaitIdle(s));
    memcpy(block_max, h_block_max_, static_cast<size_t>(nb_) * 4);
  }
  return true;
}

bool Engine::StartBlockComparisons(float* mask_scale_host) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  // ButteraugliComparator::StartBlockComparisons: Mask(rgb0, rgb0) with no
  // high-intensity masking (butteraugli_comparator.cc:72-79).
  if (!MaskPipeline(d_ref_xyb_, d_ref_xyb_, false)) return false;
  MaskPlanes mk = MaskPlanesOf(d_ma_, n_, false);
  GZ_TIMED("mask_scale", k_mask_scale<<<(nb_ + 255) / 256, 256, 0, s>>>(mk, w_, h_, bw_, nb_, d_mask_scale_));
  if (mask_scale_host)
    GZ_HIP(hipMemcpyAsync(mask_scale_host, d_mask_scale_, 3 * nb_ * 4, hipMemcpyDeviceToHost, s));
  GZ_HIP(hipStreamSynchronize(s));
  ProfFlush();
  have_mask_scale_ = true;
  return true;
}

// The per-request staging of CompareBlocks / CompareBlocksRgb: mapped pinned
// host memory the kernel reads the request from and writes the errors to, so
// a call is one launch and one wait (the comparator-level adapter makes one
// call per CompareBlock; three copy blits per call cost more than the kernel).
char* Engine::RequestStaging(size_t need, char** mapped) {
  if (need > cbreq_cap_) {
    if (h_cbreq_) {
      if (hipStreamSynchronize(static_cast<hipStream_t>(stream_)) != hipSuccess) return nullptr;
      (void)hipHostFree(h_cbreq_);
    }
    h_cbreq_ = nullptr;
    m_cbreq_ = nullptr;
    cbreq_cap_ = 0;
    const size_t cap = std::max<size_t>(need, 4096);
    if (hipHostMalloc(reinterpret_cast<void**>(&h_cbreq_), cap, hipHostMallocCoherent) != hipSuccess) {
      h_cbreq_ = nullptr;
      return nullptr;
    }
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&m_cbreq_), h_cbreq_, 0) != hipSuccess) return nullptr;
    cbreq_cap_ = cap;
  }
  *mapped = m_cbreq_;
  return h_cbreq_;
}

// A single request's error, posted by k_compare_block1(_rgb) into the first
// word of the staging buffer: the host polls it (the value replaces a NaN
// pattern no comparison yields), checking the stream now and then so a failed
// launch ends the wait.
static constexpr uint64_t kNoResult = ~0ull;
bool Engine::AwaitPosted(const char* h, double* err) {
  const volatile uint64_t* slot = reinterpret_cast<const volatile uint64_t*>(h);
  for (unsigned i = 1;; ++i) {
    uint64_t v = *slot;
    if (v != kNoResult) {
      memcpy(err, &v, 8);
      return true;
    }
    if ((i & 255) == 0) {
      const hipError_t q = hipStreamQuery(static_cast<hipStream_t>(stream_));
      if (q == hipSuccess) {
        v = *slot;
        if (v == kNoResult) return Fail("CompareBlock: no result posted", 0);
        memcpy(err, &v, 8);
        return true;
      }
      if (q != hipErrorNotReady) return Fail("CompareBlock", q);
    }
    __builtin_ia32_pause();
  }
}

bool Engine::CompareBlocks(int n, const int* blocks, const int16_t* cand, double* err) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (n <= 0) return true;
  for (int i = 0; i < n; ++i)
    if (blocks[i] < 0 || blocks[i] >= nb_) return Fail("CompareBlocks block index", 0);
  if (!have_mask_scale_ && !StartBlockComparisons(nullptr)) return false;
  if (n == 1) {
    char* m = nullptr;
    char* h = RequestStaging(64, &m);
    if (!h) return Fail("CompareBlocks staging", 0);
    CompareRequest q;
    q.block = blocks[0];
    memcpy(q.cand, cand, sizeof(q.cand));
    *reinterpret_cast<volatile uint64_t*>(h) = kNoResult;
    GZ_TIMED("compare_blocks", k_compare_block1<<<1, 64, 0, s>>>(q, d_rgb_, d_mask_scale_, w_, h_, bw_,
                                                                  reinterpret_cast<double*>(m)));
    if (!AwaitPosted(h, err)) return false;
    ProfFlush();
    return true;
  }
  // one staging buffer: block indices | candidates | errors
  const size_t o_cand = (static_cast<size_t>(n) * 4 + 15) & ~15ull;
  const size_t o_err = o_cand + ((static_cast<size_t>(n) * 384 + 15) & ~15ull);
  char* m = nullptr;
  char* h = RequestStaging(o_err + static_cast<size_t>(n) * 8, &m);
  if (!h) return Fail("CompareBlocks staging", 0);
  memcpy(h, blocks, static_cast<size_t>(n) * 4);
  memcpy(h + o_cand, cand, static_cast<size_t>(n) * 384);
  GZ_TIMED("compare_blocks", k_compare_blocks<<<n, 64, 0, s>>>(reinterpret_cast<const int*>(m),
                                                                reinterpret_cast<const int16_t*>(m + o_cand), n,
                                                                d_rgb_, d_mask_scale_, w_, h_, bw_,
                                                                reinterpret_cast<double*>(m + o_err)));
  GZ_HIP(hipStreamSynchronize(s));
  memcpy(err, h + o_err, static_cast<size_t>(n) * 8);
  ProfFlush();
  return true;
}

bool Engine::SetCandidateRgb(const uint8_t* rgb) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (!d_cand_rgb_) GZ_HIP(hipMalloc(reinterpret_cast<void**>(&d_cand_rgb_), 3 * n_));
  GZ_HIP(hipMemcpyAsync(d_cand_rgb_, rgb, 3 * n_, hipMemcpyHostToDevice, s));
  cand_src_ = kCandRgb;
  return true;
}

bool Engine::CompareBlocksRgb(int n, const int* blocks, const uint8_t* rgb, double* err) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (n <= 0) return true;
  for (int i = 0; i < n; ++i)
    if (blocks[i] < 0 || blocks[i] >= nb_) return Fail("CompareBlocksRgb block index", 0);
  if (!have_mask_scale_ && !StartBlockComparisons(nullptr)) return false;
  if (n == 1) {
    char* m = nullptr;
    char* h = RequestStaging(64, &m);
    if (!h) return Fail("CompareBlocksRgb staging", 0);
    CompareRequestRgb q;
    q.block = blocks[0];
    memcpy(q.rgb, rgb, sizeof(q.rgb));
    *reinterpret_cast<volatile uint64_t*>(h) = kNoResult;
    GZ_TIMED("compare_blocks_rgb", k_compare_block1_rgb<<<1, 64, 0, s>>>(q, d_rgb_, d_mask_scale_, w_, h_, bw_,
                                                                          reinterpret_cast<double*>(m)));
    if (!AwaitPosted(h, err)) return false;
    ProfFlush();
    return true;
  }
  // one staging buffer: block indices | windows | errors
  const size_t o_rgb = (static_cast<size_t>(n) * 4 + 15) & ~15ull;
  const size_t o_err = o_rgb + ((static_cast<size_t>(n) * 192 + 15) & ~15ull);
  char* m = nullptr;
  char* h = RequestStaging(o_err + static_cast<size_t>(n) * 8, &m);
  if (!h) return Fail("CompareBlocksRgb staging", 0);
  memcpy(h, blocks, static_cast<size_t>(n) * 4);
  memcpy(h + o_rgb, rgb, static_cast<size_t>(n) * 192);
  GZ_TIMED("compare_blocks_rgb",
           k_compare_blocks_rgb<<<n, 64, 0, s>>>(reinterpret_cast<const int*>(m),
                                                 reinterpret_cast<const uint8_t*>(m + o_rgb), n, d_rgb_,
                                                 d_mask_scale_, w_, h_, bw_, reinterpret_cast<double*>(m + o_err)));
  GZ_HIP(hipStreamSynchronize(s));
  memcpy(err, h + o_err, static_cast<size_t>(n) * 8);
  ProfFlush();
  return true;
}

// Diagnostics: with GZ_BZ_TRACE=path every zeroing search writes per block
// (start, end, steps) -- 100 MHz wall clock, int64 -- to path (the last
// search's, overwritten each time).
static long long* BzTraceBuf(int nb, void* stream) {
  static const char* path = getenv("GZ_BZ_TRACE");
  if (!path) return nullptr;
  static long long* buf = nullptr;
  static int cap = 0;
  if (nb > cap) {
    if (buf) hipFree(buf);
    buf = nullptr;
    if (hipMalloc(reinterpret_cast<void**>(&buf), static_cast<size_t>(nb) * 8 * kBzTraceWords) != hipSuccess) return nullptr;
    cap = nb;
  }
  (void)stream;
  return buf;
}
static void BzTraceDump(long long* buf, int nb, void* stream) {
  static const char* path = getenv("GZ_BZ_TRACE");
  if (!buf || !path) return;
  std::vector<long long> h(static_cast<size_t>(nb) * kBzTraceWords);  // (start, end, steps, list sorted[, phases])
  if (hipMemcpyAsync(h.data(), buf, h.size() * 8, hipMemcpyDeviceToHost, static_cast<hipStream_t>(stream)) != hipSuccess ||
      hipStreamSynchronize(static_cast<hipStream_t>(stream)) != hipSuccess)
    return;
  if (FILE* f = fopen(path, "wb")) {
    fwrite(h.data(), 8, h.size(), f);
    fclose(f);
  }
}

// Debug knob (GZ_BZ_LDS_PAD bytes of unused dynamic LDS) to probe how the
// zeroing search's speed depends on occupancy.
static size_t BzLdsPad() {
  static const size_t pad = getenv("GZ_BZ_LDS_PAD") ? static_cast<size_t>(atoi(getenv("GZ_BZ_LDS_PAD"))) : 0;
  return pad;
}

// offsets[0..n] = exclusive prefix sums of the device counts[0..n), on the stream.
bool Engine::ScanCounts(const int* counts, int n, int* offsets, const char* name, int* first,
                        const int* wg_totals) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  if (n > nb_) return Fail("ScanCounts size", 0);
  const unsigned chunks = static_cast<unsigned>((n + kScanChunk - 1) / kScanChunk);
  if (wg_totals) {
    // (per 256 counts, stride 2: k_order_local / k_order_near's partials)
    GZ_TIMED(name, k_scan_chunks<<<chunks, 256, 0, s>>>(counts, n, wg_totals, 2, kScanChunk / 256, offsets,
                                                         first));
    return true;
  }
  GZ_TIMED(name, (k_chunk_sums<<<chunks, 256, 0, s>>>(counts, n, d_scan_sums_),
                  k_scan_chunks<<<chunks, 256, 0, s>>>(counts, n, d_scan_sums_, 1, 1, offsets, first)));
  return true;
}

// d_zero_order_ = blocks by decreasing non-zero AC count (k_block_nnz / k_order_scatter).
bool Engine::OrderBlocks(int comp_mask) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const unsigned groups = static_cast<unsigned>((nb_ + kOrderGroup - 1) / kOrderGroup);
  GZ_HIP(hipMemsetAsync(d_zero_bins_, 0, 2 * kOrderBins * 4, s));
  GZ_TIMED("order_blocks", (k_block_nnz<<<groups, 256, 0, s>>>(d_cur_, nb_, comp_mask, d_zero_nnz_, d_zero_bins_),
                            k_order_scatter<<<groups, 256, 0, s>>>(d_zero_nnz_, nb_, d_zero_bins_,
                                                                 d_zero_bins_ + kOrderBins, d_zero_order_)));
  return true;
}

bool Engine::BlockZeroingOrders(int comp_mask, float limit, int lookahead, bool new_model,
                                CoeffDataHost* out) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  ord_cand_n_ = -1;
  if (!have_mask_scale_ && !StartBlockComparisons(nullptr)) return false;
  if (!OrderBlocks(comp_mask)) return false;
  long long* tr = BzTraceBuf(nb_, stream_);
  GZ_TIMED("block_zeroing", k_block_zeroing<<<nb_, 64, BzLdsPad(), s>>>(d_cur_, d_orig_, d_rgb_, d_mask_scale_, w_, h_, bw_, nb_,
                                     comp_mask, limit, lookahead, new_model ? 1 : 0,
                                     static_cast<CoeffData*>(d_zero_out_), d_zero_count_, d_zero_order_,
                                     nullptr, tr, 0));
  BzTraceDump(tr, nb_, stream_);
  GZ_HIP(hipMemcpyAsync(out, d_zero_out_, static_cast<size_t>(nb_) * 192 * sizeof(CoeffData),
                        hipMemcpyDeviceToHost, s));
  GZ_HIP(WaitOnStream(s));
  ProfFlush();
  return true;
}

bool Engine::BlockZeroingCandidates(int comp_mask, float limit, int lookahead, bool new_model,
                                    std::vector<int>* offsets, std::vector<uint8_t>* idx,
                                    std::vector<float>* err) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (!have_mask_scale_ && !StartBlockComparisons(nullptr)) return false;
  if (!OrderBlocks(comp_mask)) return false;
  long long* tr = BzTraceBuf(nb_, stream_);
  GZ_TIMED("block_zeroing", k_block_zeroing<<<nb_, 64, BzLdsPad(), s>>>(d_cur_, d_orig_, d_rgb_, d_mask_scale_, w_, h_, bw_, nb_,
                                     comp_mask, limit, lookahead, new_model ? 1 : 0,
                                     static_cast<CoeffData*>(d_zero_out_), d_zero_count_, d_zero_order_,
                                     nullptr, tr, 1));
  BzTraceDump(tr, nb_, stream_);
  if (!CompactCandidates(nb_, limit, offsets, idx, err, true)) return false;
  ord_cand_n_ = static_cast<int>(err->size());  // (the device change order may use them)
  return true;
}

// The kept entries of the first nblocks blocks' orders (d_zero_out_ /
// d_zero_count_), concatenated, to the host.
bool Engine::CompactCandidates(int nblocks, float limit, std::vector<int>* offsets,
                               std::vector<uint8_t>* idx, std::vector<float>* err, bool slots) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  ord_cand_n_ = -1;
  if (!ScanCounts(d_zero_count_, nblocks, d_zero_off_, "scan_counts")) return false;
  if (slots) {
    GZ_TIMED("compact_candidates", k_compact_slots<<<(nblocks + 3) / 4, 256, 0, s>>>(
        static_cast<const uint8_t*>(d_zero_out_), d_zero_count_, d_zero_off_, nblocks, d_cand_idx_,
        d_cand_err_));
  } else {
    GZ_TIMED("compact_candidates", k_compact_candidates<<<(nblocks + 3) / 4, 256, 0, s>>>(
        static_cast<const CoeffData*>(d_zero_out_), d_zero_off_, nblocks, limit, d_cand_idx_, d_cand_err_));
  }
  GZ_HIP(hipMemcpyAsync(h_zero_off_, d_zero_off_, static_cast<size_t>(nblocks + 1) * 4, hipMemcpyDeviceToHost, s));
  GZ_HIP(WaitOnStream(s));  // (behind the zeroing search: milliseconds, sleep through them)
  const size_t total = static_cast<size_t>(h_zero_off_[nblocks]);
  if (total > h_cand_cap_) {
    if (h_cand_idx_) GZ_HIP(hipHostFree(h_cand_idx_));
    if (h_cand_err_) GZ_HIP(hipHostFree(h_cand_err_));
    h_cand_idx_ = nullptr;
    h_cand_err_ = nullptr;
    h_cand_cap_ = 0;
    const size_t cap = total + total / 4 + 1024;
    GZ_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_cand_idx_), cap));
    GZ_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_cand_err_), cap * 4));
    h_cand_cap_ = cap;
  }
  if (total) {
    GZ_HIP(hipMemcpyAsync(h_cand_idx_, d_cand_idx_, total, hipMemcpyDeviceToHost, s));
    GZ_HIP(hipMemcpyAsync(h_cand_err_, d_cand_err_, total * 4, hipMemcpyDeviceToHost, s));
    GZ_HIP(WaitIdle(s));
  }
  ProfFlush();
  offsets->assign(h_zero_off_, h_zero_off_ + nblocks + 1);
  idx->assign(h_cand_idx_, h_cand_idx_ + total);
  err->assign(h_cand_err_, h_cand_err_ + total);
  return true;
}

// ---- the back end's change order (order_kernels.inc) ----
// The kernels read last_indexes (bytes) from the mapped pinned h_ord_ and
// write the totals after it; the entries stay in HBM (d_ord_entries_), where
// the selection of the bulk prefix and of the tail window reads them
// (OrderSelect); only the window, the per-block prefix counts and the
// selection's result cross to the host (mapped), or all entries when the
// host takes the exact path (OrderFetch).
namespace {
struct OrdLayout {
  size_t weight, active, info, arr, mbe, last, sel, cnt8, bytes;
  explicit OrdLayout(int nb) {
    const size_t n = static_cast<size_t>(nb), a = (n * 4 + 255) / 256 * 256;
    weight = 0;
    active = a;
    info = 2 * a;      // (unused; kept zero)
    arr = info + 256;  // k_order_build's arrival counters: 1 + groups / 64 + 1 (kBuildBlocks per group)
    mbe = arr + ((n / kBuildBlocks / 64 + 3) * 4 + 255) / 256 * 256;
    last = mbe + a;
    sel = last + a;                                         // the selection's counts and state
    cnt8 = sel + (SelLayout::words * 4 + 255) / 256 * 256;  // per-block prefix counts (bytes)
    bytes = cnt8 + (n + 255) / 256 * 256;
  }
};
// mapped pinned h_ord_: last_indexes [nb] bytes | totals [8] | below_floor | SelHost
constexpr int kOrdInfoInts = 8;
// | per k_order_build workgroup 4 ints (entries, blocks with entries, below
// the floor, the group's first entry)
size_t OrdHostBytes(int nb) {
  return static_cast<size_t>(nb) * 4 + 64 + (sizeof(SelHost) + 63) / 64 * 64 + 64 +
         16 * (static_cast<size_t>(nb) / kBuildBlocks + 1);
}
}  // namespace

bool Engine::OrderReset(bool* unavailable) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (unavailable) *unavailable = false;
  const OrdLayout L(nb_);
  if (!d_ord_) {
    // (all three buffers or none: they are committed together)
    void* d = nullptr;
    int* h = nullptr;
    int* m = nullptr;
    const bool ok =
        hipMalloc(&d, L.bytes) == hipSuccess &&
        hipHostMalloc(reinterpret_cast<void**>(&h), OrdHostBytes(nb_), hipHostMallocCoherent) == hipSuccess &&
        hipHostGetDevicePointer(reinterpret_cast<void**>(&m), h, 0) == hipSuccess &&
        hipMemsetAsync(static_cast<char*>(d) + L.info, 0, L.mbe - L.info, s) == hipSuccess &&  // totals, arrivals
        hipMemsetAsync(static_cast<char*>(d) + L.sel, 0, L.cnt8 - L.sel, s) == hipSuccess;  // (its arrivals)
    if (!ok) {
      if (d) (void)hipFree(d);
      if (h) (void)hipHostFree(h);
      (void)hipGetLastError();  // (the failed allocation's error is handled here)
      if (unavailable) {
        *unavailable = true;
        return true;
      }
      return Fail("OrderReset: device allocation failed", 0);
    }
    d_ord_ = d;
    h_ord_ = h;
    m_ord_ = m;
    bytes_ += L.bytes;
  }
  GZ_HIP(hipMemsetAsync(static_cast<char*>(d_ord_) + L.mbe, 0, static_cast<size_t>(nb_) * 4, s));
  // (the selection's counts and state: left zero by every completed build
  // and selection; cleared per frame so that an abandoned one leaves nothing)
  GZ_HIP(hipMemsetAsync(static_cast<char*>(d_ord_) + L.sel, 0, L.cnt8 - L.sel, s));
  ord_adv_dir_ = 0;
  ord_n_ = 0;
  return true;
}

bool Engine::OrderEntriesCapacity(size_t n) {
  const size_t bytes = n * sizeof(OrderEntry);
  if (bytes > d_ord_entries_cap_) {
    if (d_ord_entries_) GZ_HIP(hipFree(d_ord_entries_));
    d_ord_entries_ = nullptr;
    d_ord_entries_cap_ = 0;
    const size_t cap = bytes + bytes / 4 + 4096;
    GZ_HIP(hipMalloc(&d_ord_entries_, cap));
    d_ord_entries_cap_ = cap;
  }
  return true;
}

bool Engine::OrderBuild(int direction, int rblock, double target_distance, bool zero_bmax,
                        const std::vector<int>& last_indexes, size_t* n_entries, int* blocks_to_change,
                        float floor_limit, int64_t* below_floor) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (ord_cand_n_ < 0 || !d_ord_) return Fail("OrderBuild without candidates", 0);
  // (at most cand_n + nb entries: the buffer holds that many before
  // anything is queued)
  const size_t max_entries = static_cast<size_t>(ord_cand_n_) + static_cast<size_t>(nb_);
  if (!OrderEntriesCapacity(max_entries)) return false;
  if (static_cast<int>(last_indexes.size()) != nb_ || rblock < 1 || rblock > 4)
    return Fail("OrderBuild arguments", 0);
  const OrdLayout L(nb_);
  char* base = static_cast<char*>(d_ord_);
  uint32_t* sel = reinterpret_cast<uint32_t*>(base + L.sel);
  int adv_dir = 0;
  if (rblock == 1) {
    // last_indexes change between iterations only: the first radius copies
    // them to the device and applies the previous iteration's
    // max_block_error update (the previous build's kernels, which read the
    // staging, have completed: the host synchronised on them)
    // (as bytes: a block has at most 3 x 63 candidates; the kernel reads
    // them across PCIe, a quarter of the int array's bytes)
    uint8_t* l8 = reinterpret_cast<uint8_t*>(h_ord_);
    int bad = 0;
    for (int b = 0; b < nb_; ++b) {
      bad |= last_indexes[b] & ~0xff;
      l8[b] = static_cast<uint8_t>(last_indexes[b]);
    }
    if (bad) return Fail("OrderBuild: last index above 255", 0);
    adv_dir = ord_adv_dir_;
    ord_adv_dir_ = 0;
  }
  ord_h1_ ^= 1;  // this build's copy of the round-1 counts (zeroed by the previous build)
  BuildArgs g;
  g.bmax = d_block_max_;
  g.zero_bmax = zero_bmax ? 1 : 0;
  g.bw = bw_;
  g.bh = bh_;
  g.r = rblock;
  g.direction = direction;
  g.td = target_distance;
  g.weight = reinterpret_cast<float*>(base + L.weight);
  g.active = reinterpret_cast<const int*>(base + L.active);
  g.mbe = reinterpret_cast<float*>(base + L.mbe);
  g.adv_vt = ord_adv_vt_;
  g.adv_dir = adv_dir;
  g.copy_last = rblock == 1 ? 1 : 0;
  g.last = reinterpret_cast<int*>(base + L.last);
  g.last_host = reinterpret_cast<const uint8_t*>(m_ord_);
  g.off = d_zero_off_;
  g.cand_n = ord_cand_n_;
  g.cand_err = d_cand_err_;
  g.out = static_cast<OrderEntry*>(d_ord_entries_);
  g.h1 = sel + SelLayout::h1 + ord_h1_ * kSelBins;
  g.h1_next = sel + SelLayout::h1 + (ord_h1_ ^ 1) * kSelBins;
  SelState* st = reinterpret_cast<SelState*>(sel + SelLayout::state);
  g.reserve = &st->reserve[ord_h1_];
  g.reserve_next = &st->reserve[ord_h1_ ^ 1];
  const unsigned groups = static_cast<unsigned>((nb_ + kBuildBlocks - 1) / kBuildBlocks);
  g.wg_host = m_ord_ + nb_ + kOrdInfoInts + 16 + static_cast<int>((sizeof(SelHost) + 63) / 64 * 16);
  const int* wg = h_ord_ + nb_ + kOrdInfoInts + 16 + static_cast<int>((sizeof(SelHost) + 63) / 64 * 16);
  g.floor_limit = floor_limit;
  g.blo = ord_lo_;
  g.bhi = std::min(ord_hi_, nb_);
  ord_h1_summed_ = false;
  if (direction < 0 && (rblock > 1 || !GZ_FUSE_ACTIVE))  // (radius 1: formed by the build itself)
    GZ_TIMED("order_build", k_order_active<<<static_cast<unsigned>((nb_ + 255) / 256), 256, 0, s>>>(
                                d_block_max_, zero_bmax ? 1 : 0, bw_, bh_, rblock, target_distance,
                                reinterpret_cast<int*>(base + L.active)));
  GZ_TIMED("order_build", k_order_build<<<groups, 256, 0, s>>>(g));
  GZ_HIP(WaitOnStream(s));
  ProfFlush();
  long long tot[3] = {0, 0, 0};
  for (unsigned k = 0; k < groups; ++k)
    for (int x = 0; x < 3; ++x) tot[x] += wg[4 * k + x];
  *blocks_to_change = static_cast<int>(tot[1]);
  *n_entries = static_cast<size_t>(tot[0]);
  if (below_floor) *below_floor = tot[2];
  ord_n_ = *n_entries;
  return true;
}

bool Engine::OrderFetch(std::pair<int, float>* out, size_t n) {
  static_assert(sizeof(OrderEntry) == sizeof(std::pair<int, float>), "entry layout");
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (!n) return true;
  if (n != ord_n_) return Fail("OrderFetch entry count", 0);
  const size_t bytes = n * sizeof(OrderEntry);
  if (bytes > h_ord_entries_cap_) {
    if (h_ord_entries_) GZ_HIP(hipHostFree(h_ord_entries_));
    h_ord_entries_ = nullptr;
    h_ord_entries_cap_ = 0;
    const size_t cap = bytes + bytes / 4 + 4096;
    GZ_HIP(hipHostMalloc(&h_ord_entries_, cap));
    h_ord_entries_cap_ = cap;
  }
  GZ_HIP(hipMemcpyAsync(h_ord_entries_, d_ord_entries_, bytes, hipMemcpyDeviceToHost, s));
  GZ_HIP(WaitIdle(s));
  ProfFlush();
  // the build groups entries by workgroup in arrival order (blocks in order
  // within a group, a block's entries in k order), each group's position
  // from its reservation: the groups copied in workgroup order restore the
  // block order of the host's loop (one sequential pass; round 5 sorted by
  // block with a counting sort, 40 ms per fetch at 8192^2)
  const auto* src = static_cast<const std::pair<int, float>*>(h_ord_entries_);
  const int* wg = h_ord_ + nb_ + kOrdInfoInts + 16 + static_cast<int>((sizeof(SelHost) + 63) / 64 * 16);
  const int groups = (nb_ + kBuildBlocks - 1) / kBuildBlocks;
  size_t at = 0;
  for (int g = 0; g < groups; ++g) {
    const int cnt = wg[4 * g], base = wg[4 * g + 3];
    if (cnt == 0) continue;
    if (cnt < 0 || base < 0 || static_cast<size_t>(base) + cnt > n || at + cnt > n)
      return Fail("OrderFetch: workgroup ranges", 0);
    memcpy(static_cast<void*>(out + at), src + base, static_cast<size_t>(cnt) * sizeof(OrderEntry));
    at += static_cast<size_t>(cnt);
  }
  if (at != n) return Fail("OrderFetch: entry count", 0);
  return true;
}

bool Engine::BulkCountsStaging() {
  if (h_bulk_) return true;
  void* h = nullptr;
  void* m = nullptr;
  if (hipHostMalloc(&h, static_cast<size_t>(nb_) + 64, hipHostMallocCoherent) != hipSuccess) {
    return Fail("BulkApply: pinned allocation failed", 0);
  }
  if (hipHostGetDevicePointer(&m, h, 0) != hipSuccess) {
    (void)hipHostFree(h);
    return Fail("BulkApply: mapped address", 0);
  }
  h_bulk_ = static_cast<uint8_t*>(h);
  m_bulk_ = static_cast<uint8_t*>(m);
  bytes_ += static_cast<size_t>(nb_) + 64;
  return true;
}

bool Engine::BulkApplyEnqueue(int direction, const int quant[3][64], const uint8_t* cnt_dev, const uint32_t* sel,
                              const uint8_t* last8, uint8_t* cnt_host) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const OrdLayout L(nb_);
  QuantMatrix qm;
  memcpy(qm.q, quant, sizeof(qm.q));
  JpegQuantF qf;
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 64; ++k) qf.qz[c][k] = static_cast<float>(quant[c][c_natural_order[k]]);
  // (round 4 capped the grid at the histogram stage's arrival counters; kept)
  const size_t stage_groups = (3 * static_cast<size_t>(nb_) + kStageBlocks - 1) / kStageBlocks;
  const unsigned groups = static_cast<unsigned>(
      std::min(stage_groups, (static_cast<size_t>(nb_) + kBulkWaves - 1) / kBulkWaves));
  GZ_TIMED("bulk_apply", k_bulk_apply<<<groups, kBulkThreads, 0, s>>>(
      cnt_dev, reinterpret_cast<const int*>(static_cast<char*>(d_ord_) + L.last), d_zero_off_, ord_cand_n_,
      d_cand_idx_, nb_, direction, d_orig_, qm, qf, d_cur_, d_jhist_, sel, last8, cnt_host),
      k_hist_fold<<<1, 1024, 0, s>>>(d_jhist_, m_jhist_, 0));
  return true;
}

bool Engine::BulkApply(int direction, const int quant[3][64], const uint8_t* cnt, int32_t delta[3][256],
                       const std::vector<int>* last_indexes) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (last_indexes && !d_ord_ && !OrderReset()) return false;  // (the staging for the bytes)
  if (ord_cand_n_ < 0 || !d_ord_) return Fail("BulkApply without a change order", 0);
  if (!BulkCountsStaging()) return false;
  // (the previous BulkApply's kernel, which read the staging, has completed:
  // its histograms were waited for)
  memcpy(h_bulk_, cnt, static_cast<size_t>(nb_));
  const uint8_t* last8 = nullptr;
  if (last_indexes) {
    if (static_cast<int>(last_indexes->size()) != nb_) return Fail("BulkApply: last indexes", 0);
    uint8_t* l8 = reinterpret_cast<uint8_t*>(h_ord_);
    int bad = 0;
    for (int b = 0; b < nb_; ++b) {
      bad |= (*last_indexes)[b] & ~0xff;
      l8[b] = static_cast<uint8_t>((*last_indexes)[b]);
    }
    if (bad) return Fail("BulkApply: last index above 255", 0);
    last8 = reinterpret_cast<const uint8_t*>(m_ord_);
  }
  if (!BulkApplyEnqueue(direction, quant, m_bulk_, nullptr, last8, nullptr)) return false;
  // (a sleeping wait: nothing else of this frame is queued behind it)
  GZ_HIP(WaitOnStream(s));
  ProfFlush();
  for (int c = 0; c < 3; ++c)
    for (int i = 0; i < 256; ++i) delta[c][i] = static_cast<int32_t>(h_jhist_[(2 * c + 1) * 256 + i]);
  return true;
}

// k_sel_finish's dynamic LDS: the sorted keys, the scatter's copy, the bucket counts
static size_t SelCollectLds(int cap) {
  return 2 * static_cast<size_t>(cap) * sizeof(unsigned long long) + (kSelSortBins + 1) * sizeof(uint32_t);
}

bool Engine::OrderSelect(size_t bulk, size_t window, int direction, const int quant[3][64], bool apply,
                         OrderSelection* out, int32_t delta[3][256]) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (ord_cand_n_ < 0 || !d_ord_) return Fail("OrderSelect without a change order", 0);
  const size_t n = ord_n_;
  if ((ord_x_ ? ord_frame_n_ : n) == 0 || bulk >= (ord_x_ ? ord_frame_n_ : n) || window == 0)
    return Fail("OrderSelect arguments", 0);
  if (!BulkCountsStaging()) return false;
  // (the candidates -- the window and the ties at its ends -- are sorted in
  // one workgroup's LDS: at most kSelCandMax; more and the host takes the
  // exact path)
  window = std::min<size_t>(window, kSelCandMax / 2);
  if (!h_win_) {
    GZ_HIP(hipHostMalloc(&h_win_, kSelCandMax * sizeof(OrderEntry), hipHostMallocCoherent));
    GZ_HIP(hipHostGetDevicePointer(&m_win_, h_win_, 0));
    GZ_HIP(hipMalloc(&d_win_, kSelCandMax * sizeof(unsigned long long)));
    bytes_ += kSelCandMax * sizeof(unsigned long long);
    GZ_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_sel_finish),
                               hipFuncAttributeMaxDynamicSharedMemorySize,
                               static_cast<int>(SelCollectLds(kSelCandMax))));
  }
  // the sort's capacity: twice the window, 1024 .. kSelCandMax (LDS sized per launch)
  int cap = 1024;
  while (static_cast<size_t>(cap) < 2 * window && cap < kSelCandMax) cap <<= 1;
  const OrdLayout L(nb_);
  char* base = static_cast<char*>(d_ord_);
  uint32_t* sel = reinterpret_cast<uint32_t*>(base + L.sel);
  uint8_t* cnt8 = reinterpret_cast<uint8_t*>(base + L.cnt8);
  const OrderEntry* e = static_cast<const OrderEntry*>(d_ord_entries_);
  const int has_prefix = bulk > 0 ? 1 : 0;
  // (a frame split over ranks: ranks of the frame's order; this engine's
  // entries are its owned blocks')
  const size_t fn = ord_x_ ? ord_frame_n_ : n;
  const long long ta = static_cast<long long>(bulk) - 1;
  const long long tb = static_cast<long long>(std::min(fn - 1, bulk + window - 1));
  SelHost* host = reinterpret_cast<SelHost*>(h_ord_ + nb_ + kOrdInfoInts + 16);
  SelHost* mhost = reinterpret_cast<SelHost*>(m_ord_ + nb_ + kOrdInfoInts + 16);
  host->done = 0;
  // (GZ_SELECT_OPEN=1: every prefix reported open -- tests of the exact path)
  static const int force_open = getenv("GZ_SELECT_OPEN") ? atoi(getenv("GZ_SELECT_OPEN")) : 0;
  const size_t chunks = (n + 1023) / 1024;
  const unsigned rgroups = static_cast<unsigned>(std::max<size_t>(1, std::min<size_t>(512, chunks)));
  // (k_sel_collect: every workgroup first picks the 24-bit bins from round
  // 2's counts -- 32 KiB of reads and two barriers -- so the grid stays at
  // one round of resident 1024-lane workgroups, 2 per CU, each looping over
  // its share of the entries, instead of one workgroup per 1024 entries: at
  // 1080p 2050 workgroups paid that pick in 4 rounds)
  static const size_t cmax = getenv("GZ_SEL_CGROUPS") ? static_cast<size_t>(atoi(getenv("GZ_SEL_CGROUPS"))) : 512;
  const unsigned cgroups = static_cast<unsigned>(std::max<size_t>(1, std::min<size_t>(cmax, chunks)));
  uint32_t* h1 = sel + SelLayout::h1 + ord_h1_ * kSelBins;
  const int blo = ord_x_ ? ord_lo_ : 0, bhi = ord_x_ ? std::min(ord_hi_, nb_) : nb_;
  const int gbase = ord_x_ ? ord_gbase_ : 0;
  if (!ord_x_) {
    GZ_TIMED("order_select",
             (k_sel_refine<<<rgroups, 256, 0, s>>>(e, static_cast<int>(n), has_prefix, ta, tb, h1, sel,
                                                    reinterpret_cast<uint32_t*>(cnt8), (nb_ + 3) / 4),
              k_sel_collect<<<cgroups, kSelThreads, 0, s>>>(e, static_cast<int>(n), has_prefix,
                                                             static_cast<long long>(bulk), ta, tb, sel,
                                                             reinterpret_cast<uint32_t*>(cnt8),
                                                             static_cast<unsigned long long*>(d_win_), cap),
              k_sel_finish<<<1, kSelThreads, SelCollectLds(cap), s>>>(
                  static_cast<int>(n), has_prefix, static_cast<long long>(bulk), sel,
                  reinterpret_cast<uint32_t*>(cnt8), static_cast<const unsigned long long*>(d_win_), cap,
                  static_cast<OrderEntry*>(m_win_), mhost, force_open, 0, 0, nb_)));
  } else if (!OrderSelectSplit(e, n, fn, has_prefix, bulk, ta, tb, cap, rgroups, cgroups, force_open, gbase, blo,
                               bhi)) {
    return false;
  }
  if (has_prefix && apply && !BulkApplyEnqueue(direction, quant, cnt8, sel, nullptr, m_bulk_)) return false;
  GZ_HIP(WaitOnStream(s));
  ProfFlush();
  if (!host->done) return Fail("OrderSelect: no result", 0);
  out->kbits[0] = host->kbits[0];
  out->kbits[1] = host->kbits[1];
  out->below = host->below;
  out->eq = host->eq;
  out->straddle = host->straddle != 0;
  out->take = host->take;
  out->tie_block = host->tie_block;
  out->open = host->open != 0;
  out->applied = has_prefix && apply && !out->open;
  out->window_n = static_cast<size_t>(host->cand_n);
  // (GZ_SEL_OVERFLOW=1: every window reported overflowed -- tests of the
  // back end's path without a window, the bulk prefix applied or not)
  static const int force_overflow = getenv("GZ_SEL_OVERFLOW") ? atoi(getenv("GZ_SEL_OVERFLOW")) : 0;
  out->window_overflow = host->overflow != 0 || force_overflow;
  out->window_last = host->window_last != 0;
  if (out->applied) out->cnt.assign(h_bulk_, h_bulk_ + nb_);
  else out->cnt.clear();
  out->window.clear();
  out->window_ok = 0;
  if (!out->window_overflow && !out->open) {
    const auto* src = static_cast<const std::pair<int, float>*>(h_win_);
    out->window.assign(src, src + host->win_out);
    out->window_ok = static_cast<size_t>(host->win_ok);
  }
  if (out->applied)
    for (int c = 0; c < 3; ++c)
      for (int i = 0; i < 256; ++i) delta[c][i] = static_cast<int32_t>(h_jhist_[(2 * c + 1) * 256 + i]);
  return true;
}

// The selection of a frame split over ranks (SetOrderScope): the launches
// of OrderSelect with the exchanges between them -- this build's round-1
// counts summed once, round 2's summed, the candidates gathered from every
// rank (frame block indices) -- then the final step alike on every rank.
bool Engine::OrderSelectSplit(const void* entries, size_t n, size_t fn, int has_prefix, size_t bulk, long long ta,
                              long long tb, int cap, unsigned rgroups, unsigned cgroups, int force_open, int gbase,
                              int blo, int bhi) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  const OrderEntry* e = static_cast<const OrderEntry*>(entries);
  const OrdLayout L(nb_);
  char* base = static_cast<char*>(d_ord_);
  uint32_t* sel = reinterpret_cast<uint32_t*>(base + L.sel);
  uint32_t* cnt32 = reinterpret_cast<uint32_t*>(base + L.cnt8);
  uint32_t* h1 = sel + SelLayout::h1 + ord_h1_ * kSelBins;
  SelState* st = reinterpret_cast<SelState*>(sel + SelLayout::state);
  SelHost* mhost = reinterpret_cast<SelHost*>(m_ord_ + nb_ + kOrdInfoInts + 16);
  std::vector<uint32_t> h(2 * kSelBins);
  // (a local failure still takes part in the exchange, with its status)
  auto sum_counts = [&](bool ok, uint32_t* dev, int count) -> bool {
    if (ok) ok = hipMemcpyAsync(h.data(), dev, count * 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
                 WaitIdle(s) == hipSuccess;
    if (!ord_x_->SumU32(ok, h.data(), count)) return Fail("OrderSelect: exchange", 0);
    if (!ok) return Fail("OrderSelect: counts", 0);
    GZ_HIP(hipMemcpyAsync(dev, h.data(), count * 4, hipMemcpyHostToDevice, s));
    return true;
  };
  if (!ord_h1_summed_) {
    if (!sum_counts(true, h1, kSelBins)) return false;
    ord_h1_summed_ = true;
  }
  bool ok = true;
  GZ_TIMED("order_select", k_sel_refine<<<rgroups, 256, 0, s>>>(e, static_cast<int>(n), has_prefix, ta, tb, h1, sel,
                                                                 cnt32, (nb_ + 3) / 4));
  if (!sum_counts(ok, sel + SelLayout::h2, 2 * kSelBins)) return false;
  GZ_TIMED("order_select", k_sel_collect<<<cgroups, kSelThreads, 0, s>>>(
                               e, static_cast<int>(n), has_prefix, static_cast<long long>(bulk), ta, tb, sel, cnt32,
                               static_cast<unsigned long long*>(d_win_), cap));
  // this rank's candidates (their count first: more than `cap` and the
  // merged count alone tells every rank the selection overflowed)
  int nc = 0;
  ok = hipMemcpyAsync(&nc, &st->cand_n, 4, hipMemcpyDeviceToHost, s) == hipSuccess && WaitIdle(s) == hipSuccess;
  std::vector<unsigned long long> mine(1, 0ull), all;
  if (ok && nc > 0 && nc <= cap) {
    mine.resize(1 + static_cast<size_t>(nc));
    ok = hipMemcpyAsync(mine.data() + 1, d_win_, static_cast<size_t>(nc) * 8, hipMemcpyDeviceToHost, s) == hipSuccess &&
         WaitIdle(s) == hipSuccess;
    for (int i = 1; i <= nc; ++i) {
      const unsigned long long v = mine[i];
      mine[i] = (v & 0xffffffff00000000ull) | static_cast<uint32_t>(static_cast<int>(v & 0xffffffffu) + gbase);
    }
  }
  mine[0] = static_cast<unsigned long long>(std::max(nc, 0));
  if (!ord_x_->Gather(ok, mine, &all)) return Fail("OrderSelect: candidate exchange", 0);
  if (!ok) return Fail("OrderSelect: candidates", 0);
  // every rank's block: [count, candidates...]
  std::vector<unsigned long long> merged;
  size_t total = 0;
  for (size_t p = 0; p < all.size();) {
    const size_t c = static_cast<size_t>(all[p]);
    total += c;
    const size_t have = c <= static_cast<size_t>(cap) ? c : 0;
    if (p + 1 + have > all.size()) return Fail("OrderSelect: candidate blocks", 0);
    merged.insert(merged.end(), all.begin() + p + 1, all.begin() + p + 1 + have);
    p += 1 + have;
  }
  const int ntot = static_cast<int>(std::min<size_t>(total, 0x7fffffff));
  if (total <= static_cast<size_t>(cap) && total)
    GZ_HIP(hipMemcpyAsync(d_win_, merged.data(), total * 8, hipMemcpyHostToDevice, s));
  GZ_HIP(hipMemcpyAsync(&st->cand_n, &ntot, 4, hipMemcpyHostToDevice, s));
  GZ_TIMED("order_select", k_sel_finish<<<1, kSelThreads, SelCollectLds(cap), s>>>(
                               static_cast<int>(fn), has_prefix, static_cast<long long>(bulk), sel, cnt32,
                               static_cast<const unsigned long long*>(d_win_), cap,
                               static_cast<OrderEntry*>(m_win_), mhost, force_open, gbase, blo, bhi));
  // (the pageable sources above: the copies are done when the calls return;
  // ntot lives until the finish launch has read it)
  GZ_HIP(WaitIdle(s));
  return true;
}

bool Engine::SetBlockMax(const float* bmax) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  GZ_HIP(hipMemcpyAsync(d_block_max_, bmax, static_cast<size_t>(nb_) * 4, hipMemcpyHostToDevice, s));
  GZ_HIP(WaitIdle(s));
  return true;
}

// (applied by the next OrderBuild's first radius, before it overwrites the
// weights)
bool Engine::OrderAdvance(float val_threshold, int direction) {
  if (!d_ord_) return Fail("OrderAdvance without OrderReset", 0);
  ord_adv_vt_ = val_threshold;
  ord_adv_dir_ = direction;
  return true;
}

bool Engine::SetOriginal420(const int16_t* y, const int16_t* cb, const int16_t* cr) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  cbw_ = (w_ + 15) / 16;
  cbh_ = (h_ + 15) / 16;
  const size_t per = static_cast<size_t>(nb_) * 64, cper = static_cast<size_t>(cbw_) * cbh_ * 64;
  GZ_HIP(hipMemcpyAsync(d_orig_, y, per * 2, hipMemcpyHostToDevice, s));
  GZ_HIP(hipMemcpyAsync(d_orig_ + per, cb, cper * 2, hipMemcpyHostToDevice, s));
  GZ_HIP(hipMemcpyAsync(d_orig_ + 2 * per, cr, cper * 2, hipMemcpyHostToDevice, s));
  GZ_HIP(hipStreamSynchronize(s));
  return true;
}

bool Engine::Set420(const int16_t* y, const int16_t* cb, const int16_t* cr, const uint16_t* plane_cb,
                    const uint16_t* plane_cr) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  cbw_ = (w_ + 15) / 16;
  cbh_ = (h_ + 15) / 16;
  if (!d_planes_) GZ_HIP(hipMalloc(reinterpret_cast<void**>(&d_planes_), 2 * n_ * sizeof(uint16_t)));
  const size_t per = static_cast<size_t>(nb_) * 64, cper = static_cast<size_t>(cbw_) * cbh_ * 64;
  // (pageable sources: the copies are done when the calls return)
  GZ_HIP(hipMemcpyAsync(d_cur_, y, per * 2, hipMemcpyHostToDevice, s));
  GZ_HIP(hipMemcpyAsync(d_cur_ + per, cb, cper * 2, hipMemcpyHostToDevice, s));
  GZ_HIP(hipMemcpyAsync(d_cur_ + 2 * per, cr, cper * 2, hipMemcpyHostToDevice, s));
  GZ_HIP(hipMemcpyAsync(d_planes_, plane_cb, n_ * 2, hipMemcpyHostToDevice, s));
  GZ_HIP(hipMemcpyAsync(d_planes_ + n_, plane_cr, n_ * 2, hipMemcpyHostToDevice, s));
  cand_src_ = kCand420;
  return true;
}

bool Engine::BlockZeroingCandidates420(int comp_mask, float limit, int lookahead, bool new_model,
                                       std::vector<int>* offsets, std::vector<uint8_t>* idx,
                                       std::vector<float>* err, uint16_t* plane_cb,
                                       uint16_t* plane_cr) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (cand_src_ != kCand420) return Fail("BlockZeroingCandidates420 without Set420", 0);
  if (!have_mask_scale_ && !StartBlockComparisons(nullptr)) return false;
  if (comp_mask == 1) {
    if (!OrderBlocks(1)) return false;
    GZ_TIMED("block_zeroing", k_block_zeroing<<<nb_, 64, BzLdsPad(), s>>>(
        d_cur_, d_orig_, d_rgb_, d_mask_scale_, w_, h_, bw_, nb_, 1, limit, lookahead, new_model ? 1 : 0,
        static_cast<CoeffData*>(d_zero_out_), d_zero_count_, d_zero_order_, d_planes_, nullptr, 1));
    return CompactCandidates(nb_, limit, offsets, idx, err, true);
  }
  if (comp_mask != 6) return Fail("BlockZeroingCandidates420 comp_mask", 0);
  // wavefronts t = bx + 2 by (block_zeroing420.inc); by in
  // [max(0, ceil((t - cbw + 1) / 2)), min(cbh - 1, t / 2)]
  ProfBegin("block_zeroing420");
  for (int t = 0; t <= (cbw_ - 1) + 2 * (cbh_ - 1); ++t) {
    const int lo = std::max(0, (t - (cbw_ - 1) + 1) / 2), hi = std::min(cbh_ - 1, t / 2);
    if (lo > hi) continue;
    k_block_zeroing420<<<hi - lo + 1, kZ4Threads, 0, s>>>(d_cur_, d_orig_, d_rgb_, d_mask_scale_, w_, h_, bw_, nb_,
                                                  cbw_, t, lo, limit, lookahead, new_model ? 1 : 0, d_planes_,
                                                  static_cast<CoeffData*>(d_zero_out_), d_zero_count_);
    GZ_HIP(hipGetLastError());
  }
  ProfEnd();
  if (!CompactCandidates(cbw_ * cbh_, limit, offsets, idx, err)) return false;
  GZ_HIP(hipMemcpyAsync(plane_cb, d_planes_, n_ * 2, hipMemcpyDeviceToHost, s));
  GZ_HIP(hipMemcpyAsync(plane_cr, d_planes_ + n_, n_ * 2, hipMemcpyDeviceToHost, s));
  GZ_HIP(hipStreamSynchronize(s));
  return true;
}

bool Engine::JpegStage(const int q[3][64], uint32_t* hist, uint64_t* chroma_nz) {
  return JpegStageEnqueue(q) && JpegStageWait(hist, chroma_nz);
}

bool Engine::JpegStageEnqueue(const int q[3][64]) { return JpegStageEnqueueRange(q, 0, nb_); }

bool Engine::JpegStageEnqueueRange(const int q[3][64], int m0, int m1) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (m0 < 0 || m1 > nb_ || m1 <= m0) return Fail("JpegStage block range", 0);
  if (!stage_event_) {
    hipEvent_t ev;
    GZ_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    stage_event_ = ev;
  }
  JpegQuantF qf;
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 64; ++k) qf.qz[c][k] = static_cast<float>(q[c][c_natural_order[k]]);
  // (the device counts are zero: cleared at creation, and by every fold
  // after it has published them to h_jhist_)
  GZ_TIMED("jpeg_stage", (k_jpeg_stage<<<(3 * (m1 - m0) + kStageBlocks - 1) / kStageBlocks, kStageThreads, 0, s>>>(
                              d_cur_, qf, nb_, m0, m1, d_jhist_),
                          k_hist_fold<<<1, 1024, 0, s>>>(d_jhist_, m_jhist_, 1)));
  GZ_HIP(hipEventRecord(static_cast<hipEvent_t>(stage_event_), s));
  return true;
}

bool Engine::JpegStageWait(uint32_t* hist, uint64_t* chroma_nz) {
  GZ_HIP(hipEventSynchronize(static_cast<hipEvent_t>(stage_event_)));
  memcpy(hist, h_jhist_, 6 * 256 * 4);
  uint64_t nz;
  memcpy(&nz, h_jhist_ + 6 * 256, 8);
  *chroma_nz = nz;
  return true;
}

bool Engine::JpegScan(int ncomp, const int q[3][64], const JpegCodeTables& codes, uint64_t* nbits,
                      uint64_t* ff) {
  return JpegScanEnqueue(ncomp, q, codes) && Sync() && JpegScanFinish(nbits, ff);
}

// (the caller has synchronised since the previous scan: the pinned code
// staging is free)
bool Engine::JpegScanEnqueue(int ncomp, const int q[3][64], const JpegCodeTables& codes, float skip_at) {
  return JpegScanEnqueueRange(ncomp, q, codes, 0, nb_, 0, true, skip_at);
}

bool Engine::JpegScanEnqueueRange(int ncomp, const int q[3][64], const JpegCodeTables& codes, int m0, int m1,
                                  uint64_t base, bool pad_end, float skip_at) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  if (ncomp < 1 || ncomp > 3) return Fail("JpegScan component count", 0);
  if (m0 < 0 || m1 > nb_ || m1 <= m0) return Fail("JpegScan block range", 0);
  JpegCodesArg dc;
  for (int c = 0; c < 3; ++c) {
    for (int i = 0; i < 256; ++i) {
      // (an absent symbol's length is 0 or 255: HuffCodeTable's fill)
      if (i >= kJDcSyms && codes.dc_len[c][i] >= 1 && codes.dc_len[c][i] <= 16)
        return Fail("JpegScan DC category above 16", 0);
      if (i < kJDcSyms) {
        dc.dc[c][i][0] = static_cast<uint8_t>(codes.dc_code[c][i]);
        dc.dc[c][i][1] = static_cast<uint8_t>(codes.dc_code[c][i] >> 8);
        dc.dc[c][i][2] = codes.dc_len[c][i];
      }
      dc.ac[c][i][0] = static_cast<uint8_t>(codes.ac_code[c][i]);
      dc.ac[c][i][1] = static_cast<uint8_t>(codes.ac_code[c][i] >> 8);
      dc.ac[c][i][2] = codes.ac_len[c][i];
    }
  }
  // (the bits of an MCU are bounded by its 3 blocks: the capacity holds any
  // scan of these MCUs, plus the word of an unaligned start)
  uint32_t* words = d_jwords_[jslot_];
  const int groups = (m1 - m0 + kCodeMcus - 1) / kCodeMcus;
  // launch counter: tags the status words (low 14 bits)
  if ((++jepoch_ & 0x3fff) == 0) ++jepoch_;  // (0: the zeroed words' tag)
  const size_t max_groups = (static_cast<size_t>(nb_) + kCodeMcus - 1) / kCodeMcus;
  uint32_t* arr = d_jctl_ + 2 * kCodeFfCopies;
  uint64_t* status = reinterpret_cast<uint64_t*>(arr) + 1 + max_groups / 64 + 2;
  uint64_t* side = status + max_groups;
  uint32_t* seam = reinterpret_cast<uint32_t*>(side + 2 * max_groups);
  JpegQuantF qf;
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 64; ++k) qf.qz[c][k] = static_cast<float>(q[c][c_natural_order[k]]);
  GZ_TIMED("jpeg_code", k_jpeg_code<<<groups, 256, 0, s>>>(d_cur_, qf, nb_, m0, m1, ncomp, dc,
                                                            static_cast<unsigned long long>(base),
                                                            pad_end ? 1 : 0, words, m_jhist_ + kJCodeHost, status,
                                                            side, seam, jepoch_, d_dmax_, skip_at));
  jpart_[jslot_].base = base;
  jcode_groups_[jslot_] = groups;
  jcode_pad_[jslot_] = pad_end;
  // (the bit total, the shared words and every workgroup's 0xff count reach
  // h_jhist_ + kJCodeHost from the coder itself)
  return true;
}

bool Engine::JpegScanFinishPart(ScanPart* part) {
  ScanPart& p = jpart_[jslot_];
  const uint32_t* h = h_jhist_ + kJCodeHost;
  p.bits = static_cast<uint64_t>(h[kCodeHostBits]) | (static_cast<uint64_t>(h[kCodeHostBits + 1]) << 32);
  uint64_t ff = 0;
  for (int t = 0; t < jcode_groups_[jslot_]; ++t) ff += h[kCodeHostFf + t];
  p.ff = ff;
  const uint64_t end = p.base + p.bits;
  p.first_shared = (p.base & 31) != 0;
  p.last_open = !jcode_pad_[jslot_] && (end & 31) != 0;
  p.first_word = p.first_shared ? h[kCodeHostFirst] : 0u;
  p.last_word = p.last_open ? h[kCodeHostLast] : 0u;
  // (one word holding both ends of the part -- a part under 32 bits -- is
  // not supported by the seam exchange)
  if (p.first_shared && p.bits && (p.base >> 5) == ((end - 1) >> 5)) return Fail("JpegScan: a part under one word", 0);
  if ((p.base % 32 + p.bits + 31) / 32 + 1 > jwords_cap_) return Fail("JpegScan bitstream capacity", 0);
  jnbits_[jslot_] = p.bits;
  if (part) *part = p;
  return true;
}

bool Engine::JpegScanFinish(uint64_t* nbits, uint64_t* ff) {
  ScanPart p;
  if (!JpegScanFinishPart(&p)) return false;
  *nbits = p.bits;
  *ff = p.ff;
  return true;
}

bool Engine::JpegFetchPart(bool kept, std::vector<uint32_t>* words, ScanPart* part) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  const int slot = kept ? jslot_ ^ 1 : jslot_;
  const ScanPart& p = jpart_[slot];
  const size_t nw = static_cast<size_t>((p.base % 32 + p.bits + 31) / 32);
  words->assign(nw, 0u);
  if (nw) GZ_HIP(hipMemcpyAsync(words->data(), d_jwords_[slot], nw * 4, hipMemcpyDeviceToHost, s));
  GZ_HIP(hipStreamSynchronize(s));
  if (p.first_shared && nw) (*words)[0] = 0u;            // (not stored by the coder)
  if (p.last_open && nw) (*words)[nw - 1] = 0u;
  *part = p;
  return true;
}

bool Engine::JpegFetch(bool kept, const uint8_t** bytes, uint64_t* nbits) {
  hipStream_t s = static_cast<hipStream_t>(stream_);
  GZ_HIP(hipSetDevice(device_));
  const int slot = kept ? jslot_ ^ 1 : jslot_;
  const uint64_t total = jnbits_[slot];
  const size_t nbytes = static_cast<size_t>((total + 7) / 8);
  if (nbytes + 8 > h_jbytes_cap_) {
    if (h_jbytes_) GZ_HIP(hipHostFree(h_jbytes_));
    h_jbytes_ = nullptr;
    h_jbytes_cap_ = 0;
    const size_t cap = nbytes + nbytes / 4 + 4096;
    GZ_HIP(hipHostMalloc(reinterpret_cast<void**>(&h_jbytes_), cap));
    h_jbytes_cap_ = cap;
  }
  if (nbytes) GZ_HIP(hipMemcpyAsync(h_jbytes_, d_jwords_[slot], nbytes, hipMemcpyDeviceToHost, s));
  GZ_HIP(hipStreamSynchronize(s));
  *bytes = h_jbytes_;
  *nbits = total;
  return true;
}

double Engine::last_kernel_ms(const char*) const { return 0.0; }

const char* BuildInfo() {
  return "libguetzli_hip (gfx950)";
}

}  // namespace gz
