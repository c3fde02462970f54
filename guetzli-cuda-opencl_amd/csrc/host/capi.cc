// extern "C" boundary of libguetzli_hip (include/guetzli_hip.h).
#include "guetzli_hip.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include <hip/hip_runtime.h>

#include "host/jpeg_encode.h"
#include "host/jpeg_reader.h"
#include "host/png_reader.h"
#include "host/jpeg_writer.h"
#include "host/processor.h"
#include "host/rccl_collectives.h"
#include "host/strips.h"
#include "host/synthetic.h"
#include "runtime/engine.h"

namespace {

thread_local std::string g_last_error;
thread_local std::string g_last_detail = "{}";

gz_status SetError(gz_status st, const std::string& msg) {
  g_last_error = msg;
  return st;
}

// No C++ exception may cross the C ABI (it would terminate the caller's
// process): host allocation failure becomes GZ_ERR_OUT_OF_MEMORY, anything
// else GZ_ERR_INTERNAL.
#ifndef GZ_HOSTARCH
#define GZ_HOSTARCH ""
#endif

// The host objects are built for HOSTARCH (Makefile; x86-64-v3 by default:
// AVX2, FMA, BMI2).  This file is not, so every entry point can check the
// CPU before any of that code runs.
bool HostCpuOk() {
  static const bool ok = [] {
    if (std::strstr(GZ_HOSTARCH, "x86-64-v3") == nullptr) return true;
    __builtin_cpu_init();
    return __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma") &&
           __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("f16c") &&
           __builtin_cpu_supports("movbe");
  }();
  return ok;
}

gz_status CpuError(const char* what) {
  return SetError(GZ_ERR_UNSUPPORTED, std::string(what) +
                                          ": this libguetzli_hip was built for x86-64-v3 (AVX2, FMA, BMI2) "
                                          "and the CPU lacks it; rebuild with `make HOSTARCH=`");
}
#define GZ_CPU_CHECK(what) \
  if (!HostCpuOk()) return CpuError(what)

template <class F>
gz_status Guard(const char* what, F&& body) {
  GZ_CPU_CHECK(what);
  try {
    return body();
  } catch (const std::bad_alloc&) {
    return SetError(GZ_ERR_OUT_OF_MEMORY, std::string(what) + ": out of host memory");
  } catch (const std::exception& e) {
    return SetError(GZ_ERR_INTERNAL, std::string(what) + ": " + e.what());
  }
}

}  // namespace

struct gz_comparator {
  std::unique_ptr<gz::Engine> engine;
  float target = 0.0f;
  float distance = 0.0f;
  int w = 0, h = 0;
  std::vector<float> block_max;
  std::vector<int16_t> last;      // coefficients of the last compare (distmap())
  std::vector<uint8_t> last_rgb;  // ... or its sRGB pixels (gz_comparator_compare_rgb)
  // ... or a 4:2:0 candidate (gz_comparator_compare_420): Y, Cb, Cr
  // coefficients and the two factor-2 pixel planes
  std::vector<int16_t> last420_coeffs[3];
  std::vector<uint16_t> last420_planes[2];
  bool Set420Again() {
    return engine->Set420(last420_coeffs[0].data(), last420_coeffs[1].data(), last420_coeffs[2].data(),
                          last420_planes[0].data(), last420_planes[1].data());
  }
  void ForgetLast() {
    last.clear();
    last_rgb.clear();
    for (auto& v : last420_coeffs) v.clear();
    for (auto& v : last420_planes) v.clear();
  }
};

extern "C" {

const char* gz_last_error(void) { return g_last_error.c_str(); }

const char* gz_build_info(void) { return gz::BuildInfo(); }

int gz_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void gz_params_init(gz_params* p) {
  if (!p) return;
  p->butteraugli_target = 1.0f;
  p->clear_metadata = 1;
  p->try_420 = 0;
  p->force_420 = 0;
  p->use_silver_screen = 0;
  p->zeroing_greedy_lookahead = 3;
  p->new_zeroing_model = 1;
}

double gz_butteraugli_score_for_quality(double quality) {
  return gz::ButteraugliScoreForQuality(quality);
}

void gz_free(void* p) { std::free(p); }

gz_status gz_png_decode(const uint8_t* png, size_t png_len, int* width, int* height,
                        uint8_t** rgb_out) {
  return Guard("png_decode", [&]() -> gz_status {
    if (!png || !width || !height || !rgb_out) return SetError(GZ_ERR_INVALID_ARG, "png_decode: bad argument");
    std::vector<uint8_t> rgb;
    std::string err;
    int w = 0, h = 0;
    if (!gz::ReadPng(png, png_len, &w, &h, &rgb, &err))
      return SetError(GZ_ERR_INVALID_ARG, "png_decode: " + err);
    uint8_t* buf = static_cast<uint8_t*>(std::malloc(rgb.size()));
    if (!buf) return SetError(GZ_ERR_OUT_OF_MEMORY, "out of host memory");
    std::memcpy(buf, rgb.data(), rgb.size());
    *width = w;
    *height = h;
    *rgb_out = buf;
    return GZ_OK;
  });
}

gz_status gz_comparator_create(int device, int width, int height, const uint8_t* rgb,
                               float target_distance, gz_comparator** out) {
  return Guard("gz_comparator_create", [&]() -> gz_status {
    if (!out || !rgb || width < 8 || height < 8)
      return SetError(GZ_ERR_INVALID_ARG, "gz_comparator_create: bad argument");
    std::string err;
    auto eng = gz::Engine::Create(device, width, height, &err);
    if (!eng) return SetError(GZ_ERR_DEVICE, "gz_comparator_create: " + err);
    if (!eng->SetReference(rgb, false))
      return SetError(GZ_ERR_DEVICE, "gz_comparator_create: " + eng->error());
    auto* c = new gz_comparator;
    c->engine = std::move(eng);
    c->target = target_distance;
    c->w = width;
    c->h = height;
    *out = c;
    return GZ_OK;
  });
}

void gz_comparator_destroy(gz_comparator* cmp) { delete cmp; }

static gz_status CompareImpl(gz_comparator* cmp, const int16_t* coeffs, gz::CompareDebug* dbg,
                             float* distance) {
  if (!cmp || !coeffs) return SetError(GZ_ERR_INVALID_ARG, "compare: bad argument");
  gz::Engine& e = *cmp->engine;
  cmp->block_max.resize(e.blocks());
  if (!e.UploadCoeffs(coeffs) || !e.Compare(&cmp->distance, cmp->block_max.data(), dbg))
    return SetError(GZ_ERR_DEVICE, "compare: " + e.error());
  cmp->ForgetLast();
  cmp->last.assign(coeffs, coeffs + static_cast<size_t>(e.blocks()) * 192);
  if (distance) *distance = cmp->distance;
  return GZ_OK;
}

gz_status gz_comparator_compare_rgb(gz_comparator* cmp, const uint8_t* rgb, float* distance) {
  if (!cmp || !rgb) return SetError(GZ_ERR_INVALID_ARG, "compare_rgb: bad argument");
  gz::Engine& e = *cmp->engine;
  cmp->block_max.resize(e.blocks());
  if (!e.SetCandidateRgb(rgb) || !e.Compare(&cmp->distance, cmp->block_max.data(), nullptr))
    return SetError(GZ_ERR_DEVICE, "compare_rgb: " + e.error());
  cmp->ForgetLast();
  cmp->last_rgb.assign(rgb, rgb + static_cast<size_t>(3) * cmp->w * cmp->h);
  if (distance) *distance = cmp->distance;
  return GZ_OK;
}

gz_status gz_comparator_compare_420(gz_comparator* cmp, const int16_t* y, const int16_t* cb,
                                    const int16_t* cr, const uint16_t* plane_cb, const uint16_t* plane_cr,
                                    float* distance) {
  if (!cmp || !y || !plane_cb || !plane_cr) return SetError(GZ_ERR_INVALID_ARG, "compare_420: bad argument");
  gz::Engine& e = *cmp->engine;
  const size_t per = static_cast<size_t>(e.blocks()) * 64;
  const size_t cper = static_cast<size_t>((cmp->w + 15) / 16) * ((cmp->h + 15) / 16) * 64;
  const size_t n = static_cast<size_t>(cmp->w) * cmp->h;
  cmp->ForgetLast();
  cmp->last420_coeffs[0].assign(y, y + per);
  cmp->last420_coeffs[1] = cb ? std::vector<int16_t>(cb, cb + cper) : std::vector<int16_t>(cper, 0);
  cmp->last420_coeffs[2] = cr ? std::vector<int16_t>(cr, cr + cper) : std::vector<int16_t>(cper, 0);
  cmp->last420_planes[0].assign(plane_cb, plane_cb + n);
  cmp->last420_planes[1].assign(plane_cr, plane_cr + n);
  cmp->block_max.resize(e.blocks());
  if (!cmp->Set420Again() || !e.Compare(&cmp->distance, cmp->block_max.data(), nullptr)) {
    cmp->ForgetLast();
    return SetError(GZ_ERR_DEVICE, "compare_420: " + e.error());
  }
  if (distance) *distance = cmp->distance;
  return GZ_OK;
}

gz_status gz_comparator_compare(gz_comparator* cmp, const int16_t* coeffs, float* distance) {
  return CompareImpl(cmp, coeffs, nullptr, distance);
}

gz_status gz_comparator_compare_stages(gz_comparator* cmp, const int16_t* coeffs,
                                       gz_compare_stages* st, float* distance) {
  gz::CompareDebug dbg;
  if (st) {
    dbg.cand_linear = st->cand_linear;
    dbg.cand_xyb = st->cand_xyb;
    dbg.mhic0 = st->mhic0;
    dbg.mhic1 = st->mhic1;
    dbg.edge = st->edge;
    dbg.block_dc = st->block_dc;
    dbg.block_ac = st->block_ac;
    dbg.block_ac_lf = st->block_ac_lf;
    dbg.mask = st->mask;
    dbg.mask_dc = st->mask_dc;
    dbg.combined = st->combined;
    dbg.distmap = st->distmap;
  }
  return CompareImpl(cmp, coeffs, &dbg, distance);
}

gz_status gz_comparator_compare_stages_production(gz_comparator* cmp, const int16_t* coeffs,
                                                  gz_compare_stages* st, float* distance) {
  gz::CompareDebug dbg;
  dbg.production = true;
  if (st) {
    if (st->cand_linear || st->cand_xyb || st->block_ac_lf || st->mask || st->mask_dc || st->combined)
      return SetError(GZ_ERR_INVALID_ARG,
                      "compare_stages_production: only mhic0, mhic1, edge, block_dc, block_ac and distmap");
    dbg.mhic0 = st->mhic0;
    dbg.mhic1 = st->mhic1;
    dbg.edge = st->edge;
    dbg.block_dc = st->block_dc;
    dbg.block_ac = st->block_ac;
    dbg.distmap = st->distmap;
  }
  return CompareImpl(cmp, coeffs, &dbg, distance);
}

gz_status gz_comparator_distmap(gz_comparator* cmp, float* out) {
  if (!cmp || !out) return SetError(GZ_ERR_INVALID_ARG, "distmap: bad argument");
  const bool is420 = !cmp->last420_planes[0].empty();
  if (cmp->last.empty() && cmp->last_rgb.empty() && !is420)
    return SetError(GZ_ERR_INVALID_ARG, "distmap: no compare yet");
  gz::Engine& e = *cmp->engine;
  // the pass again on the same candidate, with the map read back (the
  // search's passes keep only the per-block maxima)
  gz::CompareDebug dbg;
  dbg.distmap = out;
  float d = 0.0f;
  const bool up = is420 ? cmp->Set420Again()
                  : cmp->last.empty() ? e.SetCandidateRgb(cmp->last_rgb.data())
                                      : e.UploadCoeffs(cmp->last.data());
  if (!up || !e.Compare(&d, nullptr, &dbg)) return SetError(GZ_ERR_DEVICE, "distmap: " + e.error());
  return GZ_OK;
}

gz_status gz_comparator_compare_blocks(gz_comparator* cmp, int n, const int* blocks,
                                       const int16_t* cand, double* err) {
  if (!cmp || n < 0 || (n > 0 && (!blocks || !cand || !err)))
    return SetError(GZ_ERR_INVALID_ARG, "compare_blocks: bad argument");
  gz::Engine& e = *cmp->engine;
  for (int i = 0; i < n; ++i)
    if (blocks[i] < 0 || blocks[i] >= e.blocks())
      return SetError(GZ_ERR_INVALID_ARG, "compare_blocks: block index out of range");
  if (!e.CompareBlocks(n, blocks, cand, err))
    return SetError(GZ_ERR_DEVICE, "compare_blocks: " + e.error());
  return GZ_OK;
}

gz_status gz_comparator_compare_blocks_rgb(gz_comparator* cmp, int n, const int* blocks,
                                           const uint8_t* rgb, double* err) {
  if (!cmp || n < 0 || (n > 0 && (!blocks || !rgb || !err)))
    return SetError(GZ_ERR_INVALID_ARG, "compare_blocks_rgb: bad argument");
  gz::Engine& e = *cmp->engine;
  for (int i = 0; i < n; ++i)
    if (blocks[i] < 0 || blocks[i] >= e.blocks())
      return SetError(GZ_ERR_INVALID_ARG, "compare_blocks_rgb: block index out of range");
  if (!e.CompareBlocksRgb(n, blocks, rgb, err))
    return SetError(GZ_ERR_DEVICE, "compare_blocks_rgb: " + e.error());
  return GZ_OK;
}

gz_status gz_comparator_original_coeffs(gz_comparator* cmp, int16_t* out) {
  if (!cmp || !out) return SetError(GZ_ERR_INVALID_ARG, "original_coeffs: bad argument");
  if (!cmp->engine->ComputeOriginalCoeffs(out))
    return SetError(GZ_ERR_DEVICE, "original_coeffs: " + cmp->engine->error());
  return GZ_OK;
}

gz_status gz_comparator_block_max(gz_comparator* cmp, float* out) {
  if (!cmp || !out) return SetError(GZ_ERR_INVALID_ARG, "block_max: bad argument");
  if (cmp->block_max.empty()) return SetError(GZ_ERR_INVALID_ARG, "block_max: no compare yet");
  std::memcpy(out, cmp->block_max.data(), cmp->block_max.size() * sizeof(float));
  return GZ_OK;
}

int gz_comparator_distance_ok(gz_comparator* cmp, double target_mul) {
  // butteraugli_comparator.h:52-54
  return cmp && cmp->distance <= target_mul * cmp->target;
}

double gz_comparator_score_output_size(gz_comparator* cmp, int size) {
  return cmp ? gz::ScoreJPEG(cmp->distance, size, cmp->target) : 0.0;
}

gz_status gz_comparator_start_block_comparisons(gz_comparator* cmp, float* mask_scale) {
  if (!cmp) return SetError(GZ_ERR_INVALID_ARG, "start_block_comparisons: bad argument");
  if (!cmp->engine->StartBlockComparisons(mask_scale))
    return SetError(GZ_ERR_DEVICE, "start_block_comparisons: " + cmp->engine->error());
  return GZ_OK;
}

gz_status gz_comparator_block_zeroing_orders(gz_comparator* cmp, const int16_t* cur_coeffs,
                                             const int16_t* orig_coeffs, int comp_mask,
                                             float limit, int lookahead, int new_zeroing_model,
                                             gz_coeff_data* out) {
  if (!cmp || !cur_coeffs || !orig_coeffs || !out || lookahead < 1 || comp_mask <= 0 ||
      comp_mask > 7)
    return SetError(GZ_ERR_INVALID_ARG, "block_zeroing_orders: bad argument");
  gz::Engine& e = *cmp->engine;
  static_assert(sizeof(gz_coeff_data) == sizeof(gz::CoeffDataHost), "CoeffData layout");
  if (!e.SetOriginalCoeffs(orig_coeffs, false) || !e.UploadCoeffs(cur_coeffs) ||
      !e.BlockZeroingOrders(comp_mask, limit, lookahead, new_zeroing_model != 0,
                            reinterpret_cast<gz::CoeffDataHost*>(out)))
    return SetError(GZ_ERR_DEVICE, "block_zeroing_orders: " + e.error());
  return GZ_OK;
}

static gz_status CopyOut(const std::string& s, uint8_t** jpeg_out, size_t* jpeg_size) {
  uint8_t* buf = static_cast<uint8_t*>(std::malloc(s.size() ? s.size() : 1));
  if (!buf) return SetError(GZ_ERR_OUT_OF_MEMORY, "out of host memory");
  std::memcpy(buf, s.data(), s.size());
  *jpeg_out = buf;
  *jpeg_size = s.size();
  return GZ_OK;
}

gz_status gz_comparator_write_jpeg(gz_comparator* cmp, const int16_t* coeffs, const int* quant,
                                   uint8_t** jpeg_out, size_t* jpeg_size) {
  return Guard("write_jpeg", [&]() -> gz_status {
    if (!cmp || !coeffs || !quant || !jpeg_out || !jpeg_size)
      return SetError(GZ_ERR_INVALID_ARG, "write_jpeg: bad argument");
    int q[3][64];
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 64; ++k) {
        q[c][k] = quant[c * 64 + k];
        if (q[c][k] < 1 || q[c][k] > 65535) return SetError(GZ_ERR_INVALID_ARG, "write_jpeg: quant");
      }
    gz::Engine& e = *cmp->engine;
    if (!e.UploadCoeffs(coeffs)) return SetError(GZ_ERR_DEVICE, "write_jpeg: " + e.error());
    gz::JpegData meta;
    std::string out, err;
    if (!gz::DeviceWriteJpeg(&e, cmp->w, cmp->h, q, meta, true, &out, &err))
      return SetError(GZ_ERR_DEVICE, "write_jpeg: " + err);
    return CopyOut(out, jpeg_out, jpeg_size);
  });
}

gz_status gz_write_jpeg_host(int width, int height, const int16_t* coeffs, const int* quant,
                             uint8_t** jpeg_out, size_t* jpeg_size) {
  return Guard("write_jpeg_host", [&]() -> gz_status {
    if (!coeffs || !quant || !jpeg_out || !jpeg_size || width <= 0 || height <= 0)
      return SetError(GZ_ERR_INVALID_ARG, "write_jpeg_host: bad argument");
    gz::CoeffImage img;
    img.Init(width, height);
    std::memcpy(img.coeffs.data(), coeffs, img.coeffs.size() * sizeof(int16_t));
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 64; ++k) {
        img.quant[c][k] = quant[c * 64 + k];
        if (img.quant[c][k] < 1 || img.quant[c][k] > 65535)
          return SetError(GZ_ERR_INVALID_ARG, "write_jpeg_host: quant");
      }
    gz::JpegData jpg;
    img.SaveToJpegData(&jpg);
    std::string out;
    if (!gz::WriteJpegReference(jpg, true, &out)) return SetError(GZ_ERR_INTERNAL, "write_jpeg_host");
    return CopyOut(out, jpeg_out, jpeg_size);
  });
}

size_t gz_last_process_detail(char* buf, size_t cap) {
  if (buf && cap) {
    const size_t n = std::min(cap - 1, g_last_detail.size());
    std::memcpy(buf, g_last_detail.data(), n);
    buf[n] = 0;
  }
  return g_last_detail.size() + 1;
}

void gz_profile_enable(int enable) { gz::ProfileEnable(enable != 0); }

void gz_profile_reset(void) { gz::ProfileReset(); }

int gz_profile_get(const char* name, long* count, double* total_ms) {
  if (!name || !count || !total_ms) return 0;
  return gz::ProfileGet(name, count, total_ms) ? 1 : 0;
}

size_t gz_profile_names(char* buf, size_t cap) {
  const std::string names = gz::ProfileNames();
  if (buf && cap) {
    const size_t n = std::min(cap - 1, names.size());
    std::memcpy(buf, names.data(), n);
    buf[n] = 0;
  }
  return names.size() + 1;
}

gz_status gz_synthetic_frame(uint64_t seed, int width, int height, uint8_t* rgb_out) {
  GZ_CPU_CHECK("synthetic_frame");
  if (!rgb_out || width <= 0 || height <= 0)
    return SetError(GZ_ERR_INVALID_ARG, "synthetic_frame: bad argument");
  gz::SyntheticFrame(seed, width, height, rgb_out);
  return GZ_OK;
}

gz_status gz_rgb_to_coeffs(const uint8_t* rgb, int width, int height, int16_t* coeffs_out) {
  GZ_CPU_CHECK("rgb_to_coeffs");
  if (!rgb || !coeffs_out || width <= 0 || height <= 0 || width >= (1 << 16) ||
      height >= (1 << 16))
    return SetError(GZ_ERR_INVALID_ARG, "rgb_to_coeffs: bad argument");
  gz::RgbToCoeffsQ1(rgb, width, height, coeffs_out);
  return GZ_OK;
}

size_t gz_engine_pool_trim(size_t keep_bytes) { return gz::TrimEnginePool(keep_bytes); }

size_t gz_engine_pool_idle_bytes(void) { return gz::EnginePoolIdleBytes(); }

gz_status gz_block_error_adjustment_weights(int width, int height, float target, int direction,
                                            int max_block_dist, double target_mul, int factor_x,
                                            int factor_y, const float* distmap,
                                            float* block_weight) {
  GZ_CPU_CHECK("block_error_adjustment_weights");
  if (!distmap || !block_weight || width <= 0 || height <= 0 || factor_x < 1 || factor_y < 1 ||
      (direction != 1 && direction != -1) || max_block_dist < 0)
    return SetError(GZ_ERR_INVALID_ARG, "block_error_adjustment_weights: bad argument");
  // per-block maxima of the distance map (butteraugli_comparator.cc:181-195),
  // then the weights from them (the search loop gets the maxima from the device)
  const int sx = 8 * factor_x, sy = 8 * factor_y;
  const int bw = (width + sx - 1) / sx, bh = (height + sy - 1) / sy;
  std::vector<float> bmax(static_cast<size_t>(bw) * bh);
  for (int by = 0; by < bh; ++by)
    for (int bx = 0; bx < bw; ++bx) {
      float m = 0.0f;
      for (int y = sy * by; y < std::min(height, sy * (by + 1)); ++y)
        for (int x = sx * bx; x < std::min(width, sx * (bx + 1)); ++x)
          m = std::max(m, distmap[static_cast<size_t>(y) * width + x]);
      bmax[static_cast<size_t>(by) * bw + bx] = m;
    }
  std::vector<float> wgt(block_weight, block_weight + bmax.size());
  gz::BlockErrorAdjustmentWeights(width, height, target, direction, max_block_dist, target_mul,
                                  factor_x, factor_y, bmax, &wgt);
  std::copy(wgt.begin(), wgt.end(), block_weight);
  return GZ_OK;
}

namespace {
// gz_collectives (C callback) as the host's collective interface.
class CCollectives : public gz::Collectives {
 public:
  explicit CCollectives(const gz_collectives* c) : c_(*c) {}
  int rank() const override { return c_.rank; }
  int world() const override { return c_.world; }
  bool AllGather(const void* send, size_t bytes, void* recv) override {
    return c_.allgather(c_.ctx, send, bytes, recv) == 0;
  }

 private:
  gz_collectives c_;
};

bool ValidCollectives(const gz_collectives* c) {
  return c && c->allgather && c->world >= 1 && c->rank >= 0 && c->rank < c->world;
}
}  // namespace

static gz_status Deliver(const gz::ProcessResult& res, uint8_t** jpeg_out, size_t* jpeg_size,
                         gz_process_stats* stats);

static gz::ProcessParams ToProcessParams(const gz_params* params) {
  gz::ProcessParams pp;
  pp.butteraugli_target = params->butteraugli_target;
  pp.clear_metadata = params->clear_metadata != 0;
  pp.try_420 = params->try_420 != 0;
  pp.force_420 = params->force_420 != 0;
  pp.use_silver_screen = params->use_silver_screen != 0;
  pp.zeroing_greedy_lookahead = params->zeroing_greedy_lookahead;
  pp.new_zeroing_model = params->new_zeroing_model != 0;
  return pp;
}

static gz_status ProcessImpl(int device, const gz_params* params, const uint8_t* rgb,
                             bool device_ptr, int w, int h, uint8_t** jpeg_out,
                             size_t* jpeg_size, gz_process_stats* stats,
                             const gz_collectives* coll = nullptr) {
  return Guard("process", [&]() -> gz_status {
    if (!params || !rgb || !jpeg_out || !jpeg_size || w <= 0 || h <= 0)
      return SetError(GZ_ERR_INVALID_ARG, "process: bad argument");
    // (the strip decomposition of one frame runs the 4:4:4 search only)
    if (coll && (params->try_420 || params->force_420))
      return SetError(GZ_ERR_UNSUPPORTED, "process: 4:2:0 output of a strip-decomposed frame is not supported");
    const gz::ProcessParams pp = ToProcessParams(params);
    gz::ProcessResult res;
    std::string err;
    int rc;
    if (coll) {
      CCollectives cc(coll);
      rc = gz::ProcessStrips(device, pp, rgb, w, h, &cc, &res, &err);
    } else {
      rc = gz::Process(device, pp, rgb, device_ptr, w, h, &res, &err);
    }
    if (rc != 0) return SetError(rc, "process: " + err);
    return Deliver(res, jpeg_out, jpeg_size, stats);
  });
}

// The encoded bytes (library-allocated) and statistics of a finished encode.
static gz_status Deliver(const gz::ProcessResult& res, uint8_t** jpeg_out, size_t* jpeg_size,
                         gz_process_stats* stats) {
  uint8_t* buf = static_cast<uint8_t*>(std::malloc(res.jpeg.size() ? res.jpeg.size() : 1));
  if (!buf) return SetError(GZ_ERR_OUT_OF_MEMORY, "process: out of host memory");
  std::memcpy(buf, res.jpeg.data(), res.jpeg.size());
  *jpeg_out = buf;
  *jpeg_size = res.jpeg.size();
  {
    std::string j = "{";
    char item[96];
    for (auto& kv : res.detail) {
      snprintf(item, sizeof(item), "%s\"%s\": %.6g", j.size() > 1 ? ", " : "", kv.first.c_str(), kv.second);
      j += item;
    }
    g_last_detail = j + "}";
  }
  if (stats) {
    stats->iterations = res.iterations;
    stats->iterations_up = res.iterations_up;
    stats->iterations_down = res.iterations_down;
    stats->compares = res.compares;
    stats->seconds_compare = res.seconds_compare;
    stats->seconds_zeroing = res.seconds_zeroing;
    stats->seconds_total = res.seconds_total;
    stats->seconds_setup = res.seconds_setup;
    stats->seconds_write = res.seconds_write;
    stats->seconds_quantize = res.seconds_quantize;
    stats->seconds_backend = res.seconds_backend;
  }
  return GZ_OK;
}

gz_status gz_process_rgb(int device, const gz_params* params, const uint8_t* rgb, int width,
                         int height, uint8_t** jpeg_out, size_t* jpeg_size,
                         gz_process_stats* stats) {
  return ProcessImpl(device, params, rgb, false, width, height, jpeg_out, jpeg_size, stats);
}

gz_status gz_process_rgb_device(int device, const gz_params* params, const uint8_t* rgb_dev,
                                int width, int height, uint8_t** jpeg_out, size_t* jpeg_size,
                                gz_process_stats* stats) {
  return ProcessImpl(device, params, rgb_dev, true, width, height, jpeg_out, jpeg_size, stats);
}

gz_status gz_process_jpeg(int device, const gz_params* params, const uint8_t* jpeg, size_t jpeg_len,
                          uint8_t** jpeg_out, size_t* jpeg_size, gz_process_stats* stats) {
  return Guard("process_jpeg", [&]() -> gz_status {
    if (!params || !jpeg || !jpeg_out || !jpeg_size)
      return SetError(GZ_ERR_INVALID_ARG, "process_jpeg: bad argument");
    gz::ProcessResult res;
    std::string err;
    const int rc = gz::ProcessJpeg(device, ToProcessParams(params), jpeg, jpeg_len, &res, &err);
    if (rc != 0) return SetError(rc, "process_jpeg: " + err);
    return Deliver(res, jpeg_out, jpeg_size, stats);
  });
}

gz_status gz_jpeg_decode(const uint8_t* jpeg, size_t jpeg_len, int* width, int* height,
                         int* ncomp, int16_t** coeffs_out, size_t* ncoeffs, uint8_t** rgb_out) {
  return Guard("jpeg_decode", [&]() -> gz_status {
    if (!jpeg || !width || !height || !ncomp || !coeffs_out || !ncoeffs || !rgb_out)
      return SetError(GZ_ERR_INVALID_ARG, "jpeg_decode: bad argument");
    *coeffs_out = nullptr;
    *rgb_out = nullptr;
    gz::JpegData jpg;
    std::string err;
    if (!gz::ReadJpeg(jpeg, jpeg_len, &jpg, &err)) return SetError(GZ_ERR_INVALID_ARG, "jpeg_decode: " + err);
    *width = jpg.width;
    *height = jpg.height;
    *ncomp = static_cast<int>(jpg.components.size());
    size_t n = 0;
    for (const auto& c : jpg.components) n += c.coeffs.size();
    int16_t* co = static_cast<int16_t*>(std::malloc(n ? n * sizeof(int16_t) : 1));
    if (!co) return SetError(GZ_ERR_OUT_OF_MEMORY, "jpeg_decode: out of host memory");
    size_t at = 0;
    for (const auto& c : jpg.components) {
      std::memcpy(co + at, c.coeffs.data(), c.coeffs.size() * sizeof(int16_t));
      at += c.coeffs.size();
    }
    *coeffs_out = co;
    *ncoeffs = n;
    std::vector<uint8_t> rgb;
    if (gz::DecodeJpegToRGB(jpg, &rgb)) {
      uint8_t* r = static_cast<uint8_t*>(std::malloc(rgb.size()));
      if (!r) return SetError(GZ_ERR_OUT_OF_MEMORY, "jpeg_decode: out of host memory");
      std::memcpy(r, rgb.data(), rgb.size());
      *rgb_out = r;
    }
    return GZ_OK;
  });
}

gz_status gz_process_rgb_strips(int device, const gz_params* params, const uint8_t* rgb, int width,
                                int height, const gz_collectives* coll, uint8_t** jpeg_out,
                                size_t* jpeg_size, gz_process_stats* stats) {
  if (!ValidCollectives(coll)) return SetError(GZ_ERR_INVALID_ARG, "process_strips: bad collectives");
  return ProcessImpl(device, params, rgb, false, width, height, jpeg_out, jpeg_size, stats, coll);
}

gz_status gz_strip_layout(int width, int height, int world, int rank, int* y0, int* y1, int* e0,
                          int* e1) {
  GZ_CPU_CHECK("strip_layout");
  if (width <= 0 || height <= 0 || world < 1 || rank < 0 || rank >= world || !y0 || !y1 || !e0 ||
      !e1)
    return SetError(GZ_ERR_INVALID_ARG, "strip_layout: bad argument");
  const gz::StripLayout L = gz::StripLayout::Make(width, height, world);
  *y0 = L.y0[rank];
  *y1 = L.y1[rank];
  *e0 = L.e0[rank];
  *e1 = L.e1[rank];
  return GZ_OK;
}

gz_status gz_collectives_selftest(const gz_collectives* coll) {
  GZ_CPU_CHECK("collectives_selftest");
  if (!ValidCollectives(coll)) return SetError(GZ_ERR_INVALID_ARG, "collectives: bad argument");
  CCollectives cc(coll);
  // equal-size gather of a rank-tagged pattern, then a variable-size one
  const int n = cc.world(), r = cc.rank();
  std::vector<uint32_t> mine(5), all(5 * n);
  for (int i = 0; i < 5; ++i) mine[i] = 1000u * r + i;
  if (!cc.AllGather(mine.data(), mine.size() * 4, all.data()))
    return SetError(GZ_ERR_INTERNAL, "collectives: all-gather failed");
  for (int q = 0; q < n; ++q)
    for (int i = 0; i < 5; ++i)
      if (all[5 * q + i] != 1000u * q + i) return SetError(GZ_ERR_INTERNAL, "collectives: wrong data");
  std::vector<uint8_t> v(3 * r + 1, static_cast<uint8_t>(r + 7));
  std::vector<std::vector<uint8_t>> got;
  if (!cc.AllGatherV(v, &got)) return SetError(GZ_ERR_INTERNAL, "collectives: all-gather-v failed");
  for (int q = 0; q < n; ++q)
    if (got[q] != std::vector<uint8_t>(3 * q + 1, static_cast<uint8_t>(q + 7)))
      return SetError(GZ_ERR_INTERNAL, "collectives: wrong variable-size data");
  return GZ_OK;
}

gz_status gz_rccl_unique_id(uint8_t id[128]) {
  GZ_CPU_CHECK("rccl_unique_id");
  if (!id) return SetError(GZ_ERR_INVALID_ARG, "rccl_unique_id: null id");
  std::string err;
  if (!gz::RcclUniqueId(id, &err)) return SetError(GZ_ERR_DEVICE, "rccl_unique_id: " + err);
  return GZ_OK;
}

gz_status gz_rccl_create(int device, int rank, int world, const uint8_t id[128], gz_rccl** out,
                         gz_collectives* coll) {
  GZ_CPU_CHECK("rccl_create");
  if (!id || !out || !coll || world < 1 || rank < 0 || rank >= world || device < 0)
    return SetError(GZ_ERR_INVALID_ARG, "rccl_create: bad argument");
  std::string err;
  gz::RcclComm* c = gz::RcclCreate(device, rank, world, id, &err);
  if (!c) return SetError(GZ_ERR_DEVICE, "rccl_create: " + err);
  *out = reinterpret_cast<gz_rccl*>(c);
  coll->ctx = c;
  coll->rank = rank;
  coll->world = world;
  coll->allgather = &gz::RcclAllGather;
  return GZ_OK;
}

const char* gz_rccl_library(void) {
  static thread_local std::string path;
  path = gz::RcclLibraryPath();
  return path.c_str();
}

void gz_rccl_destroy(gz_rccl* comm) { gz::RcclDestroy(reinterpret_cast<gz::RcclComm*>(comm)); }

}  // extern "C"
