// Portions restate Guetzli (Copyright 2016 Google Inc., Apache License 2.0,
// http://www.apache.org/licenses/LICENSE-2.0) as modified in
// yyamamoto79/guetzli-cuda-opencl: processor.cc, quality.cc, score.cc and butteraugli_comparator.cc
// (QuantMatrixGenerator, the back end's control flow, kLocalMaxWeight).
// Byte-exact output forces their operation order and constants; the
// code around them is this repository's own.
// The Guetzli search loop on the host (guetzli/processor.cc), driving the GPU
// comparator.  Control flow, heuristics and every floating-point decision are
// those of the reference's CPU_OPT (`guetzli --c`) path so the output bytes
// are identical; only the expensive work (Butteraugli passes, per-block
// greedy zeroing, global quantization) runs on the device.
#include "host/processor.h"

#include <algorithm>
#include <limits>
#include <time.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <set>
#include <thread>
#include <utility>

#include <hip/hip_runtime.h>

#include "guetzli_hip.h"
#include "host/jpeg_encode.h"
#include "host/jpeg_reader.h"
#include "host/jpeg_writer.h"
#include "host/lazy_sort.h"
#include "host/strips.h"
#include "host/thread_pool.h"

namespace gz {

// ---------------------------------------------------------------------------
// quality.cc / score.cc
// ---------------------------------------------------------------------------

double ButteraugliScoreForQuality(double quality) {
  static const double kScoreForQuality[] = {
      2.810761, 2.729300, 2.689687, 2.636811, 2.547863, 2.525400, 2.473416, 2.366133, 2.338078,
      2.318654, 2.201674, 2.145517, 2.087322, 2.009328, 1.945456, 1.900112, 1.805701, 1.750194,
      1.644175, 1.562165, 1.473608, 1.382021, 1.294298, 1.185402, 1.066781, 0.971769, 0.852901,
      0.724544, 0.611302, 0.443185, 0.211578, 0.209462, 0.207346, 0.205230, 0.203114, 0.200999,
      0.198883, 0.196767, 0.194651, 0.192535, 0.190420, 0.190420,
  };
  const int kLowest = 70, kHighest = 110;
  if (quality < kLowest) quality = kLowest;
  if (quality > kHighest) quality = kHighest;
  const int index = static_cast<int>(quality);
  const double mix = quality - index;
  return kScoreForQuality[index - kLowest] * (1 - mix) + kScoreForQuality[index - kLowest + 1] * mix;
}

double ScoreJPEG(double distance, int size, double target) {
  const double kScale = 50, kMaxExponent = 10, kLargeSize = 1e30;
  const double diff = distance - target;
  if (diff <= 0.0) return size;
  const double exponent = kScale * diff;
  if (exponent > kMaxExponent) return kLargeSize * std::exp(kMaxExponent) * diff + size;
  return std::exp(exponent) * size;
}

namespace {

using Clock = std::chrono::steady_clock;
inline double Since(Clock::time_point t0) {
  return std::chrono::duration<double>(Clock::now() - t0).count();
}
// CPU seconds of the calling thread (host-cost accounting in the detail map)
inline double ThreadCpu() {
  timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return static_cast<double>(ts.tv_sec) + 1e-9 * static_cast<double>(ts.tv_nsec);
}

inline int Log2FloorNonZero(uint32_t n) { return 31 ^ __builtin_clz(n); }

}  // namespace

// ---------------------------------------------------------------------------
// HipButteraugliComparator
// ---------------------------------------------------------------------------

std::unique_ptr<HipButteraugliComparator> HipButteraugliComparator::Create(
    int device, int w, int h, const uint8_t* rgb, bool device_ptr, float target, std::string* err) {
  std::unique_ptr<HipButteraugliComparator> c(new HipButteraugliComparator);
  c->engine_ = AcquireEngine(device, w, h, err);
  if (!c->engine_) return nullptr;
  if (!c->engine_->SetReference(rgb, device_ptr)) {
    if (err) *err = c->engine_->error();
    return nullptr;
  }
  c->w_ = w;
  c->h_ = h;
  c->target_ = target;
  c->block_max_.assign(c->engine_->blocks(), 0.0f);
  return c;
}

bool HipButteraugliComparator::OriginalJpegData(JpegData* jpg) {
  InitJpegDataYUV444(w_, h_, jpg);
  for (auto& q : jpg->quant)
    for (int k = 0; k < kDCTBlockSize; ++k) q.values[k] = 1;
  const size_t per = static_cast<size_t>(engine_->blocks()) * 64;
  if (orig_.size() != 3 * per) orig_.reset(3 * per);
  if (!engine_->ComputeOriginalCoeffs(orig_.data())) {
    err_ = engine_->error();
    return false;
  }
  for (int c = 0; c < 3; ++c)
    std::memcpy(jpg->components[c].coeffs.data(), orig_.data() + c * per, per * sizeof(coeff_t));
  orig_on_device_ = true;
  return true;
}

bool HipButteraugliComparator::SetOriginalCoeffs(const JpegData& jpg) {
  const size_t per = static_cast<size_t>(engine_->blocks()) * 64;
  if (orig_on_device_ && orig_.size() == 3 * per) {
    // already resident (OriginalJpegData) unless the caller changed them
    bool same = true;
    for (int c = 0; c < 3 && same; ++c)
      same = jpg.components[c].coeffs.size() == per &&
             std::memcmp(jpg.components[c].coeffs.data(), orig_.data() + c * per,
                         per * sizeof(coeff_t)) == 0;
    if (same) return true;
  }
  orig_on_device_ = false;
  size_t total = 0;
  for (int c = 0; c < 3; ++c) total += jpg.components[c].coeffs.size();
  orig_.reset(total);
  coeff_t* all = orig_.data();
  for (int c = 0; c < 3; ++c) {
    std::memcpy(all, jpg.components[c].coeffs.data(), jpg.components[c].coeffs.size() * sizeof(coeff_t));
    all += jpg.components[c].coeffs.size();
  }
  if (!engine_->SetOriginalCoeffs(orig_.data(), false)) {
    err_ = engine_->error();
    return false;
  }
  return true;
}

// img holds exactly the q=1 originals resident on the device (d_orig_).
bool HipButteraugliComparator::IsOriginal(const CoeffImage& img) const {
  if (!orig_on_device_ || img.coeffs.size() != orig_.size()) return false;
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < kDCTBlockSize; ++k)
      if (img.quant[c][k] != 1) return false;
  return std::memcmp(img.coeffs.data(), orig_.data(), orig_.size() * sizeof(coeff_t)) == 0;
}

// Brings the device copy of the coefficients up to date with img: the
// journalled edits when it is in img's epoch, else everything.
bool HipButteraugliComparator::SyncCoeffs(const CoeffImage& img) {
  if (device_.Current(img)) return true;
  // A short journal is replayed, a long one replaced by a full upload --
  // except while the host copy is partial (the back end's lazily
  // materialised blocks): then only the journalled values are current, so
  // the journal is replayed whatever its length.  (GZ_REPLAY_DIV: the
  // journal length above which the full upload is chosen, as a fraction
  // 1/GZ_REPLAY_DIV of the coefficients; tests force long tails with it.)
  static const size_t replay_div = [] {
    const char* e = std::getenv("GZ_REPLAY_DIV");
    return static_cast<size_t>(e && std::atoi(e) > 0 ? std::atoi(e) : 8);
  }();
  const bool short_journal = img.changed.size() - device_.pos < img.coeffs.size() / replay_div;
  const bool replay = device_.CanReplay(img) && (short_journal || img.host_partial);
  if (!img.host_valid || (img.host_partial && !replay)) {
    err_ = "coefficients are current on neither side";
    return false;
  }
  bool ok;
  if (replay) {
    const size_t n = img.changed.size() - device_.pos;
    const uint32_t* idx = img.changed.data() + device_.pos;
    delta_val_.resize(n);
    for (size_t i = 0; i < n; ++i) delta_val_[i] = img.coeffs[idx[i]];
    ok = engine_->UploadCoeffDelta(idx, delta_val_.data(), n);
  } else if (IsOriginal(img)) {
    // the search's first image (CopyFromJpegData of the q=1 originals) is
    // already resident: an HBM copy instead of a pageable upload
    ok = engine_->CurrentFromOriginal();
  } else {
    ok = engine_->UploadCoeffs(img.coeffs.data());
  }
  if (!ok) {
    err_ = engine_->error();
    return false;
  }
  device_.Set(img);
  return true;
}

const std::vector<float>& HipButteraugliComparator::block_max_distance() const {
  if (block_max_stale_) {
    float d = 0.0f;
    block_max_failed_ = false;
    if (engine_->CompareFinish(&d, block_max_.data())) {
      block_max_stale_ = false;
    } else {
      block_max_failed_ = true;
      err_ = engine_->error();
      std::fill(block_max_.begin(), block_max_.end(), std::numeric_limits<float>::infinity());
    }
  }
  return block_max_;
}

bool HipButteraugliComparator::Compare(const CoeffImage& img) {
  const auto t0 = Clock::now();
  if (!SyncCoeffs(img)) return false;
  if (!engine_->Compare(&distance_, nullptr, nullptr)) {
    err_ = engine_->error();
    return false;
  }
  block_max_stale_ = true;
  ++compares;
  seconds_compare += Since(t0);
  return true;
}

bool HipButteraugliComparator::QuantizeFromOriginal(const int q[3][kDCTBlockSize], CoeffImage* img,
                                                    bool need_host) {
  // CopyFromJpegData(q=1) + ApplyGlobalQuantization (processor.cc:316-317)
  // on the device copy of the originals; the host copy (a pinned DMA) only
  // when the caller will read it.
  if (!engine_->QuantizeFromOriginal(q, need_host ? img->coeffs.data() : nullptr)) {
    err_ = engine_->error();
    return false;
  }
  for (int c = 0; c < 3; ++c) std::memcpy(img->quant[c], q[c], sizeof(img->quant[c]));
  img->BulkChanged();
  img->host_valid = need_host;
  device_.Set(*img);
  return true;
}

int DeviceJpegHistograms(Engine* e, const int q[3][kDCTBlockSize], JpegHistogram dc[3],
                         JpegHistogram ac[3], std::string* err) {
  uint32_t hist[6 * 256];
  uint64_t chroma = 0;
  if (!e->JpegStage(q, hist, &chroma)) {
    if (err) *err = e->error();
    return -1;
  }
  return HistogramsFromStage(hist, chroma, dc, ac);
}

int HistogramsFromStage(const uint32_t* hist, uint64_t chroma, JpegHistogram dc[3],
                        JpegHistogram ac[3]) {
  const int ncomp = chroma > 0 ? 3 : 1;  // SaveToJpegData drops all-zero chroma
  for (int c = 0; c < 3; ++c) {
    dc[c].Clear();
    ac[c].Clear();
    if (c >= ncomp) continue;
    for (int i = 0; i < 256; ++i) {
      dc[c].counts[i] = 2 * hist[(2 * c) * 256 + i];
      ac[c].counts[i] = 2 * hist[(2 * c + 1) * 256 + i];
    }
  }
  return ncomp;
}

bool PrepareScanFor(const JpegData& hdr, bool strip_metadata, int ncomp, JpegHistogram* dc_h,
                    JpegHistogram* ac_h, std::string* prologue, JpegCodeTables* codes) {
  HuffCodeTable dc_tab[3], ac_tab[3];
  prologue->clear();
  if (!WriteJpegPrologue(hdr, strip_metadata, dc_h, ac_h, dc_tab, ac_tab, prologue)) return false;
  std::memset(codes, 0, sizeof(*codes));
  for (int c = 0; c < ncomp; ++c)
    for (int i = 0; i < 256; ++i) {
      codes->dc_len[c][i] = dc_tab[c].depth[i];
      codes->ac_len[c][i] = ac_tab[c].depth[i];
      codes->dc_code[c][i] = static_cast<uint16_t>(dc_tab[c].code[i]);
      codes->ac_code[c][i] = static_cast<uint16_t>(ac_tab[c].code[i]);
    }
  return true;
}

bool PrepareScan(int w, int h, const int q[3][kDCTBlockSize], const JpegData& meta,
                 bool strip_metadata, int ncomp, JpegHistogram* dc_h, JpegHistogram* ac_h,
                 std::string* prologue, JpegCodeTables* codes) {
  JpegData hdr;
  hdr.app_data = meta.app_data;
  hdr.com_data = meta.com_data;
  JpegHeaderFor(w, h, q, ncomp, &hdr);
  return PrepareScanFor(hdr, strip_metadata, ncomp, dc_h, ac_h, prologue, codes);
}

bool DeviceEncodeJpeg(Engine* e, int w, int h, const int q[3][kDCTBlockSize], const JpegData& meta,
                      bool strip_metadata, std::string* prologue, size_t* size, std::string* err) {
  JpegHistogram dc_h[3], ac_h[3];
  const int ncomp = DeviceJpegHistograms(e, q, dc_h, ac_h, err);
  if (ncomp < 0) return false;
  JpegCodeTables codes;
  if (!PrepareScan(w, h, q, meta, strip_metadata, ncomp, dc_h, ac_h, prologue, &codes)) {
    if (err) *err = "jpeg header";
    return false;
  }
  uint64_t nbits = 0, ff = 0;
  if (!e->JpegScan(ncomp, q, codes, &nbits, &ff)) {
    if (err) *err = e->error();
    return false;
  }
  // prologue + scan bytes (padded) + a stuffed 0x00 per 0xff + EOI
  *size = prologue->size() + static_cast<size_t>((nbits + 7) / 8 + ff) + 2;
  return true;
}

bool DeviceFetchJpeg(Engine* e, bool kept, const std::string& prologue, size_t size,
                     std::string* out, std::string* err) {
  const uint8_t* bytes = nullptr;
  uint64_t nbits = 0;
  if (!e->JpegFetch(kept, &bytes, &nbits)) {
    if (err) *err = e->error();
    return false;
  }
  *out = prologue;
  AppendStuffedScan(bytes, nbits, out);
  if (out->size() != size) {  // the device's size prediction is what the search scored
    if (err) *err = "device JPEG size prediction mismatch";
    return false;
  }
  return true;
}

bool DeviceWriteJpeg(Engine* e, int w, int h, const int q[3][kDCTBlockSize], const JpegData& meta,
                     bool strip_metadata, std::string* out, std::string* err) {
  std::string prologue;
  size_t size = 0;
  return DeviceEncodeJpeg(e, w, h, q, meta, strip_metadata, &prologue, &size, err) &&
         DeviceFetchJpeg(e, false, prologue, size, out, err);
}

int HipButteraugliComparator::DeviceHistograms(const CoeffImage& img, JpegHistogram dc[3],
                                               JpegHistogram ac[3]) {
  if (!SyncCoeffs(img)) return -1;
  return DeviceJpegHistograms(engine_.get(), img.quant, dc, ac, &err_);
}

bool HipButteraugliComparator::DeviceWriteJpeg(const CoeffImage& img, const JpegData& meta,
                                               bool strip_metadata, std::string* out) {
  if (!SyncCoeffs(img)) return false;
  return gz::DeviceWriteJpeg(engine_.get(), w_, h_, img.quant, meta, strip_metadata, out, &err_);
}

bool HipButteraugliComparator::DeviceEncodeAndCompare(const CoeffImage& img,
                                                      const JpegData& meta, bool strip_metadata,
                                                      size_t* size) {
  return EncodeAndCompareWith(img, meta, nullptr, strip_metadata, size);
}

// The reference's first output, OutputJpeg(jpg_in) (processor.cc:965-967),
// when jpg_in holds img's coefficients as they are (every quant value 1, as
// for RGB input, one block per MCU): its scan is the device coder's scan of
// img, only the headers are jpg_in's own (three quant tables where
// SaveToJpegData shares one), so the size -- and, if it is kept, the bytes --
// come from the device with jpg_in's prologue.  Not used (*used = false;
// the Compare is done) when SaveToJpegData would drop all-zero chroma that
// jpg_in keeps.
bool HipButteraugliComparator::DeviceEncodeOriginalAndCompare(const CoeffImage& img,
                                                              const JpegData& jpg_in,
                                                              bool strip_metadata, size_t* size,
                                                              bool* used) {
  JpegData hdr;
  JpegHeaderOf(jpg_in, &hdr);
  *used = true;
  if (!EncodeAndCompareWith(img, jpg_in, &hdr, strip_metadata, size)) {
    if (err_ != "jpeg header components") return false;
    err_.clear();
    *used = false;
  }
  return true;
}

bool HipButteraugliComparator::EncodeAndCompareWith(const CoeffImage& img, const JpegData& meta,
                                                    const JpegData* hdr, bool strip_metadata,
                                                    size_t* size) {
  // One stream order: histogram stage, Compare pass, then the scan; the host
  // builds the Huffman codes from the staged histograms while the Compare
  // pass runs, and waits once for both results.
  const auto t0 = Clock::now();
  const double c0 = ThreadCpu();
  if (!SyncCoeffs(img)) return false;
  Engine* e = engine_.get();
  uint32_t hist[6 * 256];
  uint64_t chroma = 0;
  if (!e->JpegStageEnqueue(img.quant) || !e->CompareEnqueue()) {
    err_ = e->error();
    return false;
  }
  const auto tw0 = Clock::now();
  const double cw0 = ThreadCpu();
  if (!e->JpegStageWait(hist, &chroma)) {
    err_ = e->error();
    return false;
  }
  seconds_wait += Since(tw0);
  cpu_wait += ThreadCpu() - cw0;
  JpegHistogram dc_h[3], ac_h[3];
  const int ncomp = HistogramsFromStage(hist, chroma, dc_h, ac_h);
  JpegCodeTables codes;
  if (hdr && static_cast<int>(hdr->components.size()) != ncomp) {
    // (the Compare is in the stream: finish it)
    if (!e->Sync()) {
      err_ = e->error();
      return false;
    }
    (void)e->CompareFinish(&distance_, nullptr);
    block_max_stale_ = true;
    ++compares;
    seconds_compare += Since(t0);
    cpu_compare += ThreadCpu() - c0;
    err_ = "jpeg header components";
    return false;
  }
  if (!(hdr ? PrepareScanFor(*hdr, strip_metadata, ncomp, dc_h, ac_h, &cur_prologue_, &codes)
            : PrepareScan(w_, h_, img.quant, meta, strip_metadata, ncomp, dc_h, ac_h, &cur_prologue_,
                          &codes))) {
    err_ = "jpeg header";
    return false;
  }
  seconds_encode += Since(t0);
  uint64_t nbits = 0, ff = 0;
  if (!e->JpegScanEnqueue(ncomp, img.quant, codes)) {
    err_ = e->error();
    return false;
  }
  const auto tw1 = Clock::now();
  const double cw1 = ThreadCpu();
  if (!e->Sync() || !e->JpegScanFinish(&nbits, &ff)) {
    err_ = e->error();
    return false;
  }
  seconds_wait += Since(tw1);
  cpu_wait += ThreadCpu() - cw1;
  (void)e->CompareFinish(&distance_, nullptr);
  block_max_stale_ = true;
  ++compares;
  // prologue + scan bytes (padded) + a stuffed 0x00 per 0xff + EOI
  cur_size_ = cur_prologue_.size() + static_cast<size_t>((nbits + 7) / 8 + ff) + 2;
  *size = cur_size_;
  seconds_compare += Since(t0);
  cpu_compare += ThreadCpu() - c0;
  return true;
}

bool HipButteraugliComparator::DeviceEncode(const CoeffImage& img, const JpegData& meta,
                                            bool strip_metadata, size_t* size) {
  if (!SyncCoeffs(img)) return false;
  if (!DeviceEncodeJpeg(engine_.get(), w_, h_, img.quant, meta, strip_metadata, &cur_prologue_,
                        &cur_size_, &err_))
    return false;
  *size = cur_size_;
  return true;
}

void HipButteraugliComparator::DeviceKeepEncoded() {
  engine_->JpegKeep();
  kept_prologue_.swap(cur_prologue_);
  kept_size_ = cur_size_;
}

bool HipButteraugliComparator::DeviceFetchKept(std::string* out) {
  return DeviceFetchJpeg(engine_.get(), true, kept_prologue_, kept_size_, out, &err_);
}

bool HipButteraugliComparator::StartBlockComparisons() {
  if (!engine_->StartBlockComparisons(nullptr)) {
    err_ = engine_->error();
    return false;
  }
  return true;
}

bool HipButteraugliComparator::BlockZeroingOrders(const CoeffImage& img, const JpegData&,
                                                  int comp_mask, int lookahead, bool new_model,
                                                  std::vector<CoeffData>* out) {
  const auto t0 = Clock::now();
  if (!SyncCoeffs(img)) return false;
  out->resize(static_cast<size_t>(img.blocks) * 192);
  static_assert(sizeof(CoeffData) == sizeof(CoeffDataHost), "CoeffData layout");
  if (!engine_->BlockZeroingOrders(comp_mask, target_, lookahead, new_model,
                                   reinterpret_cast<CoeffDataHost*>(out->data()))) {
    err_ = engine_->error();
    return false;
  }
  seconds_zeroing += Since(t0);
  return true;
}

bool Comparator::BlockZeroingCandidates(const CoeffImage& img, const JpegData& orig_jpg,
                                        int comp_mask, int lookahead, bool new_model,
                                        std::vector<int>* offsets, std::vector<uint8_t>* idx,
                                        std::vector<float>* err) {
  std::vector<CoeffData> order;
  if (!BlockZeroingOrders(img, orig_jpg, comp_mask, lookahead, new_model, &order)) return false;
  const float limit = BlockErrorLimit();
  offsets->assign(img.blocks + 1, 0);
  idx->clear();
  err->clear();
  for (int b = 0; b < img.blocks; ++b) {
    const CoeffData* p = &order[static_cast<size_t>(b) * 192];
    (*offsets)[b] = static_cast<int>(idx->size());
    for (int i = 0; i < 192; ++i) {
      if (p[i].block_err > 0 && p[i].block_err <= limit) {
        idx->push_back(static_cast<uint8_t>(p[i].idx));
        err->push_back(p[i].block_err);
      }
    }
  }
  (*offsets)[img.blocks] = static_cast<int>(idx->size());
  return true;
}

bool HipButteraugliComparator::BlockZeroingCandidates(const CoeffImage& img, const JpegData&,
                                                      int comp_mask, int lookahead, bool new_model,
                                                      std::vector<int>* offsets,
                                                      std::vector<uint8_t>* idx,
                                                      std::vector<float>* err) {
  const auto t0 = Clock::now();
  if (!SyncCoeffs(img)) return false;
  if (!engine_->BlockZeroingCandidates(comp_mask, target_, lookahead, new_model, offsets, idx,
                                       err)) {
    err_ = engine_->error();
    return false;
  }
  seconds_zeroing += Since(t0);
  return true;
}

bool HipButteraugliComparator::SetOriginalCoeffs420(const JpegData& jpg420) {
  // the luma at the engine's block width (the 4:2:0 file pads Y to whole
  // MCUs), the chroma as stored; q = 1, so these are the raw values the
  // zeroing keys and the back end read (processor.cc:653-657, 865-868)
  const int bw = engine_->block_w(), bh = engine_->block_h();
  const int cbw = (w_ + 15) / 16, cbh = (h_ + 15) / 16;
  if (jpg420.components.size() != 3) {
    err_ = "4:2:0 originals need 3 components";
    return false;
  }
  std::vector<coeff_t> y(static_cast<size_t>(bw) * bh * 64), c[2];
  const JpegComponent& jy = jpg420.components[0];
  for (int by = 0; by < bh; ++by)
    std::memcpy(&y[static_cast<size_t>(by) * bw * 64], &jy.coeffs[static_cast<size_t>(by) * jy.width_in_blocks * 64],
                static_cast<size_t>(bw) * 64 * sizeof(coeff_t));
  for (int k = 0; k < 2; ++k) {
    const JpegComponent& jc = jpg420.components[1 + k];
    c[k].resize(static_cast<size_t>(cbw) * cbh * 64);
    for (int by = 0; by < cbh; ++by)
      std::memcpy(&c[k][static_cast<size_t>(by) * cbw * 64], &jc.coeffs[static_cast<size_t>(by) * jc.width_in_blocks * 64],
                  static_cast<size_t>(cbw) * 64 * sizeof(coeff_t));
  }
  orig_on_device_ = false;  // (the 4:4:4 originals are gone from the device)
  device_ = CoeffCursor();
  if (!engine_->SetOriginal420(y.data(), c[0].data(), c[1].data())) {
    err_ = engine_->error();
    return false;
  }
  return true;
}

bool HipButteraugliComparator::Compare420(const Image420& img) {
  const auto t0 = Clock::now();
  device_ = CoeffCursor();
  if (!engine_->Set420(img.y.data(), img.c[0].data(), img.c[1].data(), img.plane[0].px.data(),
                       img.plane[1].px.data()) ||
      !engine_->Compare(&distance_, nullptr, nullptr)) {
    err_ = engine_->error();
    return false;
  }
  block_max_stale_ = true;
  ++compares;
  seconds_compare += Since(t0);
  return true;
}

bool HipButteraugliComparator::BlockZeroingCandidates420(Image420* img, int comp_mask, int lookahead,
                                                         bool new_model, std::vector<int>* offsets,
                                                         std::vector<uint8_t>* idx,
                                                         std::vector<float>* err) {
  const auto t0 = Clock::now();
  device_ = CoeffCursor();
  if (!engine_->Set420(img->y.data(), img->c[0].data(), img->c[1].data(), img->plane[0].px.data(),
                       img->plane[1].px.data()) ||
      !engine_->BlockZeroingCandidates420(comp_mask, target_, lookahead, new_model, offsets, idx, err,
                                          img->plane[0].px.data(), img->plane[1].px.data())) {
    err_ = engine_->error();
    return false;
  }
  seconds_zeroing += Since(t0);
  return true;
}

bool HipButteraugliComparator::DeviceOrderReset(bool* available) {
  *available = false;
  if (!engine_->HasOrderCandidates()) return true;
  // (an allocation failure leaves the order on the host; a stream or launch
  // error fails the encode)
  bool unavailable = false;
  if (!engine_->OrderReset(&unavailable)) {
    err_ = engine_->error();
    return false;
  }
  *available = !unavailable;
  return true;
}

bool HipButteraugliComparator::DeviceChangeOrder(int direction, double target_mul, bool zero_bmax,
                                                 const std::vector<int>& last_indexes, float floor_limit,
                                                 size_t* n_entries, int* blocks_to_change, int64_t* below_floor) {
  // (ComputeBlockErrorAdjustmentWeights' target distance: target * target_mul
  // in double, butteraugli_comparator.cc:175)
  const double td = target_ * target_mul;
  *n_entries = 0;
  for (int rblock = 1; rblock <= 4; ++rblock) {
    // (the entries are filled with the counts: one wait per radius)
    const bool ok = engine_->OrderBuild(direction, rblock, td, zero_bmax, last_indexes, n_entries,
                                        blocks_to_change, floor_limit, below_floor);
    if (!ok) err_ = engine_->error();
    if (order_x_) {
      // a frame split over ranks: the radius is the first with entries
      // anywhere in the frame; the counts are the frame's
      uint32_t t[4] = {static_cast<uint32_t>(ok ? *n_entries : 0), static_cast<uint32_t>(ok ? *blocks_to_change : 0),
                       static_cast<uint32_t>(ok && below_floor ? *below_floor : 0), 0};
      if (!order_x_->SumU32(ok, t, 3)) {
        if (ok) err_ = "change order: a rank failed";
        return false;
      }
      *n_entries = t[0];
      *blocks_to_change = static_cast<int>(t[1]);
      if (below_floor) *below_floor = t[2];
      engine_->SetOrderFrameEntries(*n_entries);
    }
    if (!ok) return false;
    if (*n_entries) break;
  }
  return true;
}

void HipButteraugliComparator::SetDeviceOrderScope(int own_lo, int own_hi, int gbase, Engine::OrderExchange* x) {
  order_x_ = x;
  order_gbase_ = x ? gbase : 0;
  if (x) engine_->SetOrderScope(own_lo, own_hi, gbase, x);
  else engine_->SetOrderScope(0, 1 << 30, 0, nullptr);
}

bool HipButteraugliComparator::DeviceSetBlockMax(const std::vector<float>& bmax) {
  if (static_cast<int>(bmax.size()) != engine_->blocks() || !engine_->SetBlockMax(bmax.data())) {
    err_ = bmax.size() != static_cast<size_t>(engine_->blocks()) ? "DeviceSetBlockMax: size" : engine_->error();
    return false;
  }
  return true;
}

bool HipButteraugliComparator::DeviceOrderEntries(std::vector<std::pair<int, float>>* order) {
  const auto t0 = Clock::now();
  order->resize(engine_->OrderEntryCount());
  if (!engine_->OrderFetch(order->data(), order->size())) {
    err_ = engine_->error();
    return false;
  }
  // (a strip's entries in frame block indices, as the host build's)
  if (order_gbase_)
    for (auto& e : *order) e.first += order_gbase_;
  seconds_bulk += Since(t0);
  return true;
}

bool HipButteraugliComparator::DeviceSelectBulk(const CoeffImage& img, size_t bulk, size_t window, int direction,
                                                Engine::OrderSelection* sel, JpegHistogram ac[3]) {
  const auto t0 = Clock::now();
  if (bulk && !SyncCoeffs(img)) return false;
  int32_t delta[3][256];
  const bool ok = engine_->OrderSelect(bulk, window, direction, img.quant, true, sel, delta);
  if (!ok) err_ = engine_->error();
  if (order_x_ && (!ok || sel->applied)) {
    // a frame split over ranks: the frame's histogram change (every rank's
    // applies to its owned blocks; the same `applied` on every rank)
    std::vector<uint32_t> d(3 * 256);
    for (int c = 0; c < 3; ++c)
      for (int i = 0; i < 256; ++i) d[c * 256 + i] = ok ? static_cast<uint32_t>(delta[c][i]) : 0u;
    if (!order_x_->SumU32(ok, d.data(), 3 * 256)) {
      if (ok) err_ = "bulk prefix: a rank failed";
      return false;
    }
    for (int c = 0; c < 3; ++c)
      for (int i = 0; i < 256; ++i) delta[c][i] = static_cast<int32_t>(d[c * 256 + i]);
  }
  if (!ok) return false;
  if (sel->applied) {
    // (the counts are stored doubled, JpegHistogram::Add)
    for (int c = 0; c < 3; ++c)
      for (int i = 0; i < 256; ++i) ac[c].counts[i] += 2u * static_cast<uint32_t>(delta[c][i]);
  }
  seconds_bulk += Since(t0);
  return true;
}

bool HipButteraugliComparator::DeviceSelectWindow(size_t from, size_t window, int direction,
                                                  Engine::OrderSelection* sel) {
  const auto t0 = Clock::now();
  int32_t delta[3][256];
  const int q[3][kDCTBlockSize] = {};
  if (!engine_->OrderSelect(from, window, direction, q, false, sel, delta)) {
    err_ = engine_->error();
    return false;
  }
  seconds_bulk += Since(t0);
  return true;
}

bool HipButteraugliComparator::DeviceBulkApplyLocal(const CoeffImage& img, int direction, const uint8_t* cnt,
                                                    const std::vector<int>& last_indexes, int32_t delta[3][256]) {
  const auto t0 = Clock::now();
  if (!SyncCoeffs(img)) return false;
  if (!engine_->BulkApply(direction, img.quant, cnt, delta, &last_indexes)) {
    err_ = engine_->error();
    return false;
  }
  seconds_bulk += Since(t0);
  return true;
}

bool HipButteraugliComparator::DeviceBulkApply(const CoeffImage& img, int direction, const uint8_t* cnt,
                                               JpegHistogram ac[3]) {
  const auto t0 = Clock::now();
  if (!SyncCoeffs(img)) return false;
  int32_t delta[3][256];
  if (!engine_->BulkApply(direction, img.quant, cnt, delta)) {
    err_ = engine_->error();
    return false;
  }
  // (the counts are stored doubled, JpegHistogram::Add)
  for (int c = 0; c < 3; ++c)
    for (int i = 0; i < 256; ++i) ac[c].counts[i] += 2u * static_cast<uint32_t>(delta[c][i]);
  seconds_bulk += Since(t0);
  return true;
}

// The scan's bit count from the histograms the candidate is coded with:
// every symbol's code length plus its extra bits (the DC category; an AC
// symbol's low nibble).  Without the 0xff stuffing and the padding this is
// what k_jpeg_code counts, so prologue + ceil(bits / 8) + EOI bounds the
// candidate's size from below.
uint64_t ScanBits(const JpegHistogram dc[3], const JpegHistogram ac[3], int ncomp,
                  const JpegCodeTables& codes) {
  uint64_t bits = 0;
  for (int c = 0; c < ncomp; ++c)
    for (int i = 0; i < 256; ++i) {
      // (the counts are stored doubled, JpegHistogram::Add)
      bits += static_cast<uint64_t>(dc[c].counts[i] / 2) * (codes.dc_len[c][i] + i);
      bits += static_cast<uint64_t>(ac[c].counts[i] / 2) * (codes.ac_len[c][i] + (i & 15));
    }
  return bits;
}

// The distance at and above which ScoreJPEG(distance, size, target) >= best
// for every size >= size_lb (processor.cc:151-160 keeps a candidate only
// when its score is below the best; ScoreJPEG, score.cc:23-34, grows with the
// distance and with the size), with a margin; -inf when no size from size_lb
// up can beat best at any distance.
static double HopelessDistance(double best, size_t size_lb, double target) {
  const double s = static_cast<double>(size_lb);
  if (s >= best) return -HUGE_VAL;
  const double kScale = 50, kMaxExponent = 10, kLargeSize = 1e30;
  double diff = std::log(best / s) / kScale;  // exp(kScale * diff) * size_lb >= best
  if (diff > kMaxExponent / kScale)           // above it the linear branch decides
    diff = std::max(kMaxExponent / kScale, (best - s) / (kLargeSize * std::exp(kMaxExponent)));
  return target + diff + 1e-6;
}

bool HipButteraugliComparator::DeviceEncodeAndCompareKnown(const CoeffImage& img, const JpegData& meta,
                                                           bool strip_metadata, const JpegHistogram dc[3],
                                                           const JpegHistogram ac[3], int ncomp,
                                                           double best_score, size_t* size, bool* skipped) {
  // the Compare pass first; the codes on the host while it runs; the scan
  // behind it (not coded when the pass's distance shows the candidate
  // cannot become the output); one wait
  const auto t0 = Clock::now();
  const double c0 = ThreadCpu();
  *skipped = false;
  if (!SyncCoeffs(img)) return false;
  Engine* e = engine_.get();
  if (!e->CompareEnqueue()) {
    err_ = e->error();
    return false;
  }
  JpegHistogram dc_h[3], ac_h[3];
  for (int c = 0; c < ncomp; ++c) {
    dc_h[c] = dc[c];
    ac_h[c] = ac[c];
  }
  JpegCodeTables codes;
  if (!PrepareScan(w_, h_, img.quant, meta, strip_metadata, ncomp, dc_h, ac_h, &cur_prologue_, &codes)) {
    err_ = "jpeg header";
    return false;
  }
  const uint64_t bound_bits = ScanBits(dc, ac, ncomp, codes);
  const size_t size_lb = cur_prologue_.size() + static_cast<size_t>((bound_bits + 7) / 8) + 2;
  float skip_at = HUGE_VALF;
  if (best_score >= 0 && scan_bound_mismatches == 0) {
    const double d = HopelessDistance(best_score, size_lb, target_);
    if (d <= -HUGE_VAL) {
      skip_at = -HUGE_VALF;
    } else if (d < 1e30) {
      skip_at = std::nextafter(static_cast<float>(d), HUGE_VALF);
    }
  }
  seconds_encode += Since(t0);
  uint64_t nbits = 0, ff = 0;
  if (!e->JpegScanEnqueue(ncomp, img.quant, codes, skip_at)) {
    err_ = e->error();
    return false;
  }
  const auto tw = Clock::now();
  const double cw = ThreadCpu();
  if (!e->Sync()) {
    err_ = e->error();
    return false;
  }
  seconds_wait += Since(tw);
  cpu_wait += ThreadCpu() - cw;
  (void)e->CompareFinish(&distance_, nullptr);
  block_max_stale_ = true;
  ++compares;
  if (skip_at != HUGE_VALF && distance_ >= skip_at) {  // (k_jpeg_code's own test, on the same float)
    if (ScoreJPEG(distance_, static_cast<int>(size_lb), target_) >= best_score) {
      *skipped = true;
      ++scans_skipped;
      seconds_compare += Since(t0);
      cpu_compare += ThreadCpu() - c0;
      return true;
    }
    // (the margin makes this unreachable; code the scan after all)
    if (!e->JpegScanEnqueue(ncomp, img.quant, codes) || !e->Sync()) {
      err_ = e->error();
      return false;
    }
  }
  if (!e->JpegScanFinish(&nbits, &ff)) {
    err_ = e->error();
    return false;
  }
  if (nbits != bound_bits) ++scan_bound_mismatches;
  cur_size_ = cur_prologue_.size() + static_cast<size_t>((nbits + 7) / 8 + ff) + 2;
  *size = cur_size_;
  seconds_compare += Since(t0);
  cpu_compare += ThreadCpu() - c0;
  return true;
}

bool HipButteraugliComparator::DeviceOrderAdvance(float val_threshold, int direction) {
  if (!engine_->OrderAdvance(val_threshold, direction)) {
    err_ = engine_->error();
    return false;
  }
  return true;
}

double HipButteraugliComparator::ScoreOutputSize(int size) const {
  return ScoreJPEG(distance_, size, target_);
}

void HipButteraugliComparator::ComputeBlockErrorAdjustmentWeights(
    int direction, int max_block_dist, double target_mul, int factor_x, int factor_y,
    const std::vector<float>& max_dist_per_block, std::vector<float>* block_weight) {
  BlockErrorAdjustmentWeights(w_, h_, target_, direction, max_block_dist, target_mul, factor_x,
                              factor_y, max_dist_per_block, block_weight);
}

void BlockErrorAdjustmentWeights(int w, int h, float target, int direction, int max_block_dist,
                                 double target_mul, int factor_x, int factor_y,
                                 const std::vector<float>& max_dist_per_block,
                                 std::vector<float>* block_weight) {
  // butteraugli_comparator.cc:169-233 (block maxima come from the device).
  // Rows of blocks in parallel; the direction < 0 scatter of the reference
  // (every over-target block raises its neighbours to 1 / (d + 1)) is formed
  // as the equivalent gather -- a max over the same values, order-free.
  const double target_distance = target * target_mul;
  const int sizex = 8 * factor_x, sizey = 8 * factor_y;
  const int bw = (w + sizex - 1) / sizex, bh = (h + sizey - 1) / sizey;
  const int r = max_block_dist;
  constexpr int kRows = 8;
  const int chunks = (bh + kRows - 1) / kRows;
  const size_t nblk = static_cast<size_t>(bw) * bh;
  // max_local(bx, by) = max(target, block maxima within Chebyshev radius r),
  // separably: the row maxima over [bx - r, bx + r], then their maximum over
  // [by - r, by + r] (a max of the same values: exact)
  std::vector<float> rowmax(nblk), local(nblk);
  ParallelFor(chunks, [&](int ch) {
    for (int by = ch * kRows; by < std::min(bh, (ch + 1) * kRows); ++by)
      for (int bx = 0; bx < bw; ++bx) {
        float m = static_cast<float>(target_distance);
        for (int x = std::max(0, bx - r); x < std::min(bw, bx + 1 + r); ++x)
          m = std::max(m, max_dist_per_block[by * bw + x]);
        rowmax[by * bw + bx] = m;
      }
  });
  ParallelFor(chunks, [&](int ch) {
    for (int by = ch * kRows; by < std::min(bh, (ch + 1) * kRows); ++by)
      for (int bx = 0; bx < bw; ++bx) {
        float m = static_cast<float>(target_distance);
        for (int y = std::max(0, by - r); y < std::min(bh, by + 1 + r); ++y) m = std::max(m, rowmax[y * bw + bx]);
        local[by * bw + bx] = m;
      }
  });
  if (direction > 0) {
    ParallelFor(chunks, [&](int ch) {
      for (int by = ch * kRows; by < std::min(bh, (ch + 1) * kRows); ++by)
        for (int bx = 0; bx < bw; ++bx) {
          const int bix = by * bw + bx;
          if (max_dist_per_block[bix] <= target_distance && local[bix] <= 1.1 * target_distance)
            (*block_weight)[bix] = 1.0;
        }
    });
    return;
  }
  constexpr double kLocalMaxWeight = 0.5;
  std::vector<uint8_t> active(nblk);
  ParallelFor(chunks, [&](int ch) {
    for (int by = ch * kRows; by < std::min(bh, (ch + 1) * kRows); ++by)
      for (int bx = 0; bx < bw; ++bx) {
        const int bix = by * bw + bx;
        active[bix] = !(max_dist_per_block[bix] <=
                        (1 - kLocalMaxWeight) * target_distance + kLocalMaxWeight * local[bix]);
      }
  });
  // every active block within Chebyshev distance d <= r raises the weight to
  // 1 / (d + 1): the largest such term is the nearest active block's, found
  // separably (nearest active in the row, then min over rows of
  // max(|dy|, that)); the weight is the max of the same float terms as the
  // per-neighbour loop
  std::vector<int> hx(nblk);
  ParallelFor(chunks, [&](int ch) {
    for (int by = ch * kRows; by < std::min(bh, (ch + 1) * kRows); ++by)
      for (int bx = 0; bx < bw; ++bx) {
        int d = r + 1;
        for (int x = std::max(0, bx - r); x < std::min(bw, bx + 1 + r); ++x)
          if (active[by * bw + x]) d = std::min(d, std::abs(x - bx));
        hx[by * bw + bx] = d;
      }
  });
  ParallelFor(chunks, [&](int ch) {
    for (int by = ch * kRows; by < std::min(bh, (ch + 1) * kRows); ++by)
      for (int bx = 0; bx < bw; ++bx) {
        const int ix = by * bw + bx;
        int d = r + 1;
        for (int y = std::max(0, by - r); y < std::min(bh, by + 1 + r); ++y)
          d = std::min(d, std::max(std::abs(y - by), hx[y * bw + bx]));
        if (d <= r) (*block_weight)[ix] = std::max<float>((*block_weight)[ix], 1.0f / (d + 1.0f));
      }
  });
}

// ---------------------------------------------------------------------------
// Processor
// ---------------------------------------------------------------------------

namespace {

struct QuantData {
  int q[3][kDCTBlockSize];
  size_t jpg_size;
  bool dist_ok;
};

double ContrastSensitivity(int k) { return 1.0 / (1.0 + kJPEGZigZagOrder[k] / 2.0); }

double QuantMatrixHeuristicScore(const int q[3][kDCTBlockSize]) {
  double score = 0.0;
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < kDCTBlockSize; ++k) score += 0.5 * (q[c][k] - 1.0) * ContrastSensitivity(k);
  return score;
}

// -1 / 0 / 1 / 2 ordering of two quant matrices (processor.cc:168-190).
int CompareQuantMatrices(const int* a, const int* b) {
  const int n = 3 * kDCTBlockSize;
  int i = 0;
  while (i < n && a[i] == b[i]) ++i;
  if (i == n) return 0;
  if (a[i] < b[i]) {
    for (++i; i < n; ++i)
      if (a[i] > b[i]) return 2;
    return -1;
  }
  for (++i; i < n; ++i)
    if (a[i] < b[i]) return 2;
  return 1;
}

bool CompareQuantData(const QuantData& a, const QuantData& b) {
  if (a.dist_ok && !b.dist_ok) return true;
  if (!a.dist_ok && b.dist_ok) return false;
  return a.jpg_size < b.jpg_size;
}

// Binary search over the heuristic quantization "score" (processor.cc:206-308).
class QuantMatrixGenerator {
 public:
  explicit QuantMatrixGenerator(bool downsample = false) : downsample_(downsample) {
    for (int k = 0; k < kDCTBlockSize; ++k) total_csf_ += 3.0 * ContrastSensitivity(k);
  }
  bool GetNext(int q[3][kDCTBlockSize]) {
    for (int iter = 0; iter < 1000; iter++) {
      double hscore;
      if (hscore_b_ == -1.0) {
        if (hscore_a_ == -1.0) {
          hscore = downsample_ ? 0.0 : total_csf_;
        } else if (hscore_a_ < 5.0 * total_csf_) {
          hscore = hscore_a_ + total_csf_;
        } else {
          hscore = 2 * (hscore_a_ + total_csf_);
        }
        if (hscore > 100 * total_csf_) return false;
      } else if (hscore_b_ == 0.0) {
        return false;
      } else if (hscore_a_ == -1.0) {
        hscore = 0.0;
      } else {
        int lower_q[3][kDCTBlockSize], upper_q[3][kDCTBlockSize];
        constexpr double kEps = 0.05;
        MatrixForScore((1 - kEps) * hscore_a_ + kEps * 0.5 * (hscore_a_ + hscore_b_), lower_q);
        MatrixForScore((1 - kEps) * hscore_b_ + kEps * 0.5 * (hscore_a_ + hscore_b_), upper_q);
        if (CompareQuantMatrices(&lower_q[0][0], &upper_q[0][0]) == 0) return false;
        hscore = (hscore_a_ + hscore_b_) * 0.5;
      }
      MatrixForScore(hscore, q);
      bool retry = false;
      for (const QuantData& d : quants_) {
        if (CompareQuantMatrices(&q[0][0], &d.q[0][0]) == 0) {
          if (d.dist_ok) hscore_a_ = hscore; else hscore_b_ = hscore;
          retry = true;
          break;
        }
      }
      if (!retry) return true;
    }
    return false;
  }
  void Add(const QuantData& d) {
    quants_.push_back(d);
    const double hscore = QuantMatrixHeuristicScore(d.q);
    if (d.dist_ok) hscore_a_ = std::max(hscore_a_, hscore);
    else hscore_b_ = hscore_b_ == -1.0 ? hscore : std::min(hscore_b_, hscore);
  }

 private:
  void MatrixForScore(double score, int q[3][kDCTBlockSize]) const {
    const int level = static_cast<int>(score / total_csf_);
    score -= level * total_csf_;
    for (int k = kDCTBlockSize - 1; k >= 0; --k) {
      for (int c = 0; c < 3; ++c) q[c][kJPEGNaturalOrder[k]] = 2 * level + (score > 0.0 ? 3 : 1);
      score -= 3.0 * ContrastSensitivity(kJPEGNaturalOrder[k]);
    }
  }
  bool downsample_;
  double hscore_a_ = -1.0, hscore_b_ = -1.0, total_csf_ = 0.0;
  std::vector<QuantData> quants_;
};

size_t ComputeEntropyCodes(const std::vector<JpegHistogram>& histograms, std::vector<uint8_t>* depths) {
  // processor.cc:517-536
  std::vector<JpegHistogram> clustered = histograms;
  size_t num = histograms.size();
  std::vector<int> indexes(num);
  std::vector<uint8_t> cdepths(num * JpegHistogram::kSize);
  ClusterHistograms(clustered.data(), &num, indexes.data(), cdepths.data());
  depths->resize(cdepths.size());
  for (size_t i = 0; i < histograms.size(); ++i)
    std::memcpy(&(*depths)[i * JpegHistogram::kSize], &cdepths[indexes[i] * JpegHistogram::kSize],
                JpegHistogram::kSize);
  size_t size = 0;
  for (size_t i = 0; i < num; ++i) size += HistogramHeaderCost(clustered[i]) / 8;
  return size;
}

// The AC histogram update of one coefficient change in the search loop
// (UpdateACHistogram(-1, block) / change / UpdateACHistogram(+1, block),
// processor.cc:491-515 and :869-874) done locally: in zigzag order a block's
// AC symbols are, per non-zero coefficient, the ZRLs and run/size symbol of
// the zero run before it, then EOB if zeros trail.  Changing the
// coefficient at zigzag position z only re-forms the symbols of the segment
// from the previous non-zero p to the next non-zero nx, so only those are
// removed and re-added (same counts as the full rescans).  raw_bits tracks
// sum_i (counts[i]/2) * (depth[i] + (i & 0xf)) -- HistogramEntropyCost
// before rounding -- for the current depths.
// The change loop's control for one back-end iteration (processor.cc:
// 836-905), shared by the 4:4:4 and the 4:2:0 back ends: the thresholds
// from the iteration's order, the decades whose entropy codes are read, when
// the size estimate is read and the break test.  The estimate is only read
// once changed > min_coeffs (and at the last step), and a decade's codes
// only if such a step reads them, so the codes of other decades are never
// built -- the same values wherever they are read.
struct ChangeLoop {
  size_t n_order;
  int min_coeffs;  // min_coeffs_to_change
  double min_size_delta;
  int changed = 0;
  float val_threshold = 0.0f;
  // factor: the searched blocks' size in 8x8 blocks (4:2:0 chroma: 2);
  // *first_up_iter: the first up iteration's floor on min_coeffs (the count
  // of keys below 0.75 x the block error limit), then cleared.
  // (n_total / below: the frame's entry count and count below the floor
  // when `order` holds only this rank's entries; else taken from order)
  ChangeLoop(int direction, bool distance_ok, int base_size, int factor, int blocks_to_change,
             bool* first_up_iter, float block_error_limit,
             const std::vector<std::pair<int, float>>& order, size_t n_total = SIZE_MAX,
             int64_t below_floor = -1)
      : n_order(n_total == SIZE_MAX ? order.size() : n_total) {
    double rel_size_delta = direction > 0 ? 0.01 : 0.0005;
    if (direction > 0 && distance_ok) rel_size_delta = 0.05;
    min_size_delta = base_size * rel_size_delta;
    const float per_block = direction > 0 ? 2.0f : factor * factor * 0.2f;
    min_coeffs = static_cast<int>(per_block * blocks_to_change);
    if (*first_up_iter) {
      const float limit = 0.75f * block_error_limit;
      // partition_point(key < limit) of the sorted order == count of keys below limit
      int below = static_cast<int>(below_floor);
      if (below_floor < 0) {
        below = 0;
        for (const auto& e : order) below += e.second < limit ? 1 : 0;
      }
      min_coeffs = std::max<int>(min_coeffs, below);
      *first_up_iter = false;
    }
  }
  void Applied(float key) {
    val_threshold = key;
    ++changed;
  }
  // after change i: its decade's codes are read (rebuild them), the estimate is read
  bool CodesRead(size_t i) const {
    return i % 10 == 0 && (i + 9 >= static_cast<size_t>(std::max(0, min_coeffs)) || i + 10 >= n_order);
  }
  bool EstimateRead(size_t i) const { return changed > min_coeffs || i + 1 == n_order; }
  bool Stop(int est, int prev) const { return changed > min_coeffs && std::abs(est - prev) > min_size_delta; }
};

struct AcBlockModel {
  std::vector<uint64_t> nz;  // [c * blocks + b]: bit z set <=> zigzag coefficient z non-zero
  float inv_q[3][kDCTBlockSize];  // 1 / quant (natural order), for Size

  void Build(const CoeffImage& img) {
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < kDCTBlockSize; ++k) inv_q[c][k] = 1.0f / static_cast<float>(img.quant[c][k]);
    nz.assign(static_cast<size_t>(3) * img.blocks, 0);
    for (int c = 0; c < 3; ++c)
      for (int b = 0; b < img.blocks; ++b) {
        const coeff_t* blk = img.block(c, b);
        uint64_t m = 0;
        for (int z = 0; z < 64; ++z) m |= static_cast<uint64_t>(blk[kJPEGNaturalOrder[z]] != 0) << z;
        nz[static_cast<size_t>(c) * img.blocks + b] = m;
      }
  }

  static int Size(coeff_t v, int q) { return Log2FloorNonZero(std::abs(v / q)) + 1; }
  // Size(v, q) without the integer division: |v| / q rounded through the
  // float reciprocal is within one of the quotient (|v| < 2^16, relative
  // error < 2^-22), and one multiply-compare settles it on the truncated one.
  static int SizeInv(coeff_t v, int q, float inv) {
    const int a = std::abs(static_cast<int>(v));
    int n = static_cast<int>(static_cast<float>(a) * inv + 0.5f);
    if (n * q > a) --n;
    return Log2FloorNonZero(static_cast<uint32_t>(n)) + 1;
  }

  // weight * symbols of the segment after non-zero position p (0 = none /
  // DC) through the non-zeros `mid` (0: none) and `nx` (0: none; then EOB
  // if the last one is below 63).
  // H: the histogram (JpegHistogram) or a recorder of the same Add calls.
  // kRaw = false: the histogram only (the bulk prefix, whose raw bits are
  // recomputed from the summed histograms)
  template <class H, bool kRaw = true>
  static void Segment(int weight, int p, int mid, int mid_size, int nx, int nx_size,
                      const uint8_t* depth, H* h, int64_t* raw) {
    int last = p;
    int64_t bits = 0;
    auto put = [&](int pos, int size) {
      int run = pos - last - 1;
      while (run > 15) {
        h->Add(0xf0, weight);
        if (kRaw) bits += depth[0xf0];
        run -= 16;
      }
      const int sym = (run << 4) + size;
      h->Add(sym, weight);
      if (kRaw) bits += depth[sym] + (sym & 0xf);
      last = pos;
    };
    if (mid) put(mid, mid_size);
    if (nx) {
      put(nx, nx_size);
    } else if (last < 63) {
      h->Add(0, weight);
      if (kRaw) bits += depth[0];
    }
    if (kRaw) *raw += weight * bits;
  }

  // The 4:2:0 image's blocks (Y, then Cb, Cr at factor 2): slot base[c] + b.
  void Build(const Image420& img, size_t base[3]) {
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < kDCTBlockSize; ++k) inv_q[c][k] = 1.0f / static_cast<float>(img.quant[c][k]);
    base[0] = 0;
    base[1] = static_cast<size_t>(img.Blocks(0));
    base[2] = base[1] + static_cast<size_t>(img.Blocks(1));
    nz.assign(base[2] + static_cast<size_t>(img.Blocks(2)), 0);
    for (int c = 0; c < 3; ++c)
      for (int b = 0; b < img.Blocks(c); ++b) {
        const coeff_t* blk = img.block(c, b);
        uint64_t m = 0;
        for (int z = 0; z < 64; ++z) m |= static_cast<uint64_t>(blk[kJPEGNaturalOrder[z]] != 0) << z;
        nz[base[c] + b] = m;
      }
  }

  // block[k] := newval with the histogram / raw-bit bookkeeping.
  template <class H, bool kRaw = true>
  void Change(int c, int bix, int blocks, coeff_t* block, int k, coeff_t newval, const int* q,
              const uint8_t* depth, H* h, int64_t* raw) {
    ChangeAt<H, kRaw>(static_cast<size_t>(c) * blocks + bix, c, block, k, newval, q, depth, h, raw);
  }
  template <class H, bool kRaw = true>
  void ChangeAt(size_t slot, int c, coeff_t* block, int k, coeff_t newval, const int* q, const uint8_t* depth,
                H* h, int64_t* raw) {
    const coeff_t old = block[k];
    block[k] = newval;
    const int z = kJPEGZigZagOrder[k];
    if (z == 0 || old == newval) return;  // DC is not an AC symbol
    uint64_t& m = nz[slot];
    const uint64_t below = m & ((1ull << z) - 1) & ~1ull;
    const uint64_t above = z < 63 ? m & ~((2ull << z) - 1) : 0;
    const int p = below ? 63 - __builtin_clzll(below) : 0;
    const int nx = above ? __builtin_ctzll(above) : 0;
    const int knx = kJPEGNaturalOrder[nx];
    const int nx_size = nx ? SizeInv(block[knx], q[knx], inv_q[c][knx]) : 0;
    Segment<H, kRaw>(-1, p, old ? z : 0, old ? SizeInv(old, q[k], inv_q[c][k]) : 0, nx, nx_size, depth, h,
                     raw);
    Segment<H, kRaw>(1, p, newval ? z : 0, newval ? SizeInv(newval, q[k], inv_q[c][k]) : 0, nx, nx_size, depth,
                     h, raw);
    if (newval) m |= 1ull << z; else m &= ~(1ull << z);
  }
};

// The symbol updates of one change, as the partitioned back end publishes
// them (the AcBlockModel::Change calls recorded instead of applied).
struct SymbolLog {
  uint8_t n = 0;
  uint8_t sym[32];
  int8_t weight[32];
  void Add(int s, int w) {
    sym[n] = static_cast<uint8_t>(s);
    weight[n] = static_cast<int8_t>(w);
    ++n;
  }
};

int64_t HistogramRawBits(const JpegHistogram& h, const uint8_t* depth) {
  int64_t bits = 0;
  for (int i = 0; i + 1 < JpegHistogram::kSize; ++i)
    bits += static_cast<int64_t>(h.counts[i] / 2) * (depth[i] + (i & 0xf));
  return bits;
}

// EntropyCodedDataSize from the per-histogram raw bit sums
// (HistogramEntropyCost's rounding applied per histogram).
int EntropySizeFromRaw(const std::vector<int64_t>& raw) {
  int64_t bits = 0;
  for (int64_t b : raw) bits += b + ((b * 3 + 512) >> 10);
  return static_cast<int>((bits + 7) / 8);
}

size_t EntropyCodedDataSize(const std::vector<JpegHistogram>& histograms,
                            const std::vector<uint8_t>& depths) {
  size_t bits = 0;
  for (size_t i = 0; i < histograms.size(); ++i)
    bits += HistogramEntropyCost(histograms[i], &depths[i * JpegHistogram::kSize]);
  return (bits + 7) / 8;
}

// The order of one back-end iteration's change entries on a frame split
// over ranks (host/strips.h), from every rank's own entries.  std::sort
// (processor.cc:840-843) is not stable, so where keys are equal its order
// is that of libstdc++'s introsort over the frame's array -- the exact path
// (LazyStdSort on every rank, after an all-gather of every entry).  But the
// loop consumes a prefix as a set and then a short tail in order, and those
// are functions of the keys alone wherever no key is shared by entries of
// two blocks (entries of one block are interchangeable: a change takes the
// block's next candidate, whichever entry named it).  So:
//   * Prefix: the bulk-th smallest key K* by a radix selection over every
//     rank's keys (three small all-sums of bucket counts); the prefix is
//     every key below K* plus the K*-keyed entries it reaches -- all of them,
//     or some of one block's; K* shared by several blocks across the
//     boundary leaves the set open (the caller takes the exact path);
//   * Next: the tail in windows, each rank's next entries (smallest first)
//     merged on every rank; a position is certified when no rank can still
//     hold a smaller key, and a tie of several blocks among the certified
//     entries ends the window there (open: the caller takes the exact path
//     from that position on -- the positions before it are the same in
//     std::sort's order).
// No rank gathers or sorts the frame's entries unless a tie leaves the
// order open.
class StripOrder {
 public:
  // Order-preserving bits of a float key (equal keys -- both zeros -- give
  // equal bits).
  static uint32_t Bits(float k) {
    if (k == 0.0f) return 0x80000000u;
    uint32_t u;
    std::memcpy(&u, &k, 4);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  }

  // cnt (num_blocks, local indices) := per owned block its entries among the
  // first `bulk` of the frame's order.  1: done; 0: open; -1: failed exchange.
  int Prefix(const std::vector<std::pair<int, float>>& local, size_t bulk, Partition* part, int gbase,
             int num_blocks, std::vector<int>* cnt) {
    // radix selection of the key of rank bulk - 1: 12 + 12 + 8 bits
    static const int kShift[3] = {20, 8, 0}, kBits[3] = {12, 12, 8};
    uint32_t prefix = 0;
    int64_t below = 0, eq = 0;
    const int64_t target = static_cast<int64_t>(bulk) - 1;
    for (int round = 0; round < 3; ++round) {
      const int sh = kShift[round], nb = kBits[round];
      std::vector<int64_t> h(static_cast<size_t>(1) << nb, 0);
      const int hi_sh = sh + nb;
      for (const auto& e : local) {
        const uint32_t u = Bits(e.second);
        if (hi_sh < 32 && (u >> hi_sh) != prefix) continue;
        ++h[(u >> sh) & ((1u << nb) - 1)];
      }
      if (!part->SumAll(h.data(), static_cast<int>(h.size()))) return -1;
      int64_t cum = below;
      uint32_t j = 0;
      for (; j + 1 < h.size() && cum + h[j] <= target; ++j) cum += h[j];
      below = cum;
      eq = h[j];
      prefix = (prefix << nb) | j;
    }
    kbits_ = prefix;
    tie_block_ = -1;
    take_ = 0;
    if (TestOpen() == 1) return 0;
    if (below + eq > static_cast<int64_t>(bulk)) {
      // K* straddles the boundary: determined only if one block holds every
      // entry keyed K* (local entries are in block order)
      std::vector<uint8_t> mine;
      int last = -1;
      for (const auto& e : local)
        if (Bits(e.second) == kbits_ && e.first != last) {
          last = e.first;
          mine.insert(mine.end(), reinterpret_cast<const uint8_t*>(&last),
                      reinterpret_cast<const uint8_t*>(&last) + 4);
        }
      std::vector<std::vector<uint8_t>> all;
      if (!part->coll->AllGatherV(mine, &all)) return -1;
      size_t blocks = 0;
      for (const auto& m : all) {
        blocks += m.size() / 4;
        if (m.size() >= 4) std::memcpy(&tie_block_, m.data(), 4);
      }
      if (blocks != 1) return 0;
      take_ = static_cast<int64_t>(bulk) - below;
    }
    cnt->assign(num_blocks, 0);
    for (const auto& e : local) {
      const uint32_t u = Bits(e.second);
      if (u < kbits_ || (u == kbits_ && tie_block_ < 0)) ++(*cnt)[e.first - gbase];
    }
    if (tie_block_ >= 0 && tie_block_ - gbase >= 0 && tie_block_ - gbase < num_blocks) {
      // (only the owner has entries of it; a halo block is never searched here)
      bool owner = false;
      for (const auto& e : local) owner = owner || e.first == tie_block_;
      if (owner) (*cnt)[tie_block_ - gbase] += static_cast<int>(take_);
    }
    have_prefix_ = true;
    return 1;
  }

  // This rank's entries after the prefix (all, without one), for Next.
  void StartTail(const std::vector<std::pair<int, float>>& local, bool after_prefix) {
    rem_.clear();
    int64_t skip = take_;
    for (const auto& e : local) {
      const uint32_t u = Bits(e.second);
      if (after_prefix) {
        if (u < kbits_) continue;
        if (u == kbits_) {
          if (tie_block_ < 0) continue;   // all K*-keyed entries are in the prefix
          if (skip > 0) {                 // the prefix's share of tie_block_'s
            --skip;
            continue;
          }
        }
      }
      rem_.push_back(Entry{u, e.first, e.second});
    }
    pos_ = 0;
    sorted_ = 0;
    static const size_t kFirst = [] {
      const char* w = std::getenv("GZ_STRIP_WINDOW");  // (tests: small windows)
      return static_cast<size_t>(w && std::atoi(w) > 0 ? std::atoi(w) : 1024);
    }();
    window_ = kFirst;
  }

  // The next certified positions of the frame's order.  *open: the position
  // after them starts a tie of several blocks.  1: ok; 0: every rank's
  // entries are consumed; -1: failed exchange.
  int Next(Partition* part, std::vector<int>* blocks, std::vector<float>* keys, bool* open) {
    *open = false;
    for (;;) {
      const size_t k = std::min(window_, rem_.size() - pos_);
      if (pos_ + k > sorted_) {
        // the smallest entries left, sorted, a good way ahead of the window
        const size_t want = std::min(rem_.size(), pos_ + std::max<size_t>(4 * k, 1 << 16));
        auto less = [](const Entry& a, const Entry& b) {
          return a.bits != b.bits ? a.bits < b.bits : a.block < b.block;
        };
        if (want < rem_.size()) std::nth_element(rem_.begin() + pos_, rem_.begin() + want, rem_.end(), less);
        std::sort(rem_.begin() + pos_, rem_.begin() + want, less);
        sorted_ = want;
      }
      std::vector<uint8_t> send(1 + 12 * k);
      send[0] = pos_ + k < rem_.size() ? 1 : 0;
      for (size_t i = 0; i < k; ++i) {
        const Entry& e = rem_[pos_ + i];
        std::memcpy(&send[1 + 12 * i], &e.bits, 4);
        std::memcpy(&send[5 + 12 * i], &e.block, 4);
        std::memcpy(&send[9 + 12 * i], &e.key, 4);
      }
      std::vector<std::vector<uint8_t>> all;
      if (!part->coll->AllGatherV(send, &all)) return -1;
      uint64_t bound = uint64_t{1} << 32;
      size_t sent = 0;
      for (const auto& m : all) {
        if (m.empty() || (m.size() - 1) % 12) return -1;
        const size_t n = (m.size() - 1) / 12;
        sent += n;
        if (m[0] && n) {
          uint32_t b;
          std::memcpy(&b, &m[1 + 12 * (n - 1)], 4);
          bound = std::min<uint64_t>(bound, b);
        }
      }
      if (sent == 0) return 0;
      struct M {
        uint32_t bits;
        int rank;
        size_t idx;
        int block;
        float key;
      };
      std::vector<M> merged;
      for (int r = 0; r < static_cast<int>(all.size()); ++r) {
        const auto& m = all[r];
        for (size_t i = 0; i < (m.size() - 1) / 12; ++i) {
          M x{0, r, i, 0, 0.0f};
          std::memcpy(&x.bits, &m[1 + 12 * i], 4);
          std::memcpy(&x.block, &m[5 + 12 * i], 4);
          std::memcpy(&x.key, &m[9 + 12 * i], 4);
          if (x.bits < bound) merged.push_back(x);
        }
      }
      if (merged.empty()) {  // every sent key at the bound: wider windows
        window_ *= 2;
        continue;
      }
      std::sort(merged.begin(), merged.end(), [](const M& a, const M& b) {
        return a.bits != b.bits ? a.bits < b.bits : (a.rank != b.rank ? a.rank < b.rank : a.idx < b.idx);
      });
      // the first tie of several blocks ends the certified positions at its group's start
      size_t end = merged.size();
      for (size_t t = 1; t < merged.size(); ++t)
        if (merged[t].bits == merged[t - 1].bits && merged[t].block != merged[t - 1].block) {
          size_t g = t - 1;
          while (g > 0 && merged[g - 1].bits == merged[t].bits) --g;
          end = g;
          *open = true;
          break;
        }
      if (TestOpen() == 2 && end > 1) {  // (tests: the fallback in mid-tail)
        end /= 2;
        *open = true;
      }
      const int me = part->rank;
      blocks->clear();
      keys->clear();
      mine_.clear();
      for (size_t t = 0; t < end; ++t) {
        blocks->push_back(merged[t].block);
        keys->push_back(merged[t].key);
        mine_.push_back(merged[t].rank == me ? 1 : 0);
      }
      return 1;
    }
  }

  // GZ_STRIP_TEST_OPEN=prefix / tail: report the prefix / the middle of the
  // first tail window as open, so that tests take the exact path from there
  // (the result must not change).
  static int TestOpen() {
    static const int v = [] {
      const char* e = std::getenv("GZ_STRIP_TEST_OPEN");
      if (!e) return 0;
      return std::strcmp(e, "prefix") == 0 ? 1 : std::strcmp(e, "tail") == 0 ? 2 : 0;
    }();
    return v;
  }

  // The caller processed the first n positions of the last window.
  void Consumed(size_t n) {
    for (size_t t = 0; t < n && t < mine_.size(); ++t) pos_ += mine_[t];
    window_ = std::min<size_t>(window_ * 2, size_t{1} << 16);
  }

 private:
  struct Entry {
    uint32_t bits;
    int block;
    float key;
  };
  uint32_t kbits_ = 0;
  bool have_prefix_ = false;
  int tie_block_ = -1;
  int64_t take_ = 0;
  std::vector<Entry> rem_;
  size_t pos_ = 0, sorted_ = 0, window_ = 1024;
  std::vector<uint8_t> mine_;
};

// GZ_STRIP_ORDER=exact: every iteration on the exact path (A/B and tests).
bool StripFastOrder() {
  static const bool fast = [] {
    const char* e = std::getenv("GZ_STRIP_ORDER");
    return !(e && std::strcmp(e, "exact") == 0);
  }();
  return fast;
}

class Processor {
 public:
  Processor(const ProcessParams& p, Comparator* cmp, ProcessResult* res, Partition* part)
      : params_(p), cmp_(cmp), res_(res), part_(part), scratch_(NewScanScratch(), FreeScanScratch) {}
  ~Processor() {
    if (writer_.joinable()) writer_.join();
  }
  int Run(const JpegData& jpg_in, std::string* err);

 private:
  bool Fail(std::string* err) {
    if (err) *err = internal_err_.empty() ? cmp_->error() : internal_err_;
    return false;
  }
  // an inconsistency found by the loop itself, not by the comparator
  std::string internal_err_;
  void OutputJpeg(const JpegData& jpg, std::string* out) {
    const auto t0 = Clock::now();
    out->clear();
    WriteJpeg(jpg, params_.clear_metadata, out);
    const double dt = Since(t0);
    res_->seconds_write += dt;
    res_->detail["write_jpeg_s"] += dt;
  }
  // Output of a search candidate: SaveToJpegData(img) over jpg + OutputJpeg
  // + MaybeOutput, pipelined.  BeginOutput stages img (quantize + count, on
  // the pool) and encodes it on a helper thread while the caller runs the
  // Compare and, in the back end, the next iteration's selection.  The
  // MaybeOutput of a candidate must see the distance of the Compare that
  // followed it, so it is applied by FlushOutput, which runs before the next
  // Compare (at the next BeginOutput) or explicitly.
  bool BeginOutput(const JpegData& jpg, const CoeffImage& img, std::string* err) {
    FlushOutput();
    const auto t0 = Clock::now();
    pending_.clear();
    if (cmp_->HasDeviceWriter()) {
      // entropy coded on the device from its resident copy (sub-ms), no
      // helper thread needed; the bytes stay there unless kept
      if (!cmp_->DeviceEncode(img, jpg, params_.clear_metadata, &pending_size_)) return Fail(err);
      has_pending_ = true;
      pending_device_ = true;
      const double dt = Since(t0);
      res_->seconds_write += dt;
      res_->detail["write_device_s"] += dt;
      return true;
    }
    pending_device_ = false;
    StageCoeffImage(img, jpg, scratch_.get());
    writer_ = std::thread([this] {
      const auto t = Clock::now();
      EncodeStaged(scratch_.get(), params_.clear_metadata, &pending_);
      encode_s_ = Since(t);
    });
    has_pending_ = true;
    const double dt = Since(t0);
    res_->seconds_write += dt;
    res_->detail["write_stage_s"] += dt;
    return true;
  }
  // BeginOutput(img) followed by the Compare of img; with a device writer
  // both run as one overlapped device call (the candidate's size and its
  // distance come back together).
  bool EncodeAndCompare(const JpegData& jpg, const CoeffImage& img, std::string* err) {
    if (!cmp_->HasDeviceWriter()) {
      if (!BeginOutput(jpg, img, err)) return false;
      return cmp_->Compare(img) || Fail(err);
    }
    FlushOutput();
    const auto t0 = Clock::now();
    size_t size = 0;
    if (!cmp_->DeviceEncodeAndCompare(img, jpg, params_.clear_metadata, &size)) return Fail(err);
    pending_.clear();
    pending_size_ = size;
    has_pending_ = true;
    pending_device_ = true;
    res_->detail["encode_compare_s"] += Since(t0);
    return true;
  }
  // EncodeAndCompare of a back-end candidate with its histograms known: the
  // DC ones of the back end's start (DC coefficients do not change) and the
  // tracked AC ones; the components SaveToJpegData keeps -- one when the
  // chroma has become all zero (no chroma DC symbol but category 0, no
  // chroma AC symbol with a magnitude) -- as the histogram pass would count.
  bool EncodeAndCompareKnown(const JpegData& jpg, const CoeffImage& img, int saved0, const JpegHistogram dc0[3],
                             const std::vector<JpegHistogram>& ac, std::string* err) {
    FlushOutput();
    const auto t0 = Clock::now();
    int ncomp = 1;
    if (saved0 > 1) {
      for (int c = 1; c < 3 && c < static_cast<int>(ac.size()) && ncomp == 1; ++c) {
        for (int i = 1; i < 256 && ncomp == 1; ++i)
          if (dc0[c].counts[i] || ((i & 0xf) && ac[c].counts[i])) ncomp = 3;
      }
    }
    JpegHistogram ach[3];
    for (int c = 0; c < ncomp && c < static_cast<int>(ac.size()); ++c) ach[c] = ac[c];
    size_t size = 0;
    bool skipped = false;
    // (FlushOutput above: final_score_ includes every earlier candidate)
    if (!cmp_->DeviceEncodeAndCompareKnown(img, jpg, params_.clear_metadata, dc0, ach, ncomp, final_score_, &size,
                                           &skipped))
      return Fail(err);
    pending_.clear();
    pending_size_ = size;
    has_pending_ = true;
    pending_device_ = true;
    pending_skipped_ = skipped;
    res_->detail["encode_compare_s"] += Since(t0);
    res_->detail["encode_known_histograms"] += 1;
    if (skipped) res_->detail["scans_skipped"] += 1;
    return true;
  }
  // Joins the pending encode and applies its MaybeOutput; returns its size.
  size_t FlushOutput() {
    if (!has_pending_) return 0;
    if (writer_.joinable()) {
      const auto t0 = Clock::now();
      writer_.join();
      const double dt = Since(t0);
      res_->seconds_write += dt;
      res_->detail["write_wait_s"] += dt;
      res_->detail["write_encode_s"] += encode_s_;
    }
    has_pending_ = false;
    if (pending_skipped_) {  // its score is not below final_score_: MaybeOutput keeps nothing
      pending_skipped_ = false;
      return 0;
    }
    if (pending_device_) {
      MaybeOutputDevice(pending_size_);
      return pending_size_;
    }
    MaybeOutput(pending_);
    return pending_.size();
  }
  // processor.cc:899-904 (the score depends on the size alone)
  void MaybeOutput(const std::string& encoded) {
    const double score = cmp_->ScoreOutputSize(static_cast<int>(encoded.size()));
    if (score < final_score_ || final_score_ < 0) {
      res_->jpeg = encoded;
      final_score_ = score;
      best_size_ = encoded.size();
      kept_on_device_ = false;
    }
  }
  void MaybeOutputDevice(size_t size) {
    const double score = cmp_->ScoreOutputSize(static_cast<int>(size));
    if (score < final_score_ || final_score_ < 0) {
      cmp_->DeviceKeepEncoded();
      final_score_ = score;
      best_size_ = size;
      kept_on_device_ = true;
    }
  }
  bool TryQuantMatrix(const JpegData& jpg_in, float target_mul, const int q[3][kDCTBlockSize],
                      CoeffImage* img, QuantData* data, std::string* err);
  bool SelectQuantMatrix(const JpegData& jpg_in, bool downsample, int best_q[3][kDCTBlockSize],
                         CoeffImage* img, bool* ok, std::string* err);
  bool SelectFrequencyMasking(const JpegData& jpg, CoeffImage* img, int comp_mask,
                              double target_mul, bool stop_early, std::string* err);
  bool SelectFrequencyBackEnd(const JpegData& jpg, CoeffImage* img, int comp_mask,
                              double target_mul, bool stop_early,
                              const std::vector<int>& offsets, const std::vector<uint8_t>& coeffs,
                              const std::vector<float>& errors, std::string* err);
  bool GatherEntries(std::vector<std::pair<int, float>>* entries, int own_lo, int own_hi, int gbase,
                     int* blocks_to_change);
  // The change entries of one back-end iteration (processor.cc:776-834), for
  // both back ends: the block weights at rblock = 1..4 until some block has
  // entries, every (owned) block's entries in block order -- built in
  // parallel over chunks of blocks -- and on a partitioned frame the frame's
  // entries from every rank.  factor: the searched blocks' size in 8x8
  // blocks; bmax: their distance maxima.  False: a failed exchange.
  bool BuildChangeOrder(int direction, int factor, double target_mul, int num_blocks, int own_lo,
                        int own_hi, int gbase, const std::vector<float>& bmax,
                        const std::vector<int>& last_indexes, const std::vector<int>& offsets,
                        const std::vector<float>& cand_err, const std::vector<float>& max_block_error,
                        std::vector<std::pair<int, float>>* order, std::vector<float>* block_weight,
                        int* blocks_to_change, size_t* frame_entries = nullptr);
  // The 4:2:0 pass (processor.cc:989-1016, downsample = 1) on the host model
  // Image420, entropy coded on the host.
  int Run420(const JpegData& jpg_in, std::string* err);
  bool TryQuantMatrix420(const JpegData& jpg, float target_mul, const int q[3][kDCTBlockSize],
                         Image420* img, QuantData* data, std::string* err);
  bool SelectFrequencyMasking420(const JpegData& jpg, Image420* img, int comp_mask,
                                 double target_mul, bool stop_early, std::string* err);
  void BeginOutput420(const JpegData& jpg, Image420* img);

  ProcessParams params_;
  Comparator* cmp_;
  ProcessResult* res_;
  Partition* part_;  // nullptr: the whole frame is this process's
  std::unique_ptr<ScanScratch, void (*)(ScanScratch*)> scratch_;
  std::thread writer_;
  std::string pending_;
  bool has_pending_ = false;
  bool pending_device_ = false;
  bool pending_skipped_ = false;  // a back-end candidate that could not win, not coded
  size_t pending_size_ = 0;
  bool kept_on_device_ = false;  // the best candidate so far is the device's kept slot
  size_t best_size_ = 0;
  double encode_s_ = 0.0;
  double final_score_ = -1;
  std::vector<int> bulk_cnt_;  // per-block change counts of a back-end bulk prefix
  size_t tail_len_[2] = {0, 0};  // the last back-end tail's length per direction (up, down)
  StripOrder strip_order;      // (a frame split over ranks)
  static constexpr int kOrderChunk = 1024;     // blocks per parallel back-end work item
  static constexpr size_t kMinBulkChanges = 64;
};

bool Processor::TryQuantMatrix(const JpegData& jpg_in, float target_mul,
                               const int q[3][kDCTBlockSize], CoeffImage* img, QuantData* data,
                               std::string* err) {
  // processor.cc:310-338
  std::memcpy(data->q, q, sizeof(data->q));
  const auto tq = Clock::now();
  if (!cmp_->QuantizeFromOriginal(q, img, /*need_host=*/!cmp_->HasDeviceWriter())) return Fail(err);
  res_->seconds_quantize += Since(tq);
  ++res_->iterations;
  if (!EncodeAndCompare(jpg_in, *img, err)) return false;
  data->dist_ok = cmp_->DistanceOK(target_mul);
  data->jpg_size = FlushOutput();
  return true;
}

bool Processor::SelectQuantMatrix(const JpegData& jpg_in, bool downsample,
                                  int best_q[3][kDCTBlockSize], CoeffImage* img, bool* ok,
                                  std::string* err) {
  // processor.cc:340-372
  QuantMatrixGenerator qgen(downsample);
  const float target_mul_high = 0.97f, target_mul_low = 0.95f;
  QuantData best;
  if (!TryQuantMatrix(jpg_in, target_mul_high, best_q, img, &best, err)) return false;
  for (;;) {
    int q_next[3][kDCTBlockSize];
    if (!qgen.GetNext(q_next)) break;
    QuantData data;
    if (!TryQuantMatrix(jpg_in, target_mul_high, q_next, img, &data, err)) return false;
    qgen.Add(data);
    if (CompareQuantData(data, best)) {
      best = data;
      if (data.dist_ok && !cmp_->DistanceOK(target_mul_low)) break;
    }
  }
  std::memcpy(best_q, best.q, sizeof(best.q));
  *ok = best.dist_ok;
  return true;
}

bool Processor::SelectFrequencyMasking(const JpegData& jpg, CoeffImage* img, int comp_mask,
                                       double target_mul, bool stop_early, std::string* err) {
  // processor.cc:559-721 (the CPU_OPT loop runs as one batched device call)
  if (!cmp_->StartBlockComparisons()) return Fail(err);
  std::vector<int> offsets;
  std::vector<uint8_t> cand;
  std::vector<float> cand_err;
  if (!cmp_->BlockZeroingCandidates(*img, jpg, comp_mask, params_.zeroing_greedy_lookahead,
                                    params_.new_zeroing_model,
                                    &offsets, &cand, &cand_err))
    return Fail(err);
  cmp_->FinishBlockComparisons();
  res_->detail["candidates"] = static_cast<double>(cand.size());
  const double c0 = ThreadCpu();
  const bool ok = SelectFrequencyBackEnd(jpg, img, comp_mask, target_mul, stop_early, offsets, cand,
                                         cand_err, err);
  res_->detail["backend_thread_cpu_s"] += ThreadCpu() - c0;
  return ok;
}

bool Processor::SelectFrequencyBackEnd(const JpegData& jpg, CoeffImage* img, int comp_mask,
                                       double target_mul, bool stop_early,
                                       const std::vector<int>& offsets,
                                       const std::vector<uint8_t>& cand,
                                       const std::vector<float>& cand_err, std::string* err) {
  // processor.cc:723-919.  With a partition (a frame split over ranks by
  // block rows, host/strips.h) img is this rank's strip: the entries, bulk
  // changes and tail changes of its owned blocks are made here, and the
  // frame-wide quantities -- the sorted change order, the histograms, the
  // entropy estimate -- are exchanged or replicated.
  const int ncomp = static_cast<int>(jpg.components.size());
  const int block_width = img->block_w;
  const int num_blocks = block_width * img->block_h;
  const int own_lo = part_ ? part_->OwnLo() : 0, own_hi = part_ ? part_->OwnHi() : num_blocks;
  const int gbase = part_ ? part_->LocalBase() : 0;  // frame index of local block 0
  (void)comp_mask;
  auto exchange_failed = [&]() {
    if (err) *err = "strip exchange failed";
    return false;
  };
  std::vector<JpegHistogram> ac_histograms(ncomp);
  int jpg_header_size, dc_size;
  // the components SaveToJpegData keeps at the start, and the DC histograms
  // (the back end changes AC coefficients only: they stay as they are)
  int saved0 = 3;
  JpegHistogram dc0[3];
  {
    JpegHistogram dc_h[3], ac_h[3];
    int saved = cmp_->DeviceHistograms(*img, dc_h, ac_h);
    if (saved < 0 && cmp_->HasDeviceWriter()) return Fail(err);
    if (saved < 0) saved = CoeffImageHistograms(*img, scratch_.get(), dc_h, ac_h);
    saved0 = saved;
    for (int c = 0; c < 3; ++c) dc0[c] = dc_h[c];
    JpegData out;
    out.app_data = jpg.app_data;
    out.com_data = jpg.com_data;
    img->SaveHeaderToJpegData(saved, &out);
    if (part_) {
      out.width = part_->width;
      out.height = part_->height;
    }
    jpg_header_size = static_cast<int>(JpegHeaderSize(out, params_.clear_metadata));
    size_t num = saved;
    int idx[3];
    std::vector<uint8_t> depths(saved * JpegHistogram::kSize);
    dc_size = static_cast<int>(ClusterHistograms(dc_h, &num, idx, depths.data()));
    for (int c = 0; c < ncomp && c < 3; ++c) ac_histograms[c] = ac_h[c];
  }
  std::vector<uint8_t> ac_depths;
  int ac_histogram_size = static_cast<int>(ComputeEntropyCodes(ac_histograms, &ac_depths));
  const int base_size = jpg_header_size + dc_size + ac_histogram_size +
                        static_cast<int>(EntropyCodedDataSize(ac_histograms, ac_depths));
  std::vector<int64_t> raw_bits(ncomp);
  auto refresh_raw = [&]() {
    for (int c = 0; c < ncomp; ++c)
      raw_bits[c] = HistogramRawBits(ac_histograms[c], &ac_depths[c * JpegHistogram::kSize]);
  };
  refresh_raw();
  AcBlockModel acm;
  acm.Build(*img);
  int prev_size = base_size;
  std::vector<float> max_block_error(num_blocks, 0.0f);
  std::vector<int> last_indexes(num_blocks, 0);
  const std::vector<float> zero_block_max(num_blocks, 0.0f);
  bool first_up_iter = true;
  const int own_chunks = (own_hi - own_lo + kOrderChunk - 1) / kOrderChunk;
  // the change order on the device (weights, entries, max_block_error there;
  // the frame's candidates and block maxima are resident) unless the frame
  // is split over ranks or the comparator has no device
  bool device_order = false;
  if (cmp_->HasDeviceBulk() && !cmp_->DeviceOrderReset(&device_order)) return Fail(err);
  // A frame split over ranks with the device order (round 6): every rank's
  // engine builds its owned blocks' entries; the selections exchange their
  // counts and candidates (the comparator's scope, Engine::OrderSelect), so
  // the bulk prefix, the windows and their certification are the frame's on
  // every rank; the owners apply the changes (their device bulk, the tail's
  // windows through tail_window below).
  const bool strip_dev = device_order && part_ && part_->world > 1;
  // With the device order the bulk prefix is selected and applied on the
  // device too (DeviceSelectBulk), with the change of the AC histograms
  // counted there.
  // The host copy of a block then follows lazily: a block's coefficients are a function of
  // its last_indexes alone -- its first last_indexes[b] candidates zeroed,
  // the others as quantized (up iterations zero candidates in order, down
  // iterations restore them in reverse) -- so mat_li[b], the last_indexes the
  // host copy reflects, is brought up to date (materialize) before the tail
  // reads or changes the block.
  const bool device_bulk = device_order && cmp_->HasDeviceBulk();
  // A frame split over ranks applies its owned blocks' bulk prefix on its
  // own device too (from the host's counts and last_indexes), its host copy
  // then following lazily as with the device order -- except the blocks
  // within the halo band of a strip edge, which the neighbours' halos need:
  // those are brought up to date and journalled at once (SyncHalo ships the
  // journal).  (GZ_STRIP_HOST_BULK=1: the host applies it, for A/B runs.)
  static const bool strip_host_bulk = getenv("GZ_STRIP_HOST_BULK") && atoi(getenv("GZ_STRIP_HOST_BULK")) != 0;
  const bool strip_bulk = part_ && !strip_host_bulk && cmp_->HasDeviceBulkLocal();
  const bool lazy_host = device_bulk || strip_bulk;
  std::vector<int> mat_li;
  std::vector<uint8_t> bulk_cnt8;
  if (lazy_host) mat_li.assign(num_blocks, 0);
  auto materialize = [&](int bix, bool journal = false) {
    int m = mat_li[bix];
    const int li = last_indexes[bix];
    if (m == li) return;
    const int offset = std::max(0, std::min(offsets[bix], static_cast<int>(cand.size()) - 1));
    const int bx = bix % block_width, by = bix / block_width;
    for (; m != li; m += m < li ? 1 : -1) {
      const int idx = cand[offset + (m < li ? m : m - 1)];
      const int c = idx / kDCTBlockSize, k = idx % kDCTBlockSize;
      coeff_t v = 0;
      if (m > li) {
        const JpegComponent& comp = jpg.components[c];
        v = QuantizeCoeff(comp.coeffs[static_cast<size_t>(by * comp.width_in_blocks + bx) * 64 + k], img->quant[c][k]);
      }
      img->block(c, bix)[k] = v;
      if (journal) img->MarkChanged(c, bix, k);
      uint64_t& nzm = acm.nz[static_cast<size_t>(c) * num_blocks + bix];
      const int z = kJPEGZigZagOrder[k];
      if (v) nzm |= 1ull << z; else nzm &= ~(1ull << z);
    }
    mat_li[bix] = li;
  };
  for (int direction : {1, -1}) {
    for (;;) {
      if (stop_early) FlushOutput();  // best_size_ must be current
      if (stop_early && direction == -1 && prev_size > 1.01 * best_size_) break;
      const auto tb = Clock::now();
      std::vector<std::pair<int, float>> global_order;
      int blocks_to_change = 0;
      std::vector<float> block_weight;
      // A frame split over ranks: by default every rank keeps its own
      // entries (StripOrder below) and the frame's std::sort order is
      // derived from them where the consumed entries' keys decide it alone;
      // strip_exact: the whole frame's entries on every rank (the fallback).
      bool strip_exact = part_ && part_->world > 1 && !strip_dev && !StripFastOrder();
      const bool strip_fast = part_ && part_->world > 1 && !strip_dev && !strip_exact;
      size_t frame_n = 0;
      int64_t device_below_floor = -1;
      if (device_order) {
        // (the entries stay on the device; the first up iteration's count of
        // keys below its floor comes back with their count)
        const float floor_limit = first_up_iter ? 0.75f * cmp_->BlockErrorLimit() : -HUGE_VALF;
        if (!cmp_->DeviceChangeOrder(direction, target_mul, first_up_iter, last_indexes, floor_limit, &frame_n,
                                     &blocks_to_change, first_up_iter ? &device_below_floor : nullptr))
          return Fail(err);
      } else if (!first_up_iter && (cmp_->block_max_distance(), cmp_->block_max_failed())) {
        return Fail(err);
      } else if (!BuildChangeOrder(direction, 1, target_mul, num_blocks, own_lo, own_hi, gbase,
                                   first_up_iter ? zero_block_max : cmp_->block_max_distance(), last_indexes,
                                   offsets, cand_err, max_block_error, &global_order, &block_weight,
                                   &blocks_to_change, strip_fast ? &frame_n : nullptr)) {
        return exchange_failed();
      }
      if (!strip_fast && !device_order) frame_n = global_order.size();
      res_->detail["backend_order_s"] += Since(tb);
      res_->detail["backend_order_entries"] += static_cast<double>(frame_n);
      if (frame_n == 0) {
        res_->seconds_backend += Since(tb);
        break;
      }
      // std::sort(global_order) by key (processor.cc:840-843), materialised
      // lazily: only the prefix the change loop consumes gets sorted.
      std::unique_ptr<LazyStdSort> sorter;
      if (!strip_fast && !device_order) sorter.reset(new LazyStdSort(global_order.data(), global_order.size()));
      // device order: the entries come to the host (all of them, in block
      // order, for std::sort's exact permutation) only where the keys leave
      // the order open
      auto fetch_exact = [&]() -> bool {
        const auto tf = Clock::now();
        if (!cmp_->DeviceOrderEntries(&global_order)) return false;
        if (global_order.size() != frame_n) {
          internal_err_ = "device order: entry count mismatch";
          return false;
        }
        sorter.reset(new LazyStdSort(global_order.data(), global_order.size()));
        res_->detail["backend_order_fetches"] += 1;
        res_->detail["backend_order_fetch_s"] += Since(tf);
        return true;
      };
      // strip_fast: this rank's entries, global_order, become the frame's (the
      // exact path) when their keys leave std::sort's order open
      auto go_exact = [&]() -> bool {
        const auto tg = Clock::now();
        int btc = blocks_to_change;
        // (the device order: this rank's entries come from its engine first)
        if (strip_dev && !cmp_->DeviceOrderEntries(&global_order)) return false;
        if (!GatherEntries(&global_order, own_lo, own_hi, gbase, &btc)) return false;
        sorter.reset(new LazyStdSort(global_order.data(), global_order.size()));
        strip_exact = true;
        res_->detail["strip_order_fallbacks"] += 1;
        res_->detail["strip_order_fallback_s"] += Since(tg);
        return true;
      };
      const auto tc = Clock::now();
      // (the frame's count of keys below the first up iteration's floor)
      int64_t below_floor = -1;
      if (strip_fast && first_up_iter) {
        const float limit = 0.75f * cmp_->BlockErrorLimit();
        below_floor = 0;
        for (const auto& e : global_order) below_floor += e.second < limit ? 1 : 0;
        if (!part_->SumAll(&below_floor, 1)) return exchange_failed();
      }
      if (device_order && first_up_iter) below_floor = device_below_floor;
      ChangeLoop loop(direction, cmp_->DistanceOK(1.0), base_size, 1, blocks_to_change, &first_up_iter,
                      cmp_->BlockErrorLimit(), global_order, frame_n, below_floor);
      int est_jpg_size = prev_size;
      // Changes before the loop's first read of an entropy code or size
      // estimate (first_read: the first i % 10 == 0 step whose codes are
      // read, the first step with changed > min_coeffs_to_change, or
      // the last one) only accumulate; their effect -- block states, AC
      // histograms, last_indexes -- depends on which changes they are, not
      // on their order.  So [0, first_read) is taken as std::sort's first
      // first_read entries as a set (LazyStdSort::SetPrefix: partitioning
      // only, no sort of the prefix) and applied per block in parallel.
      size_t bulk = 0;
      {
        const long m = std::max(0, loop.min_coeffs);
        const long n = static_cast<long>(frame_n);
        const long lo = std::max(0L, std::min(m - 9, n - 10));
        const long first_code = (lo + 9) / 10 * 10;
        const long first_read = std::min(std::min(first_code, m), n - 1);
        if (first_read >= kMinBulkChanges) bulk = static_cast<size_t>(first_read);
      }
      // The device order's selection: the bulk prefix as a set from the keys
      // (applied on the device) and the tail's window of the next entries.
      Engine::OrderSelection sel;
      std::vector<std::pair<int, float>> win;  // the tail from position win_base on, in order
      size_t win_base = bulk;
      size_t win_ok = 0;                       // ... its positions certified to be std::sort's
      bool win_last = false;                   // ... and it holds every entry left
      if (device_order) {
        const auto tbk = Clock::now();
        // (the window: twice the last tail of this direction, 512 .. 8192
        // entries -- sorted in one workgroup on the device; GZ_TAIL_WINDOW:
        // a fixed size, for tests)
        static const size_t fixed_window = [] {
          const char* w = std::getenv("GZ_TAIL_WINDOW");
          return static_cast<size_t>(w && std::atoi(w) > 0 ? std::atoi(w) : 0);
        }();
        size_t& last_tail = tail_len_[direction > 0 ? 0 : 1];
        const size_t kTailWindow =
            fixed_window ? fixed_window : std::min<size_t>(8192, std::max<size_t>(512, 2 * last_tail));
        JpegHistogram ac_now[3];
        for (int c = 0; c < ncomp && c < 3; ++c) ac_now[c] = ac_histograms[c];
        if (!cmp_->DeviceSelectBulk(*img, bulk, kTailWindow, direction, &sel, ac_now)) return Fail(err);
        // (a strip: the blocks within the halo band of its edges, which the
        // neighbours' halos need, brought up to date and journalled at once)
        auto strip_band = [&]() {
          const int band = (kStripHalo / 8) * block_width;
          for (int bix = own_lo; bix < std::min(own_hi, own_lo + band); ++bix) materialize(bix, true);
          for (int bix = std::max(own_lo + band, own_hi - band); bix < own_hi; ++bix) materialize(bix, true);
        };
        if (bulk && sel.applied) {
          for (int c = 0; c < ncomp && c < 3; ++c) ac_histograms[c] = ac_now[c];
          // (the counts include the tie block's share of the K*-keyed entries)
          for (int bix = 0; bix < num_blocks; ++bix) last_indexes[bix] += sel.cnt[bix] * direction;
          img->host_partial = true;
          if (strip_dev) strip_band();
          refresh_raw();
          loop.changed = static_cast<int>(bulk);
          res_->detail["backend_bulk_changes"] += static_cast<double>(bulk);
          res_->detail["backend_bulk_device"] += 1;
        } else if (bulk) {
          // K* shared by several blocks across the prefix's end: std::sort's
          // tie order decides which of them the prefix takes -- the exact
          // path (every entry, LazyStdSort), applied with the host's counts
          res_->detail["backend_select_open"] += 1;
          if (strip_dev) {
            // the frame's entries on every rank, the owned blocks' prefix
            // share applied on each rank's device, the histogram change summed
            if (!go_exact()) return exchange_failed();
            sorter->SetPrefix(bulk);
            bulk_cnt8.assign(num_blocks, 0);
            for (size_t i = 0; i < bulk; ++i) {
              const int b = global_order[i].first - gbase;
              if (b >= own_lo && b < own_hi) ++bulk_cnt8[b];
            }
            int32_t delta[3][256] = {};
            const bool ok = cmp_->DeviceBulkApplyLocal(*img, direction, bulk_cnt8.data(), last_indexes, delta);
            std::vector<int64_t> hsum(3 * (JpegHistogram::kSize - 1) + 1, 0);
            for (int c = 0; c < ncomp && c < 3; ++c)
              for (int q = 0; q + 1 < JpegHistogram::kSize; ++q) hsum[c * (JpegHistogram::kSize - 1) + q] = delta[c][q];
            hsum.back() = ok ? 0 : 1;
            if (!part_->SumAll(hsum.data(), static_cast<int>(hsum.size()))) return exchange_failed();
            if (!ok) return Fail(err);
            if (hsum.back()) {
              if (err) *err = "a rank's device bulk prefix failed";
              return false;
            }
            for (int bix = own_lo; bix < own_hi; ++bix) last_indexes[bix] += bulk_cnt8[bix] * direction;
            // (the counts are stored doubled, JpegHistogram::Add)
            for (int c = 0; c < ncomp && c < 3; ++c)
              for (int q = 0; q + 1 < JpegHistogram::kSize; ++q)
                ac_histograms[c].counts[q] += 2u * static_cast<uint32_t>(hsum[c * (JpegHistogram::kSize - 1) + q]);
            img->host_partial = true;
            strip_band();
            refresh_raw();
          } else {
          if (!fetch_exact()) return Fail(err);
          sorter->SetPrefix(bulk);
          bulk_cnt8.assign(num_blocks, 0);
          for (size_t i = 0; i < bulk; ++i) ++bulk_cnt8[global_order[i].first];
          for (int bix = 0; bix < num_blocks; ++bix) last_indexes[bix] += bulk_cnt8[bix] * direction;
          for (int c = 0; c < ncomp && c < 3; ++c) ac_now[c] = ac_histograms[c];
          if (!cmp_->DeviceBulkApply(*img, direction, bulk_cnt8.data(), ac_now)) return Fail(err);
          for (int c = 0; c < ncomp && c < 3; ++c) ac_histograms[c] = ac_now[c];
          img->host_partial = true;
          refresh_raw();
          }
          loop.changed = static_cast<int>(bulk);
          res_->detail["backend_bulk_changes"] += static_cast<double>(bulk);
          res_->detail["backend_bulk_device"] += 1;
        }
        if (!sorter && !sel.window_overflow) {
          // the window, sorted on the device: std::sort's order for its first
          // window_ok positions (up to the first key shared by entries of
          // several blocks; entries of one block are interchangeable: a
          // change takes the block's next candidate)
          win.swap(sel.window);
          win_ok = sel.window_ok;
          win_last = sel.window_last;
        }
        res_->detail["backend_bulk_s"] += Since(tbk);
      }
      if (bulk && !device_order) {
        const auto tbk = Clock::now();
        if (strip_fast) {
          // the prefix as a set from the keys alone (StripOrder::Prefix);
          // open (tied keys of several blocks across its boundary): exact
          const int r = strip_order.Prefix(global_order, bulk, part_, gbase, num_blocks, &bulk_cnt_);
          if (r < 0) return exchange_failed();
          if (r == 0 && !go_exact()) return exchange_failed();
        }
        if (!strip_fast || strip_exact) sorter->SetPrefix(bulk);
        res_->detail["backend_setprefix_s"] += Since(tbk);
        // per-block counts of the prefix's owned entries (parallel; blocks
        // are spread, so the atomic increments rarely meet)
        if (!strip_fast || strip_exact) {
        bulk_cnt_.assign(num_blocks, 0);
          const int kSlices = bulk >= (size_t{1} << 18) ? 64 : 1;
          int* cnt = bulk_cnt_.data();
          ParallelFor(kSlices, [&](int sl) {
            for (size_t i = bulk * sl / kSlices; i < bulk * (sl + 1) / kSlices; ++i) {
              const int b = global_order[i].first - gbase;
              if (b >= own_lo && b < own_hi) __atomic_fetch_add(&cnt[b], 1, __ATOMIC_RELAXED);
            }
          });
        }
        if (strip_bulk) {
          // the owned blocks' prefix on this rank's device; its histogram
          // delta summed over the ranks
          const auto td = Clock::now();
          bulk_cnt8.assign(num_blocks, 0);
          for (int bix = own_lo; bix < own_hi; ++bix) bulk_cnt8[bix] = static_cast<uint8_t>(bulk_cnt_[bix]);
          int32_t delta[3][256] = {};
          // (a failure on one rank fails every rank at the all-sum below:
          // its status travels with the delta)
          const bool ok = cmp_->DeviceBulkApplyLocal(*img, direction, bulk_cnt8.data(), last_indexes, delta);
          std::vector<int64_t> hsum(3 * (JpegHistogram::kSize - 1) + 1, 0);
          for (int c = 0; c < ncomp && c < 3; ++c)
            for (int q = 0; q + 1 < JpegHistogram::kSize; ++q) hsum[c * (JpegHistogram::kSize - 1) + q] = delta[c][q];
          hsum.back() = ok ? 0 : 1;
          if (!part_->SumAll(hsum.data(), static_cast<int>(hsum.size()))) return exchange_failed();
          if (!ok) return Fail(err);
          if (hsum.back()) {
            if (err) *err = "a rank's device bulk prefix failed";
            return false;
          }
          for (int bix = own_lo; bix < own_hi; ++bix) last_indexes[bix] += bulk_cnt_[bix] * direction;
          img->host_partial = true;
          // the halo bands' blocks now, journalled (the neighbours' halos)
          const int band = (kStripHalo / 8) * block_width;
          for (int bix = own_lo; bix < std::min(own_hi, own_lo + band); ++bix) materialize(bix, true);
          for (int bix = std::max(own_lo + band, own_hi - band); bix < own_hi; ++bix) materialize(bix, true);
          // (the counts are stored doubled, JpegHistogram::Add)
          for (int c = 0; c < ncomp && c < 3; ++c)
            for (int q = 0; q + 1 < JpegHistogram::kSize; ++q)
              ac_histograms[c].counts[q] += 2u * static_cast<uint32_t>(hsum[c * (JpegHistogram::kSize - 1) + q]);
          refresh_raw();
          loop.changed = static_cast<int>(bulk);
          res_->detail["backend_bulk_s"] += Since(tbk);
          res_->detail["backend_bulk_device_s"] += Since(td);
          res_->detail["backend_bulk_changes"] += static_cast<double>(bulk);
          res_->detail["backend_bulk_device"] += 1;
        }
        struct ChunkDelta {
          JpegHistogram h[3];
          std::vector<uint32_t> changed;
        };
        std::vector<ChunkDelta> deltas(strip_bulk ? 0 : own_chunks);
        if (!strip_bulk) ParallelFor(own_chunks, [&](int ch) {
          ChunkDelta& d = deltas[ch];
          int64_t raw_unused = 0;
          const int b0 = own_lo + ch * kOrderChunk, b1 = std::min(own_hi, b0 + kOrderChunk);
          size_t total = 0;
          for (int bix = b0; bix < b1; ++bix) total += bulk_cnt_[bix];
          d.changed.reserve(total);
          // the touched blocks are scattered over three 2-byte-per-coefficient
          // planes much larger than the caches: fetch a block a few touched
          // blocks ahead (its first change's plane, the mask word, and for
          // direction < 0 the original coefficients)
          constexpr int kAhead = 6;
          auto prefetch = [&](int b) {
            const int off = std::max(0, std::min(offsets[b], static_cast<int>(cand.size()) - 1));
            const int ci = off + last_indexes[b] + std::min(direction, 0);
            if (ci < 0 || ci >= static_cast<int>(cand.size())) return;
            const int c = cand[ci] / kDCTBlockSize;
            const coeff_t* blk = img->block(c, b);
            __builtin_prefetch(blk, 1);
            __builtin_prefetch(blk + 32, 1);
            __builtin_prefetch(&acm.nz[static_cast<size_t>(c) * num_blocks + b], 1);
            if (direction < 0) {
              const JpegComponent& comp = jpg.components[c];
              const coeff_t* o = comp.coeffs.data() +
                                 static_cast<size_t>((b / block_width) * comp.width_in_blocks + b % block_width) * 64;
              __builtin_prefetch(o);
              __builtin_prefetch(o + 32);
            }
          };
          int ahead = b0, pending = 0;  // next block to prefetch; touched blocks in flight
          for (int bix = b0; bix < b1; ++bix) {
            for (; ahead < b1 && pending < kAhead; ++ahead)
              if (bulk_cnt_[ahead]) {
                prefetch(ahead);
                ++pending;
              }
            const int cnt = bulk_cnt_[bix];
            if (!cnt) continue;
            --pending;
            const int bx = bix % block_width, by = bix / block_width;
            const int offset = std::max(0, std::min(offsets[bix], static_cast<int>(cand.size()) - 1));
            int li = last_indexes[bix];
            for (int t = 0; t < cnt; ++t) {
              const int idx = cand[offset + li + std::min(direction, 0)];
              const int c = idx / kDCTBlockSize, k = idx % kDCTBlockSize;
              const int* quant = img->quant[c];
              int newval = 0;
              if (direction < 0) {
                const JpegComponent& comp = jpg.components[c];
                const int jpg_bix = by * comp.width_in_blocks + bx;
                newval = QuantizeCoeff(comp.coeffs[static_cast<size_t>(jpg_bix) * 64 + k], quant[k]);
              }
              acm.Change<JpegHistogram, false>(c, bix, num_blocks, img->block(c, bix), k,
                                               static_cast<coeff_t>(newval), quant,
                                               &ac_depths[c * JpegHistogram::kSize], &d.h[c], &raw_unused);
              d.changed.push_back(static_cast<uint32_t>((static_cast<size_t>(c) * num_blocks + bix) * 64 + k));
              li += direction;
            }
            last_indexes[bix] = li;
          }
        });
        if (!strip_bulk) {
        // (symbols only: the last slot is the histogram's fixed sentinel count)
        std::vector<int64_t> hsum(3 * (JpegHistogram::kSize - 1), 0);
        for (const ChunkDelta& d : deltas) {
          for (int c = 0; c < ncomp && c < 3; ++c)
            for (int q = 0; q + 1 < JpegHistogram::kSize; ++q)
              hsum[c * (JpegHistogram::kSize - 1) + q] += static_cast<int32_t>(d.h[c].counts[q]);
          img->changed.insert(img->changed.end(), d.changed.begin(), d.changed.end());
        }
        // (the counts wrap: a chunk's removals are negative deltas)
        if (part_ && !part_->SumAll(hsum.data(), static_cast<int>(hsum.size()))) return exchange_failed();
        for (int c = 0; c < ncomp && c < 3; ++c)
          for (int q = 0; q + 1 < JpegHistogram::kSize; ++q)
            ac_histograms[c].counts[q] += static_cast<uint32_t>(hsum[c * (JpegHistogram::kSize - 1) + q]);
        refresh_raw();
        loop.changed = static_cast<int>(bulk);
        res_->detail["backend_bulk_s"] += Since(tbk);
        res_->detail["backend_bulk_changes"] += static_cast<double>(bulk);
        }
      }
      const size_t n_order = frame_n;
      double codes_s = 0.0;
      int n_codes = 0;
      double sort_s = 0.0;
      // The bookkeeping of steps [i0, i0 + n) whose changes' symbol updates
      // are known (step k: component comp[k], updates logs[k]; key keys[k]),
      // in speculative batches.  The entropy codes read at step i (i % 10
      // == 0) are a function of the AC histograms after step i alone, and
      // the histograms after every step follow from the steps' symbol
      // updates, which need no codes.  So the histograms are advanced over
      // the steps first, copied at every step whose codes are read, those
      // codes built on the pool at once, then the estimate and the break
      // test run over the steps in order with the same values as the
      // one-at-a-time loop; the histograms of the steps past
      // the break are taken back.  Returns the steps processed (through the
      // break when *stop).
      struct Snap {
        size_t step;
        JpegHistogram h[3];
        std::vector<uint8_t> depths;
        int size = 0;
        int64_t raw[3] = {0, 0, 0};
      };
      std::vector<Snap> snaps;
      auto run_steps = [&](size_t i0, size_t n, const uint8_t* comp, const SymbolLog* logs, const float* keys,
                           bool* stop) -> size_t {
        *stop = false;
        size_t ns = 0;
        for (size_t k = 0; k < n; ++k) {
          const SymbolLog& lg = logs[k];
          for (int e = 0; e < lg.n; ++e) ac_histograms[comp[k]].Add(lg.sym[e], lg.weight[e]);
          if (loop.CodesRead(i0 + k)) {
            if (ns == snaps.size()) snaps.emplace_back();
            Snap& sn = snaps[ns++];
            sn.step = i0 + k;
            for (int c = 0; c < ncomp && c < 3; ++c) sn.h[c] = ac_histograms[c];
          }
        }
        // (a task takes two consecutive rebuilds: the code-length caches are per thread)
        if (ns) {
          const auto te = Clock::now();
          const int tasks = static_cast<int>((ns + 1) / 2);
          auto build = [&](int t) {
            for (size_t q = 2 * static_cast<size_t>(t); q < std::min(ns, 2 * static_cast<size_t>(t) + 2); ++q) {
              Snap& sn = snaps[q];
              std::vector<JpegHistogram> hv(sn.h, sn.h + ncomp);
              sn.size = static_cast<int>(ComputeEntropyCodes(hv, &sn.depths));
              for (int c = 0; c < ncomp; ++c) sn.raw[c] = HistogramRawBits(sn.h[c], &sn.depths[c * JpegHistogram::kSize]);
            }
          };
          if (tasks == 1) build(0); else ParallelFor(tasks, build);
          codes_s += Since(te);
          n_codes += static_cast<int>(ns);
        }
        size_t q = 0, k = 0;
        for (; k < n; ++k) {
          const size_t s = i0 + k;
          loop.Applied(keys[k]);
          if (q < ns && snaps[q].step == s) {
            const Snap& sn = snaps[q++];
            ac_histogram_size = sn.size;
            ac_depths = sn.depths;
            for (int c = 0; c < ncomp; ++c) raw_bits[c] = sn.raw[c];
          } else {
            const SymbolLog& lg = logs[k];
            const uint8_t* d = &ac_depths[comp[k] * JpegHistogram::kSize];
            for (int e = 0; e < lg.n; ++e)
              raw_bits[comp[k]] += static_cast<int64_t>(lg.weight[e]) * (d[lg.sym[e]] + (lg.sym[e] & 0xf));
          }
          if (!loop.EstimateRead(s)) continue;
          est_jpg_size = jpg_header_size + dc_size + ac_histogram_size + EntropySizeFromRaw(raw_bits);
          if (loop.Stop(est_jpg_size, prev_size)) {
            *stop = true;
            break;
          }
        }
        if (*stop) {
          for (size_t u = k + 1; u < n; ++u)
            for (int e = 0; e < logs[u].n; ++e) ac_histograms[comp[u]].Add(logs[u].sym[e], -logs[u].weight[e]);
          res_->detail["backend_spec_wasted_codes"] += static_cast<double>(ns - q);
          return k + 1;
        }
        return n;
      };
      // the change of the next entry of owned block bix applied to img: its
      // symbol updates into the frame's histograms, or (log) recorded
      auto apply = [&](int bix, SymbolLog* log) {
        if (lazy_host) materialize(bix);
        const int bx = bix % block_width, by = bix / block_width;
        const int last_idx = last_indexes[bix];
        const int offset = std::max(0, std::min(offsets[bix], static_cast<int>(cand.size()) - 1));
        const int idx = cand[offset + last_idx + std::min(direction, 0)];
        const int c = idx / kDCTBlockSize, k = idx % kDCTBlockSize;
        const int* quant = img->quant[c];
        const JpegComponent& comp = jpg.components[c];
        const int jpg_bix = by * comp.width_in_blocks + bx;
        const int newval = direction > 0 ? 0 : QuantizeCoeff(comp.coeffs[static_cast<size_t>(jpg_bix) * 64 + k], quant[k]);
        if (log) {
          int64_t raw_unused = 0;
          acm.Change(c, bix, num_blocks, img->block(c, bix), k, static_cast<coeff_t>(newval), quant,
                     &ac_depths[c * JpegHistogram::kSize], log, &raw_unused);
        } else {
          acm.Change(c, bix, num_blocks, img->block(c, bix), k, static_cast<coeff_t>(newval), quant,
                     &ac_depths[c * JpegHistogram::kSize], &ac_histograms[c], &raw_bits[c]);
        }
        img->MarkChanged(c, bix, k);
        last_indexes[bix] += direction;
        if (lazy_host) mat_li[bix] = last_indexes[bix];
      };
      if (!part_ || part_->world == 1) {
        // Prefetch window: when the lazy sort hands out a new sorted chunk, the
        // chunk's per-block state is touched ahead of the (serial) changes in
        // three dependent passes -- block bookkeeping, then the candidate byte,
        // then the coefficient block and its non-zero mask -- so the cache
        // misses of a chunk overlap instead of chaining.  Values are only
        // prefetched; the loop below reads them as before.
        size_t prefetched = bulk;
        // The tail's entries: the device window's certified positions, else
        // (past them, or without a window) std::sort's exact order -- all
        // entries fetched once, LazyStdSort with the prefix set aside; the
        // window's positions before are the same in it (see above)
        bool tail_exact = !device_order || static_cast<bool>(sorter);
        auto tail_block = [&](size_t s) { return tail_exact ? global_order[s].first : win[s - win_base].first; };
        auto tail_key = [&](size_t s) { return tail_exact ? global_order[s].second : win[s - win_base].second; };
        auto tail_ready = [&](size_t s) -> bool {
          if (!tail_exact) {
            if (s < win_base + win_ok) return true;
            // (no window at all -- the selection's candidates overflowed, or
            // its prefix was open -- goes straight to the exact order)
            if (!win.empty() && win_ok == win.size() && !win_last && s == win_base + win_ok) {
              // the window ran out without a tie: the next one from rank s
              Engine::OrderSelection next;
              const size_t want = std::min<size_t>(8192, std::max<size_t>(512, 2 * win.size()));
              const auto tw = Clock::now();
              if (!cmp_->DeviceSelectWindow(s, want, direction, &next)) return false;
              res_->detail["backend_tail_windows"] += 1;
              res_->detail["backend_tail_window_s"] += Since(tw);
              if (!next.open && !next.window_overflow) {
                win.swap(next.window);
                win_base = s;
                win_ok = next.window_ok;
                win_last = next.window_last;
                if (s < win_base + win_ok) return true;
              }
            }
            if (!fetch_exact()) return false;
            const auto tp = Clock::now();
            if (bulk) sorter->SetPrefix(bulk);
            res_->detail["backend_setprefix_s"] += Since(tp);
            tail_exact = true;
            res_->detail["backend_tail_exact"] += 1;
            if (!bulk && win.empty()) res_->detail["backend_tail_exact_nobulk"] += 1;
          }
          if (s >= sorter->sorted()) {
            const auto ts = Clock::now();
            sorter->EnsureSorted(s);
            sort_s += Since(ts);
          }
          return true;
        };
        auto prefetch_chunk = [&](size_t lo, size_t hi) {
          for (size_t j = lo; j < hi; ++j) {
            const int b = tail_block(j);
            __builtin_prefetch(&last_indexes[b]);
            __builtin_prefetch(&offsets[b]);
          }
          for (size_t j = lo; j < hi; ++j) {
            const int b = tail_block(j);
            const int off = std::max(0, std::min(offsets[b], static_cast<int>(cand.size()) - 1));
            const int ci = off + last_indexes[b] + std::min(direction, 0);
            if (ci >= 0 && ci < static_cast<int>(cand.size())) __builtin_prefetch(&cand[ci]);
          }
          for (size_t j = lo; j < hi; ++j) {
            const int b = tail_block(j);
            const int off = std::max(0, std::min(offsets[b], static_cast<int>(cand.size()) - 1));
            const int ci = off + last_indexes[b] + std::min(direction, 0);
            if (ci < 0 || ci >= static_cast<int>(cand.size())) continue;
            const int c = cand[ci] / kDCTBlockSize;
            __builtin_prefetch(img->block(c, b), 1);
            __builtin_prefetch(&acm.nz[static_cast<size_t>(c) * num_blocks + b], 1);
          }
        };
        // The tail in speculative batches.  The entropy codes read at change
        // i (i % 10 == 0) are a function of the AC histograms after change i
        // alone, and the histograms after every change follow from the
        // changes' symbol updates, which need no codes.  So a batch applies
        // its changes first (recording each one's symbol updates and what
        // undoes it), copies the histograms at every step whose codes are
        // read, builds those codes on the pool at once, then runs the
        // estimate and the break test over the batch in order with the same
        // values as the one-at-a-time loop; the changes past the break are
        // undone.  Batches grow from 4 to kMaxDecades rebuilds (capped by
        // the pool workers this encode may use), so a tail that stops early
        // wastes at most a few rebuilds.
        struct Spec {
          int bix, k;
          coeff_t old;
          uint64_t nz;
        };
        std::vector<Spec> spec;
        std::vector<uint8_t> sp_comp;
        std::vector<SymbolLog> sp_log;
        std::vector<float> sp_key;
        const int workers = std::max(1, PoolWorkerCap());
        constexpr int kMaxDecades = 32;
        // (GZ_SPEC_DECADES: a fixed batch, for A/B runs and tests)
        static const int fixed_decades = getenv("GZ_SPEC_DECADES") ? std::max(1, atoi(getenv("GZ_SPEC_DECADES"))) : 0;
        int decades = fixed_decades ? fixed_decades : std::min(4, 2 * workers);
        size_t i = bulk;
        bool stop = false;
        while (!stop && i < n_order) {
          const size_t first_code = (i + 9) / 10 * 10;
          const size_t j = std::min(n_order, first_code + 10 * static_cast<size_t>(decades));
          spec.clear();
          sp_comp.clear();
          sp_log.clear();
          sp_key.clear();
          // A: the batch's changes, their symbol updates into the histograms
          for (size_t s = i; s < j; ++s) {
            if (!tail_ready(s)) return Fail(err);
            if (s >= prefetched) {
              prefetched = tail_exact ? std::max(sorter->sorted(), s + 1) : std::min(win_base + win_ok, s + 256);
              prefetch_chunk(s, std::min(prefetched, n_order));
            }
            const int bix = tail_block(s);
            if (lazy_host) materialize(bix);
            const int off = std::max(0, std::min(offsets[bix], static_cast<int>(cand.size()) - 1));
            const int li = last_indexes[bix] + std::min(direction, 0);
            if (li < 0 || off + li >= offsets[bix + 1]) {  // (an order entry without a candidate: a bug)
              if (err) *err = "back end: change order names a block without candidates left";
              return false;
            }
            const int idx = cand[off + li];
            Spec sp;
            sp.bix = bix;
            const int c = idx / kDCTBlockSize;
            sp.k = idx % kDCTBlockSize;
            sp.old = img->block(c, bix)[sp.k];
            sp.nz = acm.nz[static_cast<size_t>(c) * num_blocks + bix];
            sp_log.emplace_back();
            apply(bix, &sp_log.back());
            spec.push_back(sp);
            sp_comp.push_back(static_cast<uint8_t>(c));
            sp_key.push_back(tail_key(s));
          }
          // B, C: the histograms, the codes of every read step (on the pool),
          // the estimate and the break test; the changes past the break undone
          // (newest first; their journal entries stay: they name positions
          // whose values are current)
          const size_t done = run_steps(i, j - i, sp_comp.data(), sp_log.data(), sp_key.data(), &stop);
          if (stop) {
            for (size_t u = j - i; u-- > done;) {
              const Spec& sp = spec[u];
              img->block(sp_comp[u], sp.bix)[sp.k] = sp.old;
              acm.nz[static_cast<size_t>(sp_comp[u]) * num_blocks + sp.bix] = sp.nz;
              last_indexes[sp.bix] -= direction;
              if (lazy_host) mat_li[sp.bix] = last_indexes[sp.bix];
            }
            res_->detail["backend_spec_undone"] += static_cast<double>(j - i - done);
          }
          i = j;
          if (!fixed_decades) decades = std::min(std::min(kMaxDecades, std::max(4, 2 * workers)), decades * 2);
        }
      } else {
        // The tail on a partitioned frame, a window of entries at a time: the
        // owners apply theirs tentatively and publish the symbol updates,
        // every rank replays them in order into the frame's histograms and
        // finds the break; the owners undo what lies past it.
        struct Undo {
          size_t i;
          int bix, c, k;
          coeff_t old;
          uint64_t nz;
        };
        std::vector<Undo> undo;
        // the window of order positions i0 .. i0 + W - 1 (frame blocks /
        // keys); *done: positions processed (through the break if *stop)
        auto tail_window = [&](const int* blocks, const float* keys, size_t W, size_t i0, bool* stop,
                               size_t* done) -> bool {
          std::vector<uint8_t> rec;
          undo.clear();
          for (size_t j = 0; j < W; ++j) {
            const int bix = blocks[j] - gbase;
            if (bix < own_lo || bix >= own_hi) continue;
            if (lazy_host) materialize(bix);  // (the undo records current values)
            const int off = std::max(0, std::min(offsets[bix], static_cast<int>(cand.size()) - 1));
            const int idx = cand[off + last_indexes[bix] + std::min(direction, 0)];
            const int c = idx / kDCTBlockSize, k = idx % kDCTBlockSize;
            undo.push_back(Undo{i0 + j, bix, c, k, img->block(c, bix)[k],
                                acm.nz[static_cast<size_t>(c) * num_blocks + bix]});
            SymbolLog log;
            apply(bix, &log);
            const uint32_t pos = static_cast<uint32_t>(j);
            rec.insert(rec.end(), reinterpret_cast<const uint8_t*>(&pos),
                       reinterpret_cast<const uint8_t*>(&pos) + 4);
            rec.push_back(static_cast<uint8_t>(c));
            rec.push_back(log.n);
            for (int e = 0; e < log.n; ++e) {
              rec.push_back(log.sym[e]);
              rec.push_back(static_cast<uint8_t>(log.weight[e]));
            }
          }
          const auto tx = Clock::now();
          std::vector<std::vector<uint8_t>> all;
          if (!part_->coll->AllGatherV(rec, &all)) return false;
          res_->detail["strip_tail_exchange_s"] += Since(tx);
          std::vector<const uint8_t*> at(W, nullptr);
          for (const auto& m : all)
            for (const uint8_t* p = m.data(); p < m.data() + m.size();) {
              uint32_t pos;
              std::memcpy(&pos, p, 4);
              if (pos >= W) return false;
              at[pos] = p + 4;
              p += 6 + 2 * p[5];
            }
          // every rank runs the window's bookkeeping from the owners' symbol
          // updates (the speculative batches of the single-rank tail)
          std::vector<uint8_t> comp(W);
          std::vector<SymbolLog> logs(W);
          for (size_t q = 0; q < W; ++q) {
            const uint8_t* r = at[q];
            if (!r || r[1] > 32) return false;
            comp[q] = r[0];
            logs[q].n = r[1];
            for (int e = 0; e < r[1]; ++e) {
              logs[q].sym[e] = r[2 + 2 * e];
              logs[q].weight[e] = static_cast<int8_t>(r[3 + 2 * e]);
            }
          }
          size_t j = 0;
          for (size_t q0 = 0; q0 < W && !*stop;) {
            // (batches of about kMaxDecades rebuilds, ending before a read step)
            const size_t i = i0 + q0;
            const size_t first_code = (i + 9) / 10 * 10;
            const size_t q1 = std::min(W, first_code + 10 * 32 - i0);
            const size_t d = run_steps(i, q1 - q0, comp.data() + q0, logs.data() + q0, keys + q0, stop);
            q0 += d;
            j = q0 - (*stop ? 1 : 0);
          }
          if (*stop) {
            for (auto u = undo.rbegin(); u != undo.rend() && u->i > i0 + j; ++u) {
              img->block(u->c, u->bix)[u->k] = u->old;
              acm.nz[static_cast<size_t>(u->c) * num_blocks + u->bix] = u->nz;
              last_indexes[u->bix] -= direction;
              if (lazy_host) mat_li[u->bix] = last_indexes[u->bix];
            }
          }
          *done = *stop ? j + 1 : W;
          return true;
        };
        size_t i = bulk;
        bool stop = false;
        if (strip_dev && !strip_exact) {
          // the device's windows of the frame's order (certified positions);
          // a window run out without a tie asks for the next, a tie or an
          // overflow switches to the exact order (every rank's entries)
          std::vector<int> blocks;
          std::vector<float> keys;
          while (!stop && i < n_order) {
            if (i >= win_base + win_ok) {
              bool got = false;
              if (!win.empty() && win_ok == win.size() && !win_last && i == win_base + win_ok) {
                Engine::OrderSelection next;
                const size_t want = std::min<size_t>(8192, std::max<size_t>(512, 2 * win.size()));
                const auto tw = Clock::now();
                if (!cmp_->DeviceSelectWindow(i, want, direction, &next)) return Fail(err);
                res_->detail["backend_tail_windows"] += 1;
                res_->detail["backend_tail_window_s"] += Since(tw);
                if (!next.open && !next.window_overflow) {
                  win.swap(next.window);
                  win_base = i;
                  win_ok = next.window_ok;
                  win_last = next.window_last;
                  got = i < win_base + win_ok;
                }
              }
              if (!got) {
                if (!go_exact()) return exchange_failed();
                if (bulk) sorter->SetPrefix(bulk);
                res_->detail["backend_tail_exact"] += 1;
                break;
              }
            }
            const size_t W = std::min(win_base + win_ok, n_order) - i;
            blocks.resize(W);
            keys.resize(W);
            for (size_t j = 0; j < W; ++j) {
              blocks[j] = win[i - win_base + j].first;
              keys[j] = win[i - win_base + j].second;
            }
            size_t done = 0;
            const auto tw = Clock::now();
            if (!tail_window(blocks.data(), keys.data(), W, i, &stop, &done)) return exchange_failed();
            res_->detail["strip_window_s"] += Since(tw);
            i += done;
          }
        }
        if (strip_fast && !strip_exact) {
          // windows of the frame's order merged from every rank's next
          // entries (StripOrder::Next); positions whose entry the keys leave
          // open (a tie of several blocks) switch to the exact order
          strip_order.StartTail(global_order, bulk > 0);
          while (!stop && i < n_order) {
            std::vector<int> blocks;
            std::vector<float> keys;
            bool open = false;
            const auto tn = Clock::now();
            const int r = strip_order.Next(part_, &blocks, &keys, &open);
            res_->detail["strip_next_s"] += Since(tn);
            if (r < 0) return exchange_failed();
            if (r == 0) break;  // (no entries left on any rank)
            size_t done = 0;
            const size_t W = std::min(blocks.size(), n_order - i);
            const auto tw = Clock::now();
            if (W && !tail_window(blocks.data(), keys.data(), W, i, &stop, &done)) return exchange_failed();
            res_->detail["strip_window_s"] += Since(tw);
            strip_order.Consumed(done);
            i += done;
            if (!stop && open) {
              if (!go_exact()) return exchange_failed();
              if (bulk) sorter->SetPrefix(bulk);
              break;
            }
          }
          res_->detail["strip_order_fast_iters"] += strip_exact ? 0 : 1;
        }
        size_t window = 4096;
        while ((strip_dev ? strip_exact : (!strip_fast || strip_exact)) && !stop && i < n_order) {
          const size_t W = std::min(window, n_order - i);
          if (i + W > sorter->sorted()) {
            const auto ts = Clock::now();
            sorter->EnsureSorted(i + W - 1);
            sort_s += Since(ts);
          }
          std::vector<int> blocks(W);
          std::vector<float> keys(W);
          for (size_t j = 0; j < W; ++j) {
            blocks[j] = global_order[i + j].first;
            keys[j] = global_order[i + j].second;
          }
          size_t done = 0;
          const auto tw = Clock::now();
          if (!tail_window(blocks.data(), keys.data(), W, i, &stop, &done)) return exchange_failed();
          res_->detail["strip_exact_window_s"] += Since(tw);
          i += done;
          window *= 2;
        }
      }
      if (device_order) tail_len_[direction > 0 ? 0 : 1] = static_cast<size_t>(loop.changed) - bulk;
      res_->detail["backend_changes_s"] += Since(tc);
      res_->detail["backend_codes_s"] += codes_s;
      res_->detail["backend_sort_s"] += sort_s;
      res_->detail["backend_entropy_codes"] += n_codes;
      res_->detail["backend_changes"] += loop.changed;
      if (device_order) {
        if (!cmp_->DeviceOrderAdvance(loop.val_threshold, direction)) return Fail(err);
      } else {
        for (int i = 0; i < num_blocks; ++i) max_block_error[i] += block_weight[i] * loop.val_threshold * direction;
      }
      ++res_->iterations;
      if (direction > 0) ++res_->iterations_up; else ++res_->iterations_down;
      res_->seconds_backend += Since(tb);
      if (cmp_->HasKnownHistogramEncode()) {
        // the candidate's histograms are the tracked ones: no histogram pass
        if (!EncodeAndCompareKnown(jpg, *img, saved0, dc0, ac_histograms, err)) return false;
      } else if (!EncodeAndCompare(jpg, *img, err)) {
        return false;
      }
      prev_size = est_jpg_size;
    }
  }
  if (lazy_host) {
    // the device copy is the image now; nothing after the back end reads
    // the host copy before the next bulk rewrite (CopyFromJpegData) -- a
    // mirror that would have to read it fails instead (host_valid)
    img->host_valid = false;
    img->host_partial = false;
  }
  FlushOutput();
  return true;
}

bool Processor::BuildChangeOrder(int direction, int factor, double target_mul, int num_blocks,
                                 int own_lo, int own_hi, int gbase, const std::vector<float>& bmax,
                                 const std::vector<int>& last_indexes, const std::vector<int>& offsets,
                                 const std::vector<float>& cand_err,
                                 const std::vector<float>& max_block_error,
                                 std::vector<std::pair<int, float>>* order,
                                 std::vector<float>* block_weight, int* blocks_to_change,
                                 size_t* frame_entries) {
  const int own_chunks = (own_hi - own_lo + kOrderChunk - 1) / kOrderChunk;
  const int cand_n = static_cast<int>(cand_err.size());
  std::vector<float>& weight = *block_weight;
  for (int rblock = 1; rblock <= 4; ++rblock) {
    weight.assign(num_blocks, 0.0f);
    cmp_->ComputeBlockErrorAdjustmentWeights(direction, rblock, target_mul, factor, factor, bmax, &weight);
    // entry counts per chunk of blocks, their prefix sums, then each chunk
    // fills its own range
    std::vector<size_t> chunk_start(own_chunks + 1, 0);
    std::vector<int> chunk_btc(own_chunks, 0);
    auto block_entries = [&](int bix) -> int {
      if (weight[bix] == 0) return 0;
      const int last_index = last_indexes[bix];
      const int offset = std::max(0, std::min(offsets[bix], cand_n - 1));
      const int num_candidates = offsets[bix + 1] - offset;
      return direction > 0 ? std::max(0, num_candidates - last_index) : last_index;
    };
    ParallelFor(own_chunks, [&](int ch) {
      size_t n = 0;
      int btc = 0;
      for (int bix = own_lo + ch * kOrderChunk; bix < std::min(own_hi, own_lo + (ch + 1) * kOrderChunk); ++bix) {
        const int e = block_entries(bix);
        n += e;
        btc += e > 0 ? 1 : 0;
      }
      chunk_start[ch + 1] = n;
      chunk_btc[ch] = btc;
    });
    *blocks_to_change = 0;
    for (int ch = 0; ch < own_chunks; ++ch) {
      chunk_start[ch + 1] += chunk_start[ch];
      *blocks_to_change += chunk_btc[ch];
    }
    order->resize(chunk_start[own_chunks]);
    ParallelFor(own_chunks, [&](int ch) {
      std::pair<int, float>* out = order->data() + chunk_start[ch];
      for (int bix = own_lo + ch * kOrderChunk; bix < std::min(own_hi, own_lo + (ch + 1) * kOrderChunk); ++bix) {
        if (weight[bix] == 0) continue;
        const int last_index = last_indexes[bix];
        const int offset = std::max(0, std::min(offsets[bix], cand_n - 1));
        const int num_candidates = offsets[bix + 1] - offset;
        const float* errs = cand_err.data() + offset;
        const float max_err = max_block_error[bix];
        const int g = gbase + bix;
        if (direction > 0) {
          for (int i = last_index; i < num_candidates; ++i)
            *out++ = std::make_pair(g, (errs[i] - max_err) / weight[bix]);
        } else {
          for (int i = last_index - 1; i >= 0; --i)
            *out++ = std::make_pair(g, (max_err - errs[i]) / weight[bix]);
        }
      }
    });
    if (part_ && part_->world > 1 && frame_entries) {
      // this rank's entries only (StripOrder); the frame's totals
      int64_t t[2] = {static_cast<int64_t>(order->size()), *blocks_to_change};
      if (!part_->SumAll(t, 2)) return false;
      *frame_entries = static_cast<size_t>(t[0]);
      *blocks_to_change = static_cast<int>(t[1]);
      if (t[0] > 0) break;
      continue;
    }
    if (part_ && part_->world > 1) {
      // the frame's order: every rank's entries in rank (= block) order; a
      // rank sends its keys and a count per owned block
      const auto tx = Clock::now();
      if (!GatherEntries(order, own_lo, own_hi, gbase, blocks_to_change)) return false;
      res_->detail["strip_entries_s"] += Since(tx);
    }
    if (!order->empty()) break;
  }
  return true;
}

// The frame's change entries of one back-end iteration from every rank's
// owned ones (each rank sends its keys and an entry count per owned block;
// the pairs are rebuilt in rank order, which is block order).  *entries holds
// this rank's on entry, the frame's on return; *blocks_to_change becomes the
// frame's count.  Packing and unpacking run on the host pool.
bool Processor::GatherEntries(std::vector<std::pair<int, float>>* entries, int own_lo, int own_hi,
                              int gbase, int* blocks_to_change) {
  const int nown = own_hi - own_lo;
  const size_t n = entries->size();
  std::vector<uint8_t> send(8 + nown + n * 4, 0);
  const uint32_t n32 = static_cast<uint32_t>(n), btc = static_cast<uint32_t>(*blocks_to_change);
  std::memcpy(send.data(), &n32, 4);
  std::memcpy(send.data() + 4, &btc, 4);
  uint8_t* cnt = send.data() + 8;
  uint8_t* keys = send.data() + 8 + nown;
  constexpr int kSlices = 64;
  ParallelFor(kSlices, [&](int sl) {
    // (entries of one block are contiguous; a slice counts the blocks whose
    // first entry it holds, through the block's end)
    size_t i = n * sl / kSlices;
    const size_t end = n * (sl + 1) / kSlices;
    if (i > 0)
      while (i < end && (*entries)[i].first == (*entries)[i - 1].first) ++i;
    while (i < end) {
      const int b = (*entries)[i].first;
      size_t k = i;
      while (k < n && (*entries)[k].first == b) {
        std::memcpy(keys + 4 * k, &(*entries)[k].second, 4);
        ++k;
      }
      cnt[b - gbase - own_lo] = static_cast<uint8_t>(k - i);
      i = k;
    }
  });
  std::vector<std::vector<uint8_t>> all;
  if (!part_->coll->AllGatherV(send, &all)) return false;
  const int world = part_->world, bw = part_->bw;
  std::vector<size_t> rank_at(world + 1, 0);
  int frame_btc = 0;
  for (int r = 0; r < world; ++r) {
    uint32_t v;
    std::memcpy(&v, all[r].data(), 4);
    rank_at[r + 1] = rank_at[r] + v;
    std::memcpy(&v, all[r].data() + 4, 4);
    frame_btc += static_cast<int>(v);
  }
  entries->resize(rank_at[world]);
  // work items: (rank, 4096-block chunk), each filling its own range
  constexpr int kChunk = 4096;
  std::vector<std::pair<int, int>> items;
  std::vector<size_t> item_at;
  for (int r = 0; r < world; ++r) {
    const int nb = (part_->row0[r + 1] - part_->row0[r]) * bw;
    const uint8_t* c = all[r].data() + 8;
    size_t at = rank_at[r];
    for (int b0 = 0; b0 < nb; b0 += kChunk) {
      items.emplace_back(r, b0);
      item_at.push_back(at);
      for (int b = b0; b < std::min(nb, b0 + kChunk); ++b) at += c[b];
    }
  }
  ParallelFor(static_cast<int>(items.size()), [&](int it) {
    const int r = items[it].first, b0 = items[it].second;
    const int nb = (part_->row0[r + 1] - part_->row0[r]) * bw, base = part_->row0[r] * bw;
    const uint8_t* c = all[r].data() + 8;
    size_t at = item_at[it];
    const uint8_t* k = all[r].data() + 8 + nb + 4 * (at - rank_at[r]);
    for (int b = b0; b < std::min(nb, b0 + kChunk); ++b)
      for (int j = 0; j < c[b]; ++j, ++at, k += 4) {
        float key;
        std::memcpy(&key, k, 4);
        (*entries)[at] = std::make_pair(base + b, key);
      }
  });
  *blocks_to_change = frame_btc;
  return true;
}

// RemoveOriginalQuantization, processor.cc:94-107: coefficients times their
// quantization, quant tables of ones; q_in receives the originals.
void RemoveOriginalQuantization(JpegData* jpg, int q_in[3][kDCTBlockSize]) {
  for (int i = 0; i < 3; ++i) {
    JpegComponent& c = jpg->components[i];
    const int* q = jpg->quant[c.quant_idx].values;
    std::memcpy(q_in[i], q, sizeof(q_in[i]));
    bool ones = true;  // (RGB input: the q=1 originals -- nothing to multiply)
    for (int k = 0; k < kDCTBlockSize; ++k) ones = ones && q[k] == 1;
    if (ones) continue;
    for (size_t j = 0; j < c.coeffs.size(); ++j) c.coeffs[j] = static_cast<coeff_t>(c.coeffs[j] * q[j % 64]);
  }
  int ones[3][kDCTBlockSize];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < kDCTBlockSize; ++j) ones[i][j] = 1;
  SaveQuantTables(ones, jpg);
}

// IsGrayscale, processor.cc:921-929
// The 4:4:4 JpegData of a 4:2:0 one whose chroma is all zero: Y cropped to
// the image's blocks (a 4:2:0 file pads it to whole 16-pixel MCUs), chroma
// zero at full resolution.
JpegData Gray444Of420(const JpegData& jpg) {
  JpegData g = jpg;
  const int bw = (jpg.width + 7) / 8, bh = (jpg.height + 7) / 8;
  g.max_h_samp_factor = g.max_v_samp_factor = 1;
  g.mcu_cols = bw;
  g.mcu_rows = bh;
  for (int c = 0; c < 3; ++c) {
    JpegComponent& comp = g.components[c];
    comp.h_samp_factor = comp.v_samp_factor = 1;
    comp.width_in_blocks = bw;
    comp.height_in_blocks = bh;
    comp.coeffs.assign(static_cast<size_t>(bw) * bh * kDCTBlockSize, 0);
    if (c != 0) continue;
    const JpegComponent& y = jpg.components[0];
    for (int by = 0; by < bh; ++by)
      std::memcpy(&comp.coeffs[static_cast<size_t>(by) * bw * kDCTBlockSize],
                  &y.coeffs[static_cast<size_t>(by) * y.width_in_blocks * kDCTBlockSize],
                  static_cast<size_t>(bw) * kDCTBlockSize * sizeof(coeff_t));
  }
  return g;
}

bool IsGrayscale(const JpegData& jpg) {
  for (int c = 1; c < 3; ++c)
    for (coeff_t v : jpg.components[c].coeffs)
      if (v != 0) return false;
  return true;
}

// UpdateACHistogram, processor.cc:491-515
void UpdateACHistogram(int weight, const coeff_t* coeffs, const int* q, JpegHistogram* h) {
  int r = 0;
  for (int k = 1; k < 64; ++k) {
    const int k_nat = kJPEGNaturalOrder[k];
    const coeff_t coeff = coeffs[k_nat];
    if (coeff == 0) {
      ++r;
      continue;
    }
    while (r > 15) {
      h->Add(0xf0, weight);
      r -= 16;
    }
    h->Add((r << 4) + Log2FloorNonZero(std::abs(coeff / q[k_nat])) + 1, weight);
    r = 0;
  }
  if (r > 0) h->Add(0, weight);
}

int Processor::Run(const JpegData& jpg_in, std::string* err) {
  // ProcessJpegData, processor.cc:931-1020
  if (params_.butteraugli_target > 2.0f) {
    if (err) *err = "butteraugli target above 2.0 (quality below 84) is not supported";
    return GZ_ERR_INVALID_ARG;
  }
  if (jpg_in.components.size() != 3 || !HasYCbCrColorSpace(jpg_in)) {
    if (err) *err = "Only YUV color space input jpeg is supported";
    return GZ_ERR_UNSUPPORTED;
  }
  const bool input_is_420 = JpegIs420(jpg_in);
  if (!input_is_420 && !JpegIs444(jpg_in)) {
    if (err) *err = "Unsupported sampling factors";
    return GZ_ERR_UNSUPPORTED;
  }
  // The original's output (processor.cc:965-967) is written here on the
  // host unless the device coder can give it (DeviceEncodeOriginalAndCompare)
  std::string encoded;
  bool ones = true;
  for (const QuantTable& t : jpg_in.quant)
    for (int k = 0; k < kDCTBlockSize; ++k) ones = ones && t.values[k] == 1;
  const bool orig_on_device = cmp_ && cmp_->HasDeviceWriter() && !input_is_420 && ones;
  if (!orig_on_device) OutputJpeg(jpg_in, &encoded);
  final_score_ = -1;
  if (cmp_ == nullptr) {  // image too small for Butteraugli
    res_->jpeg = encoded;
    return GZ_OK;
  }
  int q_in[3][kDCTBlockSize];
  JpegData jpg = jpg_in;
  RemoveOriginalQuantization(&jpg, q_in);
  auto device_error = [&]() {
    Fail(err);
    return GZ_ERR_DEVICE;
  };
  CoeffImage img;
  // A 4:2:0 input whose chroma is all zero: DownsampleImage leaves it and
  // SaveToJpegData keeps its one component (processor.cc:990-1016), so its
  // search is the grayscale pass below on the 4:4:4 image it equals (zero
  // chroma upsamples to the same pixels at either factor)
  const bool gray420 = input_is_420 && IsGrayscale(jpg);
  JpegData jpg444;
  if (!input_is_420) {
    if (!cmp_->SetOriginalCoeffs(jpg)) return device_error();
    img.Init(jpg.width, jpg.height);
    img.CopyFromJpegData(jpg);
    if (orig_on_device) {
      size_t size = 0;
      bool used = false;
      if (!cmp_->DeviceEncodeOriginalAndCompare(img, jpg_in, params_.clear_metadata, &size, &used))
        return device_error();
      if (used) {
        MaybeOutputDevice(size);  // the first output: always kept
        if (getenv("GZ_CHECK_ORIGINAL_OUTPUT")) {  // test hook: bytes vs the host writer
          std::string host, dev;
          OutputJpeg(jpg_in, &host);
          if (!cmp_->DeviceFetchKept(&dev)) return device_error();
          if (host != dev || host.size() != size) {
            if (err) *err = "device-coded original output differs from the host writer's";
            return GZ_ERR_INTERNAL;
          }
        }
      } else {
        OutputJpeg(jpg_in, &encoded);
        MaybeOutput(encoded);
      }
    } else {
      if (!cmp_->Compare(img)) return device_error();
      MaybeOutput(encoded);
    }
  } else {
    Image420 im;
    im.Init(jpg.width, jpg.height);
    im.CopyFromJpegData(jpg);
    if (!cmp_->Compare420(im)) return device_error();
    MaybeOutput(encoded);
  }
  const int try_420 = (input_is_420 || params_.force_420 || (params_.try_420 && !IsGrayscale(jpg_in))) ? 1 : 0;
  const int force_420 = (input_is_420 || params_.force_420) ? 1 : 0;
  // DownsampleImage leaves an image whose chroma is all zero at 4:4:4
  // (output_image.cc:535-539) and SaveToJpegData keeps its one component, so
  // the "4:2:0" pass of such an image is the 4:4:4 machinery on a
  // one-component JpegData: the downsampling quantization generator, then the
  // Y search alone with ymul 1.0 (processor.cc:994-1016).
  const bool gray_pass = (!input_is_420 || gray420) && IsGrayscale(jpg);
  if (gray420) {  // (after the 4:2:0 Compare of the input above)
    jpg444 = Gray444Of420(jpg);
    if (!cmp_->SetOriginalCoeffs(jpg444)) return device_error();
    img.Init(jpg.width, jpg.height);
  }
  for (int downsample = force_420; downsample <= try_420; ++downsample) {
    if (downsample && !gray_pass) {
      const int rc = Run420(jpg_in, err);
      if (rc != GZ_OK) return rc;
      continue;
    }
    const JpegData& src = gray420 ? jpg444 : jpg;
    JpegData gray;
    const JpegData* pass_jpg = &src;
    if (downsample) {
      gray = src;
      gray.components.resize(1);
      pass_jpg = &gray;
    }
    img.CopyFromJpegData(src);
    int best_q[3][kDCTBlockSize];
    std::memcpy(best_q, q_in, sizeof(best_q));
    bool ok = false;
    if (!SelectQuantMatrix(*pass_jpg, downsample != 0, best_q, &img, &ok, err)) return GZ_ERR_DEVICE;
    if (!ok)
      for (int c = 0; c < 3; ++c)
        for (int i = 0; i < kDCTBlockSize; ++i) best_q[c][i] = 1;
    if (!cmp_->QuantizeFromOriginal(best_q, &img)) return device_error();
    if (!SelectFrequencyMasking(*pass_jpg, &img, downsample ? 1 : 7, 1.0, false, err))
      return GZ_ERR_DEVICE;
  }
  FlushOutput();
  if (kept_on_device_ && !cmp_->DeviceFetchKept(&res_->jpeg)) return device_error();
  return GZ_OK;
}

int Processor::Run420(const JpegData& jpg_in, std::string* err) {
  // processor.cc:990-1016 with downsample = 1
  FlushOutput();
  int q_in[3][kDCTBlockSize];
  JpegData jpg = jpg_in;
  RemoveOriginalQuantization(&jpg, q_in);
  JpegData jpg420;
  if (JpegIs420(jpg)) {
    // already subsampled (DownsampleImage leaves it): OutputImage of it,
    // saved back (whole MCUs, padding blocks re-derived)
    Image420 t;
    t.Init(jpg.width, jpg.height);
    t.CopyFromJpegData(jpg);
    jpg420.app_data = jpg.app_data;
    jpg420.com_data = jpg.com_data;
    t.SaveToJpegData(&jpg420);
  } else if (!DownsampleToJpegData420(jpg, params_.use_silver_screen, &jpg420)) {
    // (all-zero chroma: the reference keeps 4:4:4 and continues with one
    // grayscale component)
    if (err) *err = "4:2:0 pass of an image without chroma is not supported";
    return GZ_ERR_UNSUPPORTED;
  }
  if (jpg420.components.size() != 3) {
    if (err) *err = "4:2:0 pass of an image without chroma is not supported";
    return GZ_ERR_UNSUPPORTED;
  }
  auto device_error = [&]() {
    Fail(err);
    return GZ_ERR_DEVICE;
  };
  if (!cmp_->SetOriginalCoeffs420(jpg420)) return device_error();
  Image420 img;
  // (a candidate's bytes may still be in the writer thread, which reads
  // img's saved JpegData: joined before img goes out of scope on every
  // return -- the normal one applies its MaybeOutput first, below)
  struct JoinWriter {
    std::thread* t;
    ~JoinWriter() {
      if (t->joinable()) t->join();
    }
  } join_writer{&writer_};
  img.Init(jpg420.width, jpg420.height);
  // SelectQuantMatrix (processor.cc:340-372) with the downsampling generator
  int best_q[3][kDCTBlockSize];
  std::memcpy(best_q, q_in, sizeof(best_q));
  {
    QuantMatrixGenerator qgen(true);
    const float target_mul_high = 0.97f, target_mul_low = 0.95f;
    QuantData best;
    if (!TryQuantMatrix420(jpg420, target_mul_high, best_q, &img, &best, err)) return GZ_ERR_DEVICE;
    for (;;) {
      int q_next[3][kDCTBlockSize];
      if (!qgen.GetNext(q_next)) break;
      QuantData data;
      if (!TryQuantMatrix420(jpg420, target_mul_high, q_next, &img, &data, err)) return GZ_ERR_DEVICE;
      qgen.Add(data);
      if (CompareQuantData(data, best)) {
        best = data;
        if (data.dist_ok && !cmp_->DistanceOK(target_mul_low)) break;
      }
    }
    std::memcpy(best_q, best.q, sizeof(best.q));
    if (!best.dist_ok)
      for (int c = 0; c < 3; ++c)
        for (int i = 0; i < kDCTBlockSize; ++i) best_q[c][i] = 1;
  }
  const auto tq = Clock::now();
  img.CopyFromJpegData(jpg420);
  img.ApplyGlobalQuantization(best_q);
  res_->seconds_quantize += Since(tq);
  if (!SelectFrequencyMasking420(jpg420, &img, 1, 0.97f, false, err)) return GZ_ERR_DEVICE;
  if (!SelectFrequencyMasking420(jpg420, &img, 6, 1.0, true, err)) return GZ_ERR_DEVICE;
  FlushOutput();  // (the last candidate's MaybeOutput, with its own Compare's distance)
  return GZ_OK;
}

bool Processor::TryQuantMatrix420(const JpegData& jpg, float target_mul, const int q[3][kDCTBlockSize],
                                  Image420* img, QuantData* data, std::string* err) {
  // processor.cc:310-338
  std::memcpy(data->q, q, sizeof(data->q));
  const auto tq = Clock::now();
  img->CopyFromJpegData(jpg);
  img->ApplyGlobalQuantization(q);
  res_->seconds_quantize += Since(tq);
  FlushOutput();
  // the candidate's bytes on a helper thread while its Compare runs (the
  // size is needed at once: joined before the return)
  const auto te = Clock::now();
  const JpegData& out = img->SavedJpegData(jpg);
  res_->detail["r420_stage_s"] += Since(te);
  std::string encoded;
  double enc_s = 0.0;
  std::thread wr([&] {
    const auto t = Clock::now();
    WriteJpeg(out, params_.clear_metadata, &encoded);
    enc_s = Since(t);
  });
  ++res_->iterations;
  const auto tc = Clock::now();
  const bool ok = cmp_->Compare420(*img);
  res_->detail["r420_compare_s"] += Since(tc);
  const auto tw = Clock::now();
  wr.join();
  res_->detail["write_wait_s"] += Since(tw);
  res_->seconds_write += enc_s;
  res_->detail["write_jpeg_s"] += enc_s;
  if (!ok) return Fail(err);
  data->dist_ok = cmp_->DistanceOK(target_mul);
  data->jpg_size = encoded.size();
  MaybeOutput(encoded);
  return true;
}

// A 4:2:0 back-end candidate's output (processor.cc:899-904 after the
// iteration's changes): its bytes formed on the helper thread while the
// Compare that scores it and the next iteration's selection run;
// FlushOutput applies its MaybeOutput before the next Compare.
void Processor::BeginOutput420(const JpegData& jpg, Image420* img) {
  FlushOutput();
  const auto te = Clock::now();
  const JpegData& out = img->SavedJpegData(jpg);
  res_->detail["r420_stage_s"] += Since(te);
  pending_.clear();
  pending_device_ = false;
  pending_skipped_ = false;
  writer_ = std::thread([this, &out] {
    const auto t = Clock::now();
    WriteJpeg(out, params_.clear_metadata, &pending_);
    encode_s_ = Since(t);
  });
  has_pending_ = true;
}

bool Processor::SelectFrequencyMasking420(const JpegData& jpg, Image420* img, int comp_mask,
                                          double target_mul, bool stop_early, std::string* err) {
  // processor.cc:559-721 and the back end :723-919 for one pass of the 4:2:0
  // image (comp_mask 1: Y at factor 1; 6: Cb + Cr at factor 2), serial as
  // in the reference
  const int ncomp = static_cast<int>(jpg.components.size());
  const int last_c = Log2FloorNonZero(static_cast<uint32_t>(comp_mask));
  if (last_c >= ncomp) return true;
  const int factor = last_c == 0 ? 1 : 2;
  const int w = img->w, h = img->h;
  const int block_width = (w + 8 * factor - 1) / (8 * factor);
  const int block_height = (h + 8 * factor - 1) / (8 * factor);
  const int num_blocks = block_width * block_height;
  FlushOutput();  // (the last candidate's MaybeOutput sees its own Compare's distance)
  const auto tz = Clock::now();
  if (!cmp_->StartBlockComparisons()) return Fail(err);
  std::vector<int> offsets;
  std::vector<uint8_t> cand;
  std::vector<float> cand_err;
  if (!cmp_->BlockZeroingCandidates420(img, comp_mask, params_.zeroing_greedy_lookahead,
                                       params_.new_zeroing_model, &offsets, &cand, &cand_err))
    return Fail(err);
  cmp_->FinishBlockComparisons();
  res_->detail[comp_mask == 1 ? "r420_zeroing_y_s" : "r420_zeroing_c_s"] += Since(tz);
  res_->detail["candidates"] += static_cast<double>(cand.size());
  const auto tb0 = Clock::now();
  std::vector<JpegHistogram> ac_histograms(ncomp);
  int jpg_header_size, dc_size;
  {
    JpegData out;
    out.app_data = jpg.app_data;
    out.com_data = jpg.com_data;
    img->SaveToJpegData(&out);
    jpg_header_size = static_cast<int>(JpegHeaderSize(out, params_.clear_metadata));
    std::vector<JpegHistogram> dc(out.components.size());
    BuildDCHistograms(out, dc.data());
    size_t num = dc.size();
    std::vector<int> idx(num);
    std::vector<uint8_t> depths(num * JpegHistogram::kSize);
    dc_size = static_cast<int>(ClusterHistograms(dc.data(), &num, idx.data(), depths.data()));
    ac_histograms.resize(out.components.size());
    BuildACHistograms(out, ac_histograms.data());
  }
  std::vector<uint8_t> ac_depths;
  int ac_histogram_size = static_cast<int>(ComputeEntropyCodes(ac_histograms, &ac_depths));
  const int base_size = jpg_header_size + dc_size + ac_histogram_size +
                        static_cast<int>(EntropyCodedDataSize(ac_histograms, ac_depths));
  int prev_size = base_size;
  std::vector<float> max_block_error(num_blocks, 0.0f);
  std::vector<int> last_indexes(num_blocks, 0);
  // (a change's symbol updates from its neighbours in zigzag order, as the
  // 4:4:4 back end; UpdateACHistogram's two passes over the block give the
  // same counts)
  AcBlockModel acm;
  size_t acm_base[3];
  acm.Build(*img, acm_base);
  size_t chroma_updates = 0;
  res_->seconds_backend += Since(tb0);
  bool first_up_iter = true;
  for (int direction : {1, -1}) {
    for (;;) {
      if (stop_early && direction == -1) {
        FlushOutput();
        if (prev_size > 1.01 * best_size_) break;
      }
      const auto tb = Clock::now();
      std::vector<std::pair<int, float>> global_order;
      int blocks_to_change = 0;
      std::vector<float> block_weight;
      // the distance map's maximum per searched block (all zero on the first
      // up iteration, processor.cc:777-780)
      std::vector<float> bmax(num_blocks, 0.0f);
      if (!first_up_iter) {
        const std::vector<float>& m8 = cmp_->block_max_distance();
        if (cmp_->block_max_failed()) return Fail(err);
        const int bw8 = (w + 7) / 8, bh8 = (h + 7) / 8;
        for (int by = 0; by < bh8; ++by)
          for (int bx = 0; bx < bw8; ++bx) {
            float& d = bmax[(by / factor) * block_width + bx / factor];
            d = std::max(d, m8[by * bw8 + bx]);
          }
      }
      if (!BuildChangeOrder(direction, factor, target_mul, num_blocks, 0, num_blocks, 0, bmax,
                            last_indexes, offsets, cand_err, max_block_error, &global_order,
                            &block_weight, &blocks_to_change))
        return Fail(err);
      res_->detail["r420_order_s"] += Since(tb);
      if (global_order.empty()) {
        res_->seconds_backend += Since(tb);
        break;
      }
      // std::sort(global_order) (processor.cc:825-828), materialised lazily:
      // only the prefix the change loop consumes gets sorted (host/lazy_sort.h)
      LazyStdSort sorter(global_order.data(), global_order.size());
      ChangeLoop loop(direction, cmp_->DistanceOK(1.0), base_size, factor, blocks_to_change,
                      &first_up_iter, cmp_->BlockErrorLimit(), global_order);
      int est_jpg_size = prev_size;
      const size_t n_order = global_order.size();
      for (size_t i = 0; i < n_order; ++i) {
        if (i >= sorter.sorted()) sorter.EnsureSorted(i);
        const int bix = global_order[i].first;
        const int bx = bix % block_width, by = bix / block_width;
        const int last_idx = last_indexes[bix];
        const int offset = std::max(0, std::min(offsets[bix], static_cast<int>(cand.size()) - 1));
        const int idx = cand[offset + last_idx + std::min(direction, 0)];
        const int c = idx / kDCTBlockSize, k = idx % kDCTBlockSize;
        const int* quant = img->quant[c];
        const JpegComponent& comp = jpg.components[c];
        const int jpg_bix = by * comp.width_in_blocks + bx;
        const int newval =
            direction > 0 ? 0 : QuantizeCoeff(comp.coeffs[static_cast<size_t>(jpg_bix) * 64 + k], quant[k]);
        coeff_t* block = img->block(c, bix);
        acm.ChangeAt<JpegHistogram, false>(acm_base[c] + bix, c, block, k, static_cast<coeff_t>(newval), quant,
                                           nullptr, &ac_histograms[c], nullptr);
        img->SetCoeffBlock(c, bix, block);  // (the chroma's pixel update: 0.5 us, 0.17 s of a 1080p force_420)
        chroma_updates += c != 0;
        last_indexes[bix] += direction;
        loop.Applied(global_order[i].second);
        if (loop.CodesRead(i)) ac_histogram_size = static_cast<int>(ComputeEntropyCodes(ac_histograms, &ac_depths));
        if (!loop.EstimateRead(i)) continue;
        est_jpg_size = jpg_header_size + dc_size + ac_histogram_size +
                       static_cast<int>(EntropyCodedDataSize(ac_histograms, ac_depths));
        if (loop.Stop(est_jpg_size, prev_size)) break;
      }
      for (int i = 0; i < num_blocks; ++i) max_block_error[i] += block_weight[i] * loop.val_threshold * direction;
      ++res_->iterations;
      if (direction > 0) ++res_->iterations_up; else ++res_->iterations_down;
      res_->detail["backend420_changes"] += loop.changed;
      res_->detail["backend420_chroma_updates"] += static_cast<double>(chroma_updates);
      chroma_updates = 0;
      res_->seconds_backend += Since(tb);
      BeginOutput420(jpg, img);
      const auto tc = Clock::now();
      if (!cmp_->Compare420(*img)) return Fail(err);
      res_->detail["r420_compare_s"] += Since(tc);
      prev_size = est_jpg_size;
    }
  }
  return true;
}

}  // namespace

void EncodeRGBToJpegData(const uint8_t* rgb, int w, int h, JpegData* jpg) {
  InitJpegDataYUV444(w, h, jpg);
  for (auto& q : jpg->quant)
    for (int k = 0; k < kDCTBlockSize; ++k) q.values[k] = 1;
  const size_t nb = static_cast<size_t>(jpg->mcu_cols) * jpg->mcu_rows;
  std::vector<coeff_t> all(nb * 64 * 3);
  RgbToCoeffsQ1(rgb, w, h, all.data());
  for (int c = 0; c < 3; ++c)
    std::memcpy(jpg->components[c].coeffs.data(), all.data() + c * nb * 64, nb * 64 * sizeof(coeff_t));
}

int ProcessJpegData(const ProcessParams& params, const JpegData& jpg, Comparator* cmp,
                    ProcessResult* result, std::string* err, Partition* part) {
  if (part && (params.try_420 || params.force_420)) {
    if (err) *err = "4:2:0 output of a strip-decomposed frame is not supported";
    return GZ_ERR_UNSUPPORTED;
  }
  ActiveEncode active;  // (the host pool's worker cap)
  Processor proc(params, cmp, result, cmp ? part : nullptr);
  return proc.Run(jpg, err);
}

int Process(int device, const ProcessParams& params, const uint8_t* rgb, bool device_ptr, int w,
            int h, ProcessResult* result, std::string* err) {
  // guetzli::Process(params, stats, rgb, w, h, out), processor.cc:1157-1185
  const auto t0 = Clock::now();
  const double c0 = ThreadCpu();
  if (w <= 0 || h <= 0 || w >= (1 << 16) || h >= (1 << 16)) {
    if (err) *err = "Could not create jpg data from rgb pixels";
    return GZ_ERR_INVALID_ARG;
  }
  if (params.butteraugli_target > 2.0f) {
    // ProcessJpegData's first check (processor.cc:939-945), made before any
    // device work so that the answer does not depend on a device being there
    if (err) *err = "butteraugli target above 2.0 (quality below 84) is not supported";
    return GZ_ERR_INVALID_ARG;
  }
  JpegData jpg;
  std::unique_ptr<HipButteraugliComparator> cmp;
  if (w >= 32 && h >= 32) {
    // q=1 coefficients on the device from the resident reference image
    std::string e;
    cmp = HipButteraugliComparator::Create(device, w, h, rgb, device_ptr, params.butteraugli_target, &e);
    if (!cmp || !cmp->OriginalJpegData(&jpg)) {
      if (err) *err = cmp ? cmp->error() : e;
      return GZ_ERR_DEVICE;
    }
  } else {
    // Below 32 px guetzli::Process skips Butteraugli and writes the q=1
    // encode; that is the host encoder's job (no device work to mirror).
    std::vector<uint8_t> host_rgb;
    const uint8_t* hrgb = rgb;
    if (device_ptr) {
      host_rgb.resize(static_cast<size_t>(3) * w * h);
      if (hipSetDevice(device) != hipSuccess ||
          hipMemcpy(host_rgb.data(), rgb, host_rgb.size(), hipMemcpyDeviceToHost) != hipSuccess) {
        if (err) *err = "device rgb copy failed";
        return GZ_ERR_DEVICE;
      }
      hrgb = host_rgb.data();
    }
    EncodeRGBToJpegData(hrgb, w, h, &jpg);
  }
  result->seconds_setup = Since(t0);
  const int rc = ProcessJpegData(params, jpg, cmp.get(), result, err);
  if (cmp) {
    result->compares = cmp->compares;
    result->seconds_compare = cmp->seconds_compare;
    result->seconds_zeroing = cmp->seconds_zeroing;
    result->detail["compare_thread_cpu_s"] = cmp->cpu_compare;
    result->detail["compare_wait_s"] = cmp->seconds_wait;
    result->detail["compare_wait_cpu_s"] = cmp->cpu_wait;
    result->detail["scan_bound_mismatches"] = cmp->scan_bound_mismatches;
  }
  result->seconds_total = Since(t0);
  result->detail["thread_cpu_s"] = ThreadCpu() - c0;
  return rc;
}

int ProcessJpeg(int device, const ProcessParams& params, const uint8_t* data, size_t len,
                ProcessResult* result, std::string* err) {
  // guetzli::Process(params, stats, data, jpg_out), processor.cc:1029-1066
  const auto t0 = Clock::now();
  const double c0 = ThreadCpu();
  JpegData jpg;
  std::string rerr;
  if (!ReadJpeg(data, len, &jpg, &rerr)) {
    if (err) *err = "Can't read jpg data from input file: " + rerr;
    return GZ_ERR_INVALID_ARG;
  }
  if (!CheckJpegSanity(jpg)) {
    if (err) *err = "Unsupported input JPEG (unexpectedly large coefficient values)";
    return GZ_ERR_INVALID_ARG;
  }
  // ProcessJpegData's input checks (processor.cc:939-963), ahead of the
  // decode
  if (params.butteraugli_target > 2.0f) {
    if (err) *err = "butteraugli target above 2.0 (quality below 84) is not supported";
    return GZ_ERR_INVALID_ARG;
  }
  if (jpg.components.size() != 3 || !HasYCbCrColorSpace(jpg)) {
    if (err) *err = "Only YUV color space input jpeg is supported";
    return GZ_ERR_UNSUPPORTED;
  }
  if (!JpegIs444(jpg) && !JpegIs420(jpg)) {
    if (err) *err = "Unsupported sampling factors";
    return GZ_ERR_UNSUPPORTED;
  }

  std::vector<uint8_t> rgb;
  if (!DecodeJpegToRGB(jpg, &rgb)) {
    if (err) *err = "input JPEG could not be decoded";
    return GZ_ERR_UNSUPPORTED;
  }
  std::unique_ptr<HipButteraugliComparator> cmp;
  if (jpg.width >= 32 && jpg.height >= 32) {
    std::string e;
    cmp = HipButteraugliComparator::Create(device, jpg.width, jpg.height, rgb.data(), false,
                                           params.butteraugli_target, &e);
    if (!cmp) {
      if (err) *err = e;
      return GZ_ERR_DEVICE;
    }
  }
  result->seconds_setup = Since(t0);
  const int rc = ProcessJpegData(params, jpg, cmp.get(), result, err);
  if (cmp) {
    result->compares = cmp->compares;
    result->seconds_compare = cmp->seconds_compare;
    result->seconds_zeroing = cmp->seconds_zeroing;
    result->detail["compare_thread_cpu_s"] = cmp->cpu_compare;
    result->detail["compare_wait_s"] = cmp->seconds_wait;
    result->detail["compare_wait_cpu_s"] = cmp->cpu_wait;
    result->detail["scan_bound_mismatches"] = cmp->scan_bound_mismatches;
  }
  result->seconds_total = Since(t0);
  result->detail["thread_cpu_s"] = ThreadCpu() - c0;
  return rc;
}

}  // namespace gz
