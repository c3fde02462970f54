// Row-strip decomposition of one frame over the ranks of a job; see strips.h.
#include "host/strips.h"

#include <algorithm>
#include <chrono>
#include <cstring>

#include "host/jpeg_encode.h"
#include "host/thread_pool.h"
#include "../../include/guetzli_hip.h"

namespace gz {

namespace {
using Clock = std::chrono::steady_clock;
inline double Since(Clock::time_point t0) {
  return std::chrono::duration<double>(Clock::now() - t0).count();
}
}  // namespace

StripLayout StripLayout::Make(int width, int height, int world) {
  StripLayout L;
  L.width = width;
  L.height = height;
  L.world = world;
  const int per = (height + world - 1) / world;
  const int step = (per + kStripAlign - 1) / kStripAlign * kStripAlign;
  for (int r = 0; r < world; ++r) {
    const int y0 = std::min(height, r * step), y1 = std::min(height, (r + 1) * step);
    L.y0.push_back(y0);
    L.y1.push_back(y1);
    L.e0.push_back(y0 == y1 ? y0 : std::max(0, y0 - kStripHalo));
    L.e1.push_back(y0 == y1 ? y1 : std::min(height, y1 + kStripHalo));
  }
  return L;
}

bool Collectives::AllGatherV(const std::vector<uint8_t>& send,
                             std::vector<std::vector<uint8_t>>* out) {
  const int n = world();
  const uint64_t mine = send.size();
  std::vector<uint64_t> sizes(n);
  if (!AllGather(&mine, sizeof(mine), sizes.data())) return false;
  const uint64_t cap = std::max<uint64_t>(1, *std::max_element(sizes.begin(), sizes.end()));
  std::vector<uint8_t> padded(cap, 0), all(cap * n);
  if (!send.empty()) std::memcpy(padded.data(), send.data(), send.size());
  if (!AllGather(padded.data(), cap, all.data())) return false;
  out->resize(n);
  for (int r = 0; r < n; ++r)
    (*out)[r].assign(all.begin() + r * cap, all.begin() + r * cap + sizes[r]);
  return true;
}

StripComparator::StripComparator(const StripLayout& layout, std::unique_ptr<Comparator> inner,
                                 Collectives* coll, float target)
    : layout_(layout), inner_(std::move(inner)), coll_(coll), target_(target) {
  rank_ = coll->rank();
  bw_ = (layout.width + 7) / 8;
  blocks_ = bw_ * ((layout.height + 7) / 8);
  lb0_ = layout.e0[rank_] / 8;
  lb1_ = (layout.e1[rank_] + 7) / 8;
  ob0_ = layout.y0[rank_] / 8;
  ob1_ = (layout.y1[rank_] + 7) / 8;
  for (int r = 0; r < layout.world; ++r)
    max_owned_ = std::max(max_owned_, ((layout.y1[r] + 7) / 8 - layout.y0[r] / 8) * bw_);
  if (inner_) local_.Init(layout.width, layout.e1[rank_] - layout.e0[rank_]);
  block_max_.assign(blocks_, 0.0f);
}

bool StripComparator::Fail(const std::string& what) {
  err_ = what;
  return false;
}

bool StripComparator::Sync(const CoeffImage& img) {
  if (!inner_ || synced_.Current(img)) return true;
  if (!img.host_valid) return Fail("strip comparator: host coefficients are stale");
  const size_t per = static_cast<size_t>(img.blocks) * 64;
  const size_t lper = static_cast<size_t>(local_.blocks) * 64;
  const size_t first = static_cast<size_t>(lb0_) * bw_ * 64;  // the strip's first coefficient
  if (synced_.CanReplay(img)) {
    for (size_t i = synced_.pos; i < img.changed.size(); ++i) {
      const uint32_t idx = img.changed[i];
      const int c = static_cast<int>(idx / per);
      const size_t off = idx - c * per;
      if (off < first || off >= first + lper) continue;
      const size_t loff = off - first;
      local_.coeffs[c * lper + loff] = img.coeffs[idx];
      local_.MarkChanged(c, static_cast<int>(loff / 64), static_cast<int>(loff % 64));
    }
  } else {
    for (int c = 0; c < 3; ++c) {
      std::memcpy(&local_.coeffs[c * lper], &img.coeffs[c * per + first], lper * sizeof(coeff_t));
      std::memcpy(local_.quant[c], img.quant[c], sizeof(local_.quant[c]));
    }
    local_.BulkChanged();
  }
  synced_.Set(img);
  return true;
}

bool StripComparator::SetOriginalCoeffs(const JpegData& jpg) {
  orig_.clear();
  for (int c = 0; c < 3; ++c)
    orig_.insert(orig_.end(), jpg.components[c].coeffs.begin(), jpg.components[c].coeffs.end());
  if (!inner_) return true;
  InitJpegDataYUV444(layout_.width, layout_.e1[rank_] - layout_.e0[rank_], &local_orig_);
  local_orig_.app_data = jpg.app_data;
  local_orig_.com_data = jpg.com_data;
  local_orig_.quant = jpg.quant;
  const size_t lper = static_cast<size_t>(local_.blocks) * 64;
  const size_t first = static_cast<size_t>(lb0_) * bw_ * 64;
  for (int c = 0; c < 3; ++c) {
    JpegComponent& lc = local_orig_.components[c];
    lc.quant_idx = jpg.components[c].quant_idx;
    lc.coeffs.assign(jpg.components[c].coeffs.begin() + first,
                     jpg.components[c].coeffs.begin() + first + lper);
  }
  if (!inner_->SetOriginalCoeffs(local_orig_)) return Fail(inner_->error());
  return true;
}

bool StripComparator::QuantizeFromOriginal(const int q[3][kDCTBlockSize], CoeffImage* img,
                                           bool /*need_host*/) {
  // CopyFromJpegData(q=1) + ApplyGlobalQuantization (processor.cc:316-317):
  // the whole image on the host (every rank's search loop reads it), the
  // strip on the device.
  const size_t per = static_cast<size_t>(img->blocks) * 64;
  constexpr size_t kChunk = 1 << 16;
  const int chunks = static_cast<int>((3 * per + kChunk - 1) / kChunk);
  ParallelFor(chunks, [&](int ch) {
    const size_t lo = ch * kChunk, hi = std::min(3 * per, lo + kChunk);
    for (size_t i = lo; i < hi; ++i)
      img->coeffs[i] = QuantizeCoeff(orig_[i], q[i / per][i & 63]);
  });
  for (int c = 0; c < 3; ++c) std::memcpy(img->quant[c], q[c], sizeof(img->quant[c]));
  img->BulkChanged();
  if (inner_) {
    if (!inner_->QuantizeFromOriginal(q, &local_, true)) return Fail(inner_->error());
    synced_.Set(*img);
  }
  return true;
}

// Every exchange message starts with a status word, and a rank whose local
// step failed still takes part in the exchange: all ranks then see the
// failure in the same collective and fail together instead of leaving the
// others blocked in the next all-gather.
bool StripComparator::CheckStatus(const std::vector<uint32_t>& status, const std::string& local) {
  for (int r = 0; r < layout_.world; ++r) {
    if (status[r] == 0) continue;
    if (r == rank_) return Fail(local);
    return Fail("strip comparator: rank " + std::to_string(r) + " failed");
  }
  return true;
}

bool StripComparator::Compare(const CoeffImage& img) {
  // message: [status][owned block maxima, padded to the largest strip]
  std::vector<float> mine(1 + max_owned_, 0.0f);
  uint32_t st = 0;
  std::string local_err;
  if (!Sync(img)) {
    st = 1;
    local_err = err_;
  } else if (inner_) {
    if (!inner_->Compare(local_)) {
      st = 1;
      local_err = inner_->error();
    } else {
      const std::vector<float>& lb = inner_->block_max_distance();
      const size_t off = static_cast<size_t>(ob0_ - lb0_) * bw_;
      std::copy(lb.begin() + off, lb.begin() + off + rank_blocks(), mine.begin() + 1);
    }
  }
  std::memcpy(mine.data(), &st, sizeof(st));
  const auto t0 = Clock::now();
  const size_t stride = 1 + static_cast<size_t>(max_owned_);
  std::vector<float> all(stride * layout_.world);
  if (!coll_->AllGather(mine.data(), mine.size() * sizeof(float), all.data()))
    return Fail("strip comparator: block maxima all-gather failed");
  seconds_exchange += Since(t0);
  std::vector<uint32_t> status(layout_.world);
  for (int r = 0; r < layout_.world; ++r) std::memcpy(&status[r], &all[r * stride], sizeof(uint32_t));
  if (!CheckStatus(status, local_err)) return false;
  float d = 0.0f;
  for (int r = 0; r < layout_.world; ++r) {
    const int b0 = layout_.y0[r] / 8 * bw_;
    const int nb = ((layout_.y1[r] + 7) / 8 - layout_.y0[r] / 8) * bw_;
    for (int i = 0; i < nb; ++i) {
      const float v = all[static_cast<size_t>(r) * stride + 1 + i];
      block_max_[b0 + i] = v;
      d = std::max(d, v);
    }
  }
  // ButteraugliScoreFromDiffmap (butteraugli.cc:1233-1240): the maximum of
  // the map is the maximum of its block maxima
  distance_ = d;
  return true;
}

bool StripComparator::StartBlockComparisons() {
  if (inner_ && !inner_->StartBlockComparisons()) return Fail(inner_->error());
  return true;
}

void StripComparator::FinishBlockComparisons() {
  if (inner_) inner_->FinishBlockComparisons();
}

bool StripComparator::BlockZeroingOrders(const CoeffImage& img, const JpegData& orig_jpg,
                                         int comp_mask, int lookahead, bool new_model,
                                         std::vector<CoeffData>* out) {
  // The orders through the candidates' form (processor.cc:690-700 filter)
  // are all the search reads; the unfiltered form is not exchanged.
  (void)img;
  (void)orig_jpg;
  (void)comp_mask;
  (void)lookahead;
  (void)new_model;
  (void)out;
  return Fail("strip comparator: use BlockZeroingCandidates");
}

bool StripComparator::BlockZeroingCandidates(const CoeffImage& img, const JpegData& orig_jpg,
                                             int comp_mask, int lookahead, bool new_model,
                                             std::vector<int>* offsets, std::vector<uint8_t>* idx,
                                             std::vector<float>* err) {
  (void)orig_jpg;
  // this rank's owned blocks: [status][count per block][candidate bytes][errors]
  // (a failed rank sends its status alone and still takes part, see Compare)
  std::vector<uint8_t> send(sizeof(uint32_t), 0);
  uint32_t st = 0;
  std::string local_err;
  std::vector<int> loff;
  std::vector<uint8_t> lidx;
  std::vector<float> lerr;
  if (!Sync(img)) {
    st = 1;
    local_err = err_;
  } else if (inner_ && !inner_->BlockZeroingCandidates(local_, local_orig_, comp_mask, lookahead,
                                                       new_model, &loff, &lidx, &lerr)) {
    st = 1;
    local_err = inner_->error();
  }
  std::memcpy(send.data(), &st, sizeof(st));
  if (inner_ && st == 0) {
    const int b0 = (ob0_ - lb0_) * bw_, nb = rank_blocks();
    const int c0 = loff[b0], c1 = loff[b0 + nb];
    send.resize(sizeof(uint32_t) + sizeof(int) * nb + (c1 - c0) * (1 + sizeof(float)));
    uint8_t* p = send.data() + sizeof(uint32_t);
    for (int b = 0; b < nb; ++b) {
      const int cnt = loff[b0 + b + 1] - loff[b0 + b];
      std::memcpy(p, &cnt, sizeof(int));
      p += sizeof(int);
    }
    std::memcpy(p, lidx.data() + c0, c1 - c0);
    p += c1 - c0;
    std::memcpy(p, lerr.data() + c0, (c1 - c0) * sizeof(float));
  }
  const auto t0 = Clock::now();
  std::vector<std::vector<uint8_t>> all;
  if (!coll_->AllGatherV(send, &all)) return Fail("strip comparator: candidate all-gather failed");
  seconds_exchange += Since(t0);
  std::vector<uint32_t> status(layout_.world, 1);
  for (int r = 0; r < layout_.world; ++r)
    if (all[r].size() >= sizeof(uint32_t)) std::memcpy(&status[r], all[r].data(), sizeof(uint32_t));
  if (!CheckStatus(status, local_err)) return false;
  for (auto& m : all) m.erase(m.begin(), m.begin() + sizeof(uint32_t));
  offsets->assign(blocks_ + 1, 0);
  idx->clear();
  err->clear();
  for (int r = 0; r < layout_.world; ++r) {
    const int b0 = layout_.y0[r] / 8 * bw_;
    const int nb = ((layout_.y1[r] + 7) / 8 - layout_.y0[r] / 8) * bw_;
    if (nb == 0) continue;
    const std::vector<uint8_t>& buf = all[r];
    if (buf.size() < sizeof(int) * static_cast<size_t>(nb))
      return Fail("strip comparator: short candidate message");
    std::vector<int> cnt(nb);
    std::memcpy(cnt.data(), buf.data(), sizeof(int) * nb);
    size_t total = 0;
    for (int c : cnt) total += c;
    if (buf.size() != sizeof(int) * nb + total * (1 + sizeof(float)))
      return Fail("strip comparator: bad candidate message");
    const uint8_t* pi = buf.data() + sizeof(int) * nb;
    const uint8_t* pe = pi + total;
    const size_t base = idx->size();
    idx->insert(idx->end(), pi, pi + total);
    err->resize(base + total);
    std::memcpy(err->data() + base, pe, total * sizeof(float));
    int run = static_cast<int>(base);
    for (int b = 0; b < nb; ++b) {
      (*offsets)[b0 + b] = run;
      run += cnt[b];
    }
  }
  (*offsets)[blocks_] = static_cast<int>(idx->size());
  // blocks of no rank (none: the strips tile the image) keep offset 0
  return true;
}

void StripComparator::ComputeBlockErrorAdjustmentWeights(
    int direction, int max_block_dist, double target_mul, int factor_x, int factor_y,
    const std::vector<float>& max_dist_per_block, std::vector<float>* block_weight) {
  BlockErrorAdjustmentWeights(layout_.width, layout_.height, target_, direction, max_block_dist,
                              target_mul, factor_x, factor_y, max_dist_per_block, block_weight);
}

int ProcessStrips(int device, const ProcessParams& params, const uint8_t* rgb, int w, int h,
                  Collectives* coll, ProcessResult* result, std::string* err) {
  const auto t0 = Clock::now();
  if (w <= 0 || h <= 0 || w >= (1 << 16) || h >= (1 << 16)) {
    if (err) *err = "Could not create jpg data from rgb pixels";
    return GZ_ERR_INVALID_ARG;
  }
  JpegData jpg;
  EncodeRGBToJpegData(rgb, w, h, &jpg);
  std::unique_ptr<StripComparator> cmp;
  HipButteraugliComparator* hip = nullptr;
  if (w >= 32 && h >= 32) {
    const StripLayout L = StripLayout::Make(w, h, coll->world());
    const int r = coll->rank();
    std::unique_ptr<Comparator> inner;
    std::string e;
    if (L.y1[r] > L.y0[r]) {
      auto c = HipButteraugliComparator::Create(device, w, L.e1[r] - L.e0[r],
                                                rgb + static_cast<size_t>(3) * w * L.e0[r], false,
                                                params.butteraugli_target, &e);
      hip = c.get();
      inner = std::move(c);
    }
    // every rank reports whether its device comparator came up before any
    // rank enters the search (a rank that returned here alone would leave the
    // others waiting in the first exchange)
    const uint32_t mine = (L.y1[r] > L.y0[r] && !inner) ? 1u : 0u;
    std::vector<uint32_t> status(coll->world());
    if (!coll->AllGather(&mine, sizeof(mine), status.data())) {
      if (err) *err = "strip setup: status all-gather failed";
      return GZ_ERR_INTERNAL;
    }
    for (int q = 0; q < coll->world(); ++q) {
      if (status[q] == 0) continue;
      if (err) *err = q == r ? e : "strip setup: rank " + std::to_string(q) + " failed";
      return GZ_ERR_DEVICE;
    }
    cmp.reset(new StripComparator(L, std::move(inner), coll, params.butteraugli_target));
  }
  result->seconds_setup = Since(t0);
  const int rc = ProcessJpegData(params, jpg, cmp.get(), result, err);
  if (hip) {
    result->compares = hip->compares;
    result->seconds_compare = hip->seconds_compare;
    result->seconds_zeroing = hip->seconds_zeroing;
  }
  if (cmp) result->detail["strip_exchange_s"] = cmp->seconds_exchange;
  result->seconds_total = Since(t0);
  return rc;
}

}  // namespace gz
