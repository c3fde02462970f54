// The search loop's comparator backed by the CPU oracle (test
// infrastructure only: oracle/gz_oracle.c computes every Butteraugli value).
#pragma once

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "host/processor.h"

extern "C" {
#include "gz_oracle.h"
}

namespace gz_test {

class OracleComparator : public gz::Comparator {
 public:
  OracleComparator(int w, int h, const uint8_t* rgb, float target)
      : w_(w), h_(h), rgb_(rgb, rgb + 3 * static_cast<size_t>(w) * h), target_(target) {
    bw_ = (w + 7) / 8;
    bh_ = (h + 7) / 8;
    block_max_.assign(bw_ * bh_, 0.0f);
  }
  // Failure injection (strip tests): the n-th Compare / BlockZeroingOrders
  // call (1-based) fails; -1: never.
  int fail_compare_at = -1, fail_zeroing_at = -1;

  bool Compare(const gz::CoeffImage& img) override {
    if (++n_compare_ == fail_compare_at) {
      err_ = "injected Compare failure";
      return false;
    }
    std::vector<float> dm(static_cast<size_t>(w_) * h_);
    distance_ = gzo_compare(w_, h_, rgb_.data(), img.coeffs.data(), dm.data());
    for (int by = 0; by < bh_; ++by)
      for (int bx = 0; bx < bw_; ++bx) {
        float m = 0.0f;
        for (int y = 8 * by; y < std::min(h_, 8 * by + 8); ++y)
          for (int x = 8 * bx; x < std::min(w_, 8 * bx + 8); ++x) m = std::max(m, dm[y * w_ + x]);
        block_max_[by * bw_ + bx] = m;
      }
    return true;
  }
  bool StartBlockComparisons() override {
    const size_t n = static_cast<size_t>(w_) * h_;
    std::vector<float> ref(3 * n), dc(3 * n);
    gzo_srgb_to_linear_planes(w_, h_, rgb_.data(), ref.data());
    gzo_opsin_dynamics(w_, h_, ref.data());
    mask_.assign(3 * n, 0.0f);
    gzo_mask(w_, h_, ref.data(), ref.data(), mask_.data(), dc.data());
    return true;
  }
  void FinishBlockComparisons() override { mask_.clear(); }
  bool BlockZeroingOrders(const gz::CoeffImage& img, const gz::JpegData&, int comp_mask,
                          int lookahead, bool new_model, std::vector<gz::CoeffData>* out) override {
    if (++n_zeroing_ == fail_zeroing_at) {
      err_ = "injected zeroing failure";
      return false;
    }
    out->resize(static_cast<size_t>(img.blocks) * 192);
    gzo_block_zeroing_orders(w_, h_, rgb_.data(), mask_.data(), img.coeffs.data(), orig_.data(),
                             target_, lookahead, comp_mask, new_model ? 1 : 0,
                             reinterpret_cast<gzo_coeff_data*>(out->data()));
    return true;
  }
  bool QuantizeFromOriginal(const int q[3][64], gz::CoeffImage* img, bool) override {
    const size_t per = static_cast<size_t>(img->blocks) * 64;
    for (int c = 0; c < 3; ++c)
      for (size_t i = 0; i < per; ++i)
        img->coeffs[c * per + i] = gz::QuantizeCoeff(orig_[c * per + i], q[c][i & 63]);
    for (int c = 0; c < 3; ++c) std::memcpy(img->quant[c], q[c], sizeof(img->quant[c]));
    img->BulkChanged();
    return true;
  }
  double ScoreOutputSize(int size) const override { return gz::ScoreJPEG(distance_, size, target_); }
  bool DistanceOK(double target_mul) const override { return distance_ <= target_mul * target_; }
  float distmap_aggregate() const override { return distance_; }
  const std::vector<float>& block_max_distance() const override { return block_max_; }
  float BlockErrorLimit() const override { return target_; }
  void ComputeBlockErrorAdjustmentWeights(int direction, int max_block_dist, double target_mul,
                                          int fx, int fy, const std::vector<float>& bmax,
                                          std::vector<float>* weight) override {
    gz::BlockErrorAdjustmentWeights(w_, h_, target_, direction, max_block_dist, target_mul, fx, fy,
                                    bmax, weight);
  }
  bool SetOriginalCoeffs(const gz::JpegData& jpg) override {
    orig_.clear();
    for (int c = 0; c < 3; ++c)
      orig_.insert(orig_.end(), jpg.components[c].coeffs.begin(), jpg.components[c].coeffs.end());
    return true;
  }
  const std::string& error() const override { return err_; }
  int n_compare_ = 0, n_zeroing_ = 0;

 private:
  int w_, h_, bw_, bh_;
  std::vector<uint8_t> rgb_;
  float target_;
  float distance_ = 0.0f;
  std::vector<float> block_max_, mask_;
  std::vector<gz::coeff_t> orig_;
  std::string err_;
};

}  // namespace gz_test
