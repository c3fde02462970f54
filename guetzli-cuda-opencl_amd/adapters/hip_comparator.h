// Comparator-level drop-in for the reference tree: guetzli::Comparator
// (guetzli/comparator.h:29-96) implemented over the C ABI of libguetzli_hip
// (include/guetzli_hip.h), for callers that keep the reference's own
// Processor (guetzli/processor.cc) and swap only the comparator -- the shape
// of the reference's ButteraugliComparatorEx / --cuda design.
//
// Compiled against the reference's headers (guetzli/comparator.h,
// guetzli/output_image.h, guetzli/stats.h); it needs nothing else from the
// reference and no HIP headers.  Every call goes to the GPU; a device error
// aborts with a message (the Comparator interface has no error channel, and
// there is no CPU fallback).
//
// Images with subsampled components (the reference's 4:2:0 search): their
// pixels are state of the OutputImage, not a function of the coefficients,
// so Compare / CompareBlock send the image's sRGB pixels (ToSRGB) instead of
// its coefficients (gz_comparator_compare_rgb / _compare_blocks_rgb).
#ifndef GUETZLI_HIP_ADAPTER_HIP_COMPARATOR_H_
#define GUETZLI_HIP_ADAPTER_HIP_COMPARATOR_H_

#include <stdint.h>

#include <vector>

#include "guetzli/comparator.h"
#include "guetzli/output_image.h"
#include "guetzli/stats.h"
#include "guetzli_hip.h"

namespace guetzli {

class HipButteraugliComparator : public Comparator {
 public:
  // ButteraugliComparator(w, h, rgb, target, stats)
  // (guetzli/butteraugli_comparator.cc:48-58), on HIP device `device`.
  HipButteraugliComparator(int width, int height, const std::vector<uint8_t>* rgb,
                           float target_distance, ProcessStats* stats, int device = 0);
  ~HipButteraugliComparator() override;

  // Comparator::Compare (butteraugli_comparator.cc:60-70): the image's DCT
  // coefficients (4:4:4) or its sRGB pixels (subsampled components) go to
  // the device; distance + per-block maxima come back.
  void Compare(const OutputImage& img) override;
  // butteraugli_comparator.cc:72-83: the activity mask of the reference.
  void StartBlockComparisons() override;
  void FinishBlockComparisons() override {}
  // butteraugli_comparator.cc:85-111 (the 8x8 opsin of the original block is
  // formed on the device per CompareBlock call).
  void SwitchBlock(int block_x, int block_y, int factor_x, int factor_y) override;
  // butteraugli_comparator.cc:113-163 on the device: `candidate_block` for
  // the components in comp_mask, the image's current block for the others
  // (4:4:4); the image's 8x8 sRGB window at the block when img has
  // subsampled components (the caller has set the candidate into img,
  // processor.cc:426-431).
  double CompareBlock(const OutputImage& img, int off_x, int off_y,
                      const coeff_t* candidate_block, const int comp_mask) const override;
  // butteraugli_comparator.cc:235-237
  double ScoreOutputSize(int size) const override;
  // butteraugli_comparator.h:52-54
  bool DistanceOK(double target_mul) const override;
  // The distance map of the last Compare (recomputed on the device).
  const std::vector<float> distmap() const override;
  float distmap_aggregate() const override { return distance_; }
  float BlockErrorLimit() const override { return target_; }
  // butteraugli_comparator.cc:169-233 (gz_block_error_adjustment_weights)
  void ComputeBlockErrorAdjustmentWeights(int direction, int max_block_dist, double target_mul,
                                          int factor_x, int factor_y,
                                          const std::vector<float>& distmap,
                                          std::vector<float>* block_weight) override;

 private:
  void Die(const char* what) const;
  gz_comparator* cmp_ = nullptr;
  ProcessStats* stats_;
  const int width_, height_, block_width_, num_blocks_;
  const float target_;
  float distance_ = 0.0f;
  int block_x_ = 0, block_y_ = 0, factor_x_ = 1, factor_y_ = 1;
  std::vector<int16_t> coeffs_;  // [3][blocks][64] staging of Compare
  mutable std::vector<int16_t> cand_;  // [3][64] staging of CompareBlock
};

}  // namespace guetzli

#endif  // GUETZLI_HIP_ADAPTER_HIP_COMPARATOR_H_
