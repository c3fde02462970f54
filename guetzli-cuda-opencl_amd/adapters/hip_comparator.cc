// guetzli::Comparator over libguetzli_hip -- see hip_comparator.h.
#include "hip_comparator.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

namespace guetzli {

HipButteraugliComparator::HipButteraugliComparator(int width, int height,
                                                   const std::vector<uint8_t>* rgb,
                                                   float target_distance, ProcessStats* stats,
                                                   int device)
    : stats_(stats),
      width_(width),
      height_(height),
      block_width_((width + 7) / 8),
      num_blocks_(((width + 7) / 8) * ((height + 7) / 8)),
      target_(target_distance),
      coeffs_(static_cast<size_t>(num_blocks_) * 3 * 64),
      cand_(3 * 64) {
  if (!rgb || rgb->size() != 3u * static_cast<size_t>(width) * height)
    Die("reference image size");
  if (gz_comparator_create(device, width, height, rgb->data(), target_distance, &cmp_) != GZ_OK)
    Die("gz_comparator_create");
}

HipButteraugliComparator::~HipButteraugliComparator() { gz_comparator_destroy(cmp_); }

void HipButteraugliComparator::Die(const char* what) const {
  fprintf(stderr, "HipButteraugliComparator: %s failed: %s\n", what, gz_last_error());
  if (stats_ && stats_->debug_output) {
    *stats_->debug_output += "HipButteraugliComparator: ";
    *stats_->debug_output += what;
    *stats_->debug_output += " failed\n";
  }
  abort();
}

void HipButteraugliComparator::Compare(const OutputImage& img) {
  if (img.width() != width_ || img.height() != height_) Die("Compare: image size");
  for (int c = 0; c < 3; ++c) {
    const OutputImageComponent& comp = img.component(c);
    if (comp.factor_x() != 1 || comp.factor_y() != 1) {
      // subsampled: the pixels (ToLinearRGB's source) are the input
      const std::vector<uint8_t> rgb = img.ToSRGB();
      if (gz_comparator_compare_rgb(cmp_, rgb.data(), &distance_) != GZ_OK) Die("Compare");
      return;
    }
    // [blocks][64] per component: the layout of OutputImageComponent::coeffs()
    memcpy(&coeffs_[static_cast<size_t>(c) * num_blocks_ * 64], comp.coeffs(),
           static_cast<size_t>(num_blocks_) * 64 * sizeof(coeff_t));
  }
  if (gz_comparator_compare(cmp_, coeffs_.data(), &distance_) != GZ_OK) Die("Compare");
}

void HipButteraugliComparator::StartBlockComparisons() {
  if (gz_comparator_start_block_comparisons(cmp_, nullptr) != GZ_OK)
    Die("StartBlockComparisons");
}

void HipButteraugliComparator::SwitchBlock(int block_x, int block_y, int factor_x,
                                           int factor_y) {
  block_x_ = block_x;
  block_y_ = block_y;
  factor_x_ = factor_x;
  factor_y_ = factor_y;
}

double HipButteraugliComparator::CompareBlock(const OutputImage& img, int off_x, int off_y,
                                              const coeff_t* candidate_block,
                                              const int comp_mask) const {
  bool subsampled = factor_x_ != 1 || factor_y_ != 1;
  for (int c = 0; c < 3; ++c)
    subsampled = subsampled || img.component(c).factor_x() != 1 || img.component(c).factor_y() != 1;
  if (subsampled) {
    // (also the Y search of a 4:2:0 image: its chroma pixels are state)
    // the 8x8 block (block_x * factor_x + off_x, ...) as ToLinearRGB reads it
    const int bx = block_x_ * factor_x_ + off_x, by = block_y_ * factor_y_ + off_y;
    const std::vector<uint8_t> rgb = img.ToSRGB(8 * bx, 8 * by, 8, 8);
    const int b = by * block_width_ + bx;
    double err = 0.0;
    if (gz_comparator_compare_blocks_rgb(cmp_, 1, &b, rgb.data(), &err) != GZ_OK) Die("CompareBlock");
    return err;
  }
  if (off_x != 0 || off_y != 0) Die("CompareBlock: offset within a 4:4:4 block");
  for (int c = 0; c < 3; ++c) {
    if (comp_mask & (1 << c)) {
      memcpy(&cand_[64 * c], candidate_block + 64 * c, 64 * sizeof(coeff_t));
    } else {
      img.component(c).GetCoeffBlock(block_x_, block_y_, &cand_[64 * c]);
    }
  }
  const int b = block_y_ * block_width_ + block_x_;
  double err = 0.0;
  if (gz_comparator_compare_blocks(cmp_, 1, &b, cand_.data(), &err) != GZ_OK)
    Die("CompareBlock");
  return err;
}

double HipButteraugliComparator::ScoreOutputSize(int size) const {
  return gz_comparator_score_output_size(cmp_, size);
}

bool HipButteraugliComparator::DistanceOK(double target_mul) const {
  return gz_comparator_distance_ok(cmp_, target_mul) != 0;
}

const std::vector<float> HipButteraugliComparator::distmap() const {
  std::vector<float> out(static_cast<size_t>(width_) * height_);
  if (gz_comparator_distmap(cmp_, out.data()) != GZ_OK) Die("distmap");
  return out;
}

void HipButteraugliComparator::ComputeBlockErrorAdjustmentWeights(
    int direction, int max_block_dist, double target_mul, int factor_x, int factor_y,
    const std::vector<float>& distmap, std::vector<float>* block_weight) {
  if (distmap.size() != static_cast<size_t>(width_) * height_) Die("weights: distmap size");
  if (gz_block_error_adjustment_weights(width_, height_, target_, direction, max_block_dist,
                                        target_mul, factor_x, factor_y, distmap.data(),
                                        block_weight->data()) != GZ_OK)
    Die("ComputeBlockErrorAdjustmentWeights");
}

}  // namespace guetzli
