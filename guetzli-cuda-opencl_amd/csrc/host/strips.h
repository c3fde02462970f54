// One large frame over several GPUs (BASELINE configs[4]: 8192x8192 q=84 on
// 4 MI355X): row strips with a halo.
//
// Every rank runs the same host search loop (guetzli::ProcessJpegData,
// processor.cc:931-1020) on the whole coefficient image -- its decisions are
// deterministic, so the replicas agree without being told -- while its GPU
// evaluates Butteraugli only on the rank's strip of rows plus a halo.  The
// halo makes the owned rows exact: a strip whose first row is a multiple of
// 24 (the res grid's 3, the block size 8 and the blur decimations 2/3/4 all
// divide it) and that extends kStripHalo rows past its owned rows on each
// side computes, for the owned rows, the distance map, block maxima, mask and
// per-block zeroing orders of the full image bit for bit (the Butteraugli
// receptive field is about -60/+66 rows; the strip's own
// borders fall inside the halo).  Checked on the CPU oracle in
// tests/test_strips.py.
//
// The exchanges are the collectives of the path: per Compare an all-gather
// of the owned block maxima (the distance is their maximum), per
// SelectFrequencyMasking an all-gather of the owned blocks' zeroing
// candidates.  Coefficient edits need no exchange: every rank holds the
// whole image and applies the same edits.
#pragma once

#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "host/processor.h"

namespace gz {

constexpr int kStripAlign = 24;  // owned rows start at multiples of this
constexpr int kStripHalo = 96;   // extra rows computed above and below

struct StripLayout {
  int width = 0, height = 0, world = 1;
  std::vector<int> y0, y1;  // owned rows [y0, y1) per rank (possibly empty)
  std::vector<int> e0, e1;  // computed rows [e0, e1) per rank
  static StripLayout Make(int width, int height, int world);
};

// Equal-size all-gather across the ranks of a job: every rank contributes
// `bytes` bytes, `recv` receives world * bytes in rank order.
class Collectives {
 public:
  virtual ~Collectives() {}
  virtual int rank() const = 0;
  virtual int world() const = 0;
  virtual bool AllGather(const void* send, size_t bytes, void* recv) = 0;
  // Variable-size form built on it: out[r] = rank r's bytes.
  bool AllGatherV(const std::vector<uint8_t>& send, std::vector<std::vector<uint8_t>>* out);
};

// guetzli::Comparator for the whole image, backed by a comparator (`inner`)
// of this rank's computed strip.  `inner` may be null for a rank without
// rows (it still takes part in every exchange).
class StripComparator : public Comparator {
 public:
  StripComparator(const StripLayout& layout, std::unique_ptr<Comparator> inner, Collectives* coll,
                  float target);
  bool Compare(const CoeffImage& img) override;
  bool StartBlockComparisons() override;
  void FinishBlockComparisons() override;
  bool BlockZeroingOrders(const CoeffImage& img, const JpegData& orig_jpg, int comp_mask,
                          int lookahead, bool new_model, std::vector<CoeffData>* out) override;
  bool BlockZeroingCandidates(const CoeffImage& img, const JpegData& orig_jpg, int comp_mask,
                              int lookahead, bool new_model, std::vector<int>* offsets,
                              std::vector<uint8_t>* idx,
                              std::vector<float>* err) override;
  bool QuantizeFromOriginal(const int q[3][kDCTBlockSize], CoeffImage* img,
                            bool need_host = true) override;
  double ScoreOutputSize(int size) const override { return ScoreJPEG(distance_, size, target_); }
  bool DistanceOK(double target_mul) const override { return distance_ <= target_mul * target_; }
  float distmap_aggregate() const override { return distance_; }
  const std::vector<float>& block_max_distance() const override { return block_max_; }
  float BlockErrorLimit() const override { return target_; }
  void ComputeBlockErrorAdjustmentWeights(int direction, int max_block_dist, double target_mul,
                                          int factor_x, int factor_y,
                                          const std::vector<float>& max_dist_per_block,
                                          std::vector<float>* block_weight) override;
  bool SetOriginalCoeffs(const JpegData& jpg) override;
  const std::string& error() const override { return err_; }
  Comparator* inner() { return inner_.get(); }
  double seconds_exchange = 0.0;

 private:
  // Fails on every rank if any rank's status word is non-zero.
  bool CheckStatus(const std::vector<uint32_t>& status, const std::string& local);
  bool Fail(const std::string& what);
  bool Sync(const CoeffImage& img);  // the strip's coefficients <- the whole image's
  int rank_blocks() const { return (ob1_ - ob0_) * bw_; }

  StripLayout layout_;
  std::unique_ptr<Comparator> inner_;
  Collectives* coll_;
  float target_;
  int rank_ = 0, bw_ = 0, blocks_ = 0;
  int lb0_ = 0, lb1_ = 0;  // computed block rows
  int ob0_ = 0, ob1_ = 0;  // owned block rows
  int max_owned_ = 0;      // owned blocks of the largest strip
  CoeffImage local_;       // the computed strip's coefficients
  JpegData local_orig_;    // and its q=1 originals
  CoeffCursor synced_;     // what local_ reflects of the whole image
  std::vector<coeff_t> orig_;  // q=1 originals of the whole image
  std::vector<float> block_max_;
  float distance_ = 0.0f;
  std::string err_;
};

// guetzli::Process for one frame whose Butteraugli work is split over the
// ranks of `coll` (one GPU each, `device` on this rank): every rank passes the
// whole RGB frame and gets the same JPEG bytes.  Returns 0 or a gz_status.
int ProcessStrips(int device, const ProcessParams& params, const uint8_t* rgb, int w, int h,
                  Collectives* coll, ProcessResult* result, std::string* err);

}  // namespace gz
