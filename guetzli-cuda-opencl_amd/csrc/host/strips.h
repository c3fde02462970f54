// One large frame over several GPUs (BASELINE configs[4]: 8192x8192 q=84 on
// 4 MI355X): row strips with a halo, each rank owning the
// search state of its strip.
//
// Rank r owns block rows [ob0, ob1) and its GPU computes rows [e0, e1) =
// owned rows plus a kStripHalo-row halo on each side.  The halo makes the
// owned rows exact: a strip whose first row is a multiple of 24 (the res
// grid's 3, the block size 8 and the blur decimations 2/3/4 all divide it)
// and that extends kStripHalo rows past its owned rows computes, for the
// owned rows, the distance map, block maxima, mask and per-block zeroing
// orders of the full image bit for bit (the Butteraugli receptive field is
// about -60/+66 rows).  Checked on the CPU oracle in
// tests/test_strips.py.
//
// Every rank runs the search loop (guetzli::ProcessJpegData, processor.cc:
// 931-1020) with the same control decisions, but holds and edits only its
// strip: the back end (processor.cc:723-919) builds the change entries of
// its owned blocks, applies the changes of its owned blocks and codes its
// owned MCUs; what the decisions need from the whole frame comes from the
// exchanges below (the Partition's collectives):
//   * per Compare: the owned blocks' maxima (the distance is their maximum,
//     and the block weights of the back end read the neighbours' ones);
//   * per coded candidate: the owned MCUs' symbol histograms (the Huffman
//     codes are those of their sum; every rank derives every rank's bit
//     count from them, so each codes its MCUs at its own bit offset), then
//     the 0xff counts and the words two ranks' parts share;
//   * per back-end iteration: the change entries (std::sort's order over the
//     whole frame is computed on every rank: its ties decide), the bulk
//     prefix's histogram deltas, and per window of the serial tail the
//     symbol deltas of the owners' changes;
//   * before any device work: the owned coefficients changed within
//     kStripHalo rows of a strip edge, into the neighbours' halos.
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

// This rank's share of a frame split by block rows, and the exchanges the
// search loop makes (ProcessJpegData with a partition; see the top).
struct Partition {
  Collectives* coll = nullptr;
  int world = 1, rank = 0;
  int width = 0, height = 0;  // the frame
  int bw = 0, bh = 0;         // its 8x8 blocks
  int lb0 = 0, lb1 = 0;       // block rows of this rank's image (owned + halo)
  int ob0 = 0, ob1 = 0;       // owned block rows
  std::vector<int> row0;      // rank r owns block rows [row0[r], row0[r + 1])

  static Partition Make(const StripLayout& layout, Collectives* coll);
  int LocalBase() const { return lb0 * bw; }  // frame index of local block 0
  int OwnLo() const { return (ob0 - lb0) * bw; }
  int OwnHi() const { return (ob1 - lb0) * bw; }
  bool OwnsRow(int row) const { return row >= ob0 && row < ob1; }
  // In-place sums of n values over the ranks (an all-gather, summed in rank
  // order: integer sums, exact).
  bool SumAll(int64_t* v, int n);
};

// guetzli::Comparator for a rank's strip image (block rows [lb0, lb1) of the
// frame), backed by a comparator of the same strip (`inner`: the HIP one, or
// any other -- without a device writer the strip is entropy coded on the
// host).  Every call that reads the image first brings its halo rows up to
// date with the neighbours' owned changes (a collective); the search loop
// itself only edits owned blocks.
// The strips' device change order (StripDeviceOrder): every rank's engine
// builds its owned blocks' entries, the selection exchanges its counts and
// candidates (Engine::OrderExchange, implemented over the partition).
// GZ_STRIP_HOST_ORDER=1: the host order (StripOrder), for A/B runs.
bool StripDeviceOrder();

class PartitionComparator : public Comparator, private Engine::OrderExchange {
 public:
  PartitionComparator(Partition* part, std::unique_ptr<Comparator> inner, float target);
  ~PartitionComparator() override;
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
  bool HasDeviceWriter() const override { return true; }
  // The back end's candidates, coded from its tracked (frame) histograms:
  // not coded at all when the bound on their size shows they cannot win.
  bool HasKnownHistogramEncode() const override { return true; }
  bool DeviceEncodeAndCompareKnown(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                                   const JpegHistogram dc[3], const JpegHistogram ac[3], int ncomp,
                                   double best_score, size_t* size, bool* skipped) override;
  int scan_bound_mismatches = 0;
  int scans_skipped = 0;
  bool DeviceEncodeAndCompare(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                              size_t* size) override;
  bool DeviceEncodeOriginalAndCompare(const CoeffImage& img, const JpegData& jpg_in,
                                      bool strip_metadata, size_t* size, bool* used) override;
  void DeviceKeepEncoded() override;
  bool DeviceFetchKept(std::string* out) override;
  int DeviceHistograms(const CoeffImage& img, JpegHistogram dc[3], JpegHistogram ac[3]) override;
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
  // One rank (the degenerate split: no halo, the strip is the frame): the
  // whole device change order and bulk prefix are the inner comparator's.
  // Several: the inner engine's order scoped to the owned blocks, its
  // selection over the frame through this comparator's exchange
  // (StripDeviceOrder; else the host order).
  bool HasDeviceBulk() const override {
    return (part_->world == 1 || StripDeviceOrder()) && inner_->HasDeviceBulk();
  }
  bool DeviceOrderReset(bool* available) override;
  bool DeviceChangeOrder(int direction, double target_mul, bool zero_bmax, const std::vector<int>& last_indexes,
                         float floor_limit, size_t* n_entries, int* blocks_to_change, int64_t* below_floor) override {
    // (the frame's maxima of the strip's blocks: its own Compare's differ
    // in the halo, which the owned blocks' weights read up to 4 blocks deep)
    if (part_->world != 1 && !zero_bmax && !inner_->DeviceSetBlockMax(block_max_)) return Fail(inner_->error());
    return inner_->DeviceChangeOrder(direction, target_mul, zero_bmax, last_indexes, floor_limit, n_entries,
                                     blocks_to_change, below_floor) ||
           Fail(inner_->error());
  }
  bool DeviceOrderEntries(std::vector<std::pair<int, float>>* order) override {
    return inner_->DeviceOrderEntries(order) || Fail(inner_->error());
  }
  bool DeviceSelectBulk(const CoeffImage& img, size_t bulk, size_t window, int direction,
                        Engine::OrderSelection* sel, JpegHistogram ac[3]) override {
    return inner_->DeviceSelectBulk(img, bulk, window, direction, sel, ac) || Fail(inner_->error());
  }
  bool DeviceSelectWindow(size_t from, size_t window, int direction, Engine::OrderSelection* sel) override {
    return inner_->DeviceSelectWindow(from, window, direction, sel) || Fail(inner_->error());
  }
  bool DeviceBulkApply(const CoeffImage& img, int direction, const uint8_t* cnt, JpegHistogram ac[3]) override {
    return inner_->DeviceBulkApply(img, direction, cnt, ac) || Fail(inner_->error());
  }
  bool DeviceOrderAdvance(float val_threshold, int direction) override {
    return inner_->DeviceOrderAdvance(val_threshold, direction) || Fail(inner_->error());
  }
  // (the owned blocks' bulk prefix on this rank's device: the inner comparator's)
  bool HasDeviceBulkLocal() const override { return inner_->HasDeviceBulkLocal(); }
  bool DeviceBulkApplyLocal(const CoeffImage& img, int direction, const uint8_t* cnt,
                            const std::vector<int>& last_indexes, int32_t delta[3][256]) override {
    const bool ok = inner_->DeviceBulkApplyLocal(img, direction, cnt, last_indexes, delta);
    if (!ok) err_ = inner_->error();
    return ok;
  }
  const std::string& error() const override { return err_; }
  Comparator* inner() { return inner_.get(); }
  double seconds_exchange = 0.0;
  double seconds_halo = 0.0;

  // The part of the scan this rank codes (frame-wide bit offset, bits, the
  // words shared with its neighbours) -- Engine::ScanPart's fields.
  struct Part {
    uint64_t base = 0, bits = 0, ff = 0;
    uint32_t first_word = 0, last_word = 0;
    bool first_shared = false, last_open = false;
  };
  class Coder;  // the strip's entropy coder (device or host)

 private:
  bool Fail(const std::string& what);
  // An exchange with a status word: fails on every rank if any rank failed.
  bool Exchange(bool ok, const std::string& local_err, const std::vector<uint8_t>& send,
                std::vector<std::vector<uint8_t>>* all);
  bool Agree(bool ok, const std::string& local_err);
  // a Compare's block maxima exchange (the distance, the edge rows)
  void PackBlockMax(const std::vector<float>& bmax, std::vector<uint8_t>* send) const;
  bool UnpackBlockMax(const std::vector<float>& own, const std::vector<std::vector<uint8_t>>& all, size_t skip);
  // Engine::OrderExchange over the partition (with the status word)
  bool SumU32(bool ok, uint32_t* v, int n) override;
  bool Gather(bool ok, const std::vector<unsigned long long>& mine, std::vector<unsigned long long>* all) override;
  bool SyncHalo(const CoeffImage& img);
  // Codes img (headers: SaveToJpegData's, or *hdr's), overlapped with the
  // Compare of img; *size the whole file's size.
  bool CodeAndCompare(const CoeffImage& img, const JpegData& meta, const JpegData* hdr,
                      bool strip_metadata, size_t* size, bool compare = true);

  Partition* part_;
  std::unique_ptr<Comparator> inner_;
  std::unique_ptr<Coder> coder_;
  float target_;
  int local_blocks_ = 0;
  CoeffCursor halo_;            // the image journal position already exchanged
  std::vector<float> block_max_;  // local blocks
  float distance_ = 0.0f;
  std::string cur_prologue_, kept_prologue_;
  size_t cur_size_ = 0, kept_size_ = 0;
  std::string err_;
};

// guetzli::Process for one frame whose work is split over the ranks of
// `coll` (one GPU each, `device` on this rank): every rank passes the whole
// RGB frame and gets the same JPEG bytes.  Every rank must own rows (height
// >= 24 * world).  Returns 0 or a gz_status.
int ProcessStrips(int device, const ProcessParams& params, const uint8_t* rgb, int w, int h,
                  Collectives* coll, ProcessResult* result, std::string* err);

}  // namespace gz
