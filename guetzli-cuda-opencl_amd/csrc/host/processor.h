// Host side of the search: the Processor loop (guetzli/processor.cc) and the
// Comparator surface it drives (guetzli/comparator.h:29-96), with the
// Butteraugli comparator implemented on the GPU engine.
#pragma once

#include <stdint.h>

#include <map>
#include <memory>
#include <string>
#include <vector>

#include "host/image420.h"
#include "host/jpeg_model.h"
#include "host/jpeg_writer.h"
#include "runtime/engine.h"

namespace gz {

// guetzli/quality.cc:78-87
double ButteraugliScoreForQuality(double quality);
// guetzli/score.cc:23-43
double ScoreJPEG(double butteraugli_distance, int size, double butteraugli_target);

struct CoeffData {  // guetzli::CoeffData, processor.h:29-32
  int idx;
  float block_err;
};

// The comparator interface the search loop talks to.  Mirrors
// guetzli::Comparator (comparator.h:29-96); the per-block pair
// SwitchBlock()/CompareBlock() becomes one batched call over all blocks
// (the shape of the reference GPU fast path, processor.cc:580-634), and
// distmap() is consumed only through its per-block maxima.
class Comparator {
 public:
  virtual ~Comparator() {}
  virtual bool Compare(const CoeffImage& img) = 0;
  virtual bool StartBlockComparisons() = 0;
  virtual void FinishBlockComparisons() = 0;
  // lookahead / new_model: Params::zeroing_greedy_lookahead / new_zeroing_model.
  virtual bool BlockZeroingOrders(const CoeffImage& img, const JpegData& orig_jpg, int comp_mask,
                                  int lookahead, bool new_model, std::vector<CoeffData>* out) = 0;
  // The back end's input: per block the BlockZeroingOrders entries with
  // 0 < block_err <= BlockErrorLimit(), in order, concatenated (offsets has
  // blocks + 1 entries) -- processor.cc:690-700.  Default: filter the orders.
  virtual bool BlockZeroingCandidates(const CoeffImage& img, const JpegData& orig_jpg,
                                      int comp_mask, int lookahead, bool new_model,
                                      std::vector<int>* offsets,
                                      std::vector<uint8_t>* idx, std::vector<float>* err);
  // CopyFromJpegData(q=1) + ApplyGlobalQuantization(q) of the originals into img
  // (and into any device mirror).
  // need_host false: only the comparator's own (device) copy must be
  // current; img->coeffs may be left stale (img->host_valid = false).
  virtual bool QuantizeFromOriginal(const int q[3][kDCTBlockSize], CoeffImage* img,
                                    bool need_host = true) = 0;
  // Entropy coding of img (SaveToJpegData over meta + WriteJpeg) by the
  // comparator's device; HasDeviceWriter() false: use the host writer.
  virtual bool HasDeviceWriter() const { return false; }
  virtual bool DeviceWriteJpeg(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                               std::string* out) {
    return false;
  }
  // The search's per-candidate form of it: the candidate stays on the device
  // and only its file size comes back; DeviceKeepEncoded marks the last
  // encoded candidate as the one to keep (the next encode may overwrite any
  // other), DeviceFetchKept returns the kept candidate's bytes.
  virtual bool DeviceEncode(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                            size_t* size) {
    return false;
  }
  // DeviceEncode of img followed by Compare(img), for comparators that can
  // overlap the two (the default runs them one after the other).
  virtual bool DeviceEncodeAndCompare(const CoeffImage& img, const JpegData& meta,
                                      bool strip_metadata, size_t* size) {
    return DeviceEncode(img, meta, strip_metadata, size) && Compare(img);
  }
  // Compare(img) and, when the comparator's device can code it, the size of
  // WriteJpeg(jpg_in) for a jpg_in holding img's coefficients unquantized
  // (its kept form via DeviceKeepEncoded); *used = false: write it on the host.
  virtual bool DeviceEncodeOriginalAndCompare(const CoeffImage& img, const JpegData& jpg_in,
                                              bool strip_metadata, size_t* size, bool* used) {
    *used = false;
    return Compare(img);
  }
  virtual void DeviceKeepEncoded() {}
  virtual bool DeviceFetchKept(std::string* out) { return false; }
  // DC / AC histograms of img as SaveToJpegData stores it (comps at or above
  // the returned count cleared) from the device copy; -1 if unsupported.
  virtual int DeviceHistograms(const CoeffImage& img, JpegHistogram dc[3], JpegHistogram ac[3]) {
    return -1;
  }
  virtual double ScoreOutputSize(int size) const = 0;
  virtual bool DistanceOK(double target_mul) const = 0;
  virtual float distmap_aggregate() const = 0;
  virtual const std::vector<float>& block_max_distance() const = 0;
  // True when the last block_max_distance() could not be formed (a failed
  // device copy): its values are then not the maxima and error() says why.
  virtual bool block_max_failed() const { return false; }
  virtual float BlockErrorLimit() const = 0;
  virtual void ComputeBlockErrorAdjustmentWeights(int direction, int max_block_dist,
                                                  double target_mul, int factor_x, int factor_y,
                                                  const std::vector<float>& max_dist_per_block,
                                                  std::vector<float>* block_weight) = 0;
  // The 4:4:4 back end's change order built where the candidates of the
  // last BlockZeroingCandidates and the last Compare's block maxima are (the
  // device): DeviceOrderReset before an iteration loop (max_block_error :=
  // 0), DeviceChangeOrder per iteration (the weights at radius 1..4 until
  // some block has entries; the entries in block order, as
  // Processor::BuildChangeOrder makes them, stay on the device: their count
  // and the blocks with entries come back, and with floor_limit > -inf the
  // count of keys below it), DeviceSelectBulk (the bulk prefix selected and
  // applied there, and the tail's window), DeviceOrderEntries (every entry,
  // for std::sort's exact order where the keys leave it open),
  // DeviceOrderAdvance after the iteration.
  // DeviceOrderReset: false on an engine error (error() says which);
  // *available = false: no device order, build on the host.
  virtual bool DeviceOrderReset(bool* available) {
    *available = false;
    return true;
  }
  virtual bool DeviceChangeOrder(int direction, double target_mul, bool zero_bmax,
                                 const std::vector<int>& last_indexes, float floor_limit, size_t* n_entries,
                                 int* blocks_to_change, int64_t* below_floor) {
    return false;
  }
  virtual bool DeviceOrderEntries(std::vector<std::pair<int, float>>* order) { return false; }
  // The first `bulk` entries of std::sort's order as a set, selected and
  // applied on the device (Engine::OrderSelect: nothing applied when sel->open),
  // ac updated as DeviceBulkApply does, and the tail's window of entries.
  virtual bool DeviceSelectBulk(const CoeffImage& img, size_t bulk, size_t window, int direction,
                                Engine::OrderSelection* sel, JpegHistogram ac[3]) {
    return false;
  }
  // The tail's next window: the entries after the first `from` of std::sort's
  // order (as a set), selected on the device as DeviceSelectBulk's window is.
  virtual bool DeviceSelectWindow(size_t from, size_t window, int direction, Engine::OrderSelection* sel) {
    return false;
  }
  virtual bool DeviceOrderAdvance(float val_threshold, int direction) { return false; }
  // A frame split over ranks (host/strips.h): the device change order over
  // this rank's owned blocks [own_lo, own_hi) of its strip, its selection
  // over the frame through the ranks' exchange (Engine::SetOrderScope).
  // DeviceChangeOrder's counts are then the frame's, DeviceSelectBulk's
  // histograms the frame's change, the windows and DeviceOrderEntries in
  // frame block indices (the entries: the owned blocks').
  virtual void SetDeviceOrderScope(int own_lo, int own_hi, int gbase, Engine::OrderExchange* x) {}
  // The block maxima the device change order reads: the frame's values for
  // the strip's blocks (its own Compare's differ in the halo).
  virtual bool DeviceSetBlockMax(const std::vector<float>& bmax) { return false; }
  // DeviceEncodeAndCompare of a candidate whose symbol histograms the caller
  // already has (the search back end tracks them exactly): the DC / AC
  // histograms SaveToJpegData + WriteJpeg would count (comps at or above
  // ncomp cleared), so the device only codes the scan -- no histogram pass,
  // no wait for one.  HasKnownHistogramEncode() false: not supported.
  // best_score >= 0: the score the candidate must beat to become the output
  // (MaybeOutput); when its distance and a lower bound of its size show it
  // cannot, the scan is not coded and *skipped is set (*size undefined).
  virtual bool HasKnownHistogramEncode() const { return false; }
  virtual bool DeviceEncodeAndCompareKnown(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                                           const JpegHistogram dc[3], const JpegHistogram ac[3], int ncomp,
                                           double best_score, size_t* size, bool* skipped) {
    return false;
  }
  // The back end's bulk prefix on the device (with the device order only):
  // cnt[b] (< 256) changes of block b from the last_indexes of the last
  // DeviceChangeOrder, in `direction`, applied to the device copy of img
  // alone (the caller brings its host copy along lazily, host_partial); ac
  // holds every component's AC histograms before the changes on entry and
  // after them on return (the same counts as the host's per-change updates).
  // HasDeviceBulk() false: apply it on the host.
  virtual bool HasDeviceBulk() const { return false; }
  virtual bool DeviceBulkApply(const CoeffImage& img, int direction, const uint8_t* cnt, JpegHistogram ac[3]) {
    return false;
  }
  // The same without the device order (a frame split over ranks): from the
  // host's last_indexes; delta[c][symbol] (unscaled) the change of the AC
  // symbol counts of the changed blocks, for the caller to sum over ranks.
  virtual bool HasDeviceBulkLocal() const { return false; }
  virtual bool DeviceBulkApplyLocal(const CoeffImage& img, int direction, const uint8_t* cnt,
                                    const std::vector<int>& last_indexes, int32_t delta[3][256]) {
    return false;
  }
  // Makes the q=1 coefficients of the original image available to
  // QuantizeFromOriginal / BlockZeroingOrders.
  virtual bool SetOriginalCoeffs(const JpegData& jpg) = 0;
  virtual const std::string& error() const = 0;

  // ---- the 4:2:0 pass (processor.cc:989-1016 with downsample = 1) ----
  // The downsampled image's own q=1 coefficients as the originals
  // (SaveToJpegData's 4:2:0 layout).
  virtual bool SetOriginalCoeffs420(const JpegData& jpg420) { return false; }
  // Compare of the 4:2:0 image: Y from its coefficients, Cb / Cr from the
  // factor-2 pixel planes as they are.
  virtual bool Compare420(const Image420& img) { return false; }
  // The zeroing search of comp_mask 1 (Y) or 6 (Cb + Cr at factor 2) on img;
  // for 6 the search's SetCoeffBlock calls leave img's chroma pixel state
  // where the reference's leave it (the kept entries as BlockZeroingCandidates).
  virtual bool BlockZeroingCandidates420(Image420* img, int comp_mask, int lookahead,
                                         bool new_model, std::vector<int>* offsets,
                                         std::vector<uint8_t>* idx, std::vector<float>* err) {
    return false;
  }
};

// ComputeBlockErrorAdjustmentWeights of butteraugli_comparator.cc:169-233
// given the per-block maxima of the distance map.
void BlockErrorAdjustmentWeights(int w, int h, float target, int direction, int max_block_dist,
                                 double target_mul, int factor_x, int factor_y,
                                 const std::vector<float>& max_dist_per_block,
                                 std::vector<float>* block_weight);

// SaveToJpegData + WriteJpeg of the engine's current coefficients (quant q,
// image w x h, metadata of meta) entropy coded on the device.
bool DeviceWriteJpeg(Engine* e, int w, int h, const int q[3][kDCTBlockSize], const JpegData& meta,
                     bool strip_metadata, std::string* out, std::string* err);
// The same leaving the scan in the engine's current JPEG slot: *prologue
// (headers), *size the file size; DeviceFetchJpeg assembles a slot's file.
bool DeviceEncodeJpeg(Engine* e, int w, int h, const int q[3][kDCTBlockSize], const JpegData& meta,
                      bool strip_metadata, std::string* prologue, size_t* size, std::string* err);
bool DeviceFetchJpeg(Engine* e, bool kept, const std::string& prologue, size_t size,
                     std::string* out, std::string* err);
// The histogram stage of it alone (for the search back end's size model).
int DeviceJpegHistograms(Engine* e, const int q[3][kDCTBlockSize], JpegHistogram dc[3],
                         JpegHistogram ac[3], std::string* err);
// Staged histograms (6 x 256 plain counts, the non-zero chroma count) ->
// per-component DC / AC histograms as SaveToJpegData stores them; returns
// the component count (1 when the chroma is all zero).
int HistogramsFromStage(const uint32_t* hist, uint64_t chroma, JpegHistogram dc[3],
                        JpegHistogram ac[3]);
// Headers (*prologue) and Huffman code tables of an image with these
// histograms (WriteJpeg's table choice, jpeg_data_writer.cc): for the
// header hdr, or for SaveToJpegData's header of a w x h image with quant q
// and meta's APPn / COM data.
bool PrepareScanFor(const JpegData& hdr, bool strip_metadata, int ncomp, JpegHistogram* dc_h,
                    JpegHistogram* ac_h, std::string* prologue, JpegCodeTables* codes);
bool PrepareScan(int w, int h, const int q[3][kDCTBlockSize], const JpegData& meta,
                 bool strip_metadata, int ncomp, JpegHistogram* dc_h, JpegHistogram* ac_h,
                 std::string* prologue, JpegCodeTables* codes);
// The scan's bit count from the histograms it is coded with (code lengths
// plus extra bits; no stuffing, no padding): prologue + ceil(bits / 8) + EOI
// bounds the file's size from below.
uint64_t ScanBits(const JpegHistogram dc[3], const JpegHistogram ac[3], int ncomp, const JpegCodeTables& codes);

// guetzli::ButteraugliComparator on the HIP engine.
class HipButteraugliComparator : public Comparator {
 public:
  static std::unique_ptr<HipButteraugliComparator> Create(int device, int w, int h,
                                                          const uint8_t* rgb, bool device_ptr,
                                                          float target, std::string* err);
  ~HipButteraugliComparator() override { ReleaseEngine(std::move(engine_)); }
  bool Compare(const CoeffImage& img) override;
  bool StartBlockComparisons() override;
  void FinishBlockComparisons() override {}
  bool BlockZeroingOrders(const CoeffImage& img, const JpegData& orig_jpg, int comp_mask,
                          int lookahead, bool new_model, std::vector<CoeffData>* out) override;
  bool BlockZeroingCandidates(const CoeffImage& img, const JpegData& orig_jpg, int comp_mask,
                              int lookahead, bool new_model, std::vector<int>* offsets,
                              std::vector<uint8_t>* idx,
                              std::vector<float>* err) override;
  bool QuantizeFromOriginal(const int q[3][kDCTBlockSize], CoeffImage* img,
                            bool need_host = true) override;
  bool HasDeviceWriter() const override { return true; }
  bool DeviceWriteJpeg(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                       std::string* out) override;
  bool DeviceEncode(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                    size_t* size) override;
  bool DeviceEncodeAndCompare(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                              size_t* size) override;
  bool DeviceEncodeOriginalAndCompare(const CoeffImage& img, const JpegData& jpg_in,
                                      bool strip_metadata, size_t* size, bool* used) override;
  void DeviceKeepEncoded() override;
  bool DeviceFetchKept(std::string* out) override;
  double seconds_encode = 0.0;  // host part of the overlapped encodes
  int DeviceHistograms(const CoeffImage& img, JpegHistogram dc[3], JpegHistogram ac[3]) override;
  double ScoreOutputSize(int size) const override;
  bool DistanceOK(double target_mul) const override { return distance_ <= target_mul * target_; }
  float distmap_aggregate() const override { return distance_; }
  // (copied from the device on first use after a Compare: the device change
  // order reads them in HBM, so the search itself never asks)
  const std::vector<float>& block_max_distance() const override;
  bool block_max_failed() const override { return block_max_failed_; }
  float BlockErrorLimit() const override { return target_; }
  void ComputeBlockErrorAdjustmentWeights(int direction, int max_block_dist, double target_mul,
                                          int factor_x, int factor_y,
                                          const std::vector<float>& max_dist_per_block,
                                          std::vector<float>* block_weight) override;
  const std::string& error() const override { return err_; }
  bool DeviceOrderReset(bool* available) override;
  bool DeviceChangeOrder(int direction, double target_mul, bool zero_bmax, const std::vector<int>& last_indexes,
                         float floor_limit, size_t* n_entries, int* blocks_to_change, int64_t* below_floor) override;
  bool DeviceOrderEntries(std::vector<std::pair<int, float>>* order) override;
  bool DeviceSelectBulk(const CoeffImage& img, size_t bulk, size_t window, int direction,
                        Engine::OrderSelection* sel, JpegHistogram ac[3]) override;
  bool DeviceSelectWindow(size_t from, size_t window, int direction, Engine::OrderSelection* sel) override;
  bool DeviceOrderAdvance(float val_threshold, int direction) override;
  void SetDeviceOrderScope(int own_lo, int own_hi, int gbase, Engine::OrderExchange* x) override;
  bool DeviceSetBlockMax(const std::vector<float>& bmax) override;
  bool HasDeviceBulk() const override { return true; }
  bool HasKnownHistogramEncode() const override { return true; }
  bool DeviceEncodeAndCompareKnown(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                                   const JpegHistogram dc[3], const JpegHistogram ac[3], int ncomp,
                                   double best_score, size_t* size, bool* skipped) override;
  bool DeviceBulkApply(const CoeffImage& img, int direction, const uint8_t* cnt, JpegHistogram ac[3]) override;
  bool HasDeviceBulkLocal() const override { return true; }
  bool DeviceBulkApplyLocal(const CoeffImage& img, int direction, const uint8_t* cnt,
                            const std::vector<int>& last_indexes, int32_t delta[3][256]) override;
  bool SetOriginalCoeffs(const JpegData& jpg) override;
  bool SetOriginalCoeffs420(const JpegData& jpg420) override;
  bool Compare420(const Image420& img) override;
  bool BlockZeroingCandidates420(Image420* img, int comp_mask, int lookahead, bool new_model,
                                 std::vector<int>* offsets, std::vector<uint8_t>* idx,
                                 std::vector<float>* err) override;
  // EncodeRGBToJpegData of the reference image, with the coefficients
  // computed on the device (and left resident as the originals).
  bool OriginalJpegData(JpegData* jpg);
  Engine* engine() { return engine_.get(); }
  // Brings the device copy of the coefficients up to date with img.
  bool Sync(const CoeffImage& img) { return SyncCoeffs(img); }
  double seconds_compare = 0.0;
  double cpu_compare = 0.0;  // calling thread's CPU seconds in the compares
  double seconds_wait = 0.0, cpu_wait = 0.0;  // of which waiting for the device (wall, CPU)
  double seconds_zeroing = 0.0;
  double seconds_bulk = 0.0;  // DeviceBulkApply (wall)
  int compares = 0;
  int scans_skipped = 0;  // back-end candidates not coded (DeviceEncodeAndCompareKnown)
  // coded back-end scans whose bit count differed from the histogram bound
  // (never expected; the first one turns the skipping off)
  int scan_bound_mismatches = 0;

 private:
  bool SyncCoeffs(const CoeffImage& img);
  // DeviceEncodeAndCompare with the headers of *hdr (nullptr: SaveToJpegData's)
  bool EncodeAndCompareWith(const CoeffImage& img, const JpegData& meta, const JpegData* hdr,
                            bool strip_metadata, size_t* size);

  std::unique_ptr<Engine> engine_;
  // q=1 coefficients of the original (host copy; 12 MB at 1080p, allocated
  // without the zero fill a std::vector would write first)
  struct CoeffBuffer {
    std::unique_ptr<coeff_t[]> p;
    size_t n = 0;
    void reset(size_t count) {
      if (count != n) p.reset(new coeff_t[count]);
      n = count;
    }
    size_t size() const { return n; }
    coeff_t* data() { return p.get(); }
    const coeff_t* data() const { return p.get(); }
  } orig_;
  bool orig_on_device_ = false;
  std::vector<coeff_t> delta_val_;
  int w_ = 0, h_ = 0;
  float target_ = 0.0f;
  float distance_ = 0.0f;
  mutable std::vector<float> block_max_;
  mutable bool block_max_failed_ = false;
  Engine::OrderExchange* order_x_ = nullptr;  // a frame split over ranks (SetDeviceOrderScope)
  int order_gbase_ = 0;
  mutable bool block_max_stale_ = false;  // the last Compare's maxima are on the device only
  CoeffCursor device_;  // what the device copy of the coefficients reflects
  bool IsOriginal(const CoeffImage& img) const;
  std::string cur_prologue_, kept_prologue_;  // headers of the encoded / kept candidates
  size_t cur_size_ = 0, kept_size_ = 0;
  mutable std::string err_;
};

struct ProcessParams {  // guetzli::Params, processor.h:34-42
  float butteraugli_target = 1.0f;
  bool clear_metadata = true;
  bool try_420 = false;
  bool force_420 = false;
  bool use_silver_screen = false;
  int zeroing_greedy_lookahead = 3;
  bool new_zeroing_model = true;
};

struct ProcessResult {
  std::string jpeg;
  int iterations = 0, iterations_up = 0, iterations_down = 0, compares = 0;
  double seconds_compare = 0.0, seconds_zeroing = 0.0, seconds_total = 0.0;
  // host-side breakdown
  double seconds_setup = 0.0;      // RGB -> q=1 coefficients, engine creation, reference upload
  double seconds_write = 0.0;      // SaveToJpegData + WriteJpeg per iteration
  double seconds_quantize = 0.0;   // global quantization (device copy + host copy)
  double seconds_backend = 0.0;    // SelectFrequencyBackEnd selection / size estimation
  // finer breakdown / counters (reported as JSON by gz_last_process_detail)
  std::map<std::string, double> detail;
};

// guetzli::Process(params, stats, rgb, w, h, &out) (processor.cc:1157-1185).
// Returns 0 or a gz_status error code.
int Process(int device, const ProcessParams& params, const uint8_t* rgb, bool device_ptr, int w,
            int h, ProcessResult* result, std::string* err);

// guetzli::Process(params, stats, jpeg_bytes, out) (processor.cc:1029-1066):
// ReadJpeg, CheckJpegSanity, DecodeJpegToRGB as the comparator's reference,
// ProcessJpegData on the input's own coefficients.  4:4:4 and 4:2:0 YCbCr
// inputs (a 4:2:0 input forces the downsampled search).
int ProcessJpeg(int device, const ProcessParams& params, const uint8_t* data, size_t len,
                ProcessResult* result, std::string* err);

// The q=1 4:4:4 JPEG model of an RGB image (EncodeRGBToJpeg).
void EncodeRGBToJpegData(const uint8_t* rgb, int w, int h, JpegData* jpg);

struct Partition;  // host/strips.h

// guetzli::ProcessJpegData (processor.cc:931-1020) with any comparator
// (nullptr: image too small for Butteraugli).  With a partition, jpg and
// the comparator are this rank's strip of a frame split over ranks
// (host/strips.h).  Returns 0 or a gz_status.
int ProcessJpegData(const ProcessParams& params, const JpegData& jpg, Comparator* cmp,
                    ProcessResult* result, std::string* err, Partition* part = nullptr);

}  // namespace gz
