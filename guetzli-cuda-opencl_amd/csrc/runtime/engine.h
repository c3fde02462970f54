// Device engine: one Butteraugli comparison context for one image size on
// one GPU (one HIP stream, persistent HBM buffers sized at creation).
//
// Replaces the reference's per-call pooled allocations + synchronous
// launches (clguetzli/cuguetzli.cpp, cumem_pool.cpp, ocu.cpp): every buffer
// is allocated once in Create(), the reference image's XYB is cached, and a
// Compare is one stream-ordered sequence of kernels followed by a single
// small device->host copy (distance + per-block maxima).
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

namespace gz {

struct CoeffDataHost {  // guetzli::CoeffData (processor.h:29-32)
  int idx;
  float block_err;
};

// Per component Huffman code (length, code) of every symbol, as the device
// entropy coder consumes them.
struct JpegCodeTables {
  uint8_t dc_len[3][256];
  uint8_t ac_len[3][256];
  uint16_t dc_code[3][256];
  uint16_t ac_code[3][256];
};

// Optional host destinations for stage-level parity tests.
struct CompareDebug {
  float* cand_linear = nullptr;   // 3*w*h
  float* cand_xyb = nullptr;      // 3*w*h
  float* mhic0 = nullptr;         // 3*w*h
  float* mhic1 = nullptr;         // 3*w*h
  float* edge = nullptr;          // 3*rw*rh
  float* block_dc = nullptr;      // 3*rw*rh
  float* block_ac = nullptr;      // 3*rw*rh (before the low-frequency term)
  float* block_ac_lf = nullptr;   // 3*rw*rh
  float* mask = nullptr;          // 3*w*h
  float* mask_dc = nullptr;       // 3*w*h
  float* combined = nullptr;      // rw*rh
  float* distmap = nullptr;       // w*h
  // Dump from the search's own kernel variants (the corner edge term fused
  // into k_block_diff2, the low-frequency term into k_combine_channels, the
  // subsampled B mask, the mask LUTs in the vertical blur's epilogue) instead
  // of switching to the stand-alone dump kernels.  Only the planes those
  // variants leave in HBM can be dumped: mhic0, mhic1, edge, block_dc,
  // block_ac (before the low-frequency term) and distmap.
  bool production = false;
};

class Engine {
 public:
  // Returns nullptr and sets *err on failure.
  static std::unique_ptr<Engine> Create(int device, int w, int h, std::string* err);
  ~Engine();

  int device() const { return device_; }
  int width() const { return w_; }
  int height() const { return h_; }
  // HBM + pinned host bytes held (the pool's accounting unit).
  size_t bytes() const { return bytes_; }
  // An operation on this engine failed: it is not returned to the pool.
  bool failed() const { return failed_; }
  int blocks() const { return nb_; }
  int block_w() const { return bw_; }
  int block_h() const { return bh_; }

  // Reference image (RGB8 interleaved); computes and caches its XYB.
  bool SetReference(const uint8_t* rgb, bool device_ptr);
  // q=1 coefficients of the reference ([3][blocks][64]); kept resident.
  bool SetOriginalCoeffs(const int16_t* coeffs, bool device_ptr);
  // EncodeRGBToJpeg's q=1 coefficients of the reference image (set by
  // SetReference) computed on the device into the originals, and copied to
  // host_out ([3][blocks][64]).
  bool ComputeOriginalCoeffs(int16_t* host_out);
  // Candidate coefficients ([3][blocks][64]).
  bool UploadCoeffs(const int16_t* coeffs);
  // The current coefficients <- the q=1 originals (an HBM copy, stream-ordered).
  bool CurrentFromOriginal();
  // Applies coeffs[idx[i]] = val[i] to the device copy (stream-ordered before
  // the next pass): the search loop's per-iteration edits, a few 10k values.
  bool UploadCoeffDelta(const uint32_t* idx, const int16_t* val, size_t n);
  // cur = Quantize(orig, q) on device, copied back to host_out if non-null.
  bool QuantizeFromOriginal(const int q[3][64], int16_t* host_out);

  // Butteraugli distance of the current candidate.  block_max (blocks
  // floats, may be null) receives the per-8x8 maximum of the distance map.
  bool Compare(float* distance, float* block_max, CompareDebug* dbg);

  // Mask(ref, ref) sampled at block corners (StartBlockComparisons).
  bool StartBlockComparisons(float* mask_scale_host /* 3*blocks, may be null */);
  // Per-block greedy zeroing orders for the current candidate.
  // new_model: Params::new_zeroing_model (false: the old candidate key,
  // processor.cc:400-405).
  bool BlockZeroingOrders(int comp_mask, float limit, int lookahead, bool new_model,
                          CoeffDataHost* out);
  // The same search, reduced on the device to what the back end consumes:
  // per block the entries with 0 < block_err <= limit, in order, concatenated
  // (offsets: blocks + 1 entries).  Moves ~5 B per kept entry instead of the
  // 1.5 KB-per-block order table.
  bool BlockZeroingCandidates(int comp_mask, float limit, int lookahead, bool new_model,
                              std::vector<int>* offsets,
                              std::vector<uint8_t>* idx, std::vector<float>* err);
  // SwitchBlock + CompareBlock for n (block, candidate [3][64]) requests;
  // err[i] receives CompareBlock's double (the comparator-level adapter's
  // per-block entry; the search itself uses the batched calls above).
  bool CompareBlocks(int n, const int* blocks, const int16_t* cand, double* err);

  // ---- the 4:2:0 pass (Params::try_420 / force_420, 4:2:0 input) ----
  // Coefficients: Y at component 0 with luma block indices (blocks()), Cb /
  // Cr at components 1 / 2 with chroma block indices (ceil(w/16) x
  // ceil(h/16) blocks); the chroma pixels are the factor-2 planes' state
  // (16-bit, [w*h] each), uploaded by the host.  Set420 switches the engine
  // to it (Compare then reads the chroma pixels from the planes) until the
  // next 4:4:4 upload / quantization.
  bool SetOriginal420(const int16_t* y, const int16_t* cb, const int16_t* cr);
  bool Set420(const int16_t* y, const int16_t* cb, const int16_t* cr, const uint16_t* plane_cb,
              const uint16_t* plane_cr);
  // The zeroing search of the 4:2:0 pass: comp_mask 1 (Y, with the chroma
  // planes as they are) or 6 (Cb + Cr at factor 2, in wavefronts; the
  // planes' state after the search comes back in plane_cb / plane_cr).
  // Output as BlockZeroingCandidates, over the searched component's blocks.
  bool BlockZeroingCandidates420(int comp_mask, float limit, int lookahead, bool new_model,
                                 std::vector<int>* offsets, std::vector<uint8_t>* idx,
                                 std::vector<float>* err, uint16_t* plane_cb, uint16_t* plane_cr);

  // ---- candidates given as pixels (the comparator-level drop-in for any
  // OutputImage, subsampled components included) ----
  // The next Compare reads the candidate as sRGB (3*w*h bytes, ToSRGB).
  bool SetCandidateRgb(const uint8_t* rgb);
  // CompareBlock of n requests with 8x8 sRGB windows rgb[192 * i ..].
  bool CompareBlocksRgb(int n, const int* blocks, const uint8_t* rgb, double* err);

  // Device entropy coding of the current coefficients with quant q (the
  // per-iteration JPEG of the search).  JpegStage: quantized zigzag
  // coefficients, symbol histograms hist[comp*2 + {0:DC, 1:AC}][256] (plain
  // counts) and the number of non-zero chroma coefficients.  JpegScan: the
  // scan bitstream of the staged image for `ncomp` components with `codes`
  // into the current slot (padded to a byte with ones): *nbits bits, *ff
  // bytes 0xff (the stuffing doubles them).  Two slots: JpegKeep makes the
  // current one the kept one (the next scan overwrites the other);
  // JpegFetch copies a slot's bytes (MSB-first, valid until the next call).
  bool JpegStage(const int q[3][64], uint32_t* hist, uint64_t* chroma_nz);
  bool JpegScan(int ncomp, const int q[3][64], const JpegCodeTables& codes, uint64_t* nbits, uint64_t* ff);
  void JpegKeep() { jslot_ ^= 1; }
  bool JpegFetch(bool kept, const uint8_t** bytes, uint64_t* nbits);
  // The same steps split for overlap within one stream order: *Enqueue
  // queues work without waiting; JpegStageWait waits for the staged
  // histograms only (an event), Sync for everything queued, after which
  // CompareFinish / JpegScanFinish read the results.  The search runs
  // stage -> Compare pass -> (host builds the codes while the pass runs)
  // -> scan, with one full synchronisation per candidate.
  bool JpegStageEnqueue(const int q[3][64]);
  bool JpegStageWait(uint32_t* hist, uint64_t* chroma_nz);
  bool CompareEnqueue();
  // skip_at: the scan is not coded when the distance of the Compare pass
  // queued before it is at or above skip_at (the caller knows the candidate
  // cannot become the output; JpegScanFinish must not be called then).
  bool JpegScanEnqueue(int ncomp, const int q[3][64], const JpegCodeTables& codes,
                       float skip_at = __builtin_inff());
  bool Sync();
  // distance: the pass's maximum (from mapped memory); block_max (may be
  // null): the per-block maxima, copied from HBM.
  bool CompareFinish(float* distance, float* block_max);
  bool JpegScanFinish(uint64_t* nbits, uint64_t* ff);

  // The coder over a part of the scan (a frame split over ranks by block
  // rows): the MCUs [m0, m1) (4:4:4, one block per component), their DC
  // predicted from block m0 - 1, their bits starting at bit `base` of the
  // whole stream; pad_end for the stream's last part.  The words this part
  // shares with its neighbours (first_word when base is not a multiple of
  // 32, last_word when the end is neither padded nor word-aligned) are not
  // stored: they come back here, in memory byte order, for the ranks to
  // combine; ff counts the 0xff bytes of the words the part stores.
  struct ScanPart {
    uint64_t base = 0, bits = 0, ff = 0;
    uint32_t first_word = 0, last_word = 0;
    bool first_shared = false, last_open = false;
  };
  bool JpegStageEnqueueRange(const int q[3][64], int m0, int m1);
  bool JpegScanEnqueueRange(int ncomp, const int q[3][64], const JpegCodeTables& codes, int m0, int m1,
                            uint64_t base, bool pad_end, float skip_at = __builtin_inff());
  bool JpegScanFinishPart(ScanPart* part);
  // The stored words of a slot's part (memory byte order; words[0] is the
  // stream's word base >> 5, the shared ones zero) and its ScanPart.
  bool JpegFetchPart(bool kept, std::vector<uint32_t>* words, ScanPart* part);
  // offsets[i] = counts[0] + ... + counts[i - 1] on the device (n + 1
  // entries); first (optional): the index holding element 256 c, per c
  // wg_totals (optional): the totals of every 256 counts at stride 2 (a
  // counting kernel's partials) -- the chunk sums without a launch
  bool ScanCounts(const int* counts, int n, int* offsets, const char* name, int* first = nullptr,
                  const int* wg_totals = nullptr);
  bool OrderBlocks(int comp_mask);

  // The search back end's change order on the device (SelectFrequencyBackEnd,
  // processor.cc:776-834, 4:4:4 whole frame) over the candidates of the last
  // BlockZeroingCandidates (HasOrderCandidates) and the block maxima of the
  // last Compare.  OrderReset zeroes max_block_error; OrderBuild computes the
  // weights at radius rblock (zero_bmax: every block maximum taken as 0) and
  // the entries from last_indexes (host state, uploaded) in one launch
  // (k_order_build) and returns their total and the blocks with entries;
  // OrderFetch downloads the n entries (block, key) in block order; OrderAdvance adds
  // weight * val_threshold * direction to max_block_error (applied by the
  // next OrderBuild, ahead of its weights).
  bool HasOrderCandidates() const { return ord_cand_n_ >= 0; }
  // (*unavailable: the order's buffers could not be allocated -- the caller
  // builds the order on the host; false is then not returned for it)
  bool OrderReset(bool* unavailable = nullptr);
  // OrderBuild: the entries of the radius are filled into HBM, grouped by
  // workgroup (with the selection's first counts); floor_limit > -inf: *below_floor =
  // the entries keyed below it (the first up iteration's floor).
  bool OrderBuild(int direction, int rblock, double target_distance, bool zero_bmax,
                  const std::vector<int>& last_indexes, size_t* n_entries, int* blocks_to_change,
                  float floor_limit = -__builtin_inff(), int64_t* below_floor = nullptr);
  size_t OrderEntryCount() const { return ord_n_; }
  // the n entries (block, key) of the last OrderBuild, in block order
  bool OrderFetch(std::pair<int, float>* out, size_t n);
  bool OrderAdvance(float val_threshold, int direction);
  // The back end's bulk prefix applied to the device copy (k_bulk_apply):
  // cnt[b] changes of block b from the last_indexes of this iteration's
  // OrderBuild, zeroed (direction 1) or restored to Quantize(orig, quant),
  // and the change of every component's AC symbol counts it makes
  // (delta[c][symbol], unscaled), waited for.
  // (last_indexes: the host's, for a back end without the device order --
  // a frame split over ranks; else the last OrderBuild's copy)
  bool BulkApply(int direction, const int quant[3][64], const uint8_t* cnt, int32_t delta[3][256],
                 const std::vector<int>* last_indexes = nullptr);
  // The first `bulk` entries of the last OrderBuild's std::sort order as a
  // set, selected on the device by their keys (radix selection of the key
  // of rank bulk - 1, K*), applied there (k_bulk_apply) -- unless K* is
  // shared by entries of several blocks across the prefix's end (open: the
  // keys leave the set to std::sort's tie order, nothing is applied) -- and
  // the tail's window: every entry keyed from K* up to the key of rank
  // bulk + window - 1 (K2), in no order, the prefix's K*-keyed entries
  // among them.  bulk 0: no prefix, the window from the smallest key.
  struct OrderSelection {
    uint32_t kbits[2] = {0, 0};  // K*, K2 (StripOrder::Bits order)
    int below = 0, eq = 0;       // entries keyed below K*, at K*
    bool straddle = false;       // the prefix takes only `take` of the K*-keyed entries ...
    int take = 0;
    int tie_block = -1;          // ... all of tie_block's (when not open)
    bool open = false;
    bool applied = false;        // the prefix was applied (cnt: per block, tie_block's take included)
    std::vector<uint8_t> cnt;
    size_t window_n = 0;
    bool window_overflow = false;  // more than the staging holds: window empty
    bool window_last = false;      // K2 is the largest key: the window holds every entry left
    // the tail from position bulk on, in order (the prefix's entries
    // dropped); its first window_ok positions are std::sort's
    std::vector<std::pair<int, float>> window;
    size_t window_ok = 0;
  };
  // (apply false: the selection and the window only -- a later window of
  // the tail, from rank `bulk` on)
  bool OrderSelect(size_t bulk, size_t window, int direction, const int quant[3][64], bool apply,
                   OrderSelection* out, int32_t delta[3][256]);

  // A frame split over ranks (host/strips.h): this engine's image is a
  // strip (local blocks; frame block = gbase + local), and the change order
  // is the frame's.  OrderBuild then forms the entries of the owned local
  // blocks [own_lo, own_hi) only (its totals stay local: the caller sums
  // them), and OrderSelect runs the frame-wide selection with the exchange's
  // collectives between its launches: the round-1 and round-2 counts summed
  // over the ranks, every rank's candidates gathered (block indices as frame
  // indices), the final step on every rank alike -- the window in frame block
  // indices, the prefix counts of the owned blocks.  `frame_n`: the frame's
  // entry count (SetOrderFrameEntries after each build).  Every exchange
  // carries a status: a rank that failed fails every rank there.
  struct OrderExchange {
    virtual ~OrderExchange() = default;
    virtual bool SumU32(bool ok, uint32_t* v, int n) = 0;  // in place, over the ranks
    virtual bool Gather(bool ok, const std::vector<unsigned long long>& mine,
                        std::vector<unsigned long long>* all) = 0;  // every rank's, concatenated
  };
  void SetOrderScope(int own_lo, int own_hi, int gbase, OrderExchange* x) {
    ord_lo_ = own_lo;
    ord_hi_ = own_hi;
    ord_gbase_ = gbase;
    ord_x_ = x;
  }
  void SetOrderFrameEntries(size_t n) { ord_frame_n_ = n; }
  // The block maxima the change order's weights read (the frame's values,
  // exchanged: a strip's halo blocks differ from its own Compare's), [nb].
  bool SetBlockMax(const float* bmax);

  const std::string& error() const { return err_; }
  void* stream() const { return stream_; }
  double last_kernel_ms(const char* which) const;

 private:
  Engine() = default;
  bool OrderEntriesCapacity(size_t n);
  bool OrderSelectSplit(const void* entries, size_t n, size_t fn, int has_prefix, size_t bulk, long long ta,
                        long long tb, int cap, unsigned rgroups, unsigned cgroups, int force_open, int gbase,
                        int blo, int bhi);
  char* RequestStaging(size_t need, char** mapped);  // CompareBlocks* mapped staging
  bool AwaitPosted(const char* h, double* err);
  bool BulkCountsStaging();
  bool BulkApplyEnqueue(int direction, const int quant[3][64], const uint8_t* cnt_dev, const uint32_t* sel,
                        const uint8_t* last8, uint8_t* cnt_host);
  bool Fail(const char* what, int code);
  void ProfBegin(const char* name);
  void ProfEnd();
  void ProfMark(const char* name);
  void ProfFlush();
  struct PendingEvent {
    std::string name;
    void* start;
    void* stop;
  };
  std::vector<PendingEvent> pending_;
  // MaskOpt's chain into d_ma_ (front: the mask front from xyb0 / xyb1 into
  // d_mb_ first; false when the Compare pass's fused edge_mask made it).
  bool MaskPipeline(const float* xyb0, const float* xyb1, bool sub_b, bool front = true);
  bool EnqueueCompare(CompareDebug* dbg);
  // slots: k_block_zeroing's kept entries per block (else CoeffData orders)
  bool CompactCandidates(int nblocks, float limit, std::vector<int>* offsets,
                         std::vector<uint8_t>* idx, std::vector<float>* err, bool slots = false);
  // what Compare's first stage reads (and its hipGraphExec_t each)
  enum CandSource { kCandCoeffs = 0, kCand420 = 1, kCandRgb = 2 };
  int cand_src_ = kCandCoeffs;
  void* compare_graph_[3] = {nullptr, nullptr, nullptr};
  void* stage_event_ = nullptr;    // hipEvent_t: the staged histograms reached the host

  int device_ = 0;
  int w_ = 0, h_ = 0, bw_ = 0, bh_ = 0, nb_ = 0, rw_ = 0, rh_ = 0;
  size_t n_ = 0;
  void* stream_ = nullptr;
  std::string err_;
  bool failed_ = false;
  size_t bytes_ = 0;
  bool have_mask_scale_ = false;
  int cbw_ = 0, cbh_ = 0;     // chroma blocks of the 4:2:0 pass

  // device buffers
  uint8_t* d_rgb_ = nullptr;
  int16_t* d_orig_ = nullptr;
  int16_t* d_cur_ = nullptr;
  float* d_ref_xyb_ = nullptr;
  float* d_lin_ = nullptr;    // the reference's linear planes (and the stage dumps')
  uint32_t* d_px8_ = nullptr;  // the candidate's sRGB pixels, packed (the Compare pass's input)
  float* d_xyb_ = nullptr;
  float* d_m0_ = nullptr;
  float* d_m1_ = nullptr;
  float* d_tmp_ = nullptr;   // 6 planes
  float* d_bl_ = nullptr;    // 6 planes
  float* d_ma_ = nullptr;    // 3 planes
  float* d_mb_ = nullptr;    // 3 planes
  float* d_edge_ = nullptr;  // 3R
  float* d_dc_ = nullptr;    // 3R
  float* d_ac_ = nullptr;    // 3R
  float* d_resval_ = nullptr;
  float* d_block_max_ = nullptr;
  uint16_t* d_planes_ = nullptr;   // 4:2:0: Cb / Cr pixel state [2][w*h] (allocated on first use)
  uint8_t* d_cand_rgb_ = nullptr;  // sRGB candidate [3*w*h] (allocated on first use)
  float* d_mask_scale_ = nullptr;
  void* d_zero_out_ = nullptr;
  int* d_zero_count_ = nullptr;    // [blocks] kept entries per block
  int* d_zero_order_ = nullptr;    // [blocks] zeroing-search processing order
  int* d_zero_off_ = nullptr;      // [blocks + 1] their offsets
  int* d_zero_nnz_ = nullptr;      // [blocks] non-zero AC counts (processing order)
  int* d_zero_bins_ = nullptr;     // [2][193] count histogram, scatter cursors
  int* d_scan_sums_ = nullptr;     // [blocks / 4 + 2] chunk totals / 4-MCU group totals
  uint8_t* d_cand_idx_ = nullptr;  // [blocks * 192] compacted candidates
  float* d_cand_err_ = nullptr;
  int16_t* h_coeffs_ = nullptr;    // pinned [3][blocks][64] staging
  uint32_t* d_jhist_ = nullptr;    //   kJHistCopies x 6 x 256 counts + chroma non-zeros (u64) + done counter
  uint32_t* d_jwords_[2] = {nullptr, nullptr};  // scan bitstreams: current / kept slot
  uint64_t jnbits_[2] = {0, 0};
  ScanPart jpart_[2];
  int jcode_groups_[2] = {0, 0};   // the coder launch's workgroups, per slot
  bool jcode_pad_[2] = {false, false};
  int jslot_ = 0;                  // current slot (kept = jslot_ ^ 1)
  uint32_t* d_jctl_ = nullptr;     //   k_jpeg_code: 0xff counters | arrivals | status | shared words
  uint32_t jepoch_ = 0;            //   launches so far (status tags)
  size_t jwords_cap_ = 0;
  uint32_t* h_jhist_ = nullptr;    // pinned: counts + chroma + (0xff count, total bits),
  uint32_t* m_jhist_ = nullptr;    //   written by the kernels through this mapped address
  uint8_t* h_jbytes_ = nullptr;
  size_t h_jbytes_cap_ = 0;
  int* h_zero_off_ = nullptr;      // pinned
  uint8_t* h_cand_idx_ = nullptr;  // pinned, h_cand_cap_ entries
  float* h_cand_err_ = nullptr;
  size_t h_cand_cap_ = 0;
  float* d_scales_ = nullptr;  // [sigma][axis][scale_stride_] border scales
  uint32_t* h_delta_idx_ = nullptr;   // UploadCoeffDelta staging (pinned host)
  int16_t* h_delta_val_ = nullptr;
  uint32_t* m_delta_idx_ = nullptr;   // ... their device-side (mapped) addresses
  int16_t* m_delta_val_ = nullptr;
  size_t delta_cap_ = 0;
  char* h_cbreq_ = nullptr;  // CompareBlocks staging, mapped (indices | candidates | errors)
  char* m_cbreq_ = nullptr;
  size_t cbreq_cap_ = 0;
  int scale_stride_ = 0;
  // pinned host staging
  float* h_block_max_ = nullptr;   // pinned: the block maxima on request; [nb_ + 4 ..]: k_diffmap's tile maxima (mapped)
  float* m_block_max_ = nullptr;
  uint32_t* d_dmax_ = nullptr;      // k_diffmap's kDmMaxWords maxima words (the coder's skip test)
  // device change order (allocated on first use): weight f32 | active i32 |
  // counts i32 | offsets i32 [nb + 1] | totals i32 [8] | arrival counters |
  // max_block_error f32 | last_indexes i32
  int ord_cand_n_ = -1;             // candidates of the last 4:4:4 zeroing search (-1: none)
  float ord_adv_vt_ = 0.0f;         // pending max_block_error update (OrderAdvance)
  int ord_h1_ = 0;                  // the last build's copy of the selection's round-1 counts
  int ord_adv_dir_ = 0;
  void* d_ord_ = nullptr;
  int* h_ord_ = nullptr;            // mapped pinned: last_indexes [nb] | totals [8]
  int* m_ord_ = nullptr;            //   (its device address)
  size_t ord_n_ = 0;                // entries of the last OrderBuild
  // (a frame split over ranks: SetOrderScope)
  int ord_lo_ = 0, ord_hi_ = 1 << 30, ord_gbase_ = 0;
  OrderExchange* ord_x_ = nullptr;
  size_t ord_frame_n_ = 0;          // the frame's entries of the last build
  bool ord_h1_summed_ = false;      // its round-1 counts are the frame's
  void* d_ord_entries_ = nullptr;   // the entries (HBM)
  size_t d_ord_entries_cap_ = 0;
  void* h_ord_entries_ = nullptr;   // pinned: OrderFetch's staging
  size_t h_ord_entries_cap_ = 0;
  void* h_win_ = nullptr;           // mapped pinned: OrderSelect's window, in order
  void* m_win_ = nullptr;
  void* d_win_ = nullptr;           // ... compacted, in no order (HBM)
  uint8_t* h_bulk_ = nullptr;       // mapped pinned: BulkApply's per-block change counts
  uint8_t* m_bulk_ = nullptr;
};

// Process-wide pool of idle engines keyed by (device, width, height): an
// encode reuses the HBM buffers, stream and tables of an earlier encode of
// the same size instead of re-allocating ~40 planes.  Idle engines are kept
// in least-recently-released order under a byte cap (GZ_ENGINE_POOL_BYTES,
// default 16 GiB of HBM + pinned memory, and at most 8 per size); an engine
// whose last operation failed is destroyed instead of pooled.
std::unique_ptr<Engine> AcquireEngine(int device, int w, int h, std::string* err);
void ReleaseEngine(std::unique_ptr<Engine> e);
// Destroys least recently used idle engines until at most keep_bytes stay
// pooled; returns the bytes released.
size_t TrimEnginePool(size_t keep_bytes);
size_t EnginePoolIdleBytes();

// Per-launch HIP-event timing (off by default).
void ProfileEnable(bool on);
void ProfileReset();
bool ProfileGet(const char* name, long* count, double* total_ms);
std::string ProfileNames();

// Version / build string of the device library.
const char* BuildInfo();

}  // namespace gz
