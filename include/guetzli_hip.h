/*
 * guetzli_hip.h — C ABI of the MI355X-native Guetzli search path
 * (libguetzli_hip.so, built from guetzli-cuda-opencl_amd/csrc).
 *
 * Drop-in boundary for the reference's hot path (yyamamoto79/guetzli-cuda-
 * opencl): the library-level encode call `guetzli::Process`
 * (guetzli/processor.h:62-64) and the comparator that the search loop talks
 * to (`guetzli::Comparator`, guetzli/comparator.h:29-96, implemented by
 * `guetzli::ButteraugliComparator`, guetzli/butteraugli_comparator.h:33-81),
 * plus the batched per-block zeroing entry of the reference GPU fast path
 * (`cuComputeBlockZeroingOrder`, clguetzli/cuguetzli.h:30-40).
 *
 * Conventions
 *  - Plain pointers and sizes only.  Every call returns gz_status; on failure
 *    gz_last_error() (thread-local) describes it.  No call silently falls
 *    back to the CPU: without a usable HIP device they fail with
 *    GZ_ERR_DEVICE.
 *  - Images: 8-bit RGB, interleaved, row-major, no padding (3*w*h bytes).
 *  - Coefficients: int16, [3][blocks][64], natural (row-major) order inside
 *    a block, blocks row-major with ceil(w/8) blocks per row (the layout of
 *    guetzli::JPEGComponent::coeffs, guetzli/jpeg_data.h:138-204).
 *  - One gz_comparator / gz_encoder owns one HIP stream and its device
 *    buffers; distinct objects may be used from distinct host threads.
 */
#ifndef GUETZLI_HIP_H_
#define GUETZLI_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int gz_status;
enum {
  GZ_OK = 0,
  GZ_ERR_INVALID_ARG = 1,
  GZ_ERR_DEVICE = 2,
  GZ_ERR_OUT_OF_MEMORY = 3,
  GZ_ERR_UNSUPPORTED = 4,
  GZ_ERR_INTERNAL = 5,
};

/* guetzli::CoeffData (guetzli/processor.h:29-32). */
typedef struct {
  int idx;
  float block_err;
} gz_coeff_data;

/* guetzli::Params (guetzli/processor.h:34-42); same defaults via
 * gz_params_init().  try_420 / force_420 / use_silver_screen run the 4:2:0
 * pass of ProcessJpegData (processor.cc:986-1016); on an image whose chroma
 * is all zero that pass keeps one component at 4:4:4, as the reference does
 * (output_image.cc:535-539).  A butteraugli_target above 2.0 (quality below
 * 84) returns GZ_ERR_INVALID_ARG (processor.cc:939-945).  The strip
 * decomposition of one frame (gz_process_rgb_strips) supports the 4:4:4
 * search only. */
typedef struct {
  float butteraugli_target;
  int clear_metadata;
  int try_420;
  int force_420;
  int use_silver_screen;
  int zeroing_greedy_lookahead;
  int new_zeroing_model;
} gz_params;

/* guetzli::ProcessStats counters (guetzli/stats.h:26-41). */
typedef struct {
  int iterations;        /* "number of iterations" */
  int iterations_up;     /* "number of iterations up" */
  int iterations_down;   /* "number of iterations down" */
  int compares;          /* full-image Butteraugli passes */
  double seconds_compare;   /* wall time inside Compare calls */
  double seconds_zeroing;   /* wall time of the per-block search */
  double seconds_total;
  double seconds_setup;     /* initial coefficients, device context, reference */
  double seconds_write;     /* JPEG serialisation of every candidate */
  double seconds_quantize;  /* device quantization + coefficient download */
  double seconds_backend;   /* host coefficient selection / size estimation */
} gz_process_stats;

/* Stage dumps of one compare (parity tests); any pointer may be NULL.
 * Plane arrays are 3*w*h floats, res arrays 3*ceil(w/3)*ceil(h/3). */
typedef struct {
  float* cand_linear;
  float* cand_xyb;
  float* mhic0;
  float* mhic1;
  float* edge;
  float* block_dc;
  float* block_ac;
  float* block_ac_lf;
  float* mask;
  float* mask_dc;
  float* combined;   /* ceil(w/3)*ceil(h/3) */
  float* distmap;    /* w*h */
} gz_compare_stages;

typedef struct gz_comparator gz_comparator;

/* ---- library ---------------------------------------------------------- */
const char* gz_last_error(void);
const char* gz_build_info(void);
/* Number of visible HIP devices (0 when none; never fails). */
int gz_device_count(void);
void gz_params_init(gz_params* params);
/* guetzli::ButteraugliScoreForQuality (guetzli/quality.cc:78-87). */
double gz_butteraugli_score_for_quality(double quality);
void gz_free(void* p);

/* ---- encode (guetzli::Process, guetzli/processor.h:62-64) -------------- */
/* Encodes an RGB image; *jpeg_out is allocated by the library (gz_free).
 * Images under 32 pixels in either dimension are written at quantization 1
 * without a search and without device work (processor.cc:1170-1181). */
gz_status gz_process_rgb(int device, const gz_params* params, const uint8_t* rgb, int width,
                         int height, uint8_t** jpeg_out, size_t* jpeg_size,
                         gz_process_stats* stats);
/* Same, with the RGB image already resident on `device` (HBM pointer). */
gz_status gz_process_rgb_device(int device, const gz_params* params, const uint8_t* rgb_dev,
                                int width, int height, uint8_t** jpeg_out, size_t* jpeg_size,
                                gz_process_stats* stats);

/* Encodes a JPEG file: guetzli::Process(params, stats, jpeg_bytes, out)
 * (guetzli/processor.h:44-46, processor.cc:1029-1066) -- the input's own
 * coefficients and quantization start the search, its decoded pixels are the
 * Butteraugli reference.  Baseline / extended / progressive Huffman JPEGs with
 * 4:4:4 or 4:2:0 YCbCr sampling (4:2:0 forces the downsampled search); other
 * layouts and 1-component files return GZ_ERR_UNSUPPORTED (the reference's
 * Process returns false for them), unreadable input GZ_ERR_INVALID_ARG.  *jpeg_out: library-allocated
 * (gz_free). */
gz_status gz_process_jpeg(int device, const gz_params* params, const uint8_t* jpeg, size_t jpeg_len,
                          uint8_t** jpeg_out, size_t* jpeg_size, gz_process_stats* stats);
/* ReadJpeg (guetzli/jpeg_data_reader.cc:931-1079, JPEG_READ_ALL) and
 * DecodeJpegToRGB (jpeg_data_decoder.cc:45-55) of a JPEG file, host only:
 * *coeffs_out the quantized coefficients of every component ([comp][blocks]
 * [64], natural order, MCU-padded grid; *ncoeffs values), *rgb_out the RGB8
 * image for 4:4:4 and 4:2:0 YCbCr inputs, else NULL.  Both library-allocated (gz_free). */
gz_status gz_jpeg_decode(const uint8_t* jpeg, size_t jpeg_len, int* width, int* height,
                         int* ncomp, int16_t** coeffs_out, size_t* ncoeffs, uint8_t** rgb_out);

/* ReadPNG of the reference CLI (guetzli/guetzli.cc:51-156; libpng with
 * PACKING | EXPAND | STRIP_16, alpha blended on black), host only: every PNG
 * colour type and bit depth, interlaced or not, tRNS.  *rgb_out: RGB8,
 * 3*w*h bytes, library-allocated (gz_free).  GZ_ERR_INVALID_ARG for what
 * ReadPNG rejects (the CLI then fails, guetzli.cc:326-330). */
gz_status gz_png_decode(const uint8_t* png, size_t png_len, int* width, int* height,
                        uint8_t** rgb_out);

/* ---- one frame over several GPUs (row strips + halo) ------------------ */
/* The exchange a multi-rank encode needs: an equal-size all-gather (every
 * rank contributes `bytes` bytes, `recv` receives world*bytes in rank order);
 * returns 0 on success.  Bound to torch.distributed (RCCL over xGMI, or gloo)
 * by the Python package. */
typedef struct {
  void* ctx;
  int rank;
  int world;
  int (*allgather)(void* ctx, const void* send, size_t bytes, void* recv);
} gz_collectives;
/* guetzli::Process (processor.h:62-64) for one frame whose Butteraugli passes
 * are split over the ranks of `coll` by rows: every rank passes the whole
 * RGB frame (host memory) and its own device, and receives the same bytes as
 * gz_process_rgb.  A rank computes its owned rows plus a 96-row halo. */
gz_status gz_process_rgb_strips(int device, const gz_params* params, const uint8_t* rgb, int width,
                                int height, const gz_collectives* coll, uint8_t** jpeg_out,
                                size_t* jpeg_size, gz_process_stats* stats);
/* Rows rank `rank` owns [y0, y1) and computes [e0, e1). */
gz_status gz_strip_layout(int width, int height, int world, int rank, int* y0, int* y1, int* e0,
                          int* e1);
/* Exercises `coll` (fixed- and variable-size gathers); GZ_OK if consistent. */
gz_status gz_collectives_selftest(const gz_collectives* coll);
/* gz_collectives over RCCL (NCCL's API on ROCm: all-gathers over xGMI
 * between the GPUs of a node), for C/C++ callers running one process per
 * GPU without torch.distributed (the reference has no collectives,
 * SURVEY.md §5).  One rank calls gz_rccl_unique_id and
 * hands the 128 bytes to the others by its own means (MPI, a file, a
 * socket); every rank then calls gz_rccl_create (ncclCommInitRank: returns
 * when all have), which fills *coll for gz_process_rgb_strips.  RCCL is
 * loaded on first use: the librccl beside the HIP runtime the process has
 * mapped (torch's own in a process that imported torch, else ROCm's), then
 * librccl.so.1 from the search path.  gz_rccl_destroy after the last encode
 * that uses *coll. */
typedef struct gz_rccl gz_rccl;
gz_status gz_rccl_unique_id(uint8_t id[128]);
gz_status gz_rccl_create(int device, int rank, int world, const uint8_t id[128], gz_rccl** out,
                         gz_collectives* coll);
void gz_rccl_destroy(gz_rccl* comm);
/* Path of the librccl loaded (empty before the first gz_rccl_* call or if
 * none could be loaded). */
const char* gz_rccl_library(void);

/* ---- comparator (guetzli::ButteraugliComparator) ---------------------- */
/* ButteraugliComparator(w, h, rgb, target, stats) ctor
 * (guetzli/butteraugli_comparator.cc:48-58); width, height >= 8. */
gz_status gz_comparator_create(int device, int width, int height, const uint8_t* rgb,
                               float target_distance, gz_comparator** out);
void gz_comparator_destroy(gz_comparator* cmp);
/* Comparator::Compare (guetzli/butteraugli_comparator.cc:60-70) on the image
 * whose DCT coefficients are `coeffs`; distance = distmap_aggregate(). */
gz_status gz_comparator_compare(gz_comparator* cmp, const int16_t* coeffs, float* distance);
/* Comparator::Compare of an image given as its sRGB pixels (3*w*h bytes,
 * RGB interleaved -- OutputImage::ToSRGB(), output_image.cc:654-701): the
 * entry for images whose pixels are not a function of their coefficients
 * alone (4:2:0: the subsampled components' upsampled pixels are state). */
gz_status gz_comparator_compare_rgb(gz_comparator* cmp, const uint8_t* rgb, float* distance);
/* Compare of a 4:2:0 candidate (OutputImage with factor-2 chroma,
 * output_image.cc:642-716): Y coefficients ([blocks][64]), Cb / Cr
 * coefficients ([ceil(w/16)*ceil(h/16)][64] each; NULL = zeros -- the
 * Compare pass reads the chroma from the planes) and the factor-2 components'
 * 16-bit pixel state (w*h each, wrapping: ToPixels' byte is
 * ((p + 8 - (x & 1)) >> 4) & 0xff, output_image.cc:83). */
gz_status gz_comparator_compare_420(gz_comparator* cmp, const int16_t* y, const int16_t* cb,
                                    const int16_t* cr, const uint16_t* plane_cb, const uint16_t* plane_cr,
                                    float* distance);
/* Same, with stage dumps. */
gz_status gz_comparator_compare_stages(gz_comparator* cmp, const int16_t* coeffs,
                                       gz_compare_stages* stages, float* distance);
/* Same, dumped from the search's own (fused) kernel variants instead of the
 * stand-alone dump kernels -- the corner edge term as k_block_diff leaves it,
 * block_ac before the low-frequency term, the distance map after the fused
 * combine (low-frequency term, subsampled B mask, LUT'd mask samples).  Only
 * mhic0, mhic1, edge, block_dc, block_ac and distmap may be non-NULL
 * (GZ_ERR_INVALID_ARG otherwise).  Parity evidence for the kernels the search
 * runs (clbutter_comparator.cpp:1387-1417). */
gz_status gz_comparator_compare_stages_production(gz_comparator* cmp, const int16_t* coeffs,
                                                  gz_compare_stages* stages, float* distance);
/* EncodeRGBToJpeg's q=1 coefficients of the comparator's reference image
 * ([3][blocks][64] int16, natural order) computed on the device: YUV16 +
 * integer FDCT + q=1 quantizer (guetzli/jpeg_data_encoder.cc:66-136,
 * guetzli/fdct.cc). */
gz_status gz_comparator_original_coeffs(gz_comparator* cmp, int16_t* out);
/* Comparator::distmap() (comparator.h:71-75): the distance map of the last
 * gz_comparator_compare (w*h floats; recomputed on the device from the same
 * candidate -- the search's own passes keep only per-block maxima). */
gz_status gz_comparator_distmap(gz_comparator* cmp, float* out);
/* Per-8x8-block maxima of the last distance map (ceil(w/8)*ceil(h/8)). */
gz_status gz_comparator_block_max(gz_comparator* cmp, float* out);
/* ComputeBlockErrorAdjustmentWeights (butteraugli_comparator.cc:169-233) on
 * the host: per-(8*factor)-block maxima of `distmap` (width*height floats),
 * then the neighbourhood weights.  block_weight (one float per block) is
 * updated in place -- the caller zero-fills it first, as the search loop does
 * (processor.cc:779-783).  No device needed. */
gz_status gz_block_error_adjustment_weights(int width, int height, float target, int direction,
                                            int max_block_dist, double target_mul, int factor_x,
                                            int factor_y, const float* distmap,
                                            float* block_weight);
/* Comparator::DistanceOK (butteraugli_comparator.h:52-54). */
int gz_comparator_distance_ok(gz_comparator* cmp, double target_mul);
/* Comparator::ScoreOutputSize (butteraugli_comparator.cc:235-237). */
double gz_comparator_score_output_size(gz_comparator* cmp, int size);
/* StartBlockComparisons (butteraugli_comparator.cc:72-79); mask_scale may be
 * NULL, else receives 3 floats per block (mask_xyz at the block corner). */
gz_status gz_comparator_start_block_comparisons(gz_comparator* cmp, float* mask_scale);
/* Batched per-block greedy zeroing of SelectFrequencyMasking's CPU_OPT loop
 * (processor.cc:376-487, 641-672) for the candidate `cur_coeffs` against
 * the original q=1 coefficients `orig_coeffs`; out: blocks*192 entries,
 * zero-filled tails.  Replaces cuComputeBlockZeroingOrder
 * (clguetzli/cuguetzli.h:30-40).  comp_mask: components searched (the
 * others keep cur_coeffs' values in the pixels); lookahead /
 * new_zeroing_model: Params::zeroing_greedy_lookahead / new_zeroing_model
 * (0: the old candidate key of processor.cc:400-405). */
gz_status gz_comparator_block_zeroing_orders(gz_comparator* cmp, const int16_t* cur_coeffs,
                                             const int16_t* orig_coeffs, int comp_mask,
                                             float limit, int lookahead, int new_zeroing_model,
                                             gz_coeff_data* out);

/* SwitchBlock(bx, by, 1, 1) + CompareBlock(img, 0, 0, candidate, comp_mask)
 * (butteraugli_comparator.cc:85-163) for n requests at once: request i
 * compares 8x8 block blocks[i] (row-major block index) of the reference image
 * with candidate coefficients cand[192*i ..] -- [3][64], natural order,
 * dequantized, every component as the image holds it (the masked
 * components' candidate values, the image's current values for the others)
 * -- and err[i] receives CompareBlock's double.  Uses the activity mask of
 * StartBlockComparisons (run first if needed).  The per-block entry of the
 * comparator-level drop-in; the search itself uses the
 * batched gz_comparator_block_zeroing_orders. */
gz_status gz_comparator_compare_blocks(gz_comparator* cmp, int n, const int* blocks,
                                       const int16_t* cand, double* err);
/* The same with each candidate given as its 8x8 sRGB window rgb[192*i ..]
 * (row major, RGB interleaved, as OutputImage::ToSRGB(8 bx, 8 by, 8, 8)
 * returns it, edge pixels replicated): CompareBlock(img, off_x, off_y, ...)
 * of any image, subsampled components included (butteraugli_comparator.cc:
 * 113-163 reads the image only through ToLinearRGB). */
gz_status gz_comparator_compare_blocks_rgb(gz_comparator* cmp, int n, const int* blocks,
                                           const uint8_t* rgb, double* err);

/* SaveToJpegData + WriteJpeg (guetzli/output_image.cc:579-640,
 * jpeg_data_writer.cc:540-553) of dequantized coefficients `coeffs`
 * ([3][blocks][64], multiples of quant) with quant tables `quant` ([3][64],
 * natural order), entropy coded on the comparator's device; metadata
 * stripped.  *jpeg_out is allocated by the library (gz_free). */
gz_status gz_comparator_write_jpeg(gz_comparator* cmp, const int16_t* coeffs, const int* quant,
                                   uint8_t** jpeg_out, size_t* jpeg_size);
/* The same on the host (the library's serial writer; no device needed). */
gz_status gz_write_jpeg_host(int width, int height, const int16_t* coeffs, const int* quant,
                             uint8_t** jpeg_out, size_t* jpeg_size);

/* ---- device memory ---------------------------------------------------- */
/* Encodes keep their per-size engines (HBM buffers, stream, graph) in a
 * process-wide pool for reuse: least recently used first out, capped at
 * GZ_ENGINE_POOL_BYTES (environment, default 16 GiB) and 8 per image size;
 * engines whose last operation failed are never pooled.  trim destroys idle
 * engines until at most keep_bytes remain and returns the bytes released. */
size_t gz_engine_pool_trim(size_t keep_bytes);
size_t gz_engine_pool_idle_bytes(void);

/* ---- measurement ------------------------------------------------------ */
/* Per-launch timing with HIP events on each object's own stream (off by
 * default).  Regions are named after the pass stage ("block_diff",
 * "mask_blur_h", "block_zeroing", ... and "compare_pass" for a whole
 * Butteraugli pass). */
void gz_profile_enable(int enable);
void gz_profile_reset(void);
/* Returns 1 and fills count / total milliseconds if `name` was recorded. */
int gz_profile_get(const char* name, long* count, double* total_ms);
/* Comma-separated recorded region names; returns the length needed. */
size_t gz_profile_names(char* buf, size_t cap);
/* JSON object of host-side timers / counters of this thread's last encode;
 * returns the length needed. */
size_t gz_last_process_detail(char* buf, size_t cap);

/* ---- helpers used by the host search loop ----------------------------- */
/* Synthetic sRGB test frame (SURVEY.md §8d generator), 3*w*h bytes. */
gz_status gz_synthetic_frame(uint64_t seed, int width, int height, uint8_t* rgb_out);
/* EncodeRGBToJpeg at q=1 (guetzli/jpeg_data_encoder.cc:66-136): coefficient
 * planes [3][blocks][64]. */
gz_status gz_rgb_to_coeffs(const uint8_t* rgb, int width, int height, int16_t* coeffs_out);

#ifdef __cplusplus
}
#endif

#endif /* GUETZLI_HIP_H_ */
