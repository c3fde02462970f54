/*
 * gz_oracle — CPU restatement of the reference's `guetzli --c` hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the checker the HIP product is compared
 * against; it is never linked into guetzli-cuda-opencl_amd/ and only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may call it.
 *
 * Pinned against the real reference (oracle/_ref, built from /root/reference
 * by oracle/Makefile) through the stage fixtures in tests/golden/ and the
 * reference's known answer for tests/bees.png.
 *
 * Layouts: images are planar float [3][h][w]; 8-bit RGB is interleaved
 * [h][w][3]; coefficients are [3][blocks][64] int16 in natural order, block
 * index = by * ceil(w/8) + bx (jpeg_data.h:138-204).
 */
#ifndef GZ_ORACLE_H_
#define GZ_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int idx;
  float block_err;
} gzo_coeff_data; /* guetzli::CoeffData, processor.h:29-32 */

/* Intermediate planes of one DiffmapOpsinDynamicsImageOpt call; any pointer
 * may be NULL.  Sizes: planes 3*w*h, res arrays 3*rw*rh (rw = ceil(w/3)). */
typedef struct {
  float* mhic0;
  float* mhic1;
  float* edge;
  float* block_dc;
  float* block_ac;
  float* block_ac_lf;
  float* mask;
  float* mask_dc;
  float* combined; /* rw*rh */
} gzo_stages;

void gzo_init(void);

/* gamma_correct.cc:23-38 */
double gzo_srgb8_to_linear(int v);
/* guetzli/idct.cc:139-161 */
void gzo_block_idct(const int16_t* block, uint8_t* out);
/* color_transform.h:211-218 */
void gzo_ycbcr_to_rgb(uint8_t* px);
/* OutputImage::ToSRGB for a 4:4:4 image whose pixels are IDCT(coeffs)<<4
 * (output_image.cc:68-98, 124-146, 642-661). */
void gzo_coeffs_to_srgb(int w, int h, const int16_t* coeffs, uint8_t* rgb);
/* RGB8 -> planar linear float (butteraugli_comparator.cc:37-44). */
void gzo_srgb_to_linear_planes(int w, int h, const uint8_t* rgb, float* planes);

/* clbutter_comparator.cpp:57-94 */
void gzo_blur(size_t xsize, size_t ysize, float* channel, float sigma, float border_ratio);
/* clbutter_comparator.cpp:881-912 (in place: linear -> XYB) */
void gzo_opsin_dynamics(size_t xsize, size_t ysize, float* planes);
/* clbutter_comparator.cpp:729-781 */
void gzo_mask_high_intensity_change(size_t xsize, size_t ysize, const float* c0,
                                    const float* c1, float* xyb0, float* xyb1);
/* clbutter_comparator.cpp:1213-1264 */
void gzo_mask(size_t xsize, size_t ysize, const float* xyb0, const float* xyb1, float* mask,
              float* mask_dc);
/* clbutter_comparator.cpp:1387-1417; xyb0/xyb1 are mutated (as in the
 * reference).  Returns 0 and leaves distmap untouched for w<8 or h<8. */
int gzo_diffmap(size_t xsize, size_t ysize, float* xyb0, float* xyb1, float* distmap,
                gzo_stages* stages);
/* butteraugli.cc:1233-1240 */
float gzo_score_from_diffmap(const float* distmap, size_t n);

/* ButteraugliComparator::Compare: reference RGB8 vs candidate coefficients.
 * Returns the distance; distmap (w*h) may be NULL. */
float gzo_compare(int w, int h, const uint8_t* ref_rgb, const int16_t* cand_coeffs,
                  float* distmap);

/* butteraugli.cc:602-684 (double) */
void gzo_block_diff_double(double* xyb0, double* xyb1, double dc[3], double ac[3],
                           double edge_dc[3]);

/* libstdc++ std::sort of (idx, key) pairs by key ascending, reproducing its
 * exact (unstable) tie order: introsort + final insertion sort. */
void gzo_sort_pairs(int* idx, float* key, int n);

/* SwitchBlock(bx, by, 1, 1) + CompareBlock (butteraugli_comparator.cc:85-163)
 * of 8x8 block `bix` with candidate coefficients block[3][64] (ref_mask as
 * below); returns CompareBlock's double. */
double gzo_compare_block(int w, int h, const uint8_t* ref_rgb, const float* ref_mask, int bix,
                         const int16_t* block);

/* Per-block greedy zeroing order of the CPU_OPT loop
 * (processor.cc:376-487, 641-672; butteraugli_comparator.cc:72-163).
 * ref_mask: MaskOpt(ref_xyb, ref_xyb).mask (3*w*h), i.e. mask_xyz_.
 * comp_mask: components searched (others keep cur's values); new_model:
 * Params::new_zeroing_model (false: the oldCsf / kWeight key, :400-405).
 * out: blocks*192 entries, zero-filled tails. */
void gzo_block_zeroing_orders(int w, int h, const uint8_t* ref_rgb, const float* ref_mask,
                              const int16_t* cur_coeffs, const int16_t* orig_coeffs,
                              float limit, int lookahead, int comp_mask, int new_model,
                              gzo_coeff_data* out);

#ifdef __cplusplus
}
#endif

#endif /* GZ_ORACLE_H_ */
