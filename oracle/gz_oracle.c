/*
 * gz_oracle.c — scalar C restatement of the reference's `guetzli --c` hot path
 * (float Butteraugli "Opt" functions + double per-block diff + integer IDCT).
 *
 * TEST INFRASTRUCTURE ONLY (see gz_oracle.h).  Build: gcc -O2 -std=c99
 * -ffp-contract=off (the x86-64 oracle has no FMA).
 *
 * Precision follows C promotion exactly as the reference is written: an
 * expression that contains a double literal is evaluated in double and
 * rounded once on assignment to float.  Transcendental tables (blur taps,
 * sRGB, mask LUTs) use glibc exp/pow in double, as the reference does.
 *
 * The algorithms restated are Guetzli's and Butteraugli's (Copyright 2016
 * Google Inc., Apache License 2.0) as modified in
 * yyamamoto79/guetzli-cuda-opencl (clguetzli/clbutter_comparator.cpp).
 */
#include "gz_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Tables                                                                    */
/* ------------------------------------------------------------------------ */

static double g_srgb[256];             /* gamma_correct.cc:23-38 */
static int g_cr_r[256], g_cb_b[256];   /* color_transform.h:22-141 (libjpeg FIX) */
static int g_cr_g[256], g_cb_g[256];
static float g_hf_dx[21], g_hf_dy[21], g_lf_dy[21]; /* clbutter_comparator.cpp:146-193 */
static float g_mask_lut[6][512];                    /* clbutter_comparator.cpp:980-1064 */
static int g_inited = 0;

/* csf / bias of the "new zeroing model" (guetzli/order.inc:3, :198); bias is
 * all zeros there.  Values are data, reproduced verbatim. */
static const float kZeroingCsf[192] = {
#include "zeroing_csf.inc"
};

/* CSF weights of the 8x8 block diff (clbutter_comparator.cpp:103-144 float,
 * butteraugli.cc:157-198 double). */
static const double kBlockCsf[37] = {
    5.28270670524, 0.0, 0.0, 0.0, 0.3831134973, 0.676303603859, 3.58927792424, 18.6104367002,
    18.6104367002, 3.09093131948, 1.0, 0.498250875965, 0.36198671102, 0.308982169883,
    0.1312701920435, 2.37370549629, 3.58927792424, 1.0, 2.37370549629, 0.991205724152,
    1.05178802919, 0.627264168628, 0.4, 0.1312701920435, 0.676303603859, 0.498250875965,
    0.991205724152, 0.5, 0.3831134973, 0.349686450518, 0.627264168628, 0.308982169883,
    0.3831134973, 0.36198671102, 1.05178802919, 0.3831134973, 0.12,
};

static const int kNaturalOrder[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
};

/* Mask LUT parameters (extmul, extoff, offset, scaler, mul) in the order
 * MaskX, MaskY, MaskB, MaskDcX, MaskDcY, MaskDcB (clbutter_comparator.cpp:994-1064). */
static const float kMaskParams[6][5] = {
    {0.975741017749f, -4.25328244168f, 0.454909521427f, 0.0738288224836f, 20.8029176447f},
    {0.373995618954f, 1.5307267433f, 0.911952641929f, 1.1731667845f, 16.2447033988f},
    {0.61582234137f, -4.25376118646f, 1.05105070921f, 0.47434643535f, 31.1444967089f},
    {1.79116943438f, -3.86797479189f, 0.670960225853f, 0.486575865525f, 20.4563479139f},
    {0.212223514236f, -3.65647120524f, 1.73396799447f, 0.170392660501f, 21.6566724788f},
    {0.349376011816f, -0.894711072781f, 0.901647926679f, 0.380086095024f, 18.0373825149f},
};

static int fix16(double x) { return (int)(x * 65536.0 + 0.5); }

void gzo_init(void) {
  if (g_inited) return;
  for (int i = 0; i < 256; ++i) {
    g_srgb[i] = i < 11 ? i / 12.92 : 255.0 * pow(((i / 255.0) + 0.055) / 1.055, 2.4);
    /* libjpeg jdcolor.c build_ycc_rgb_table, SCALEBITS 16 */
    const int x = i - 128;
    g_cr_r[i] = (fix16(1.40200) * x + 32768) >> 16;
    g_cb_b[i] = (fix16(1.77200) * x + 32768) >> 16;
    g_cr_g[i] = -fix16(0.71414) * x;
    g_cb_g[i] = -fix16(0.34414) * x + 32768;
  }
  {
    const float dx_off = 11.38708334481672f, dx_inc = 14.550189611520716f;
    const float dy_off = 1.4103373714040413f, dy_inc = 0.7084088867024f;
    const float lf_inc = 5.2511644570349185f;
    g_hf_dx[0] = 0.0f; g_hf_dx[1] = dx_off;
    g_hf_dy[0] = 0.0f; g_hf_dy[1] = dy_off;
    g_lf_dy[0] = 0.0f;
    for (int i = 2; i < 21; ++i) {
      g_hf_dx[i] = g_hf_dx[i - 1] + dx_inc;
      g_hf_dy[i] = g_hf_dy[i - 1] + dy_inc;
    }
    for (int i = 1; i < 21; ++i) g_lf_dy[i] = g_lf_dy[i - 1] + lf_inc;
  }
  for (int m = 0; m < 6; ++m) {
    const float extmul = kMaskParams[m][0], extoff = kMaskParams[m][1];
    const float offset = kMaskParams[m][2], scaler = kMaskParams[m][3];
    const float mul = kMaskParams[m][4];
    for (size_t i = 0; i < 512; ++i) {
      const float c = (float)(mul / ((0.01 * scaler * i) + offset));
      float v = (float)(1.0 + extmul * (c + extoff));
      g_mask_lut[m][i] = v * v;
    }
  }
  g_inited = 1;
}

double gzo_srgb8_to_linear(int v) { gzo_init(); return g_srgb[v & 255]; }

/* ------------------------------------------------------------------------ */
/* Pixels: IDCT and colour                                                   */
/* ------------------------------------------------------------------------ */

/* kIDCTMatrix of guetzli/idct.cc:29-38 (libjpeg-compatible 13-bit constants). */
static const int kIdctM[64] = {
    8192, 11363, 10703, 9633,   8192,  6437,   4433,   2260,   8192, 9633,  4433,  -2259, -8192,
    -11362, -10704, -6436, 8192, 6437, -4433,  -11362, -8192, 2261,   10704,  9633, 8192,  2260,
    -10703, -6436, 8192, 9633,  -4433, -11363, 8192,   -2260, -10703, 6436,   8192, -9633, -4433,
    11363,  8192,  -6437, -4433, 11362, -8192, -2261,  10704, -9633,  8192,   -9633, 4433, 2259,
    -8192,  11362, -10704, 6436, 8192,  -11363, 10703, -9633, 8192,   -6437,  4433,  -2260,
};

/* out[x] = sum_u M[8x+u] * in[u*stride], 32-bit wrap-around (idct.cc:41-137). */
static void idct_1d(const int* in, int stride, int* out) {
  for (int x = 0; x < 8; ++x) {
    unsigned acc = 0;
    for (int u = 0; u < 8; ++u) acc += (unsigned)(kIdctM[8 * x + u] * in[u * stride]);
    out[x] = (int)acc;
  }
}

void gzo_block_idct(const int16_t* block, uint8_t* out) {
  int col[64], tmp[8], in[8];
  for (int x = 0; x < 8; ++x) {
    for (int u = 0; u < 8; ++u) in[u] = block[8 * u + x];
    idct_1d(in, 1, tmp);
    for (int y = 0; y < 8; ++y) col[8 * y + x] = (int16_t)((tmp[y] + (1 << 10)) >> 11);
  }
  for (int y = 0; y < 8; ++y) {
    idct_1d(&col[8 * y], 1, tmp);
    for (int x = 0; x < 8; ++x) {
      int v = (tmp[x] + (257 << 17)) >> 18;
      out[8 * y + x] = (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
  }
}

static int clamp255(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }

void gzo_ycbcr_to_rgb(uint8_t* px) {
  gzo_init();
  const int y = px[0], cb = px[1], cr = px[2];
  px[0] = (uint8_t)clamp255(y + g_cr_r[cr]);
  px[1] = (uint8_t)clamp255(y + ((g_cr_g[cr] + g_cb_g[cb]) >> 16));
  px[2] = (uint8_t)clamp255(y + g_cb_b[cb]);
}

void gzo_coeffs_to_srgb(int w, int h, const int16_t* coeffs, uint8_t* rgb) {
  const int bw = (w + 7) / 8, bh = (h + 7) / 8;
  const size_t nb = (size_t)bw * bh;
  uint8_t pix[64];
  for (int c = 0; c < 3; ++c)
    for (int by = 0; by < bh; ++by)
      for (int bx = 0; bx < bw; ++bx) {
        gzo_block_idct(&coeffs[(c * nb + (size_t)by * bw + bx) * 64], pix);
        for (int iy = 0; iy < 8; ++iy)
          for (int ix = 0; ix < 8; ++ix) {
            const int x = 8 * bx + ix, y = 8 * by + iy;
            if (x < w && y < h) {
              /* pixels_ = idct << 4 ; ToPixels: (p + 8 - (x&1)) >> 4 == idct */
              const int p = pix[8 * iy + ix] << 4;
              rgb[3 * ((size_t)y * w + x) + c] = (uint8_t)((p + 8 - (x & 1)) >> 4);
            }
          }
      }
  for (size_t p = 0; p < (size_t)w * h; ++p) gzo_ycbcr_to_rgb(&rgb[3 * p]);
}

void gzo_srgb_to_linear_planes(int w, int h, const uint8_t* rgb, float* planes) {
  gzo_init();
  const size_t n = (size_t)w * h;
  for (int c = 0; c < 3; ++c)
    for (size_t i = 0; i < n; ++i) planes[c * n + i] = (float)g_srgb[rgb[3 * i + c]];
}

/* ------------------------------------------------------------------------ */
/* Separable blur (clbutter_comparator.cpp:25-94)                            */
/* ------------------------------------------------------------------------ */

static void convolution(size_t xsize, size_t ysize, size_t xstep, size_t len, size_t offset,
                       const float* mult, const float* inp, float border_ratio,
                       float* result) {
  float weight_no_border = 0;
  for (size_t j = 0; j <= 2 * offset; ++j) weight_no_border += mult[j];
  for (size_t x = 0, ox = 0; x < xsize; x += xstep, ox++) {
    const int minx = x < offset ? 0 : (int)(x - offset);
    const int maxx = (int)((xsize < x + len - offset ? xsize : x + len - offset) - 1);
    float weight = 0.0f;
    for (int j = minx; j <= maxx; ++j) weight += mult[j - (int)x + (int)offset];
    weight = (float)((1.0 - border_ratio) * weight + border_ratio * weight_no_border);
    const float scale = (float)(1.0 / weight);
    for (size_t y = 0; y < ysize; ++y) {
      float sum = 0.0f;
      for (int j = minx; j <= maxx; ++j) sum += inp[y * xsize + j] * mult[j - (int)x + (int)offset];
      result[ox * ysize + y] = sum * scale;
    }
  }
}

void gzo_blur(size_t xsize, size_t ysize, float* channel, float sigma, float border_ratio) {
  const float m = 2.25f;
  const float scaler = (float)(-1.0 / (2 * sigma * sigma));
  int diff = (int)(m * fabsf(sigma));
  if (diff < 1) diff = 1;
  const int expn_size = 2 * diff + 1;
  float expn[256];
  for (int i = -diff; i <= diff; ++i) expn[i + diff] = (float)exp(scaler * i * i);
  int xstep = (int)(sigma / 3);
  if (xstep < 1) xstep = 1;
  const size_t dxsize = (xsize + xstep - 1) / xstep;
  const size_t dysize = (ysize + xstep - 1) / xstep;
  float* tmp = (float*)malloc(sizeof(float) * dxsize * ysize);
  convolution(xsize, ysize, xstep, expn_size, diff, expn, channel, border_ratio, tmp);
  float* down = channel;
  if (xstep > 1) down = (float*)malloc(sizeof(float) * dxsize * dysize);
  convolution(ysize, dxsize, xstep, expn_size, diff, expn, tmp, border_ratio, down);
  if (xstep > 1) {
    for (size_t y = 0; y < ysize; y++)
      for (size_t x = 0; x < xsize; x++)
        channel[y * xsize + x] = down[(y / xstep) * dxsize + (x / xstep)];
    free(down);
  }
  free(tmp);
}

/* ------------------------------------------------------------------------ */
/* Opsin dynamics (clbutter_comparator.cpp:690-912)                          */
/* ------------------------------------------------------------------------ */

static const float kOpsinMix[12] = {
    0.348036746003f, 0.577814843137f, 0.0544556093735f, 0.774145581713f,
    0.26922717275f,  0.767247733938f, 0.0366922708552f, 0.920130265014f,
    0.0882062883536f, 0.158581714673f, 0.712857943858f, 10.6524069248f,
};

static void opsin_absorbance(const float in[3], float out[3]) {
  const float* m = kOpsinMix;
  out[0] = m[0] * in[0] + m[1] * in[1] + m[2] * in[2] + m[3];
  out[1] = m[4] * in[0] + m[5] * in[1] + m[6] * in[2] + m[7];
  out[2] = m[8] * in[0] + m[9] * in[1] + m[10] * in[2] + m[11];
}

static float clenshaw6(float x, const float* c) {
  float b1 = 0.0f, b2 = 0.0f;
  for (int k = 5; k >= 1; --k) {
    const float xb1 = x * b1;
    const float t = (xb1 + xb1) - b2 + c[k];
    b2 = b1;
    b1 = t;
  }
  const float xb1 = x * b1;
  return xb1 - b2 + c[0];
}

static float gamma_poly(float x) {
  static const float p[6] = {881.979476556478289f, 1496.058452015812463f, 908.662212739659481f,
                             373.566100223287378f, 85.840860336314364f,   6.683258861509244f};
  static const float q[6] = {12.262350348616792f, 20.557285797683576f, 12.161463238367844f,
                             4.711532733641639f,  0.899112889751053f,  0.035662329617191f};
  const float lo = 0.770000000000000f, hi = 274.579999999999984f;
  const float x01 = (x - lo) / (hi - lo);
  const float xc = (float)(2.0 * x01 - 1.0);
  const float yp = clenshaw6(xc, p);
  const float yq = clenshaw6(xc, q);
  if (yq == 0.0f) return 0.0f;
  return yp / yq;
}

void gzo_opsin_dynamics(size_t xsize, size_t ysize, float* planes) {
  const size_t n = xsize * ysize;
  float* blurred = (float*)malloc(sizeof(float) * 3 * n);
  memcpy(blurred, planes, sizeof(float) * 3 * n);
  for (int c = 0; c < 3; ++c) gzo_blur(xsize, ysize, blurred + c * n, 1.1f, 0.0f);
  for (size_t i = 0; i < n; ++i) {
    float pre[3] = {blurred[i], blurred[n + i], blurred[2 * n + i]};
    float mixed[3], sens[3];
    opsin_absorbance(pre, mixed);
    for (int c = 0; c < 3; ++c) sens[c] = gamma_poly(mixed[c]) / mixed[c];
    float cur[3] = {planes[i], planes[n + i], planes[2 * n + i]};
    float cm[3];
    opsin_absorbance(cur, cm);
    for (int c = 0; c < 3; ++c) cm[c] *= sens[c];
    planes[i] = 1.01611726948f * cm[0] - 0.982482243696f * cm[1];
    planes[n + i] = 1.43571362627f * cm[0] + 0.896039849412f * cm[1];
    planes[2 * n + i] = cm[2];
  }
  free(blurred);
}

/* ------------------------------------------------------------------------ */
/* High intensity change masking (clbutter_comparator.cpp:729-781)           */
/* ------------------------------------------------------------------------ */

void gzo_mask_high_intensity_change(size_t xsize, size_t ysize, const float* c0,
                                    const float* c1, float* xyb0, float* xyb1) {
  const size_t n = xsize * ysize;
  for (size_t y = 0; y < ysize; ++y)
    for (size_t x = 0; x < xsize; ++x) {
      const size_t ix = y * xsize + x;
      float ave[3];
      for (int c = 0; c < 3; ++c) ave[c] = (float)((c0[c * n + ix] + c1[c * n + ix]) * 0.5);
      float sqr_max_diff = -1;
      const long off[4] = {-1, 1, -(long)xsize, (long)xsize};
      const int border[4] = {x == 0, x + 1 == xsize, y == 0, y + 1 == ysize};
      for (int d = 0; d < 4; ++d) {
        if (border[d]) continue;
        const size_t ix2 = (size_t)((long)ix + off[d]);
        float diff = (float)(0.5 * (c0[n + ix2] + c1[n + ix2]) - ave[1]);
        diff *= diff;
        if (sqr_max_diff < diff) sqr_max_diff = diff;
      }
      const float kRX = 275.19165240059317f, kRY = 18599.41286306991f;
      const float kRZ = 410.8995306951065f, kChroma = 106.95800948271017f;
      const float chroma_scale = kChroma / (ave[1] + kChroma);
      const float mix[3] = {chroma_scale * kRX / (sqr_max_diff + kRX),
                            kRY / (sqr_max_diff + kRY),
                            chroma_scale * kRZ / (sqr_max_diff + kRZ)};
      for (int c = 0; c < 3; ++c) {
        xyb0[c * n + ix] = mix[c] * c0[c * n + ix] + (1 - mix[c]) * ave[c];
        xyb1[c * n + ix] = mix[c] * c1[c * n + ix] + (1 - mix[c]) * ave[c];
      }
    }
}

/* ------------------------------------------------------------------------ */
/* Colour-distance helpers (clbutter_comparator.cpp:195-299)                 */
/* ------------------------------------------------------------------------ */

static float interp(const float* a, int size, float sx) {
  const float ix = fabsf(sx);
  const int base = (int)ix;
  float res;
  if (base >= size - 1) {
    res = a[size - 1];
  } else {
    const float mix = ix - base;
    res = a[base] + mix * (a[base + 1] - a[base]);
  }
  if (sx < 0) res = -res;
  return res;
}

static float interp_clamp_neg(const float* a, int size, float sx) {
  if (sx < 0) sx = 0;
  const float ix = fabsf(sx);
  const int base = (int)ix;
  if (base >= size - 1) return a[size - 1];
  const float mix = ix - base;
  return a[base] + mix * (a[base + 1] - a[base]);
}

static void lowfreq_vals(float x, float y, float z, float* vx, float* vy, float* vz) {
  z += 0.0812519812628f * y;
  *vz = z * 7.34905756986f;
  *vx = x * 6.64482198135f;
  *vy = interp(g_lf_dy, 21, y * 0.837846224276f);
}

static void lowfreq_sq_acc(float r0, float g0, float b0, float r1, float g1, float b1,
                           float factor, float res[3]) {
  float vx0, vy0, vz0;
  lowfreq_vals(r0, g0, b0, &vx0, &vy0, &vz0);
  if (r1 == 0.0 && g1 == 0.0 && b1 == 0.0) {
    res[0] += factor * vx0 * vx0;
    res[1] += factor * vy0 * vy0;
    res[2] += factor * vz0 * vz0;
    return;
  }
  float vx1, vy1, vz1;
  lowfreq_vals(r1, g1, b1, &vx1, &vy1, &vz1);
  const float dx = vx0 - vx1, dy = vy0 - vy1, dz = vz0 - vz1;
  res[0] += factor * dx * dx;
  res[1] += factor * dy * dy;
  res[2] += factor * dz * dz;
}

static void xyb_to_vals(float x, float y, float z, float* vx, float* vy, float* vz) {
  *vx = interp(g_hf_dx, 21, x * 0.758304045695f);
  *vy = interp(g_hf_dy, 21, y * 2.28148649801f);
  *vz = 1.87816926918f * z;
}

/* ------------------------------------------------------------------------ */
/* 8-point FFTs (D. J. Bernstein's in-place FFT as used by butteraugli,      */
/* clbutter_comparator.cpp:320-546).  re/im split arrays; the butterfly       */
/* sequence is kept exactly because float results depend on it.              */
/* ------------------------------------------------------------------------ */

#define DEF_FFT(T, SUF)                                                                  \
  static void fft4_##SUF(T* re, T* im) {                                                 \
    T t1, t2, t3, t4, t5, t6, t7, t8;                                                    \
    t5 = re[2]; t1 = re[0] - t5; t7 = re[3]; t5 += re[0]; t3 = re[1] - t7; t7 += re[1]; \
    t8 = t5 + t7; re[0] = t8; t5 -= t7; re[1] = t5;                                      \
    t6 = im[2]; t2 = im[0] - t6; t6 += im[0]; t5 = im[3];                                \
    im[2] = t2 + t3; t2 -= t3; im[3] = t2;                                               \
    t4 = im[1] - t5; re[3] = t1 + t4; t1 -= t4; re[2] = t1;                              \
    t5 += im[1]; im[0] = t6 + t5; t6 -= t5; im[1] = t6;                                  \
  }                                                                                      \
  static void reorder8_##SUF(T* re, T* im) {                                             \
    T tr = re[2], ti = im[2];                                                            \
    re[2] = re[3]; im[2] = im[3]; re[3] = re[5]; im[3] = im[5];                          \
    re[5] = re[7]; im[5] = im[7]; re[7] = re[4]; im[7] = im[4];                          \
    re[4] = re[1]; im[4] = im[1]; re[1] = re[6]; im[1] = im[6];                          \
    re[6] = tr; im[6] = ti;                                                              \
  }                                                                                      \
  static void fft8_##SUF(T* re, T* im, T sqrt_half) {                                   \
    T t1, t2, t3, t4, t5, t6, t7, t8;                                                    \
    t7 = im[4]; t4 = im[0] - t7; t7 += im[0]; im[0] = t7;                                \
    t8 = re[6]; t5 = re[2] - t8; t8 += re[2]; re[2] = t8;                                \
    t7 = im[6]; im[6] = t4 - t5; t4 += t5; im[4] = t4;                                   \
    t6 = im[2] - t7; t7 += im[2]; im[2] = t7;                                            \
    t8 = re[4]; t3 = re[0] - t8; t8 += re[0]; re[0] = t8;                                \
    re[4] = t3 - t6; t3 += t6; re[6] = t3;                                               \
    t7 = re[5]; t3 = re[1] - t7; t7 += re[1]; re[1] = t7;                                \
    t8 = im[7]; t6 = im[3] - t8; t8 += im[3]; im[3] = t8;                                \
    t1 = t3 - t6; t3 += t6;                                                              \
    t7 = im[5]; t4 = im[1] - t7; t7 += im[1]; im[1] = t7;                                \
    t8 = re[7]; t5 = re[3] - t8; t8 += re[3]; re[3] = t8;                                \
    t2 = t4 - t5; t4 += t5;                                                              \
    t6 = t1 - t4; t8 = sqrt_half; t6 *= t8; re[5] = re[4] - t6;                          \
    t1 += t4; t1 *= t8; im[5] = im[4] - t1;                                              \
    t6 += re[4]; re[4] = t6; t1 += im[4]; im[4] = t1;                                    \
    t5 = t2 - t3; t5 *= t8; im[7] = im[6] - t5;                                          \
    t2 += t3; t2 *= t8; re[7] = re[6] - t2;                                              \
    t2 += re[6]; re[6] = t2; t5 += im[6]; im[6] = t5;                                    \
    fft4_##SUF(re, im);                                                                  \
    reorder8_##SUF(re, im);                                                              \
  }                                                                                      \
  static void real_fft8_##SUF(const T* in, T* re, T* im, T sqrt_half) {                 \
    T t1, t2, t3, t5, t6, t7, t8;                                                        \
    t8 = in[6]; t5 = in[2] - t8; t8 += in[2]; re[2] = t8; im[6] = -t5; im[4] = t5;       \
    t8 = in[4]; t3 = in[0] - t8; t8 += in[0]; re[0] = t8; re[4] = t3; re[6] = t3;        \
    t7 = in[5]; t3 = in[1] - t7; t7 += in[1]; re[1] = t7;                                \
    t8 = in[7]; t5 = in[3] - t8; t8 += in[3]; re[3] = t8;                                \
    t2 = -t5; t6 = t3 - t5; t8 = sqrt_half; t6 *= t8; re[5] = re[4] - t6;                \
    t1 = t3 + t5; t1 *= t8; im[5] = im[4] - t1;                                          \
    t6 += re[4]; re[4] = t6; t1 += im[4]; im[4] = t1;                                    \
    t5 = t2 - t3; t5 *= t8; im[7] = im[6] - t5;                                          \
    t2 += t3; t2 *= t8; re[7] = re[6] - t2;                                              \
    t2 += re[6]; re[6] = t2; t5 += im[6]; im[6] = t5;                                    \
    t5 = re[2]; t1 = re[0] - t5; t7 = re[3]; t5 += re[0]; t3 = re[1] - t7; t7 += re[1];  \
    t8 = t5 + t7; re[0] = t8; t5 -= t7; re[1] = t5;                                      \
    im[2] = t3; im[3] = -t3; re[3] = t1; re[2] = t1; im[0] = 0; im[1] = 0;               \
    reorder8_##SUF(re, im);                                                              \
  }                                                                                      \
  /* ButteraugliFFTSquared: fills block[4..36] with |F|^2 * 0.000064 */                 \
  static void fft_squared_##SUF(T* block, T sqrt_half) {                                 \
    T re[64], im[64], r0[8], r1[8];                                                      \
    const T global_mul = (T)0.000064;                                                    \
    for (int y = 0; y < 8; ++y) real_fft8_##SUF(block + 8 * y, re + 8 * y, im + 8 * y,   \
                                                sqrt_half);                              \
    for (int i = 0; i < 8; ++i)                                                          \
      for (int j = 0; j < i; ++j) {                                                      \
        T a = re[8 * i + j]; re[8 * i + j] = re[8 * j + i]; re[8 * j + i] = a;           \
        a = im[8 * i + j]; im[8 * i + j] = im[8 * j + i]; im[8 * j + i] = a;             \
      }                                                                                  \
    for (int x = 0; x < 8; ++x) { r0[x] = re[x]; r1[x] = re[32 + x]; }                   \
    real_fft8_##SUF(r0, re, im, sqrt_half);                                              \
    real_fft8_##SUF(r1, re + 32, im + 32, sqrt_half);                                    \
    for (int y = 1; y < 4; ++y) fft8_##SUF(re + 8 * y, im + 8 * y, sqrt_half);           \
    for (int i = 4; i < 37; ++i) {                                                       \
      block[i] = re[i] * re[i] + im[i] * im[i];                                          \
      block[i] *= global_mul;                                                            \
    }                                                                                    \
  }

DEF_FFT(float, f)
DEF_FFT(double, d)

static const float kSqrtHalfF = 0.70710678118654752440084436210484903f;
static const double kSqrtHalfD = 0.70710678118654752440084436210484903;

static float remove_range_f(float v, float range) {
  if (v >= -range && v < range) return 0;
  return v < 0 ? v + range : v - range;
}

/* ButteraugliBlockDiffOpt, clbutter_comparator.cpp:551-633 (float) */
static void block_diff_float(float* xyb0, float* xyb1, float dc[3], float ac[3], float edge[3]) {
  float avg[3] = {0, 0, 0};
  float avg_edge[3][4] = {{0}};
  for (int i = 0; i < 192; ++i) {
    const float d = xyb0[i] - xyb1[i];
    const int c = i / 64, k = i % 64, kx = k % 8, ky = k / 8;
    avg[c] += d / 64.0f;
    const int h = ky == 0 ? 1 : ky == 7 ? 3 : -1;
    const int v = kx == 0 ? 0 : kx == 7 ? 2 : -1;
    if (h >= 0) avg_edge[c][h] += d / 8.0f;
    if (v >= 0) avg_edge[c][v] += d / 8.0f;
  }
  const float csf0 = (float)kBlockCsf[0];
  lowfreq_sq_acc(avg[0], avg[1], avg[2], 0, 0, 0, csf0, dc);
  for (int i = 0; i < 4; ++i)
    lowfreq_sq_acc(avg_edge[0][i], avg_edge[1][i], avg_edge[2][i], 0, 0, 0, csf0, edge);
  for (int i = 0; i < 192; ++i) {
    const float a = (xyb0[i] + xyb1[i]) / 2;
    const float hd = (xyb0[i] - xyb1[i]) / 2;
    xyb0[i] = a;
    xyb1[i] = hd;
  }
  float* y_avg = xyb0 + 64;
  float* x_hd = xyb1;
  float* y_hd = xyb1 + 64;
  float* z_hd = xyb1 + 128;
  fft_squared_f(y_avg, kSqrtHalfF);
  fft_squared_f(x_hd, kSqrtHalfF);
  fft_squared_f(y_hd, kSqrtHalfF);
  fft_squared_f(z_hd, kSqrtHalfF);
  const float xmul = 64.8f, ymul = 1.753123908348329f, ymul2 = 1.51983458269f, zmul = 2.4f;
  for (int i = 4; i < 37; ++i) {
    const float d = (float)kBlockCsf[i];
    ac[0] += d * xmul * x_hd[i];
    ac[2] += d * zmul * z_hd[i];
    y_avg[i] = sqrtf(y_avg[i]);
    y_hd[i] = sqrtf(y_hd[i]);
    float y0 = y_avg[i] - y_hd[i];
    float y1 = y_avg[i] + y_hd[i];
    y0 = remove_range_f(y0, 0.04f);
    y1 = remove_range_f(y1, 0.04f);
    if (y0 != y1) {
      const float v0 = interp(g_hf_dy, 21, y0 * ymul2);
      const float v1 = interp(g_hf_dy, 21, y1 * ymul2);
      const float vy = ymul * (v0 - v1);
      ac[1] += d * vy * vy;
    }
  }
}

/* ------------------------------------------------------------------------ */
/* Double-precision helpers for ButteraugliBlockDiff (butteraugli.cc)        */
/* ------------------------------------------------------------------------ */

static double g_hf_dy_d[21], g_lf_dy_d[21];
static int g_d_inited = 0;
static void init_double_tables(void) {
  if (g_d_inited) return;
  g_hf_dy_d[0] = 0.0; g_hf_dy_d[1] = 1.4103373714040413;
  for (int i = 2; i < 21; ++i) g_hf_dy_d[i] = g_hf_dy_d[i - 1] + 0.7084088867024;
  g_lf_dy_d[0] = 0.0;
  for (int i = 1; i < 21; ++i) g_lf_dy_d[i] = g_lf_dy_d[i - 1] + 5.2511644570349185;
  g_d_inited = 1;
}

static double interp_d(const double* a, int size, double sx) {
  const double ix = fabs(sx);
  const int base = (int)ix;
  double res;
  if (base >= size - 1) {
    res = a[size - 1];
  } else {
    const double mix = ix - base;
    res = a[base] + mix * (a[base + 1] - a[base]);
  }
  if (sx < 0) res = -res;
  return res;
}

static void lowfreq_sq_acc_zero_d(double x, double y, double z, double factor, double res[3]) {
  z += 0.0812519812628 * y;
  const double vz = z * 7.34905756986;
  const double vx = x * 6.64482198135;
  const double vy = interp_d(g_lf_dy_d, 21, y * 0.837846224276);
  res[0] += factor * vx * vx;
  res[1] += factor * vy * vy;
  res[2] += factor * vz * vz;
}

static double remove_range_d(double v, double range) {
  if (v >= -range && v < range) return 0;
  return v < 0 ? v + range : v - range;
}

void gzo_block_diff_double(double* xyb0, double* xyb1, double dc[3], double ac[3],
                           double edge[3]) {
  init_double_tables();
  double avg[3] = {0, 0, 0};
  double avg_edge[3][4] = {{0}};
  for (int i = 0; i < 192; ++i) {
    const double d = xyb0[i] - xyb1[i];
    const int c = i / 64, k = i % 64, kx = k % 8, ky = k / 8;
    avg[c] += d / 64;
    const int h = ky == 0 ? 1 : ky == 7 ? 3 : -1;
    const int v = kx == 0 ? 0 : kx == 7 ? 2 : -1;
    if (h >= 0) avg_edge[c][h] += d / 8;
    if (v >= 0) avg_edge[c][v] += d / 8;
  }
  /* XybDiffLowFreqSquaredAccumulate with r1=g1=b1=0 (butteraugli.cc:328-340) */
  lowfreq_sq_acc_zero_d(avg[0], avg[1], avg[2], kBlockCsf[0], dc);
  for (int i = 0; i < 4; ++i)
    lowfreq_sq_acc_zero_d(avg_edge[0][i], avg_edge[1][i], avg_edge[2][i], kBlockCsf[0], edge);
  for (int i = 0; i < 192; ++i) {
    const double a = (xyb0[i] + xyb1[i]) / 2;
    const double hd = (xyb0[i] - xyb1[i]) / 2;
    xyb0[i] = a;
    xyb1[i] = hd;
  }
  double* y_avg = xyb0 + 64;
  double* x_hd = xyb1;
  double* y_hd = xyb1 + 64;
  double* z_hd = xyb1 + 128;
  fft_squared_d(y_avg, kSqrtHalfD);
  fft_squared_d(x_hd, kSqrtHalfD);
  fft_squared_d(y_hd, kSqrtHalfD);
  fft_squared_d(z_hd, kSqrtHalfD);
  const double xmul = 64.8, ymul = 1.753123908348329, ymul2 = 1.51983458269, zmul = 2.4;
  for (int i = 4; i < 37; ++i) {
    const double d = kBlockCsf[i];
    ac[0] += d * xmul * x_hd[i];
    ac[2] += d * zmul * z_hd[i];
    y_avg[i] = sqrt(y_avg[i]);
    y_hd[i] = sqrt(y_hd[i]);
    double y0 = y_avg[i] - y_hd[i];
    double y1 = y_avg[i] + y_hd[i];
    y0 = remove_range_d(y0, 0.04);
    y1 = remove_range_d(y1, 0.04);
    if (y0 != y1) {
      const double v0 = interp_d(g_hf_dy_d, 21, y0 * ymul2);
      const double v1 = interp_d(g_hf_dy_d, 21, y1 * ymul2);
      const double vy = ymul * (v0 - v1);
      ac[1] += d * vy * vy;
    }
  }
}

/* ------------------------------------------------------------------------ */
/* Edge detectors (clbutter_comparator.cpp:638-687, 1456-1540)               */
/* ------------------------------------------------------------------------ */

static void corner_edge_diff(size_t px, size_t py, size_t xsize, size_t ysize, const float* b0,
                             const float* b1, float diff[3]) {
  const size_t n = xsize * ysize;
  int count = 0;
  float local[3] = {0, 0, 0};
  const float w = 0.711100840192f;
  static const size_t off[4][2] = {{0, 0}, {0, 7}, {7, 0}, {7, 7}};
  for (int k = 0; k < 4; ++k) {
    const size_t step = 3;
    const size_t x = px + off[k][0], y = py + off[k][1];
    if (x >= step && x + step < xsize) {
      const size_t ix = y * xsize + (x - step), ix2 = ix + 2 * step;
      lowfreq_sq_acc(w * (b0[ix] - b0[ix2]), w * (b0[n + ix] - b0[n + ix2]),
                     w * (b0[2 * n + ix] - b0[2 * n + ix2]), w * (b1[ix] - b1[ix2]),
                     w * (b1[n + ix] - b1[n + ix2]), w * (b1[2 * n + ix] - b1[2 * n + ix2]),
                     1.0f, local);
      ++count;
    }
    if (y >= step && y + step < ysize) {
      const size_t ix = (y - step) * xsize + x, ix2 = ix + 2 * step * xsize;
      lowfreq_sq_acc(w * (b0[ix] - b0[ix2]), w * (b0[n + ix] - b0[n + ix2]),
                     w * (b0[2 * n + ix] - b0[2 * n + ix2]), w * (b1[ix] - b1[ix2]),
                     w * (b1[n + ix] - b1[n + ix2]), w * (b1[2 * n + ix] - b1[2 * n + ix2]),
                     1.0f, local);
      ++count;
    }
  }
  const float weight = 0.01617112696f;
  const float mul = (float)(weight * 8.0 / count);
  for (int i = 0; i < 3; ++i) diff[i] += mul * local[i];
}

/* ------------------------------------------------------------------------ */
/* Mask (clbutter_comparator.cpp:1070-1264, butteraugli.cc:1379-1438)        */
/* ------------------------------------------------------------------------ */

static void min_square_val4(size_t xsize, size_t ysize, float* values) {
  const size_t sq = 4;
  float* tmp = (float*)malloc(sizeof(float) * xsize * ysize);
  for (size_t y = 0; y < ysize; ++y) {
    const size_t maxh = ysize < y + sq ? ysize : y + sq;
    for (size_t x = 0; x < xsize; ++x) {
      float mn = values[x + y * xsize];
      for (size_t j = y + 1; j < maxh; ++j) {
        const float t = values[x + j * xsize];
        if (t < mn) mn = t;
      }
      tmp[x + y * xsize] = mn;
    }
  }
  for (size_t x = 0; x < xsize; ++x) {
    const size_t maxw = xsize < x + sq ? xsize : x + sq;
    for (size_t y = 0; y < ysize; ++y) {
      float mn = tmp[x + y * xsize];
      for (size_t j = x + 1; j < maxw; ++j) {
        const float t = tmp[j + y * xsize];
        if (t < mn) mn = t;
      }
      values[x + y * xsize] = mn;
    }
  }
  free(tmp);
}

/* _Average5x5 (butteraugli.cc:1379-1438), written per output element: the
 * reference scatters into result in an order that, for each output, adds
 * (row above: left*w, centre, right*w), (same row: left, right), (row below:
 * left*w, centre, right*w). */
static void average5x5(int xsize, int ysize, float* d) {
  if (xsize < 4 || ysize < 4) return;
  const float w = 0.679144890667f;
  const float scale = 1.0f / (5.0f + 4 * w);
  const size_t n = (size_t)xsize * ysize;
  float* r = (float*)malloc(sizeof(float) * n);
  float* dw = (float*)malloc(sizeof(float) * n);
  for (size_t i = 0; i < n; ++i) dw[i] = d[i] * w;
  for (int y = 0; y < ysize; ++y)
    for (int x = 0; x < xsize; ++x) {
      float acc = d[y * xsize + x];
      if (y > 0) {
        const int row = (y - 1) * xsize;
        if (x > 0) acc += dw[row + x - 1];
        acc += d[row + x];
        if (x + 1 < xsize) acc += dw[row + x + 1];
      }
      if (x > 0) acc += d[y * xsize + x - 1];
      if (x + 1 < xsize) acc += d[y * xsize + x + 1];
      if (y + 1 < ysize) {
        const int row = (y + 1) * xsize;
        if (x > 0) acc += dw[row + x - 1];
        acc += d[row + x];
        if (x + 1 < xsize) acc += dw[row + x + 1];
      }
      r[y * xsize + x] = acc;
    }
  for (size_t i = 0; i < n; ++i) d[i] = r[i] * scale;
  free(r);
  free(dw);
}

static void diff_precompute(const float* xyb0, const float* xyb1, size_t xsize, size_t ysize,
                            float* mask) {
  const size_t n = xsize * ysize;
  float h0[3] = {0}, v0[3] = {0}, h1[3] = {0}, v1[3] = {0};
  for (size_t y = 0; y < ysize; ++y)
    for (size_t x = 0; x < xsize; ++x) {
      const size_t ix = x + xsize * y;
      size_t ix2 = x + 1 < xsize ? ix + 1 : ix - 1;
      xyb_to_vals(xyb0[ix] - xyb0[ix2], xyb0[n + ix] - xyb0[n + ix2],
                  xyb0[2 * n + ix] - xyb0[2 * n + ix2], &h0[0], &h0[1], &h0[2]);
      xyb_to_vals(xyb1[ix] - xyb1[ix2], xyb1[n + ix] - xyb1[n + ix2],
                  xyb1[2 * n + ix] - xyb1[2 * n + ix2], &h1[0], &h1[1], &h1[2]);
      ix2 = y + 1 < ysize ? ix + xsize : ix - xsize;
      xyb_to_vals(xyb0[ix] - xyb0[ix2], xyb0[n + ix] - xyb0[n + ix2],
                  xyb0[2 * n + ix] - xyb0[2 * n + ix2], &v0[0], &v0[1], &v0[2]);
      xyb_to_vals(xyb1[ix] - xyb1[ix2], xyb1[n + ix] - xyb1[n + ix2],
                  xyb1[2 * n + ix] - xyb1[2 * n + ix2], &v1[0], &v1[1], &v1[2]);
      for (int i = 0; i < 3; ++i) {
        const float s0 = fabsf(h0[i]) + fabsf(v0[i]);
        const float s1 = fabsf(h1[i]) + fabsf(v1[i]);
        mask[i * n + ix] = s0 < s1 ? s0 : s1;
      }
    }
}

void gzo_mask(size_t xsize, size_t ysize, const float* xyb0, const float* xyb1, float* mask,
              float* mask_dc) {
  gzo_init();
  const size_t n = xsize * ysize;
  diff_precompute(xyb0, xyb1, xsize, ysize, mask);
  static const float sigma[3] = {9.65781083553f, 14.2644604355f, 4.53358927369f};
  for (int i = 0; i < 3; ++i) {
    average5x5((int)xsize, (int)ysize, mask + i * n);
    min_square_val4(xsize, ysize, mask + i * n);
    gzo_blur(xsize, ysize, mask + i * n, sigma[i], 0.0f);
  }
  const float w00 = 232.206464018f, w11 = 22.9455222245f, w22 = 503.962310606f;
  for (size_t i = 0; i < n; ++i) {
    const float p0 = w00 * mask[i], p1 = w11 * mask[n + i], p2 = w22 * mask[2 * n + i];
    mask[i] = interp_clamp_neg(g_mask_lut[0], 512, p0);
    mask[n + i] = interp_clamp_neg(g_mask_lut[1], 512, p1);
    mask[2 * n + i] = interp_clamp_neg(g_mask_lut[2], 512, p2);
    mask_dc[i] = interp_clamp_neg(g_mask_lut[3], 512, p0);
    mask_dc[n + i] = interp_clamp_neg(g_mask_lut[4], 512, p1);
    mask_dc[2 * n + i] = interp_clamp_neg(g_mask_lut[5], 512, p2);
  }
  const float gs = (float)(1.0 / 14.921561160295326f);
  const float gs2 = gs * gs;
  for (size_t i = 0; i < 3 * n; ++i) {
    mask[i] *= gs2;
    mask_dc[i] *= gs2;
  }
}

/* ------------------------------------------------------------------------ */
/* Full diffmap (clbutter_comparator.cpp:923-978, 1387-1565)                 */
/* ------------------------------------------------------------------------ */

int gzo_diffmap(size_t xsize, size_t ysize, float* xyb0, float* xyb1, float* distmap,
                gzo_stages* st) {
  gzo_init();
  if (xsize < 8 || ysize < 8) return 0;
  const size_t n = xsize * ysize, step = 3;
  const size_t rw = (xsize + step - 1) / step, rh = (ysize + step - 1) / step, rn = rw * rh;
  {
    float* c0 = (float*)malloc(sizeof(float) * 3 * n);
    float* c1 = (float*)malloc(sizeof(float) * 3 * n);
    memcpy(c0, xyb0, sizeof(float) * 3 * n);
    memcpy(c1, xyb1, sizeof(float) * 3 * n);
    gzo_mask_high_intensity_change(xsize, ysize, c0, c1, xyb0, xyb1);
    free(c0);
    free(c1);
  }
  if (st && st->mhic0) memcpy(st->mhic0, xyb0, sizeof(float) * 3 * n);
  if (st && st->mhic1) memcpy(st->mhic1, xyb1, sizeof(float) * 3 * n);

  float* edge = (float*)calloc(3 * rn, sizeof(float));
  float* dc = (float*)calloc(3 * rn, sizeof(float));
  float* ac = (float*)calloc(3 * rn, sizeof(float));
  float* b0 = (float*)malloc(sizeof(float) * 3 * n);
  float* b1 = (float*)malloc(sizeof(float) * 3 * n);

  /* EdgeDetectorMapOpt */
  {
    static const float s[3] = {1.5f, 0.586f, 0.4f};
    memcpy(b0, xyb0, sizeof(float) * 3 * n);
    memcpy(b1, xyb1, sizeof(float) * 3 * n);
    for (int i = 0; i < 3; ++i) {
      gzo_blur(xsize, ysize, b0 + i * n, s[i], 0.0f);
      gzo_blur(xsize, ysize, b1 + i * n, s[i], 0.0f);
    }
    for (size_t ry = 0; ry + (8 - step) < ysize; ry += step)
      for (size_t rx = 0; rx + (8 - step) < xsize; rx += step) {
        const size_t rix = (ry * rw + rx) / step;
        float d[3] = {0, 0, 0};
        corner_edge_diff(rx < xsize - 8 ? rx : xsize - 8, ry < ysize - 8 ? ry : ysize - 8, xsize,
                         ysize, b0, b1, d);
        for (int i = 0; i < 3; ++i) edge[3 * rix + i] = d[i];
      }
  }
  if (st && st->edge) memcpy(st->edge, edge, sizeof(float) * 3 * rn);

  /* BlockDiffMapOpt */
  for (size_t ry = 0; ry + (8 - step - 1) < ysize; ry += step)
    for (size_t rx = 0; rx + (8 - step - 1) < xsize; rx += step) {
      const size_t rix = (ry * rw + rx) / step;
      const size_t off = (ry < ysize - 8 ? ry : ysize - 8) * xsize + (rx < xsize - 8 ? rx : xsize - 8);
      float blk0[192], blk1[192];
      for (int i = 0; i < 3; ++i)
        for (size_t y = 0; y < 8; ++y)
          for (size_t x = 0; x < 8; ++x) {
            blk0[i * 64 + 8 * y + x] = xyb0[i * n + off + y * xsize + x];
            blk1[i * 64 + 8 * y + x] = xyb1[i * n + off + y * xsize + x];
          }
      float ddc[3] = {0, 0, 0}, dac[3] = {0, 0, 0}, ded[3] = {0, 0, 0};
      block_diff_float(blk0, blk1, ddc, dac, ded);
      for (int i = 0; i < 3; ++i) {
        dc[3 * rix + i] = ddc[i];
        ac[3 * rix + i] = dac[i];
      }
    }
  if (st && st->block_dc) memcpy(st->block_dc, dc, sizeof(float) * 3 * rn);
  if (st && st->block_ac) memcpy(st->block_ac, ac, sizeof(float) * 3 * rn);

  /* EdgeDetectorLowFreqOpt */
  {
    memcpy(b0, xyb0, sizeof(float) * 3 * n);
    memcpy(b1, xyb1, sizeof(float) * 3 * n);
    for (int i = 0; i < 3; ++i) {
      gzo_blur(xsize, ysize, b0 + i * n, 14.0f, 0.0f);
      gzo_blur(xsize, ysize, b1 + i * n, 14.0f, 0.0f);
    }
    const size_t s8 = 8;
    for (size_t y = 0; y + s8 < ysize; y += step) {
      const int resy = (int)(y / step);
      int resx = (int)(s8 / step);
      for (size_t x = 0; x + s8 < xsize; x += step, resx++) {
        const size_t ix = y * xsize + x;
        const size_t rix = (size_t)resy * rw + resx;
        float diff[4][3];
        for (int i = 0; i < 3; ++i) {
          const float* p0 = b0 + i * n;
          const float* p1 = b1 + i * n;
          size_t ix2 = ix + 8;
          diff[0][i] = (p1[ix] - p0[ix]) + (p0[ix2] - p1[ix2]);
          ix2 = ix + 8 * xsize;
          diff[1][i] = (p1[ix] - p0[ix]) + (p0[ix2] - p1[ix2]);
          ix2 = ix + 6 * xsize + 6;
          diff[2][i] = (p1[ix] - p0[ix]) + (p0[ix2] - p1[ix2]);
          ix2 = ix + 6 * xsize - 6;
          diff[3][i] = x < s8 ? 0 : (p1[ix] - p0[ix]) + (p0[ix2] - p1[ix2]);
        }
        float mx[3] = {0, 0, 0};
        for (int k = 0; k < 4; ++k) {
          float dd[3] = {0, 0, 0};
          lowfreq_sq_acc(diff[k][0], diff[k][1], diff[k][2], 0, 0, 0, 1.0f, dd);
          for (int i = 0; i < 3; ++i) mx[i] = mx[i] < dd[i] ? dd[i] : mx[i];
        }
        for (int i = 0; i < 3; ++i) ac[3 * rix + i] += 10.0f * mx[i];
      }
    }
  }
  if (st && st->block_ac_lf) memcpy(st->block_ac_lf, ac, sizeof(float) * 3 * rn);

  /* MaskOpt + CombineChannelsOpt */
  float* res = (float*)calloc(rn, sizeof(float));
  {
    float* mask = b0;  /* reuse */
    float* mask_dc = b1;
    gzo_mask(xsize, ysize, xyb0, xyb1, mask, mask_dc);
    if (st && st->mask) memcpy(st->mask, mask, sizeof(float) * 3 * n);
    if (st && st->mask_dc) memcpy(st->mask_dc, mask_dc, sizeof(float) * 3 * n);
    for (size_t ry = 0; ry + (8 - step) < ysize; ry += step)
      for (size_t rx = 0; rx + (8 - step) < xsize; rx += step) {
        const size_t rix = (ry * rw + rx) / step;
        const size_t pix = (ry + 3) * xsize + (rx + 3);
        float mk[3], mdc[3];
        for (int i = 0; i < 3; ++i) {
          mk[i] = mask[i * n + pix];
          mdc[i] = mask_dc[i * n + pix];
        }
        const float* pdc = &dc[3 * rix];
        const float* pac = &ac[3 * rix];
        const float* ped = &edge[3 * rix];
        res[rix] = (pdc[0] * mdc[0] + pdc[1] * mdc[1] + pdc[2] * mdc[2]) +
                   (pac[0] * mk[0] + pac[1] * mk[1] + pac[2] * mk[2]) +
                   (ped[0] * mk[0] + ped[1] * mk[1] + ped[2] * mk[2]);
      }
  }
  if (st && st->combined) memcpy(st->combined, res, sizeof(float) * rn);

  /* CalculateDiffmapOpt */
  {
    const size_t s2 = (8 - step) / 2;
    float* out = distmap;
    memset(out, 0, sizeof(float) * n);
    for (size_t ry = 0; ry + 8 - step < ysize; ry += step)
      for (size_t rx = 0; rx + 8 - step < xsize; rx += step) {
        const size_t rix = (ry * rw + rx) / step;
        const float orig = res[rix];
        const float kSlope = 100;
        const float val = orig < (1.0 / (kSlope * kSlope)) ? kSlope * orig : sqrtf(orig);
        for (size_t oy = 0; oy < step; ++oy)
          for (size_t ox = 0; ox < step; ++ox) out[(ry + oy + s2) * xsize + rx + ox + s2] = val;
      }
    const float mul1 = 24.8235314874f;
    const float scale = (float)(1.0 / (1.0 + mul1));
    const size_t s = 8 - step, bxs = xsize - s, bys = ysize - s;
    float* blurred = (float*)malloc(sizeof(float) * bxs * bys);
    for (size_t y = 0; y < bys; ++y)
      for (size_t x = 0; x < bxs; ++x) blurred[y * bxs + x] = out[(y + s2) * xsize + x + s2];
    gzo_blur(bxs, bys, blurred, 8.8510880283f, 0.03027655136f);
    for (size_t y = 0; y < bys; ++y)
      for (size_t x = 0; x < bxs; ++x) out[(y + s2) * xsize + x + s2] += mul1 * blurred[y * bxs + x];
    for (size_t i = 0; i < n; ++i) out[i] *= scale;
    free(blurred);
  }
  free(res);
  free(edge);
  free(dc);
  free(ac);
  free(b0);
  free(b1);
  return 1;
}

float gzo_score_from_diffmap(const float* distmap, size_t n) {
  float r = 0.0f;
  for (size_t i = 0; i < n; ++i) r = r < distmap[i] ? distmap[i] : r;
  return r;
}

float gzo_compare(int w, int h, const uint8_t* ref_rgb, const int16_t* cand_coeffs,
                  float* distmap) {
  gzo_init();
  const size_t n = (size_t)w * h;
  float* x0 = (float*)malloc(sizeof(float) * 3 * n);
  float* x1 = (float*)malloc(sizeof(float) * 3 * n);
  uint8_t* srgb = (uint8_t*)malloc(3 * n);
  float* dm = distmap ? distmap : (float*)malloc(sizeof(float) * n);
  gzo_srgb_to_linear_planes(w, h, ref_rgb, x0);
  gzo_opsin_dynamics(w, h, x0);
  gzo_coeffs_to_srgb(w, h, cand_coeffs, srgb);
  gzo_srgb_to_linear_planes(w, h, srgb, x1);
  gzo_opsin_dynamics(w, h, x1);
  float d = 0.0f;
  if (gzo_diffmap(w, h, x0, x1, dm, NULL)) d = gzo_score_from_diffmap(dm, n);
  if (!distmap) free(dm);
  free(x0);
  free(x1);
  free(srgb);
  return d;
}

/* ------------------------------------------------------------------------ */
/* libstdc++ std::sort emulation (bits/stl_algo.h, bits/stl_heap.h)          */
/* ------------------------------------------------------------------------ */

typedef struct {
  int idx;
  float key;
} pair_t;

static void swap_p(pair_t* a, pair_t* b) { pair_t t = *a; *a = *b; *b = t; }

static void push_heap_(pair_t* f, long hole, long top, pair_t v) {
  long parent = (hole - 1) / 2;
  while (hole > top && f[parent].key < v.key) {
    f[hole] = f[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  f[hole] = v;
}

static void adjust_heap_(pair_t* f, long hole, long len, pair_t v) {
  const long top = hole;
  long child = hole;
  while (child < (len - 1) / 2) {
    child = 2 * (child + 1);
    if (f[child].key < f[child - 1].key) child--;
    f[hole] = f[child];
    hole = child;
  }
  if ((len & 1) == 0 && child == (len - 2) / 2) {
    child = 2 * (child + 1);
    f[hole] = f[child - 1];
    hole = child - 1;
  }
  push_heap_(f, hole, top, v);
}

static void heap_sort_(pair_t* f, pair_t* l) {
  const long len = l - f;
  if (len >= 2) {
    for (long parent = (len - 2) / 2;; --parent) {
      adjust_heap_(f, parent, len, f[parent]);
      if (parent == 0) break;
    }
  }
  while (l - f > 1) {
    --l;
    pair_t v = *l;
    *l = *f;
    adjust_heap_(f, 0, l - f, v);
  }
}

static void move_median_to_first_(pair_t* r, pair_t* a, pair_t* b, pair_t* c) {
  if (a->key < b->key) {
    if (b->key < c->key) swap_p(r, b);
    else if (a->key < c->key) swap_p(r, c);
    else swap_p(r, a);
  } else if (a->key < c->key) {
    swap_p(r, a);
  } else if (b->key < c->key) {
    swap_p(r, c);
  } else {
    swap_p(r, b);
  }
}

static pair_t* unguarded_partition_(pair_t* f, pair_t* l, pair_t* pivot) {
  for (;;) {
    while (f->key < pivot->key) ++f;
    --l;
    while (pivot->key < l->key) --l;
    if (!(f < l)) return f;
    swap_p(f, l);
    ++f;
  }
}

static void introsort_loop_(pair_t* f, pair_t* l, int depth) {
  while (l - f > 16) {
    if (depth == 0) {
      heap_sort_(f, l);
      return;
    }
    --depth;
    pair_t* mid = f + (l - f) / 2;
    move_median_to_first_(f, f + 1, mid, l - 1);
    pair_t* cut = unguarded_partition_(f + 1, l, f);
    introsort_loop_(cut, l, depth);
    l = cut;
  }
}

static void unguarded_linear_insert_(pair_t* last) {
  pair_t v = *last;
  pair_t* next = last - 1;
  while (v.key < next->key) {
    *last = *next;
    last = next;
    --next;
  }
  *last = v;
}

static void insertion_sort_(pair_t* f, pair_t* l) {
  if (f == l) return;
  for (pair_t* i = f + 1; i != l; ++i) {
    if (i->key < f->key) {
      pair_t v = *i;
      memmove(f + 1, f, sizeof(pair_t) * (size_t)(i - f));
      *f = v;
    } else {
      unguarded_linear_insert_(i);
    }
  }
}

void gzo_sort_pairs(int* idx, float* key, int n) {
  if (n <= 1) return;
  pair_t* a = (pair_t*)malloc(sizeof(pair_t) * n);
  for (int i = 0; i < n; ++i) { a[i].idx = idx[i]; a[i].key = key[i]; }
  int lg = 0;
  while ((2L << lg) <= n) ++lg;
  introsort_loop_(a, a + n, 2 * lg);
  if (n > 16) {
    insertion_sort_(a, a + 16);
    for (pair_t* i = a + 16; i != a + n; ++i) unguarded_linear_insert_(i);
  } else {
    insertion_sort_(a, a + n);
  }
  for (int i = 0; i < n; ++i) { idx[i] = a[i].idx; key[i] = a[i].key; }
  free(a);
}

/* ------------------------------------------------------------------------ */
/* Per-block compare and greedy zeroing                                      */
/* ------------------------------------------------------------------------ */

/* 8x8 edge-clamped block of an RGB8 image -> planar linear float [3][64]. */
static void block_linear(int w, int h, const uint8_t* rgb, int bx, int by, float* out) {
  for (int iy = 0, i = 0; iy < 8; ++iy)
    for (int ix = 0; ix < 8; ++ix, ++i) {
      int x = 8 * bx + ix, y = 8 * by + iy;
      if (x > w - 1) x = w - 1;
      if (y > h - 1) y = h - 1;
      const size_t p = (size_t)y * w + x;
      for (int c = 0; c < 3; ++c) out[c * 64 + i] = (float)g_srgb[rgb[3 * p + c]];
    }
}

/* Candidate block pixels: ToLinearRGB(8bx, 8by, 8, 8) of an image whose
 * block (bx,by) carries `block` and whose pixels are IDCT(coeffs)<<4.
 * Only the block itself is read (edge replication stays inside it). */
static void candidate_linear(int w, int h, int bx, int by, const int16_t* block, float* out) {
  uint8_t pix[3][64];
  for (int c = 0; c < 3; ++c) gzo_block_idct(block + 64 * c, pix[c]);
  for (int iy = 0, i = 0; iy < 8; ++iy)
    for (int ix = 0; ix < 8; ++ix, ++i) {
      int x = 8 * bx + ix, y = 8 * by + iy;
      int lx = ix, ly = iy;
      if (x > w - 1) lx = w - 1 - 8 * bx;
      if (y > h - 1) ly = h - 1 - 8 * by;
      const int gx = 8 * bx + lx;
      uint8_t px[3];
      for (int c = 0; c < 3; ++c) {
        const int p = pix[c][8 * ly + lx] << 4;
        px[c] = (uint8_t)((p + 8 - (gx & 1)) >> 4);
      }
      gzo_ycbcr_to_rgb(px);
      for (int c = 0; c < 3; ++c) out[c * 64 + i] = (float)g_srgb[px[c]];
    }
}

static double compare_block(const float* rgb0_c, const float* cand_lin, const float scale_f[3]) {
  float rgb1_c[192];
  memcpy(rgb1_c, cand_lin, sizeof(rgb1_c));
  gzo_opsin_dynamics(8, 8, rgb1_c);
  float m0[192], m1[192];
  gzo_mask_high_intensity_change(8, 8, rgb0_c, rgb1_c, m0, m1);
  double b0[192], b1[192];
  for (int i = 0; i < 192; ++i) { b0[i] = m0[i]; b1[i] = m1[i]; }
  double dc[3] = {0, 0, 0}, ac[3] = {0, 0, 0}, ed[3] = {0, 0, 0};
  gzo_block_diff_double(b0, b1, dc, ac, ed);
  double diff = 0.0, diff_edge = 0.0;
  for (int c = 0; c < 3; ++c) {
    const double s = scale_f[c];
    diff += dc[c] * s;
    diff += ac[c] * s;
    diff_edge += ed[c] * s;
  }
  const double kEdgeWeight = 0.05;
  return sqrt((1 - kEdgeWeight) * diff + kEdgeWeight * diff_edge);
}

/* SwitchBlock(bx, by, 1, 1) + CompareBlock (butteraugli_comparator.cc:85-163)
 * of block `bix` with candidate coefficients block[3][64]. */
double gzo_compare_block(int w, int h, const uint8_t* ref_rgb, const float* ref_mask, int bix,
                         const int16_t* block) {
  gzo_init();
  const int bw = (w + 7) / 8, bx = bix % bw, by = bix / bw;
  const size_t n = (size_t)w * h;
  float rgb0_c[192];
  block_linear(w, h, ref_rgb, bx, by, rgb0_c);
  gzo_opsin_dynamics(8, 8, rgb0_c);
  const size_t corner = (size_t)(8 * by) * w + 8 * bx;
  const float scale[3] = {ref_mask[corner], ref_mask[n + corner], ref_mask[2 * n + corner]};
  float lin[192];
  candidate_linear(w, h, bx, by, block, lin);
  return compare_block(rgb0_c, lin, scale);
}

void gzo_block_zeroing_orders(int w, int h, const uint8_t* ref_rgb, const float* ref_mask,
                              const int16_t* cur_coeffs, const int16_t* orig_coeffs,
                              float limit, int lookahead, int comp_mask, int new_model,
                              gzo_coeff_data* out) {
  /* old zeroing model (processor.cc:381-405) */
  static const uint8_t kOldCsf[64] = {
      10, 10, 20, 40, 60, 70, 80, 90, 10, 20, 30, 60, 70, 80, 90, 90,
      20, 30, 60, 70, 80, 90, 90, 90, 40, 60, 70, 80, 90, 90, 90, 90,
      60, 70, 80, 90, 90, 90, 90, 90, 70, 80, 90, 90, 90, 90, 90, 90,
      80, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90, 90};
  static const double kWeight[3] = {1.0, 0.22, 0.20};
  /* kJPEGZigZagOrder, jpeg_data.h:73-82: zigzag position of natural index k */
  static const int kZigZagOrder[64] = {
      0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
      3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
      10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
      21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
  gzo_init();
  const int bw = (w + 7) / 8, bh = (h + 7) / 8;
  const size_t nb = (size_t)bw * bh, n = (size_t)w * h;
  memset(out, 0, sizeof(gzo_coeff_data) * nb * 192);
  for (int by = 0, bix = 0; by < bh; ++by)
    for (int bx = 0; bx < bw; ++bx, ++bix) {
      int16_t block[192], orig[192];
      for (int c = 0; c < 3; ++c) {
        memcpy(block + 64 * c, cur_coeffs + (c * nb + bix) * 64, 128);
        memcpy(orig + 64 * c, orig_coeffs + (c * nb + bix) * 64, 128);
      }
      int idxs[192];
      float keys[192];
      int ncand = 0;
      /* SelectFrequencyMasking passes only the masked components
       * (processor.cc:645-655); the image keeps the others' current values */
      for (int c = 0; c < 3; ++c) {
        if (!(comp_mask & (1 << c))) continue;
        for (int k = 1; k < 64; ++k) {
          const int idx = c * 64 + k;
          if (block[idx] != 0) {
            idxs[ncand] = idx;
            if (new_model)
              keys[ncand] = abs(orig[idx]) * kZeroingCsf[idx] + 0.0f;
            else
              keys[ncand] = (float)((abs(orig[idx]) - kZigZagOrder[k] / 64.0) * kWeight[c] /
                                    kOldCsf[k]);
            ++ncand;
          }
        }
      }
      gzo_sort_pairs(idxs, keys, ncand);
      /* SwitchBlock: 8x8-local opsin of the original block */
      float rgb0_c[192];
      block_linear(w, h, ref_rgb, bx, by, rgb0_c);
      gzo_opsin_dynamics(8, 8, rgb0_c);
      const size_t corner = (size_t)(8 * by) * w + 8 * bx;
      const float scale[3] = {ref_mask[corner], ref_mask[n + corner], ref_mask[2 * n + corner]};

      int16_t processed[192];
      memcpy(processed, block, sizeof(processed));
      gzo_coeff_data order[192];
      int norder = 0;
      while (ncand > 0) {
        float best_err = 1e17f;
        int best_i = 0;
        const int look = ncand < lookahead ? ncand : lookahead;
        for (int i = 0; i < look; ++i) {
          int16_t cand[192];
          memcpy(cand, processed, sizeof(cand));
          cand[idxs[i]] = 0;
          float lin[192];
          candidate_linear(w, h, bx, by, cand, lin);
          const float err = (float)compare_block(rgb0_c, lin, scale);
          const float max_err = 0.0f < err ? err : 0.0f;
          if (max_err < best_err) {
            best_err = max_err;
            best_i = i;
          }
        }
        const int idx = idxs[best_i];
        processed[idx] = 0;
        memmove(idxs + best_i, idxs + best_i + 1, sizeof(int) * (ncand - best_i - 1));
        memmove(keys + best_i, keys + best_i + 1, sizeof(float) * (ncand - best_i - 1));
        --ncand;
        order[norder].idx = idx;
        order[norder].block_err = best_err;
        ++norder;
        if (best_err >= limit) break;
      }
      float min_err = 1e10f;
      for (int i = norder - 1; i >= 0; --i) {
        if (order[i].block_err < min_err) min_err = order[i].block_err;
        order[i].block_err = min_err;
      }
      int num = 0;
      while (num < norder && order[num].block_err <= limit) ++num;
      for (int i = 0; i < num; ++i) out[(size_t)bix * 192 + i] = order[i];
    }
}
