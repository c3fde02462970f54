// Portions restate Guetzli (Copyright 2016 Google Inc., Apache License 2.0,
// http://www.apache.org/licenses/LICENSE-2.0) as modified in
// yyamamoto79/guetzli-cuda-opencl: preprocess_downsample.cc (PreProcessChannel, Sharpen, Erode, Dilate,
// RGBToYUV420), output_image.cc (the factor-2 SetCoeffBlock / Downsample /
// SaveToJpegData) and dct_double.cc.
// Byte-exact output forces their operation order and constants; the
// code around them is this repository's own.
#include "host/image420.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "host/jpeg_reader.h"

namespace gz {

namespace {

// libjpeg-exact integer IDCT coefficients (guetzli/idct.cc:29-38)
const int kIdctM[64] = {
    8192, 11363, 10703, 9633,   8192,  6437,   4433,   2260,   8192, 9633,  4433,  -2259, -8192,
    -11362, -10704, -6436, 8192, 6437, -4433,  -11362, -8192, 2261,   10704,  9633, 8192,  2260,
    -10703, -6436, 8192, 9633,  -4433, -11363, 8192,   -2260, -10703, 6436,   8192, -9633, -4433,
    11363,  8192,  -6437, -4433, 11362, -8192, -2261,  10704, -9633,  8192,   -9633, 4433, 2259,
    -8192,  11362, -10704, 6436, 8192,  -11363, 10703, -9633, 8192,   -6437,  4433,  -2260,
};

inline int Clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// kDCTMatrix of dct_double.cc:26-45: 0.5 * alpha(u) * cos((2x + 1) u pi / 16)
// to the reference's ten digits.
const double kDctD[64] = {
    0.3535533906,  0.3535533906,  0.3535533906,  0.3535533906,  0.3535533906,  0.3535533906,
    0.3535533906,  0.3535533906,  0.4903926402,  0.4157348062,  0.2777851165,  0.0975451610,
    -0.0975451610, -0.2777851165, -0.4157348062, -0.4903926402, 0.4619397663,  0.1913417162,
    -0.1913417162, -0.4619397663, -0.4619397663, -0.1913417162, 0.1913417162,  0.4619397663,
    0.4157348062,  -0.0975451610, -0.4903926402, -0.2777851165, 0.2777851165,  0.4903926402,
    0.0975451610,  -0.4157348062, 0.3535533906,  -0.3535533906, -0.3535533906, 0.3535533906,
    0.3535533906,  -0.3535533906, -0.3535533906, 0.3535533906,  0.2777851165,  -0.4903926402,
    0.0975451610,  0.4157348062,  -0.4157348062, -0.0975451610, 0.4903926402,  -0.2777851165,
    0.1913417162,  -0.4619397663, 0.4619397663,  -0.1913417162, -0.1913417162, 0.4619397663,
    -0.4619397663, 0.1913417162,  0.0975451610,  -0.2777851165, 0.4157348062,  -0.4903926402,
    0.4903926402,  -0.4157348062, 0.2777851165,  -0.0975451610,
};

// One 1-D pass over 8 values at `stride`: out[x] = sum_u M(x, u) in[u], the
// sum formed in u order starting from 0.0 (dct_double.cc:47-63).
template <bool kInverse>
void Transform1d(const double* in, int stride, double* out) {
  for (int x = 0; x < 8; ++x) {
    double acc = 0.0;
    for (int u = 0; u < 8; ++u) acc += (kInverse ? kDctD[8 * u + x] : kDctD[8 * x + u]) * in[u * stride];
    out[x * stride] = acc;
  }
}

template <bool kInverse>
void TransformBlock(double block[64]) {
  double tmp[64];
  for (int x = 0; x < 8; ++x) Transform1d<kInverse>(&block[x], 8, &tmp[x]);
  for (int y = 0; y < 8; ++y) Transform1d<kInverse>(&tmp[8 * y], 1, &block[8 * y]);
}

// ---- PreProcessChannel (preprocess_downsample.cc:26-279) ----

using Plane = std::vector<float>;

// Convolve2D with a size x size kernel, skipping the border (:29-50).
Plane Convolve2D(const Plane& image, int w, int h, const double* kernel, int size) {
  Plane result = image;
  const int s2 = size / 2;
  for (int y = s2; y + size - s2 - 1 < h; ++y)
    for (int x = s2; x + size - s2 - 1 < w; ++x) {
      float v = 0;
      for (int j = 0; j < size * size; ++j)
        v += static_cast<float>(kernel[j]) * image[(y + j / size - s2) * w + x + j % size - s2];
      result[static_cast<size_t>(y) * w + x] = v;
    }
  return result;
}

// Horizontal then vertical 1-D kernel, each pass scaled by (float)mul (:53-83).
Plane Convolve2X(const Plane& image, int w, int h, const double* kernel, int size, double mul) {
  const int s2 = size / 2;
  const float fmul = static_cast<float>(mul);
  Plane temp = image;
  for (int y = 0; y < h; ++y)
    for (int x = s2; x + size - s2 - 1 < w; ++x) {
      float v = 0;
      for (int j = 0; j < size; ++j) v += static_cast<float>(kernel[j]) * image[static_cast<size_t>(y) * w + x + j - s2];
      temp[static_cast<size_t>(y) * w + x] = v * fmul;
    }
  Plane result = temp;
  for (int y = s2; y + size - s2 - 1 < h; ++y)
    for (int x = 0; x < w; ++x) {
      float v = 0;
      for (int j = 0; j < size; ++j) v += static_cast<float>(kernel[j]) * temp[static_cast<size_t>(y + j - s2) * w + x];
      result[static_cast<size_t>(y) * w + x] = v * fmul;
    }
  return result;
}

double Normal(double x, double sigma) {
  static const double kInvSqrt2Pi = 0.3989422804014327;
  return std::exp(-x * x / (2 * sigma * sigma)) * kInvSqrt2Pi / sigma;
}

// The 5-tap normalised Gaussian of Sharpen / Blur (:90-149); sigma arrives
// as a double (Sharpen's float sigma widened, Blur's constant 1.3).
void Gauss5(double sigma, double kernel[5], double* mul) {
  double sum = 0;
  for (int i = 0; i < 5; ++i) kernel[i] = Normal(1.0 * i - 2, sigma);
  for (int i = 0; i < 5; ++i) sum += kernel[i];
  *mul = 1.0 / sum;
}

Plane Sharpen(const Plane& image, int w, int h, float sigma, float amount) {
  double k[5], mul;
  Gauss5(sigma, k, &mul);
  Plane result = Convolve2X(image, w, h, k, 5, mul);
  for (size_t i = 0; i < image.size(); ++i) result[i] = image[i] + (image[i] - result[i]) * amount;
  return result;
}

Plane BlurPlane(const Plane& image, int w, int h) {
  double k[5], mul;
  Gauss5(1.3, k, &mul);
  return Convolve2X(image, w, h, k, 5, mul);
}

// 4-neighbour erosion / dilation of the interior (:110-134).
void Erode(int w, int h, std::vector<uint8_t>* m) {
  const std::vector<uint8_t> t = *m;
  for (int y = 1; y + 1 < h; ++y)
    for (int x = 1; x + 1 < w; ++x) {
      const size_t i = static_cast<size_t>(y) * w + x;
      if (!(t[i] && t[i - 1] && t[i + 1] && t[i - w] && t[i + w])) (*m)[i] = 0;
    }
}

void Dilate(int w, int h, std::vector<uint8_t>* m) {
  const std::vector<uint8_t> t = *m;
  for (int y = 1; y + 1 < h; ++y)
    for (int x = 1; x + 1 < w; ++x) {
      const size_t i = static_cast<size_t>(y) * w + x;
      if (t[i] || t[i - 1] || t[i + 1] || t[i - w] || t[i + w]) (*m)[i] = 1;
    }
}

// Sharpens channel `channel` (2: v, 1: u) where it helps and blurs it where
// it is smooth (:157-279).  The float / double mix of every expression is
// the reference's.
void PreProcessChannel(int w, int h, int channel, float sigma, float amount, bool blur,
                       bool sharpen, std::vector<Plane>* image) {
  if (!blur && !sharpen) return;
  std::vector<Plane>& yuv = *image;
  const size_t n = yuv[0].size();
  for (size_t i = 0; i < n; ++i) {
    yuv[0][i] /= 255.0;
    yuv[1][i] = yuv[1][i] / 255.0f - 0.5f;
    yuv[2][i] = yuv[2][i] / 255.0f - 0.5f;
  }
  std::vector<uint8_t> darkmap(n, 0);
  for (size_t i = 0; i < n; ++i) {
    const float y = yuv[0][i], u = yuv[1][i], v = yuv[2][i];
    const float r = y + 1.402f * v;
    const float g = y - 0.34414f * u - 0.71414f * v;
    const float b = y + 1.772f * u;
    if (channel == 2 && g < 0.85 && b < 0.85 && r < 0.9) darkmap[i] = 1;
    if (channel == 1 && r < 0.85 && g < 0.85 && b < 0.9) darkmap[i] = 1;
  }
  for (int k = 0; k < 3; ++k) Erode(w, h, &darkmap);
  std::vector<uint8_t> redmap(n, 0);
  for (size_t i = 0; i < n; ++i) {
    const float u = yuv[1][i], v = yuv[2][i];
    if (channel == 2 && 2.116 * v > -0.34414 * u + 0.2 && 1.402 * v > 1.772 * u + 0.2) redmap[i] = 1;
    if (channel == 1 && v < 1.263 * u - 0.1 && u > -0.33741 * v) redmap[i] = 1;
  }
  for (int k = 0; k < 3; ++k) Dilate(w, h, &redmap);
  std::vector<uint8_t> sharpenmap(n);
  for (size_t i = 0; i < n; ++i) sharpenmap[i] = redmap[i] && darkmap[i];
  const double threshold = (channel == 2 ? 0.02 : 1.0) * 127.5;
  static const double kEdgeMatrix[9] = {0, -1, 0, -1, 4, -1, 0, -1, 0};
  std::vector<uint8_t> blurmap(n, 0);
  const Plane edge = Convolve2D(yuv[channel], w, h, kEdgeMatrix, 3);
  for (size_t i = 0; i < n; ++i) {
    const float u = yuv[1][i], v = yuv[2][i];
    if (sharpenmap[i] || !darkmap[i]) continue;
    if (std::fabs(edge[i]) < threshold && v < -0.162 * u) blurmap[i] = 1;
  }
  Erode(w, h, &blurmap);
  Erode(w, h, &blurmap);
  const Plane sharpened = Sharpen(yuv[channel], w, h, sigma, amount);
  const Plane blurred = BlurPlane(yuv[channel], w, h);
  for (size_t i = 0; i < n; ++i) {
    if (sharpenmap[i]) {
      if (sharpen) yuv[channel][i] = sharpened[i];
    } else if (blurmap[i]) {
      if (blur) yuv[channel][i] = blurred[i];
    }
  }
  for (size_t i = 0; i < n; ++i) {
    yuv[0][i] *= 255.0;
    yuv[1][i] = (yuv[1][i] + 0.5f) * 255.0f;
    yuv[2][i] = (yuv[2][i] + 0.5f) * 255.0f;
  }
}

// ---- RGBToYUV420, the "silver screen" downsampler (:283-476) ----

inline float Clip(float v) { return std::max(0.0f, std::min(255.0f, v)); }
inline float RGBToY(float r, float g, float b) { return 0.299f * r + 0.587f * g + 0.114f * b; }
inline float RGBToU(float r, float g, float b) { return -0.16874f * r - 0.33126f * g + 0.5f * b + 128.0f; }
inline float RGBToV(float r, float g, float b) { return 0.5f * r - 0.41869f * g - 0.08131f * b + 128.0f; }
inline float YUVToR(float y, float, float v) { return y + 1.402f * (v - 128.0f); }
inline float YUVToG(float y, float u, float v) { return y - 0.344136f * (u - 128.0f) - 0.714136f * (v - 128.0f); }
inline float YUVToB(float y, float u, float) { return y + 1.772f * (u - 128.0f); }
inline float GammaToLinear(float x) { return static_cast<float>(std::pow(x / 255.0f, 2.2)); }
inline float LinearToGamma(float x) { return 255.0 * std::pow(x, 1.0 / 2.2); }

Plane LinearlyAveragedLuma(const Plane& rgb) {
  Plane y(rgb.size() / 3);
  for (size_t i = 0, p = 0; p < rgb.size(); ++i, p += 3)
    y[i] = LinearToGamma(RGBToY(GammaToLinear(rgb[p]), GammaToLinear(rgb[p + 1]), GammaToLinear(rgb[p + 2])));
  return y;
}

Plane LinearlyDownsample2x2(const Plane& in, int width, int height) {
  const int w = (width + 1) / 2, h = (height + 1) / 2;
  Plane out(static_cast<size_t>(3) * w * h);
  for (int y = 0, p = 0; y < h; ++y)
    for (int x = 0; x < w; ++x)
      for (int i = 0; i < 3; ++i, ++p) {
        out[p] = 0.0;
        for (int iy = 0; iy < 2; ++iy)
          for (int ix = 0; ix < 2; ++ix) {
            const int yy = std::min(height - 1, 2 * y + iy), xx = std::min(width - 1, 2 * x + ix);
            out[p] += GammaToLinear(in[3 * (static_cast<size_t>(yy) * width + xx) + i]);
          }
        out[p] = LinearToGamma(0.25f * out[p]);
      }
  return out;
}

std::vector<Plane> RGBToYUV(const Plane& rgb) {
  std::vector<Plane> yuv(3, Plane(rgb.size() / 3));
  for (size_t i = 0, p = 0; p < rgb.size(); ++i, p += 3) {
    const float r = rgb[p], g = rgb[p + 1], b = rgb[p + 2];
    yuv[0][i] = RGBToY(r, g, b);
    yuv[1][i] = RGBToU(r, g, b);
    yuv[2][i] = RGBToV(r, g, b);
  }
  return yuv;
}

Plane YUVToRGB(const std::vector<Plane>& yuv) {
  Plane rgb(3 * yuv[0].size());
  for (size_t i = 0, p = 0; p < rgb.size(); ++i, p += 3) {
    const float y = yuv[0][i], u = yuv[1][i], v = yuv[2][i];
    rgb[p] = Clip(YUVToR(y, u, v));
    rgb[p + 1] = Clip(YUVToG(y, u, v));
    rgb[p + 2] = Clip(YUVToB(y, u, v));
  }
  return rgb;
}

Plane Upsample2x2(const Plane& in, int width, int height) {
  const int w = (width + 1) / 2, h = (height + 1) / 2;
  Plane out(static_cast<size_t>(width) * height);
  for (int y = 0, p = 0; y < h; ++y)
    for (int x = 0; x < w; ++x, ++p)
      for (int iy = 0; iy < 2; ++iy)
        for (int ix = 0; ix < 2; ++ix) {
          const int yy = std::min(height - 1, 2 * y + iy), xx = std::min(width - 1, 2 * x + ix);
          out[static_cast<size_t>(yy) * width + xx] = in[p];
        }
  return out;
}

// libjpeg's fancy upsampling filter in float (:405-426).
Plane FancyBlur(const Plane& img, int width, int height) {
  Plane out(static_cast<size_t>(width) * height);
  for (int y0 = 0; y0 < height; y0 += 2)
    for (int x0 = 0; x0 < width; x0 += 2)
      for (int iy = 0; iy < 2 && y0 + iy < height; ++iy)
        for (int ix = 0; ix < 2 && x0 + ix < width; ++ix) {
          const int x1 = std::min(width - 1, std::max(0, x0 + 4 * ix - 2));
          const int y1 = std::min(height - 1, std::max(0, y0 + 4 * iy - 2));
          out[static_cast<size_t>(y0 + iy) * width + x0 + ix] =
              (9.0f * img[static_cast<size_t>(y0) * width + x0] + 3.0f * img[static_cast<size_t>(y0) * width + x1] +
               3.0f * img[static_cast<size_t>(y1) * width + x0] + 1.0f * img[static_cast<size_t>(y1) * width + x1]) /
              16.0f;
        }
  return out;
}

Plane YUV420ToRGB(const std::vector<Plane>& yuv420, int width, int height) {
  std::vector<Plane> yuv;
  yuv.push_back(yuv420[0]);
  yuv.push_back(FancyBlur(Upsample2x2(yuv420[1], width, height), width, height));
  yuv.push_back(FancyBlur(Upsample2x2(yuv420[2], width, height), width, height));
  return YUVToRGB(yuv);
}

void UpdateGuess(const Plane& target, const Plane& rec, Plane* guess) {
  for (size_t i = 0; i < guess->size(); ++i) (*guess)[i] = Clip((*guess)[i] - (rec[i] - target[i]));
}

std::vector<Plane> RGBToYUV420(const std::vector<uint8_t>& rgb_in, int width, int height) {
  Plane rgbf(rgb_in.size());
  for (size_t i = 0; i < rgb_in.size(); ++i) rgbf[i] = static_cast<float>(rgb_in[i]);
  const Plane y_target = LinearlyAveragedLuma(rgbf);
  const std::vector<Plane> yuv_target = RGBToYUV(LinearlyDownsample2x2(rgbf, width, height));
  std::vector<Plane> guess = yuv_target;
  guess[0] = Upsample2x2(guess[0], width, height);
  for (int iter = 0; iter < 20; ++iter) {
    const Plane rgb_rec = YUV420ToRGB(guess, width, height);
    const Plane y_rec = LinearlyAveragedLuma(rgb_rec);
    const std::vector<Plane> yuv_rec = RGBToYUV(LinearlyDownsample2x2(rgb_rec, width, height));
    UpdateGuess(y_target, y_rec, &guess[0]);
    UpdateGuess(yuv_target[1], yuv_rec[1], &guess[1]);
    UpdateGuess(yuv_target[2], yuv_rec[2], &guess[2]);
  }
  guess[1] = Upsample2x2(guess[1], width, height);
  guess[2] = Upsample2x2(guess[2], width, height);
  return guess;
}

// SetDownsampledCoefficients (output_image.cc:496-531): per block the
// factor x factor average (float, edge-clamped), float64 DCT, DC level shift,
// rounded.  Returns the [bw * bh][64] coefficients at blocks of 8 * factor.
std::vector<coeff_t> DownsampledCoefficients(const Plane& pixels, int w, int h, int factor) {
  const int bw = (w + 8 * factor - 1) / (8 * factor), bh = (h + 8 * factor - 1) / (8 * factor);
  std::vector<coeff_t> out(static_cast<size_t>(bw) * bh * 64);
  for (int by = 0; by < bh; ++by)
    for (int bx = 0; bx < bw; ++bx) {
      double blockd[64];
      const int x0 = 8 * bx * factor, y0 = 8 * by * factor;
      for (int iy = 0; iy < 8; ++iy)
        for (int ix = 0; ix < 8; ++ix) {
          float avg = 0.0;
          for (int j = 0; j < factor; ++j)
            for (int i = 0; i < factor; ++i) {
              const int x = std::min(x0 + ix * factor + i, w - 1), y = std::min(y0 + iy * factor + j, h - 1);
              avg += pixels[static_cast<size_t>(y) * w + x];
            }
          avg /= factor * factor;
          blockd[8 * iy + ix] = avg;
        }
      BlockDctDouble(blockd);
      blockd[0] -= 1024.0;
      coeff_t* dst = &out[(static_cast<size_t>(by) * bw + bx) * 64];
      for (int k = 0; k < 64; ++k) dst[k] = static_cast<coeff_t>(std::round(blockd[k]));
    }
  return out;
}

}  // namespace

void BlockIdctBytes(const coeff_t* in, uint8_t out[64]) {
  // column pass rounded to int16 at scale 2^11, row pass with the +128 level
  // shift folded into the rounding term; sums mod 2^32
  int16_t col[64];
  for (int iy = 0; iy < 8; ++iy)
    for (int ix = 0; ix < 8; ++ix) {
      unsigned acc = 0;
      for (int u = 0; u < 8; ++u) acc += static_cast<unsigned>(kIdctM[8 * iy + u] * in[8 * u + ix]);
      col[8 * iy + ix] = static_cast<int16_t>((static_cast<int>(acc) + (1 << 10)) >> 11);
    }
  for (int iy = 0; iy < 8; ++iy)
    for (int ix = 0; ix < 8; ++ix) {
      unsigned acc = 0;
      for (int u = 0; u < 8; ++u) acc += static_cast<unsigned>(kIdctM[8 * ix + u] * col[8 * iy + u]);
      out[8 * iy + ix] = static_cast<uint8_t>(Clamp255((static_cast<int>(acc) + (257 << 17)) >> 18));
    }
}

void BlockDctDouble(double block[64]) { TransformBlock<false>(block); }
void BlockIdctDouble(double block[64]) { TransformBlock<true>(block); }

void SubsampledPlane::Reset(int width, int height, int factor) {
  w = width;
  h = height;
  f = factor;
  wib = (w + 8 * f - 1) / (8 * f);
  hib = (h + 8 * f - 1) / (8 * f);
  px.assign(static_cast<size_t>(w) * h, 128 << 4);
}

void SubsampledPlane::Update(int bx, int by, const uint8_t idct[64]) {
  if (f == 1) {
    for (int iy = 0; iy < 8 && 8 * by + iy < h; ++iy)
      for (int ix = 0; ix < 8 && 8 * bx + ix < w; ++ix)
        px[static_cast<size_t>(8 * by + iy) * w + 8 * bx + ix] = static_cast<uint16_t>(idct[8 * iy + ix] << 4);
    return;
  }
  // The 10x10 subsampled neighbourhood (the block's IDCT bytes, a ring
  // rebuilt from the upsampled pixels as they are by inverting the fancy
  // upsampler, edge replication outside the image; rows 1..9 then row 0,
  // columns 1..9 then column 0), then the fancy upsampler over the block's
  // 16x16 area plus one pixel around (clipped to the image).  Stored values
  // wrap at 16 bits as the reference's uint16_t arrays do.
  constexpr int E = 10;
  uint16_t sub[E * E];
  for (int j = 0; j < E; ++j) {
    const int row = j < 9 ? j + 1 : 0;
    const int y0 = by * 16 + (j < 9 ? 2 * j : -2);
    for (int i = 0; i < E; ++i) {
      const int col = i < 9 ? i + 1 : 0;
      const int x0 = bx * 16 + (i < 9 ? 2 * i : -2);
      uint16_t* d = &sub[row * E + col];
      if (x0 < 0) {
        *d = d[1];
      } else if (y0 < 0) {
        *d = d[E];
      } else if (x0 >= w) {
        *d = d[-1];
      } else if (y0 >= h) {
        *d = d[-E];
      } else if (i < 8 && j < 8) {
        *d = static_cast<uint16_t>(idct[8 * j + i] << 4);
      } else {
        const int y1 = y0 > 0 ? y0 - 1 : 0, x1 = x0 > 0 ? x0 - 1 : 0;
        const size_t r0 = static_cast<size_t>(y0) * w, r1 = static_cast<size_t>(y1) * w;
        *d = static_cast<uint16_t>((px[r0 + x0] * 9 + px[r1 + x1] - 3 * px[r0 + x1] - 3 * px[r1 + x0]) >> 2);
      }
    }
  }
  const int xa = std::max(bx * 16 - 1, 0), xb = std::min(bx * 16 + 16, w - 1);
  const int ya = std::max(by * 16 - 1, 0), yb = std::min(by * 16 + 16, h - 1);
  for (int y = ya; y <= yb; ++y) {
    const int r0 = ((y & ~1) / 2 - by * 8 + 1) * E, dr = (y & 1) ? E : -E;
    for (int x = xa; x <= xb; ++x) {
      const int k = r0 + (x & ~1) / 2 - bx * 8 + 1, dc = (x & 1) ? 1 : -1;
      px[static_cast<size_t>(y) * w + x] =
          static_cast<uint16_t>((sub[k] * 9 + sub[k + dr] * 3 + sub[k + dc] * 3 + sub[k + dc + dr]) >> 4);
    }
  }
}

void Image420::Init(int width, int height) {
  SavedReset();
  w = width;
  h = height;
  bw = (w + 7) / 8;
  bh = (h + 7) / 8;
  cbw = (w + 15) / 16;
  cbh = (h + 15) / 16;
  y.assign(static_cast<size_t>(bw) * bh * 64, 0);
  for (int k = 0; k < 2; ++k) {
    c[k].assign(static_cast<size_t>(cbw) * cbh * 64, 0);
    plane[k].Reset(w, h, 2);
  }
  for (int q = 0; q < 3; ++q)
    for (int k = 0; k < 64; ++k) quant[q][k] = 1;
}

void Image420::SetCoeffBlock(int comp, int b, const coeff_t* blk) {
  coeff_t* dst = block(comp, b);
  if (dst != blk) std::memcpy(dst, blk, 64 * sizeof(coeff_t));
  if (saved_ok_) dirty_[comp].push_back(b);
  if (comp == 0) return;  // factor 1: the pixels are the IDCT, formed on the device
  uint8_t idct[64];
  BlockIdctBytes(dst, idct);
  plane[comp - 1].Update(b % cbw, b / cbw, idct);
}

void Image420::CopyFromJpegData(const JpegData& jpg) {
  SavedReset();
  for (int comp = 0; comp < 3; ++comp) {
    const JpegComponent& jc = jpg.components[comp];
    const int* q = jpg.quant[jc.quant_idx].values;
    const int nbw = BlockWidth(comp), nbh = comp == 0 ? bh : cbh;
    if (comp > 0) plane[comp - 1].Reset(w, h, 2);
    for (int by = 0; by < nbh; ++by)
      for (int bx = 0; bx < nbw; ++bx) {
        const coeff_t* src = &jc.coeffs[(static_cast<size_t>(by) * jc.width_in_blocks + bx) * 64];
        coeff_t blk[64];
        for (int k = 0; k < 64; ++k) blk[k] = static_cast<coeff_t>(src[k] * q[k]);
        SetCoeffBlock(comp, by * nbw + bx, blk);
      }
    std::memcpy(quant[comp], q, sizeof(quant[comp]));
  }
}

void Image420::ApplyGlobalQuantization(const int q[3][kDCTBlockSize]) {
  SavedReset();
  for (int comp = 0; comp < 3; ++comp) {
    const int nb = Blocks(comp);
    for (int b = 0; b < nb; ++b) {
      coeff_t* blk = block(comp, b);
      bool changed = false;
      for (int k = 0; k < 64; ++k) {
        const coeff_t v = QuantizeCoeff(blk[k], q[comp][k]);
        changed = changed || v != blk[k];
        blk[k] = v;
      }
      if (changed) SetCoeffBlock(comp, b, blk);
    }
    std::memcpy(quant[comp], q[comp], sizeof(quant[comp]));
  }
}

bool Image420::ChromaAllZero() const {
  for (int k = 0; k < 2; ++k)
    for (coeff_t v : c[k])
      if (v != 0) return false;
  return true;
}

void Image420::SaveToJpegData(JpegData* jpg) const {
  jpg->width = w;
  jpg->height = h;
  const int ncomp = ChromaAllZero() ? 1 : 3;
  // (the reference's max_v_samp_factor = max(max_h_samp_factor, factor_y)
  // is 2 for 2x2 chroma all the same)
  jpg->max_h_samp_factor = ncomp == 3 ? 2 : 1;
  jpg->max_v_samp_factor = ncomp == 3 ? 2 : 1;
  jpg->mcu_cols = ncomp == 3 ? std::min(bw, cbw) : bw;
  jpg->mcu_rows = ncomp == 3 ? std::min(bh, cbh) : bh;
  jpg->components.resize(ncomp);
  for (int comp = 0; comp < ncomp; ++comp) {
    JpegComponent& jc = jpg->components[comp];
    const int f = comp == 0 ? 1 : 2;
    jc.id = comp;
    jc.h_samp_factor = jpg->max_h_samp_factor / f;
    jc.v_samp_factor = jpg->max_v_samp_factor / f;
    jc.width_in_blocks = jpg->mcu_cols * jc.h_samp_factor;
    jc.height_in_blocks = jpg->mcu_rows * jc.v_samp_factor;
    jc.coeffs.resize(static_cast<size_t>(jc.width_in_blocks) * jc.height_in_blocks * 64);
    const int nbw = BlockWidth(comp), nbh = comp == 0 ? bh : cbh;
    int last_dc = 0;
    coeff_t* dst = jc.coeffs.data();
    int src_b = 0;
    for (int by = 0; by < jc.height_in_blocks; ++by)
      for (int bx = 0; bx < jc.width_in_blocks; ++bx, dst += 64) {
        if (by >= nbh || bx >= nbw) {
          dst[0] = static_cast<coeff_t>(last_dc);
          for (int k = 1; k < 64; ++k) dst[k] = 0;
        } else {
          // (the reference walks its source blocks sequentially)
          const coeff_t* src = block(comp, src_b++);
          for (int k = 0; k < 64; ++k) dst[k] = static_cast<coeff_t>(src[k] / quant[comp][k]);
        }
        last_dc = dst[0];
      }
  }
  SaveQuantTables(quant, jpg);
}

const JpegData& Image420::SavedJpegData(const JpegData& meta) {
  const int ncomp = ChromaAllZero() ? 1 : 3;
  bool whole = !saved_ok_ || static_cast<int>(saved_.components.size()) != ncomp;
  for (int comp = 0; comp < ncomp && !whole; ++comp) {
    JpegComponent& jc = saved_.components[comp];
    const int nbw = BlockWidth(comp);
    for (const int b : dirty_[comp]) {
      const coeff_t* src = block(comp, b);
      coeff_t* dst = &jc.coeffs[(static_cast<size_t>(b / nbw) * jc.width_in_blocks + b % nbw) * 64];
      const coeff_t dc = static_cast<coeff_t>(src[0] / quant[comp][0]);
      if (dc != dst[0]) {
        whole = true;
        break;
      }
      for (int k = 1; k < 64; ++k) dst[k] = static_cast<coeff_t>(src[k] / quant[comp][k]);
    }
  }
  if (whole) {
    SaveToJpegData(&saved_);
    saved_.app_data = meta.app_data;
    saved_.com_data = meta.com_data;
    saved_ok_ = true;
  }
  for (auto& d : dirty_) d.clear();
  return saved_;
}

bool DownsampleToJpegData420(const JpegData& jpg444, bool silver_screen, JpegData* jpg420) {
  const int w = jpg444.width, h = jpg444.height;
  // OutputImage img; img.CopyFromJpegData(jpg444) at quant 1
  Image420 img;
  img.Init(w, h);
  {
    const JpegComponent& jc = jpg444.components[0];
    const int* q = jpg444.quant[jc.quant_idx].values;
    for (int by = 0; by < img.bh; ++by)
      for (int bx = 0; bx < img.bw; ++bx) {
        const coeff_t* src = &jc.coeffs[(static_cast<size_t>(by) * jc.width_in_blocks + bx) * 64];
        coeff_t* dst = img.block(0, by * img.bw + bx);
        for (int k = 0; k < 64; ++k) dst[k] = static_cast<coeff_t>(src[k] * q[k]);
      }
  }
  bool chroma_zero = true;
  for (int comp = 1; comp < 3 && chroma_zero; ++comp) {
    const JpegComponent& jc = jpg444.components[comp];
    const int* q = jpg444.quant[jc.quant_idx].values;
    for (int by = 0; by < img.bh && chroma_zero; ++by)
      for (int bx = 0; bx < img.bw; ++bx) {
        const coeff_t* src = &jc.coeffs[(static_cast<size_t>(by) * jc.width_in_blocks + bx) * 64];
        for (int k = 0; k < 64; ++k)
          if (static_cast<coeff_t>(src[k] * q[k]) != 0) chroma_zero = false;
      }
  }
  if (chroma_zero) return false;
  std::vector<Plane> yuv(3, Plane(static_cast<size_t>(w) * h));
  std::vector<coeff_t> down[3];
  if (silver_screen) {
    // ToSRGB of the 4:4:4 image, then the iterative 4:2:0 fit; all three
    // components are re-derived from it
    std::vector<uint8_t> rgb;
    if (!DecodeJpegToRGB(jpg444, &rgb)) return false;
    yuv = RGBToYUV420(rgb, w, h);
    down[0] = DownsampledCoefficients(yuv[0], w, h, 1);
  } else {
    // ToFloatPixels (output_image.cc:100-122): float64 IDCT + 128 per
    // component, then PreProcessChannel for u and v
    for (int comp = 0; comp < 3; ++comp) {
      const JpegComponent& jc = jpg444.components[comp];
      const int* q = jpg444.quant[jc.quant_idx].values;
      for (int by = 0; by < img.bh; ++by)
        for (int bx = 0; bx < img.bw; ++bx) {
          const coeff_t* src = &jc.coeffs[(static_cast<size_t>(by) * jc.width_in_blocks + bx) * 64];
          double blockd[64];
          for (int k = 0; k < 64; ++k) blockd[k] = static_cast<coeff_t>(src[k] * q[k]);
          BlockIdctDouble(blockd);
          for (int iy = 0; iy < 8; ++iy)
            for (int ix = 0; ix < 8; ++ix) {
              const int yy = 8 * by + iy, xx = 8 * bx + ix;
              if (yy >= h || xx >= w) continue;
              yuv[comp][static_cast<size_t>(yy) * w + xx] = static_cast<float>(blockd[8 * iy + ix] + 128.0);
            }
        }
    }
    // (the reference passes u_sharpen / u_blur in the blur / sharpen slots;
    // both are true in the default DownsampleConfig)
    PreProcessChannel(w, h, 2, 1.3f, 0.5f, true, true, &yuv);
    PreProcessChannel(w, h, 1, 1.3f, 0.5f, true, true, &yuv);
  }
  if (!down[0].empty()) img.y = down[0];
  img.c[0] = DownsampledCoefficients(yuv[1], w, h, 2);
  img.c[1] = DownsampledCoefficients(yuv[2], w, h, 2);
  *jpg420 = JpegData();
  jpg420->app_data = jpg444.app_data;
  jpg420->com_data = jpg444.com_data;
  img.SaveToJpegData(jpg420);
  return true;
}

}  // namespace gz
