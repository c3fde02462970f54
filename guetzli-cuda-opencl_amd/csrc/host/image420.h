// The YUV 4:2:0 side of the search (Params::try_420 / force_420 and 4:2:0
// JPEG input): guetzli::OutputImage with Y at factor 1 and Cb / Cr at factor
// 2 (guetzli/output_image.cc), and OutputImage::Downsample with
// PreProcessChannel (output_image.cc:494-571, preprocess_downsample.cc).
//
// A factor-2 component's pixels are state, not a function of its
// coefficients: SetCoeffBlock rebuilds the subsampled ring around the block
// by inverting the fancy upsampler on the pixels as they are
// (output_image.cc:147-204), so the pixels depend on the order of every
// block update since the last Reset.  Image420 keeps that state on the host
// exactly as the reference evolves it; the zeroing search of the chroma
// (the device kernel k_block_zeroing420) continues it on the GPU and hands it
// back.
#pragma once

#include <stdint.h>

#include <vector>

#include "host/jpeg_model.h"

namespace gz {

// ComputeBlockIDCT (idct.cc:139-161): libjpeg-exact integer IDCT -> bytes.
void BlockIdctBytes(const coeff_t* in, uint8_t out[64]);

// One OutputImageComponent's pixel plane (output_image.cc:36-50): 16-bit
// values (sample << 4) at full image resolution, blocks at 1 / factor.
struct SubsampledPlane {
  int w = 0, h = 0, f = 1, wib = 0, hib = 0;
  std::vector<uint16_t> px;
  // Reset(factor) (output_image.cc:41-50): every pixel 128 << 4.
  void Reset(int width, int height, int factor);
  // UpdatePixelsForBlock (output_image.cc:135-205) with the block's IDCT bytes.
  void Update(int bx, int by, const uint8_t idct[64]);
};

// ToPixels' byte of a 16-bit pixel at column x (output_image.cc:83).
inline uint8_t PixelByte(uint16_t p, int x) { return static_cast<uint8_t>((p + 8 - (x & 1)) >> 4); }

struct Image420 {
  int w = 0, h = 0;
  int bw = 0, bh = 0;    // Y blocks (8x8 pixels)
  int cbw = 0, cbh = 0;  // Cb / Cr blocks (16x16 pixels)
  std::vector<coeff_t> y;     // [bw * bh][64], dequantized (value * quant)
  std::vector<coeff_t> c[2];  // [cbw * cbh][64], dequantized
  SubsampledPlane plane[2];   // Cb, Cr pixels (state)
  int quant[3][kDCTBlockSize];

  void Init(int width, int height);
  int Blocks(int comp) const { return comp == 0 ? bw * bh : cbw * cbh; }
  int BlockWidth(int comp) const { return comp == 0 ? bw : cbw; }
  coeff_t* block(int comp, int b) {
    return comp == 0 ? &y[static_cast<size_t>(b) * 64] : &c[comp - 1][static_cast<size_t>(b) * 64];
  }
  const coeff_t* block(int comp, int b) const {
    return comp == 0 ? &y[static_cast<size_t>(b) * 64] : &c[comp - 1][static_cast<size_t>(b) * 64];
  }
  // SetCoeffBlock (output_image.cc:124-133): the coefficients, and for the
  // chroma the pixel update.
  void SetCoeffBlock(int comp, int b, const coeff_t* blk);
  // CopyFromJpegData (output_image.cc:481-492, 212-228) of a 3-component
  // 4:2:0 JpegData (Y 2x2, Cb / Cr 1x1): Reset, then every block in raster
  // order, dequantized.
  void CopyFromJpegData(const JpegData& jpg);
  // ApplyGlobalQuantization (output_image.cc:349-360, 573-577): changed
  // blocks only, raster order.
  void ApplyGlobalQuantization(const int q[3][kDCTBlockSize]);
  bool ChromaAllZero() const;
  // SaveToJpegData (output_image.cc:579-640): Y 2x2 / chroma 1x1 MCUs
  // (1 component when both chroma planes are all zero).
  void SaveToJpegData(JpegData* jpg) const;
  // SaveToJpegData over meta's app / com data, kept current between calls:
  // the blocks SetCoeffBlock changed since the last call re-quantized, the
  // rest as saved (a whole SaveToJpegData after Init / CopyFromJpegData /
  // ApplyGlobalQuantization, a changed DC -- padding blocks repeat the last
  // DC -- or a changed component count).  The search writes one candidate
  // per iteration and changes few blocks between them.
  const JpegData& SavedJpegData(const JpegData& meta);

  JpegData saved_;
  bool saved_ok_ = false;
  std::vector<int> dirty_[3];  // blocks set since the last SavedJpegData
 private:
  void SavedReset() {
    saved_ok_ = false;
    for (auto& d : dirty_) d.clear();
  }
};

// Processor::DownsampleImage + OutputImage::Downsample + SaveToJpegData
// (processor.cc:109-116, 994-997; output_image.cc:535-571) of a 3-component
// 4:4:4 JpegData at quant 1: the chroma through PreProcessChannel (u, then
// v) and SetDownsampledCoefficients (2x2 average, float64 DCT), or with
// silver_screen the whole image through RGBToYUV420 (preprocess_downsample.cc:
// 452-476).  False when both chroma components are all zero (the reference
// leaves such an image at 4:4:4 and saves it as one grayscale component).
bool DownsampleToJpegData420(const JpegData& jpg444, bool silver_screen, JpegData* jpg420);

// ComputeBlockDCTDouble / ComputeBlockIDCTDouble (dct_double.cc:79-85).
void BlockDctDouble(double block[64]);
void BlockIdctDouble(double block[64]);

}  // namespace gz
