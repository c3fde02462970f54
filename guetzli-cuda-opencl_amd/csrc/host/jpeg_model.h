// Host-side JPEG container model of the search loop (the subset of
// guetzli::JPEGData, guetzli/jpeg_data.h:138-204, that a 4:4:4 baseline
// Huffman encode needs) and the coefficient image the loop edits
// (guetzli::OutputImage restricted to factor-1 components,
// guetzli/output_image.h).
#pragma once

#include <stdint.h>

#include <string>
#include <vector>

namespace gz {

using coeff_t = int16_t;
constexpr int kDCTBlockSize = 64;

extern const int kJPEGNaturalOrder[64];  // zigzag position -> natural index
extern const int kJPEGZigZagOrder[64];   // natural index -> zigzag position

struct QuantTable {
  int values[kDCTBlockSize];
  int precision = 0;
  int index = 0;
};

struct JpegComponent {
  int id = 0;
  int h_samp_factor = 1;
  int v_samp_factor = 1;
  int quant_idx = 0;
  int width_in_blocks = 0;
  int height_in_blocks = 0;
  std::vector<coeff_t> coeffs;  // [blocks][64], natural order
};

struct JpegData {
  int width = 0;
  int height = 0;
  int max_h_samp_factor = 1;
  int max_v_samp_factor = 1;
  int mcu_rows = 0;
  int mcu_cols = 0;
  std::vector<std::string> app_data;
  std::vector<std::string> com_data;
  std::vector<QuantTable> quant;
  std::vector<JpegComponent> components;
};

// InitJPEGDataForYUV444 + AddApp0Data (jpeg_data.cc:49-69,
// jpeg_data_encoder.cc:51-63).
void InitJpegDataYUV444(int w, int h, JpegData* jpg);
// SaveQuantTables (jpeg_data.cc:71-101): de-duplicates identical tables.
void SaveQuantTables(const int q[3][kDCTBlockSize], JpegData* jpg);

// Coefficient image (4:4:4).  coeffs is [3][blocks][64] of DEQUANTISED
// values (quantized value * quant), as OutputImageComponent stores them.
struct CoeffImage {
  int width = 0, height = 0, block_w = 0, block_h = 0, blocks = 0;
  std::vector<coeff_t> coeffs;
  int quant[3][kDCTBlockSize];
  // Change journal for mirrors of the coefficients (the device copy, the
  // writer's quantized copy): `epoch` changes on every bulk rewrite, within
  // an epoch every single-coefficient write appends its flat index to
  // `changed`.  A mirror remembers the (epoch, journal length) it reflects.
  uint64_t epoch = 0;
  std::vector<uint32_t> changed;
  // False while only a device mirror holds the current coefficients (after a
  // device-side global quantization whose host copy was not requested).
  bool host_valid = true;
  // True while the search back end keeps the host copy lazily: some blocks
  // lag changes made on the device copy alone (Processor materialises a
  // block before it reads or journals it).  The journalled entries are
  // current, so a mirror may replay the journal but not re-read the rest.
  bool host_partial = false;
  void MarkChanged(int c, int block_ix, int k) {
    changed.push_back(static_cast<uint32_t>((static_cast<size_t>(c) * blocks + block_ix) * 64 + k));
  }
  void BulkChanged() {  // (also: the host copy is the authoritative one)
    ++epoch;
    changed.clear();
    host_valid = true;
    host_partial = false;
  }

  void Init(int w, int h);
  coeff_t* block(int c, int block_ix) { return &coeffs[(static_cast<size_t>(c) * blocks + block_ix) * 64]; }
  const coeff_t* block(int c, int block_ix) const {
    return &coeffs[(static_cast<size_t>(c) * blocks + block_ix) * 64];
  }
  // CopyFromJpegData (output_image.cc:481-492, 212-228)
  void CopyFromJpegData(const JpegData& jpg);
  // ApplyGlobalQuantization on the host (output_image.cc:349-360, 573-577)
  void ApplyGlobalQuantization(const int q[3][kDCTBlockSize]);
  // SaveToJpegData (output_image.cc:579-640)
  void SaveToJpegData(JpegData* jpg) const;
  // Everything SaveToJpegData sets except the coefficient arrays (left empty),
  // for a component count already known.
  void SaveHeaderToJpegData(int ncomp, JpegData* jpg) const;
  bool ComponentIsAllZero(int c) const;
};

// What a mirror of a CoeffImage reflects (see CoeffImage::epoch).
struct CoeffCursor {
  uint64_t epoch = ~0ull;
  size_t pos = 0;
  bool Current(const CoeffImage& img) const { return epoch == img.epoch && pos == img.changed.size(); }
  bool CanReplay(const CoeffImage& img) const { return epoch == img.epoch && pos <= img.changed.size(); }
  void Set(const CoeffImage& img) {
    epoch = img.epoch;
    pos = img.changed.size();
  }
};

// The header part of SaveToJpegData for a w x h 4:4:4 image with quant q and
// ncomp stored components (components without coefficients).
void JpegHeaderFor(int w, int h, const int q[3][kDCTBlockSize], int ncomp, JpegData* jpg);
// jpg's header fields (frame, components without coefficients, quant
// tables, APPn / COM data) into *hdr.
void JpegHeaderOf(const JpegData& jpg, JpegData* hdr);

// Quantize (guetzli/quantize.h:25-30)
inline coeff_t QuantizeCoeff(coeff_t raw, int quant) {
  const int r = raw % quant;
  const coeff_t delta = 2 * r > quant ? quant - r : (-2) * r > quant ? -quant - r : -r;
  return static_cast<coeff_t>(raw + delta);
}

}  // namespace gz
