#include "host/jpeg_model.h"

#include <cstring>

namespace gz {

const int kJPEGNaturalOrder[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63,
};

const int kJPEGZigZagOrder[64] = {
    0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42, 3,  8,  12, 17, 25, 30,
    41, 43, 9,  11, 18, 24, 31, 40, 44, 53, 10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38,
    46, 51, 55, 60, 21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63,
};

void InitJpegDataYUV444(int w, int h, JpegData* jpg) {
  jpg->width = w;
  jpg->height = h;
  jpg->max_h_samp_factor = 1;
  jpg->max_v_samp_factor = 1;
  jpg->mcu_rows = (h + 7) >> 3;
  jpg->mcu_cols = (w + 7) >> 3;
  jpg->quant.assign(3, QuantTable());
  jpg->components.assign(3, JpegComponent());
  for (int i = 0; i < 3; ++i) {
    JpegComponent& c = jpg->components[i];
    c.id = i;
    c.quant_idx = i;
    c.width_in_blocks = jpg->mcu_cols;
    c.height_in_blocks = jpg->mcu_rows;
    c.coeffs.assign(static_cast<size_t>(c.width_in_blocks) * c.height_in_blocks * 64, 0);
  }
  static const unsigned char kApp0[] = {0xe0, 0x00, 0x10, 0x4a, 0x46, 0x49, 0x46, 0x00, 0x01,
                                        0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
  jpg->app_data.assign(1, std::string(reinterpret_cast<const char*>(kApp0), sizeof(kApp0)));
}

void SaveQuantTables(const int q[3][kDCTBlockSize], JpegData* jpg) {
  jpg->quant.clear();
  for (size_t i = 0; i < jpg->components.size(); ++i) {
    JpegComponent& comp = jpg->components[i];
    int found = -1;
    for (size_t j = 0; j < jpg->quant.size(); ++j) {
      if (std::memcmp(q[i], jpg->quant[j].values, sizeof(jpg->quant[j].values)) == 0) {
        found = static_cast<int>(j);
        break;
      }
    }
    if (found < 0) {
      QuantTable t;
      std::memcpy(t.values, q[i], sizeof(t.values));
      t.precision = 0;
      for (int k = 0; k < kDCTBlockSize; ++k)
        if (t.values[k] > 0xff) t.precision = 1;
      t.index = static_cast<int>(jpg->quant.size());
      found = t.index;
      jpg->quant.push_back(t);
    }
    comp.quant_idx = found;
  }
}

void CoeffImage::Init(int w, int h) {
  width = w;
  height = h;
  block_w = (w + 7) / 8;
  block_h = (h + 7) / 8;
  blocks = block_w * block_h;
  coeffs.assign(static_cast<size_t>(blocks) * 64 * 3, 0);
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 64; ++k) quant[c][k] = 1;
  BulkChanged();
}

void CoeffImage::CopyFromJpegData(const JpegData& jpg) {
  for (int c = 0; c < 3; ++c) {
    const JpegComponent& comp = jpg.components[c];
    const int* q = jpg.quant[comp.quant_idx].values;
    for (int by = 0; by < block_h; ++by)
      for (int bx = 0; bx < block_w; ++bx) {
        const coeff_t* src = &comp.coeffs[(static_cast<size_t>(by) * comp.width_in_blocks + bx) * 64];
        coeff_t* dst = block(c, by * block_w + bx);
        for (int k = 0; k < 64; ++k) dst[k] = static_cast<coeff_t>(src[k] * q[k]);
      }
    std::memcpy(quant[c], q, sizeof(quant[c]));
  }
  BulkChanged();
}

void CoeffImage::ApplyGlobalQuantization(const int q[3][kDCTBlockSize]) {
  for (int c = 0; c < 3; ++c) {
    coeff_t* p = block(c, 0);
    const size_t n = static_cast<size_t>(blocks) * 64;
    for (size_t i = 0; i < n; ++i) p[i] = QuantizeCoeff(p[i], q[c][i & 63]);
    std::memcpy(quant[c], q[c], sizeof(quant[c]));
  }
  BulkChanged();
}

bool CoeffImage::ComponentIsAllZero(int c) const {
  const coeff_t* p = block(c, 0);
  const size_t n = static_cast<size_t>(blocks) * 64;
  for (size_t i = 0; i < n; ++i)
    if (p[i] != 0) return false;
  return true;
}

void JpegHeaderFor(int w, int h, const int q[3][kDCTBlockSize], int ncomp, JpegData* jpg) {
  jpg->width = w;
  jpg->height = h;
  jpg->max_h_samp_factor = 1;
  jpg->max_v_samp_factor = 1;
  jpg->mcu_cols = (w + 7) / 8;
  jpg->mcu_rows = (h + 7) / 8;
  jpg->components.resize(ncomp);
  for (int c = 0; c < ncomp; ++c) {
    JpegComponent& comp = jpg->components[c];
    comp.id = c;
    comp.h_samp_factor = 1;
    comp.v_samp_factor = 1;
    comp.width_in_blocks = jpg->mcu_cols;
    comp.height_in_blocks = jpg->mcu_rows;
    comp.coeffs.clear();
  }
  SaveQuantTables(q, jpg);
}

void JpegHeaderOf(const JpegData& jpg, JpegData* hdr) {
  hdr->width = jpg.width;
  hdr->height = jpg.height;
  hdr->max_h_samp_factor = jpg.max_h_samp_factor;
  hdr->max_v_samp_factor = jpg.max_v_samp_factor;
  hdr->mcu_cols = jpg.mcu_cols;
  hdr->mcu_rows = jpg.mcu_rows;
  hdr->app_data = jpg.app_data;
  hdr->com_data = jpg.com_data;
  hdr->quant = jpg.quant;
  hdr->components.resize(jpg.components.size());
  for (size_t c = 0; c < jpg.components.size(); ++c) {
    const JpegComponent& src = jpg.components[c];
    JpegComponent& dst = hdr->components[c];
    dst.id = src.id;
    dst.h_samp_factor = src.h_samp_factor;
    dst.v_samp_factor = src.v_samp_factor;
    dst.quant_idx = src.quant_idx;
    dst.width_in_blocks = src.width_in_blocks;
    dst.height_in_blocks = src.height_in_blocks;
    dst.coeffs.clear();
  }
}

void CoeffImage::SaveHeaderToJpegData(int ncomp, JpegData* jpg) const {
  JpegHeaderFor(width, height, quant, ncomp, jpg);
}

void CoeffImage::SaveToJpegData(JpegData* jpg) const {
  jpg->width = width;
  jpg->height = height;
  jpg->max_h_samp_factor = 1;
  jpg->max_v_samp_factor = 1;
  jpg->mcu_cols = block_w;
  jpg->mcu_rows = block_h;
  const int ncomp = ComponentIsAllZero(1) && ComponentIsAllZero(2) ? 1 : 3;
  jpg->components.resize(ncomp);
  for (int c = 0; c < ncomp; ++c) {
    JpegComponent& comp = jpg->components[c];
    comp.id = c;
    comp.h_samp_factor = 1;
    comp.v_samp_factor = 1;
    comp.width_in_blocks = block_w;
    comp.height_in_blocks = block_h;
    const size_t n = static_cast<size_t>(blocks) * 64;
    comp.coeffs.resize(n);
    const coeff_t* src = block(c, 0);
    for (size_t i = 0; i < n; ++i) comp.coeffs[i] = static_cast<coeff_t>(src[i] / quant[c][i & 63]);
  }
  SaveQuantTables(quant, jpg);
}

}  // namespace gz
