// Initial q=1 coefficients of an RGB image (EncodeRGBToJpeg,
// guetzli/jpeg_data_encoder.cc:66-136).
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace gz {

// In-place 16-bit scaled integer forward DCT of one 8x8 block
// (ComputeBlockDCT, guetzli/fdct.cc:230-240).
void ForwardDct8x8(int16_t* block);

// coeffs: [3][ceil(h/8)*ceil(w/8)][64], natural order.
void RgbToCoeffsQ1(const uint8_t* rgb, int w, int h, int16_t* coeffs);

}  // namespace gz
