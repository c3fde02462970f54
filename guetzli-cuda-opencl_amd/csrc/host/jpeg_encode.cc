// Initial 4:4:4 JPEG coefficients from RGB at quantization 1
// (EncodeRGBToJpeg, guetzli/jpeg_data_encoder.cc:66-136): fixed-point
// RGB->YUV, the 16-bit scaled integer forward DCT of guetzli/fdct.cc and the
// reciprocal-multiply quantizer.  All arithmetic is 32-bit integer with the
// reference's truncations to int16 at every store.
#include "host/jpeg_encode.h"
#include "host/thread_pool.h"

#include <algorithm>
#include <cstring>

namespace gz {
namespace {

inline int16_t S16(int v) { return static_cast<int16_t>(v); }
inline int MulHi(int a, int b) { return (a * b) >> 16; }  // MULT(), fdct.cc:151

// Column pass of the forward DCT on column `col` (stride 8): the butterfly /
// rotation network of fdct.cc:68-145 (constants: tan(pi/16), tan(pi/8),
// tan(3pi/16)-1, 1/(2 sqrt 2) in 16-bit fixed point).
void ForwardDctColumn(int16_t* d) {
  const int kTan1 = 13036, kTan2 = 27146, kTan3m1 = -21746, k2Sqrt2 = 23170;
  int a0 = d[0], a1 = d[8], a2 = d[16], a3 = d[24];
  int a4 = d[32], a5 = d[40], a6 = d[48], a7 = d[56];
  // stage 1: sums / differences of mirrored samples
  int s07 = a0 + a7, d07 = a0 - a7;
  int s25 = a2 + a5, d25 = a2 - a5;
  int s34 = a3 + a4, d34 = a3 - a4;
  int s16 = a1 + a6, d16 = a1 - a6;
  // even part
  int e0 = s07 + s34, e1 = s07 - s34;   // (m4, m7) after BUTTERFLY(m7, m4)
  int e2 = s16 + s25, e3 = s16 - s25;   // (m5, m6) after BUTTERFLY(m6, m5)
  e0 <<= 3;
  e2 <<= 3;
  d[0] = S16(e0 + e2);
  d[32] = S16(e0 - e2);
  e1 <<= 3;
  e3 <<= 3;
  d[16] = S16(MulHi(kTan2, e3) + e1);
  d[48] = S16(MulHi(kTan2, e1) - e3);
  // odd part
  d34 <<= 3;
  d07 <<= 3;
  d25 <<= 4;
  d16 <<= 4;
  const int p = MulHi(d16 + d25, k2Sqrt2);
  const int q = MulHi(d16 - d25, k2Sqrt2);
  const int o3 = d34 - q, o1 = d34 + q;
  const int o0 = d07 - p, o2 = d07 + p;
  const int r3 = MulHi(o3, kTan3m1) + o3 + 1;
  const int r1 = MulHi(o1, kTan1) + o2 + 1;
  d[8] = S16(r1);
  d[24] = S16(o0 - r3);
  d[40] = S16(o3 + (MulHi(kTan3m1, o0) + o0));
  d[56] = S16(MulHi(kTan1, o2) - o1);
}

// Row pass (RowDct, fdct.cc:173-208) with per-row constant tables.
void ForwardDctRow(int16_t* in, const int16_t* t) {
  const int a0 = in[0] + in[7], b0 = in[0] - in[7];
  const int a1 = in[1] + in[6], b1 = in[1] - in[6];
  const int a2 = in[2] + in[5], b2 = in[2] - in[5];
  const int a3 = in[3] + in[4], b3 = in[3] - in[4];
  const int c0 = a0 + a3, c1 = a0 - a3, c2 = a1 + a2, c3 = a1 - a2;
  const int C1 = t[0], C2 = t[1], C3 = t[2], C4 = t[3], C5 = t[4], C6 = t[5], C7 = t[6];
  in[0] = S16((C4 * (c0 + c2)) >> 16);
  in[4] = S16((C4 * (c0 - c2)) >> 16);
  in[2] = S16((C2 * c1 + C6 * c3) >> 16);
  in[6] = S16((C6 * c1 - C2 * c3) >> 16);
  in[1] = S16((C1 * b0 + C3 * b1 + C5 * b2 + C7 * b3) >> 16);
  in[3] = S16((C3 * b0 - C7 * b1 - C1 * b2 - C5 * b3) >> 16);
  in[5] = S16((C5 * b0 - C1 * b1 + C7 * b2 + C3 * b3) >> 16);
  in[7] = S16((C7 * b0 - C5 * b1 + C3 * b2 - C1 * b3) >> 16);
}

// cos(k pi/16)/sqrt(2) scaled per row pair (fdct.cc:31-38).
const int16_t kRow04[7] = {22725, 21407, 19266, 16384, 12873, 8867, 4520};
const int16_t kRow17[7] = {31521, 29692, 26722, 22725, 17855, 12299, 6270};
const int16_t kRow26[7] = {29692, 27969, 25172, 21407, 16819, 11585, 5906};
const int16_t kRow35[7] = {26722, 25172, 22654, 19266, 15137, 10426, 5315};

}  // namespace

void ForwardDct8x8(int16_t* block) {
  for (int i = 0; i < 8; ++i) ForwardDctColumn(block + i);
  static const int16_t* const kRows[8] = {kRow04, kRow17, kRow26, kRow35,
                                          kRow04, kRow35, kRow26, kRow17};
  for (int r = 0; r < 8; ++r) ForwardDctRow(block + 8 * r, kRows[r]);
}

void RgbToCoeffsQ1(const uint8_t* rgb, int w, int h, int16_t* coeffs) {
  const int bw = (w + 7) / 8, bh = (h + 7) / 8;
  const size_t nb = static_cast<size_t>(bw) * bh;
  // quantizer at q = 1: iquant = ((1 << 16) + 1) / 1, bias 0x80 << 12, shift 20
  const uint32_t kIQuant = 65537u, kBias = 0x80u << 12;
  // block rows are independent: spread them over the host pool
  ParallelFor(bh, [&](int by) {
    for (int bx = 0; bx < bw; ++bx) {
      int16_t blk[3][64];
      for (int iy = 0; iy < 8; ++iy) {
        for (int ix = 0; ix < 8; ++ix) {
          const int y = std::min(h - 1, 8 * by + iy), x = std::min(w - 1, 8 * bx + ix);
          const uint8_t* px = rgb + 3 * (static_cast<size_t>(y) * w + x);
          const int r = px[0], g = px[1], b = px[2];
          // RGBToYUV16, jpeg_data_encoder.cc:40-49
          blk[0][8 * iy + ix] = S16((19595 * r + 38469 * g + 7471 * b - (128 << 16) + 32768) >> 16);
          blk[1][8 * iy + ix] = S16((-11059 * r - 21709 * g + 32768 * b + 32767) >> 16);
          blk[2][8 * iy + ix] = S16((32768 * r - 27439 * g - 5329 * b + 32767) >> 16);
        }
      }
      for (int c = 0; c < 3; ++c) {
        ForwardDct8x8(blk[c]);
        int16_t* dst = coeffs + (c * nb + static_cast<size_t>(by) * bw + bx) * 64;
        for (int k = 0; k < 64; ++k) {
          const uint32_t v = static_cast<uint32_t>(static_cast<int>(blk[c][k])) * kIQuant + kBias;
          dst[k] = S16(static_cast<int>(v) >> 20);
        }
      }
    }
  });
}

}  // namespace gz
