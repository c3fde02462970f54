// Host writer check: the direct multithreaded CoeffImage encoder must produce
// the same bytes as SaveToJpegData + WriteJpeg; prints timings.
//   writer_check RGB W H [QUANT_SCALE]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "host/jpeg_writer.h"
#include "host/processor.h"

int main(int argc, char** argv) {
  if (argc < 4) return 1;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  const int w = atoi(argv[2]), h = atoi(argv[3]);
  const int scale = argc > 4 ? atoi(argv[4]) : 3;
  std::vector<uint8_t> rgb(3 * static_cast<size_t>(w) * h);
  if (fread(rgb.data(), 1, rgb.size(), f) != rgb.size()) return 2;
  fclose(f);
  gz::JpegData jpg;
  gz::EncodeRGBToJpegData(rgb.data(), w, h, &jpg);
  gz::CoeffImage img;
  img.Init(w, h);
  img.CopyFromJpegData(jpg);
  int q[3][64];
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 64; ++k) q[c][k] = 1 + (k * scale + c) % 23;
  img.ApplyGlobalQuantization(q);
  using Clock = std::chrono::steady_clock;
  std::string a, b;
  auto t0 = Clock::now();
  const int reps = 5;
  for (int r = 0; r < reps; ++r) {
    a.clear();
    gz::JpegData out = jpg;
    img.SaveToJpegData(&out);
    gz::WriteJpegReference(out, true, &a);
  }
  auto t1 = Clock::now();
  gz::ScanScratch* s = gz::NewScanScratch();
  for (int r = 0; r < reps; ++r) {
    b.clear();
    gz::WriteCoeffImageJpeg(img, jpg, true, s, &b);
  }
  auto t2 = Clock::now();
  gz::FreeScanScratch(s);
  // the staged path of WriteJpeg on a JpegData (3 quant tables, q=1 input)
  std::string c, d;
  gz::WriteJpegReference(jpg, false, &c);
  gz::WriteJpeg(jpg, false, &d);
  if (c != d) {
    printf("{\"equal\": 0, \"what\": \"jpegdata\"}\n");
    return 4;
  }
  const double ta = std::chrono::duration<double>(t1 - t0).count() / reps;
  const double tb = std::chrono::duration<double>(t2 - t1).count() / reps;
  printf("{\"bytes\": %zu, \"equal\": %d, \"serial_ms\": %.3f, \"direct_ms\": %.3f}\n", a.size(),
         a == b ? 1 : 0, ta * 1e3, tb * 1e3);
  return a == b ? 0 : 3;
}
