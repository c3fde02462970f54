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
  const bool direct_equal = a == b;
  // incremental restaging from the change journal: random edits (AC zeroing,
  // AC re-quantized values, DC moves, finally all chroma cleared) between
  // writes must give the bytes of a fresh SaveToJpegData + WriteJpeg
  {
    uint64_t rs = 12345;
    auto rnd = [&rs]() {
      rs = rs * 6364136223846793005ull + 1442695040888963407ull;
      return static_cast<uint32_t>(rs >> 33);
    };
    for (int round = 0; round < 6; ++round) {
      const int nchange = round == 0 ? 1 : 200 * round;
      for (int i = 0; i < nchange; ++i) {
        const int c = rnd() % 3, b = rnd() % img.blocks;
        int k = rnd() % 64;
        if (round < 3 && k == 0) k = 1;
        gz::coeff_t* blk = img.block(c, b);
        const int q = img.quant[c][k];
        blk[k] = static_cast<gz::coeff_t>((round & 1) ? 0 : q * (static_cast<int>(rnd() % 41) - 20));
        img.MarkChanged(c, b, k);
      }
      if (round == 5) {
        for (int c = 1; c < 3; ++c)
          for (int b = 0; b < img.blocks; ++b)
            for (int k = 0; k < 64; ++k)
              if (img.block(c, b)[k] != 0) {
                img.block(c, b)[k] = 0;
                img.MarkChanged(c, b, k);
              }
      }
      std::string ref, got;
      gz::JpegData out = jpg;
      img.SaveToJpegData(&out);
      gz::WriteJpegReference(out, true, &ref);
      gz::WriteCoeffImageJpeg(img, jpg, true, s, &got);
      if (ref != got) {
        printf("{\"equal\": 0, \"what\": \"incremental round %d\"}\n", round);
        return 5;
      }
    }
  }
  // stage / encode split (single call each, after warm-up)
  double t_stage = 0, t_enc = 0;
  for (int r = 0; r < reps; ++r) {
    auto ta = Clock::now();
    gz::StageCoeffImage(img, jpg, s);
    auto tb = Clock::now();
    b.clear();
    gz::EncodeStaged(s, true, &b);
    auto tc = Clock::now();
    t_stage += std::chrono::duration<double>(tb - ta).count() / reps;
    t_enc += std::chrono::duration<double>(tc - tb).count() / reps;
  }
  fprintf(stderr, "stage_ms %.3f encode_ms %.3f\n", t_stage * 1e3, t_enc * 1e3);
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
         direct_equal ? 1 : 0, ta * 1e3, tb * 1e3);
  return direct_equal ? 0 : 3;
}
