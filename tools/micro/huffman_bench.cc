// Host micro-benchmark of the back end's entropy-code rebuilds (ClusterHistograms
// over the three AC histograms, as ComputeEntropyCodes calls it every 10
// coefficient changes): realistic 1080p histograms from a synthetic frame's
// q=1 coefficients quantized with q95-like tables, then zeroing changes in
// random blocks with a rebuild after every 10.  Prints the time per rebuild
// and a checksum of every depth array (to compare builds of the Huffman code).
//
//   make -C tools/micro huffman_bench && tools/micro/huffman_bench [frames.rgb]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <cmath>
#include <cstring>
#include <random>
#include <vector>

#include "host/jpeg_writer.h"
#include "guetzli_hip.h"

using namespace gz;

namespace {
const int kZig[64] = {0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
                      3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
                      10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
                      21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};

int Log2Floor(uint32_t v) { return 31 - __builtin_clz(v); }

// AC symbols of one block (quantized values, natural order) with weight w
void BlockSymbols(const int16_t* q, int w, JpegHistogram* h) {
  int z[64];
  for (int k = 0; k < 64; ++k) z[kZig[k]] = q[k];
  int r = 0;
  for (int k = 1; k < 64; ++k) {
    if (z[k] == 0) {
      ++r;
      continue;
    }
    while (r > 15) {
      h->counts[0xf0] += 2 * w;
      r -= 16;
    }
    const int a = z[k] < 0 ? -z[k] : z[k];
    h->counts[(r << 4) + Log2Floor(a) + 1] += 2 * w;
    r = 0;
  }
  if (r > 0) h->counts[0] += 2 * w;
}
}  // namespace

int main(int argc, char** argv) {
  const int W = 1920, H = 1080, bw = W / 8, bh = (H + 7) / 8, nb = bw * bh;
  std::vector<uint8_t> rgb(static_cast<size_t>(3) * W * H);
  if (argc > 1) {
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(rgb.data(), 1, rgb.size(), f) != rgb.size()) {
      fprintf(stderr, "cannot read %s\n", argv[1]);
      return 1;
    }
    fclose(f);
  } else {
    std::mt19937 g(1);
    for (int y = 0; y < H; ++y)
      for (int x = 0; x < W; ++x)
        for (int c = 0; c < 3; ++c)
          rgb[(static_cast<size_t>(y) * W + x) * 3 + c] =
              static_cast<uint8_t>(128 + 60 * std::sin(0.01 * x * (c + 1) + 0.013 * y) + (g() % 24));
  }
  std::vector<int16_t> co(static_cast<size_t>(3) * nb * 64);
  if (gz_rgb_to_coeffs(rgb.data(), W, H, co.data()) != 0) {
    fprintf(stderr, "rgb_to_coeffs failed\n");
    return 1;
  }
  // q95-like: small luma steps, larger chroma
  int qt[3][64];
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 64; ++k) qt[c][k] = (c == 0 ? 2 : 3) + (k / 8 + k % 8) / (c == 0 ? 3 : 2);
  std::vector<int16_t> q(co.size());
  for (size_t i = 0; i < co.size(); ++i) {
    const int c = static_cast<int>(i / (static_cast<size_t>(nb) * 64)), k = static_cast<int>(i % 64);
    q[i] = static_cast<int16_t>(co[i] / qt[c][k]);
  }
  std::vector<JpegHistogram> hist(3);
  for (int c = 0; c < 3; ++c)
    for (int b = 0; b < nb; ++b) BlockSymbols(&q[(static_cast<size_t>(c) * nb + b) * 64], 1, &hist[c]);
  std::mt19937 g(7);
  const int kRebuilds = 2000;
  double secs = 0.0;
  uint64_t sum = 0;
  for (int it = 0; it < kRebuilds; ++it) {
    for (int t = 0; t < 10; ++t) {  // ten changes: a non-zero AC coefficient zeroed
      for (;;) {
        const int c = static_cast<int>(g() % 3), b = static_cast<int>(g() % nb), k = 1 + static_cast<int>(g() % 63);
        int16_t* blk = &q[(static_cast<size_t>(c) * nb + b) * 64];
        if (!blk[k]) continue;
        BlockSymbols(blk, -1, &hist[c]);
        blk[k] = 0;
        BlockSymbols(blk, 1, &hist[c]);
        break;
      }
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<JpegHistogram> clustered = hist;
    size_t num = 3;
    int idx[3];
    std::vector<uint8_t> depths(3 * JpegHistogram::kSize);
    const size_t bytes = ClusterHistograms(clustered.data(), &num, idx, depths.data());
    secs += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    for (size_t i = 0; i < depths.size(); ++i) sum = sum * 1099511628211ull + depths[i] + 1;
    sum += bytes + num;
  }
  printf("%d rebuilds: %.2f us each; checksum %016llx\n", kRebuilds, 1e6 * secs / kRebuilds,
         static_cast<unsigned long long>(sum));
  return 0;
}
