// Deterministic synthetic sRGB frames for benchmarks and parity tests
// (generator specified in SURVEY.md §8(d)): per channel a base of 128 plus
// four sinusoids, N(0, 8^2) noise smoothed by [1,4,6,4,1]/16, and
// max(4, P/200000) rectangles blended 50 % toward a mid-range colour;
// rounded and clipped to [16, 240].  splitmix64-seeded, bit-reproducible on
// the same libm.
#include "host/synthetic.h"

#include <algorithm>
#include <cmath>
#include <vector>

namespace gz {
namespace {

struct SplitMix64 {
  uint64_t s;
  uint64_t Next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double Uniform() { return static_cast<double>(Next() >> 11) * (1.0 / 9007199254740992.0); }
  double Range(double lo, double hi) { return lo + (hi - lo) * Uniform(); }
};

}  // namespace

void SyntheticFrame(uint64_t seed, int w, int h, uint8_t* rgb) {
  SplitMix64 rng{seed * 0x2545F4914F6CDD1Dull + 0x1234567ull};
  const size_t n = static_cast<size_t>(w) * h;
  std::vector<double> img(3 * n);
  std::vector<double> sx(w), cx(w), sy(h), cy(h);
  for (int c = 0; c < 3; ++c) {
    double* p = &img[c * n];
    std::fill(p, p + n, 128.0);
    for (int k = 0; k < 4; ++k) {
      const double a = rng.Range(5.0, 20.0);
      const double fx = rng.Range(0.002, 0.05), fy = rng.Range(0.002, 0.05);
      const double phase = rng.Range(0.0, 2.0 * M_PI);
      // sin(fx x + fy y + phase), separated into row and column factors
      for (int x = 0; x < w; ++x) {
        sx[x] = std::sin(fx * x);
        cx[x] = std::cos(fx * x);
      }
      for (int y = 0; y < h; ++y) {
        sy[y] = std::sin(fy * y + phase);
        cy[y] = std::cos(fy * y + phase);
      }
      for (int y = 0; y < h; ++y)
        for (int x = 0; x < w; ++x) p[static_cast<size_t>(y) * w + x] += a * (sx[x] * cy[y] + cx[x] * sy[y]);
    }
  }
  // Gaussian noise (Box-Muller), smoothed by a separable [1 4 6 4 1]/16 kernel
  std::vector<double> noise(n), tmp(n);
  const double kW[5] = {1.0 / 16, 4.0 / 16, 6.0 / 16, 4.0 / 16, 1.0 / 16};
  for (int c = 0; c < 3; ++c) {
    for (size_t i = 0; i < n; i += 2) {
      const double u1 = 1.0 - rng.Uniform(), u2 = rng.Uniform();
      const double r = std::sqrt(-2.0 * std::log(u1)) * 8.0;
      noise[i] = r * std::cos(2.0 * M_PI * u2);
      if (i + 1 < n) noise[i + 1] = r * std::sin(2.0 * M_PI * u2);
    }
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        double acc = 0.0;
        for (int k = -2; k <= 2; ++k) {
          const int xx = std::min(w - 1, std::max(0, x + k));
          acc += kW[k + 2] * noise[static_cast<size_t>(y) * w + xx];
        }
        tmp[static_cast<size_t>(y) * w + x] = acc;
      }
    double* p = &img[c * n];
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        double acc = 0.0;
        for (int k = -2; k <= 2; ++k) {
          const int yy = std::min(h - 1, std::max(0, y + k));
          acc += kW[k + 2] * tmp[static_cast<size_t>(yy) * w + x];
        }
        p[static_cast<size_t>(y) * w + x] += acc;
      }
  }
  // rectangles
  const int nrect = std::max<int>(4, static_cast<int>(n / 200000));
  for (int r = 0; r < nrect; ++r) {
    const int rw = std::max(1, 8 + static_cast<int>(rng.Uniform() * std::max(1, w / 6 - 8)));
    const int rh = std::max(1, 8 + static_cast<int>(rng.Uniform() * std::max(1, h / 6 - 8)));
    const int x0 = static_cast<int>(rng.Uniform() * std::max(1, w - rw));
    const int y0 = static_cast<int>(rng.Uniform() * std::max(1, h - rh));
    double col[3];
    for (int c = 0; c < 3; ++c) col[c] = rng.Range(64.0, 192.0);
    for (int c = 0; c < 3; ++c) {
      double* p = &img[c * n];
      for (int y = y0; y < std::min(h, y0 + rh); ++y)
        for (int x = x0; x < std::min(w, x0 + rw); ++x) {
          double& v = p[static_cast<size_t>(y) * w + x];
          v = 0.5 * v + 0.5 * col[c];
        }
    }
  }
  for (size_t i = 0; i < n; ++i)
    for (int c = 0; c < 3; ++c) {
      const double v = std::floor(img[c * n + i] + 0.5);
      rgb[3 * i + c] = static_cast<uint8_t>(std::min(240.0, std::max(16.0, v)));
    }
}

}  // namespace gz
