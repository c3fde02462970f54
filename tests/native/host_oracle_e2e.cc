// CPU end-to-end check of the product's HOST logic (search loop, quantizer,
// JPEG writer, size estimator) with the comparator backed by the CPU oracle
// instead of the GPU.  Test infrastructure only: links the product library
// for gz::ProcessJpegData and oracle/gz_oracle.c for the comparator.
//
//   host_oracle_e2e RGB W H QUALITY OUT.jpg
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "host/processor.h"

extern "C" {
#include "gz_oracle.h"
}

namespace {

class OracleComparator : public gz::Comparator {
 public:
  OracleComparator(int w, int h, const uint8_t* rgb, float target)
      : w_(w), h_(h), rgb_(rgb, rgb + 3 * static_cast<size_t>(w) * h), target_(target) {
    bw_ = (w + 7) / 8;
    bh_ = (h + 7) / 8;
    block_max_.assign(bw_ * bh_, 0.0f);
  }
  bool Compare(const gz::CoeffImage& img) override {
    std::vector<float> dm(static_cast<size_t>(w_) * h_);
    distance_ = gzo_compare(w_, h_, rgb_.data(), img.coeffs.data(), dm.data());
    for (int by = 0; by < bh_; ++by)
      for (int bx = 0; bx < bw_; ++bx) {
        float m = 0.0f;
        for (int y = 8 * by; y < std::min(h_, 8 * by + 8); ++y)
          for (int x = 8 * bx; x < std::min(w_, 8 * bx + 8); ++x) m = std::max(m, dm[y * w_ + x]);
        block_max_[by * bw_ + bx] = m;
      }
    return true;
  }
  bool StartBlockComparisons() override {
    const size_t n = static_cast<size_t>(w_) * h_;
    std::vector<float> ref(3 * n), dc(3 * n);
    gzo_srgb_to_linear_planes(w_, h_, rgb_.data(), ref.data());
    gzo_opsin_dynamics(w_, h_, ref.data());
    mask_.assign(3 * n, 0.0f);
    gzo_mask(w_, h_, ref.data(), ref.data(), mask_.data(), dc.data());
    return true;
  }
  void FinishBlockComparisons() override { mask_.clear(); }
  bool BlockZeroingOrders(const gz::CoeffImage& img, const gz::JpegData&, int comp_mask,
                          int lookahead, std::vector<gz::CoeffData>* out) override {
    if (comp_mask != 7) return false;
    out->resize(static_cast<size_t>(img.blocks) * 192);
    gzo_block_zeroing_orders(w_, h_, rgb_.data(), mask_.data(), img.coeffs.data(), orig_.data(),
                             target_, lookahead, reinterpret_cast<gzo_coeff_data*>(out->data()));
    return true;
  }
  bool QuantizeFromOriginal(const int q[3][64], gz::CoeffImage* img, bool) override {
    const size_t per = static_cast<size_t>(img->blocks) * 64;
    for (int c = 0; c < 3; ++c)
      for (size_t i = 0; i < per; ++i)
        img->coeffs[c * per + i] = gz::QuantizeCoeff(orig_[c * per + i], q[c][i & 63]);
    for (int c = 0; c < 3; ++c) std::memcpy(img->quant[c], q[c], sizeof(img->quant[c]));
    img->BulkChanged();
    return true;
  }
  double ScoreOutputSize(int size) const override { return gz::ScoreJPEG(distance_, size, target_); }
  bool DistanceOK(double target_mul) const override { return distance_ <= target_mul * target_; }
  float distmap_aggregate() const override { return distance_; }
  const std::vector<float>& block_max_distance() const override { return block_max_; }
  float BlockErrorLimit() const override { return target_; }
  void ComputeBlockErrorAdjustmentWeights(int direction, int max_block_dist, double target_mul,
                                          int fx, int fy, const std::vector<float>& bmax,
                                          std::vector<float>* weight) override {
    gz::BlockErrorAdjustmentWeights(w_, h_, target_, direction, max_block_dist, target_mul, fx, fy,
                                    bmax, weight);
  }
  bool SetOriginalCoeffs(const gz::JpegData& jpg) override {
    orig_.clear();
    for (int c = 0; c < 3; ++c)
      orig_.insert(orig_.end(), jpg.components[c].coeffs.begin(), jpg.components[c].coeffs.end());
    return true;
  }
  const std::string& error() const override { return err_; }

 private:
  int w_, h_, bw_, bh_;
  std::vector<uint8_t> rgb_;
  float target_;
  float distance_ = 0.0f;
  std::vector<float> block_max_, mask_;
  std::vector<gz::coeff_t> orig_;
  std::string err_;
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: host_oracle_e2e RGB W H QUALITY OUT.jpg\n");
    return 1;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  const int w = atoi(argv[2]), h = atoi(argv[3]), q = atoi(argv[4]);
  std::vector<uint8_t> rgb(3 * static_cast<size_t>(w) * h);
  if (fread(rgb.data(), 1, rgb.size(), f) != rgb.size()) return 2;
  fclose(f);
  gz::ProcessParams params;
  params.butteraugli_target = static_cast<float>(gz::ButteraugliScoreForQuality(q));
  gz::JpegData jpg;
  gz::EncodeRGBToJpegData(rgb.data(), w, h, &jpg);
  OracleComparator cmp(w, h, rgb.data(), params.butteraugli_target);
  gz::ProcessResult res;
  std::string err;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = gz::ProcessJpegData(params, jpg, (w >= 32 && h >= 32) ? &cmp : nullptr, &res, &err);
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (rc != 0) {
    fprintf(stderr, "ProcessJpegData failed: %d %s\n", rc, err.c_str());
    return 3;
  }
  FILE* o = fopen(argv[5], "wb");
  fwrite(res.jpeg.data(), 1, res.jpeg.size(), o);
  fclose(o);
  printf("{\"bytes\": %zu, \"iters\": %d, \"seconds\": %.4f", res.jpeg.size(), res.iterations, dt);
  printf(", \"write_s\": %.4f, \"backend_s\": %.4f", res.seconds_write, res.seconds_backend);
  for (auto& kv : res.detail) printf(", \"%s\": %.6g", kv.first.c_str(), kv.second);
  printf("}\n");
  return 0;
}
