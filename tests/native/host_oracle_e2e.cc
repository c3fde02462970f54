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
#include "oracle_comparator.h"

using gz_test::OracleComparator;


int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: host_oracle_e2e RGB W H QUALITY OUT.jpg [lookahead=N] [new_model=0|1]\n");
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
  // optional Params overrides (as oracle/ref_driver encode): lookahead=N new_model=0|1
  for (int i = 6; i < argc; ++i) {
    const std::string kv = argv[i];
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) return 1;
    const int v = atoi(kv.c_str() + eq + 1);
    if (kv.compare(0, eq, "lookahead") == 0) params.zeroing_greedy_lookahead = v;
    else if (kv.compare(0, eq, "new_model") == 0) params.new_zeroing_model = v != 0;
    else if (kv.compare(0, eq, "force_420") == 0) params.force_420 = v != 0;
    else if (kv.compare(0, eq, "try_420") == 0) params.try_420 = v != 0;
    else return 1;
  }
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
