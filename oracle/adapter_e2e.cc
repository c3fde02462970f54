// Test-infrastructure driver for the drop-in adapters (not product code).
//
// Links the REFERENCE's own Processor (guetzli/processor.cc, compiled from
// /root/reference by oracle/Makefile) with the comparator-level adapter
// guetzli::HipButteraugliComparator, and the whole-encode adapter
// guetzli::ProcessHip -- both product sources under
// guetzli-cuda-opencl_amd/adapters/, compiled here against the reference's
// headers.  The GPU tests check both encodes against the reference's known
// answers (tests/golden/manifest.json).
//
//   adapter_e2e comparator RGB W H QUALITY OUT.jpg [k=v ...]  reference Processor + HIP comparator
//   adapter_e2e process    RGB W H QUALITY OUT.jpg [k=v ...]  ProcessHip (gz_process_rgb)
// k=v: Params overrides try_420 / force_420 / silver (use_silver_screen).
//
// Prints "iterations N" on success; exits 1 on a failed encode.

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "clguetzli/clguetzli.h"
#include "guetzli/jpeg_data.h"
#include "guetzli/jpeg_data_encoder.h"
#include "guetzli/processor.h"
#include "guetzli/quality.h"
#include "guetzli/stats.h"
#include "hip_comparator.h"
#include "process_hip.h"

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: %s comparator|process RGB W H QUALITY OUT.jpg [k=v ...]\n", argv[0]);
    return 2;
  }
  const std::string mode = argv[1];
  const int w = atoi(argv[3]), h = atoi(argv[4]);
  const double quality = atof(argv[5]);
  std::vector<uint8_t> rgb(3u * static_cast<size_t>(w) * h);
  FILE* f = fopen(argv[2], "rb");
  if (!f || fread(rgb.data(), 1, rgb.size(), f) != rgb.size()) {
    fprintf(stderr, "cannot read %s\n", argv[2]);
    return 2;
  }
  fclose(f);
  g_mathMode = MODE_CPU_OPT;  // the `guetzli --c` search loop (guetzli.cc)
  guetzli::Params params;
  params.butteraugli_target = static_cast<float>(guetzli::ButteraugliScoreForQuality(quality));
  for (int i = 7; i < argc; ++i) {
    const std::string kv = argv[i];
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) return 2;
    const std::string k = kv.substr(0, eq);
    const bool v = atoi(kv.c_str() + eq + 1) != 0;
    if (k == "try_420") params.try_420 = v;
    else if (k == "force_420") params.force_420 = v;
    else if (k == "silver") params.use_silver_screen = v;
    else return 2;
  }
  guetzli::ProcessStats stats;
  std::string out;
  bool ok = false;
  if (mode == "comparator") {
    guetzli::JPEGData jpg;
    if (!guetzli::EncodeRGBToJpeg(rgb, w, h, &jpg)) return 1;
    guetzli::HipButteraugliComparator cmp(w, h, &rgb, params.butteraugli_target, &stats);
    guetzli::GuetzliOutput go;
    ok = guetzli::ProcessJpegData(params, jpg, &cmp, &go, &stats);
    out = go.jpeg_data;
  } else if (mode == "process") {
    ok = guetzli::ProcessHip(params, &stats, rgb, w, h, &out);
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  if (!ok) return 1;
  FILE* o = fopen(argv[6], "wb");
  if (!o || fwrite(out.data(), 1, out.size(), o) != out.size()) return 1;
  fclose(o);
  printf("iterations %d\n", stats.counters[guetzli::kNumItersCnt]);
  return 0;
}
