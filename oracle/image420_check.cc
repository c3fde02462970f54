// Test-infrastructure check of the 4:2:0 host model (not product code).
//
// Links the REFERENCE's OutputImage / Downsample / JPEG writer (compiled from
// /root/reference by oracle/Makefile) with the product's host model
// (gz::DownsampleToJpegData420, gz::Image420, gz::WriteJpeg from
// libguetzli_hip.so; no GPU calls) and compares them stage by stage on one
// RGB image:
//   1. Downsample + SaveToJpegData (output_image.cc:535-571, 579-640):
//      every coefficient and header field of the 4:2:0 JPEGData;
//   2. CopyFromJpegData of that data, then ApplyGlobalQuantization with a
//      seeded quantization matrix, then a seeded run of single-block
//      SetCoeffBlock edits in arbitrary order: the Cb / Cr 16-bit pixel
//      planes after each step (the fancy-upsampler state);
//   3. SaveToJpegData + WriteJpeg of the final image: the file bytes.
//
//   image420_check RGB W H SILVER(0|1) SEED
// Prints "ok" and exits 0, or names the first difference and exits 1.

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "clguetzli/clguetzli.h"
#include "guetzli/jpeg_data.h"
#include "guetzli/jpeg_data_encoder.h"
#include "guetzli/jpeg_data_writer.h"
#include "guetzli/output_image.h"
#include "guetzli/quantize.h"
#include "host/image420.h"
#include "host/jpeg_writer.h"
#include "host/processor.h"

namespace {

uint64_t g_rng = 1;
uint32_t Next() {
  g_rng = g_rng * 6364136223846793005ull + 1442695040888963407ull;
  return static_cast<uint32_t>(g_rng >> 33);
}

int StringOut(void* data, const uint8_t* buf, size_t n) {
  static_cast<std::string*>(data)->append(reinterpret_cast<const char*>(buf), n);
  return static_cast<int>(n);
}

bool SameJpegData(const guetzli::JPEGData& r, const gz::JpegData& o) {
  if (r.width != o.width || r.height != o.height || r.max_h_samp_factor != o.max_h_samp_factor ||
      r.max_v_samp_factor != o.max_v_samp_factor || r.MCU_rows != o.mcu_rows || r.MCU_cols != o.mcu_cols ||
      r.components.size() != o.components.size()) {
    fprintf(stderr, "header: ref %dx%d f%d%d mcu %dx%d nc %zu / ours %dx%d f%d%d mcu %dx%d nc %zu\n", r.width,
            r.height, r.max_h_samp_factor, r.max_v_samp_factor, r.MCU_cols, r.MCU_rows, r.components.size(),
            o.width, o.height, o.max_h_samp_factor, o.max_v_samp_factor, o.mcu_cols, o.mcu_rows,
            o.components.size());
    return false;
  }
  for (size_t c = 0; c < r.components.size(); ++c) {
    const auto& rc = r.components[c];
    const auto& oc = o.components[c];
    if (rc.h_samp_factor != oc.h_samp_factor || rc.v_samp_factor != oc.v_samp_factor ||
        rc.width_in_blocks != oc.width_in_blocks || rc.height_in_blocks != oc.height_in_blocks ||
        rc.coeffs.size() != oc.coeffs.size()) {
      fprintf(stderr, "component %zu layout differs\n", c);
      return false;
    }
    for (size_t i = 0; i < rc.coeffs.size(); ++i)
      if (rc.coeffs[i] != oc.coeffs[i]) {
        fprintf(stderr, "component %zu coeff %zu (block %zu k %zu): ref %d ours %d\n", c, i, i / 64, i % 64,
                rc.coeffs[i], oc.coeffs[i]);
        return false;
      }
  }
  return true;
}

bool SamePlanes(const guetzli::OutputImage& r, const gz::Image420& o, const char* what) {
  for (int c = 1; c < 3; ++c) {
    const uint16_t* rp = r.component(c).pixels();
    const std::vector<uint16_t>& op = o.plane[c - 1].px;
    for (size_t i = 0; i < op.size(); ++i)
      if (rp[i] != op[i]) {
        fprintf(stderr, "%s: plane %d pixel (%zu, %zu): ref %u ours %u\n", what, c, i % o.w, i / o.w, rp[i],
                op[i]);
        return false;
      }
    const guetzli::coeff_t* rc = r.component(c).coeffs();
    for (size_t i = 0; i < o.c[c - 1].size(); ++i)
      if (rc[i] != o.c[c - 1][i]) {
        fprintf(stderr, "%s: coeffs %d differ at %zu\n", what, c, i);
        return false;
      }
  }
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: %s RGB W H SILVER SEED\n", argv[0]);
    return 2;
  }
  const int w = atoi(argv[2]), h = atoi(argv[3]);
  const bool silver = atoi(argv[4]) != 0;
  g_rng = static_cast<uint64_t>(atoll(argv[5])) * 2654435761ull + 1;
  std::vector<uint8_t> rgb(3u * static_cast<size_t>(w) * h);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(rgb.data(), 1, rgb.size(), f) != rgb.size()) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  fclose(f);
  g_mathMode = MODE_CPU_OPT;

  // 1. Downsample (ProcessJpegData's downsample pass, processor.cc:990-997)
  guetzli::JPEGData rjpg;
  if (!guetzli::EncodeRGBToJpeg(rgb, w, h, &rjpg)) return 2;
  guetzli::OutputImage rimg(w, h);
  rimg.CopyFromJpegData(rjpg);
  guetzli::OutputImage::DownsampleConfig cfg;
  cfg.use_silver_screen = silver;
  rimg.Downsample(cfg);
  rimg.SaveToJpegData(&rjpg);

  gz::JpegData ojpg444, ojpg;
  gz::EncodeRGBToJpegData(rgb.data(), w, h, &ojpg444);
  if (!gz::DownsampleToJpegData420(ojpg444, silver, &ojpg)) {
    fprintf(stderr, "ours: chroma all zero\n");
    return 1;
  }
  if (!SameJpegData(rjpg, ojpg)) return 1;

  // 2. the pixel state through CopyFromJpegData / ApplyGlobalQuantization /
  // single-block edits
  rimg.CopyFromJpegData(rjpg);
  gz::Image420 oimg;
  oimg.Init(w, h);
  oimg.CopyFromJpegData(ojpg);
  if (!SamePlanes(rimg, oimg, "CopyFromJpegData")) return 1;
  int q[3][64];
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 64; ++k) q[c][k] = 1 + static_cast<int>(Next() % (k == 0 ? 8 : 24));
  rimg.ApplyGlobalQuantization(q);
  oimg.ApplyGlobalQuantization(q);
  if (!SamePlanes(rimg, oimg, "ApplyGlobalQuantization")) return 1;
  // (with Y edits too, and Image420::SavedJpegData -- the search's
  // incrementally kept SaveToJpegData -- checked against the reference's
  // whole SaveToJpegData eight times along the way)
  const int nb = oimg.cbw * oimg.cbh;
  const int steps = 4 * nb;
  oimg.SavedJpegData(ojpg);
  for (int step = 0; step < steps; ++step) {
    const int c = static_cast<int>(Next() % 3);
    const int nbc = c == 0 ? oimg.bw * oimg.bh : nb, bwc = c == 0 ? oimg.bw : oimg.cbw;
    const int b = static_cast<int>(Next() % nbc);
    gz::coeff_t blk[64];
    std::memcpy(blk, oimg.block(c, b), sizeof(blk));
    const int k = static_cast<int>(Next() % 64);
    blk[k] = static_cast<gz::coeff_t>(Next() % 3 == 0 ? 0 : blk[k] + q[c][k] * (static_cast<int>(Next() % 5) - 2));
    rimg.component(c).SetCoeffBlock(b % bwc, b / bwc, blk);
    oimg.SetCoeffBlock(c, b, blk);
    if ((step + 1) % ((steps + 7) / 8) == 0 || step + 1 == steps) {
      guetzli::JPEGData rj = rjpg;
      rimg.SaveToJpegData(&rj);
      if (!SameJpegData(rj, oimg.SavedJpegData(ojpg))) {
        fprintf(stderr, "SavedJpegData after %d edits\n", step + 1);
        return 1;
      }
    }
  }
  if (!SamePlanes(rimg, oimg, "SetCoeffBlock sequence")) return 1;

  // 3. SaveToJpegData + WriteJpeg
  guetzli::JPEGData rout = rjpg;
  rimg.SaveToJpegData(&rout);
  std::string rbytes;
  guetzli::JPEGOutput out(StringOut, &rbytes);
  if (!guetzli::WriteJpeg(rout, true, out)) return 2;
  gz::JpegData oout = ojpg;
  oimg.SaveToJpegData(&oout);
  if (!SameJpegData(rout, oout)) return 1;
  std::string obytes;
  if (!gz::WriteJpeg(oout, true, &obytes)) return 1;
  if (rbytes != obytes) {
    size_t i = 0;
    while (i < rbytes.size() && i < obytes.size() && rbytes[i] == obytes[i]) ++i;
    fprintf(stderr, "jpeg bytes differ at %zu (ref %zu B, ours %zu B)\n", i, rbytes.size(), obytes.size());
    return 1;
  }
  printf("ok %zu\n", obytes.size());
  return 0;
}
