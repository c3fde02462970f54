// Test-infrastructure driver around the REFERENCE build (oracle/_ref).
//
// Not product code.  Linked against oracle/_ref/libguetzli_ref.a, which is
// compiled from /root/reference by oracle/Makefile.  It runs the reference's
// own `--c` path (g_mathMode = MODE_CPU_OPT, clguetzli/clguetzli.h:17-27) and
// dumps end-to-end JPEG bytes and stage-level intermediates that the clean-room
// restatement (oracle/gz_oracle.c) and the HIP product are pinned against.
//
//   guetzli_ref encode  RGB W H QUALITY OUT.jpg [c|cpu] [lookahead=N new_model=0|1
//                       try_420=0|1 force_420=0|1]       guetzli.cc:247-368
//   guetzli_ref stages  RGB W H QSEED OUTDIR [nozero]        see Stages()
//   guetzli_ref zero_variants RGB W H QSEED OUTDIR           see ZeroVariants()
//   guetzli_ref encode_jpeg IN.jpg QUALITY OUT.jpg            processor.cc:1029-1066
//   guetzli_ref decode  IN.jpg OUT.rgb OUT.coeffs             ReadJpeg + DecodeJpegToRGB
//
// RGB files are raw interleaved 8-bit (no header).  All dumps are raw
// little-endian arrays; OUTDIR/meta.txt lists them.

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

// The reference's Processor lives in an anonymous namespace inside
// processor.cc; compile that file as part of this TU (in place, from
// /root/reference) with member access opened so the per-block greedy
// zeroing (processor.cc:376-487) can be driven directly.
#define private public
#include "guetzli/processor.cc"
#undef private

#include "guetzli/butteraugli_comparator.h"
#include "guetzli/jpeg_data_encoder.h"
#include "guetzli/output_image.h"
#include "guetzli/quality.h"
#include "guetzli/gamma_correct.h"
#include "clguetzli/clguetzli.h"
#include "clguetzli/clbutter_comparator.h"

namespace guetzli {
// Defined (non-static) in guetzli/butteraugli_comparator.cc:31-46.
std::vector<std::vector<float> > ComputeOpsinDynamicsImage(int, int, const std::vector<uint8_t>&);
}

namespace butteraugli {
// Defined (non-static) in clguetzli/clbutter_comparator.cpp.
void MaskHighIntensityChangeOpt(size_t, size_t, const std::vector<std::vector<float> >&,
                                const std::vector<std::vector<float> >&,
                                std::vector<std::vector<float> >&,
                                std::vector<std::vector<float> >&);
void MaskOpt(const std::vector<std::vector<float> >&, const std::vector<std::vector<float> >&,
             size_t, size_t, std::vector<std::vector<float> >*, std::vector<std::vector<float> >*);
void CalculateDiffmapOpt(const size_t, const size_t, const size_t, std::vector<float>*);
void OpsinDynamicsImageOpt(size_t, size_t, std::vector<std::vector<float> >&);
void BlurOpt(size_t, size_t, float*, float, float);
}

namespace {

std::vector<uint8_t> ReadAll(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  std::vector<uint8_t> d;
  uint8_t buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof(buf), f)) > 0) d.insert(d.end(), buf, buf + n);
  fclose(f);
  return d;
}

void WriteAll(const std::string& path, const void* p, size_t n) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) { perror(path.c_str()); exit(2); }
  if (n && fwrite(p, 1, n, f) != n) { perror(path.c_str()); exit(2); }
  fclose(f);
}

void DumpPlanes(const std::string& path, const std::vector<std::vector<float> >& p) {
  std::vector<float> flat;
  for (auto& v : p) flat.insert(flat.end(), v.begin(), v.end());
  WriteAll(path, flat.data(), flat.size() * sizeof(float));
}

int Encode(int argc, char** argv) {
  if (argc < 7) return 1;
  std::vector<uint8_t> rgb = ReadAll(argv[2]);
  int w = atoi(argv[3]), h = atoi(argv[4]), quality = atoi(argv[5]);
  std::string mode = argc > 7 ? argv[7] : "c";
  g_mathMode = mode == "cpu" ? MODE_CPU : MODE_CPU_OPT;
  guetzli::Params params;
  params.butteraugli_target =
      static_cast<float>(guetzli::ButteraugliScoreForQuality(quality));
  // optional Params overrides: lookahead=N new_model=0|1 try_420=0|1 force_420=0|1
  // silver=0|1 (use_silver_screen)
  for (int i = 8; i < argc; ++i) {
    const std::string kv = argv[i];
    const size_t eq = kv.find('=');
    if (eq == std::string::npos) return 1;
    const std::string k = kv.substr(0, eq);
    const int v = atoi(kv.c_str() + eq + 1);
    if (k == "lookahead") params.zeroing_greedy_lookahead = v;
    else if (k == "new_model") params.new_zeroing_model = v != 0;
    else if (k == "try_420") params.try_420 = v != 0;
    else if (k == "force_420") params.force_420 = v != 0;
    else if (k == "silver") params.use_silver_screen = v != 0;
    else return 1;
  }
  guetzli::ProcessStats stats;
  if (getenv("GZ_REF_LOG")) stats.debug_output_file = stderr;  // the search's per-iteration log
  std::string out;
  auto t0 = std::chrono::steady_clock::now();
  bool ok = guetzli::Process(params, &stats, rgb, w, h, &out);
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (!ok) { fprintf(stderr, "Process failed\n"); return 3; }
  WriteAll(argv[6], out.data(), out.size());
  fprintf(stdout, "{\"bytes\": %zu, \"seconds\": %.6f, \"iters\": %d}\n", out.size(), dt,
          stats.counters[guetzli::kNumItersCnt]);
  return 0;
}

// guetzli::Process on a JPEG file (processor.cc:1029-1066), --c mode:
//   guetzli_ref encode_jpeg IN.jpg QUALITY OUT.jpg [keep]   (keep: clear_metadata = false)
int EncodeJpeg(int argc, char** argv) {
  if (argc < 5) return 1;
  std::vector<uint8_t> in = ReadAll(argv[2]);
  const int quality = atoi(argv[3]);
  g_mathMode = MODE_CPU_OPT;
  guetzli::Params params;
  if (argc > 5 && !strcmp(argv[5], "keep")) params.clear_metadata = false;
  params.butteraugli_target =
      static_cast<float>(guetzli::ButteraugliScoreForQuality(quality));
  guetzli::ProcessStats stats;
  std::string out;
  const std::string data(in.begin(), in.end());
  auto t0 = std::chrono::steady_clock::now();
  const bool ok = guetzli::Process(params, &stats, data, &out);
  double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  if (!ok) { fprintf(stderr, "Process failed\n"); return 3; }
  WriteAll(argv[4], out.data(), out.size());
  fprintf(stdout, "{\"bytes\": %zu, \"seconds\": %.6f, \"iters\": %d}\n", out.size(), dt,
          stats.counters[guetzli::kNumItersCnt]);
  return 0;
}

// ReadJpeg + DecodeJpegToRGB (jpeg_data_reader.cc, jpeg_data_decoder.cc:45-53):
//   guetzli_ref decode IN.jpg OUT.rgb OUT.coeffs
// OUT.coeffs: int16 [3][blocks][64] quantized coefficients, natural order.
int Decode(int argc, char** argv) {
  if (argc < 5) return 1;
  std::vector<uint8_t> in = ReadAll(argv[2]);
  guetzli::JPEGData jpg;
  if (!guetzli::ReadJpeg(in.data(), in.size(), guetzli::JPEG_READ_ALL, &jpg)) {
    fprintf(stderr, "ReadJpeg failed\n");
    return 3;
  }
  std::vector<uint8_t> rgb = guetzli::DecodeJpegToRGB(jpg);
  WriteAll(argv[3], rgb.data(), rgb.size());
  std::vector<int16_t> co;
  for (const auto& c : jpg.components) co.insert(co.end(), c.coeffs.begin(), c.coeffs.end());
  WriteAll(argv[4], co.data(), co.size() * sizeof(int16_t));
  fprintf(stdout, "{\"w\": %d, \"h\": %d, \"ncomp\": %zu, \"rgb_bytes\": %zu}\n", jpg.width,
          jpg.height, jpg.components.size(), rgb.size());
  return 0;
}

// Deterministic quantization matrix for stage fixtures (any valid matrix
// exercises the same code; it only needs to be reproducible).
void MakeQ(int seed, int q[3][64]) {
  uint32_t s = 2463534242u ^ static_cast<uint32_t>(seed * 7919);
  for (int c = 0; c < 3; ++c)
    for (int k = 0; k < 64; ++k) {
      s ^= s << 13; s ^= s >> 17; s ^= s << 5;
      int zz = guetzli::kJPEGZigZagOrder[k];
      q[c][k] = 1 + (zz * (2 + c)) / 8 + static_cast<int>(s % 3);
    }
}

// Per-block greedy zeroing orders of every block (the CPU_OPT loop of
// SelectFrequencyMasking, processor.cc:641-672, factor 1) for the given
// Params::zeroing_greedy_lookahead / new_zeroing_model and comp_mask.  As in
// SelectFrequencyMasking, only the masked components of the current and
// original blocks are passed (ComputeBlockZeroingOrder's REQUIRES, :374);
// the image keeps every component's current coefficients.
std::vector<guetzli::CoeffData> ZeroOrders(const std::vector<uint8_t>& rgb, int w, int h,
                                           float target, const guetzli::JPEGData& jpg,
                                           guetzli::OutputImage* img, int lookahead,
                                           int comp_mask, bool new_model) {
  guetzli::ProcessStats stats;
  guetzli::Processor proc;
  guetzli::Params params;
  params.butteraugli_target = target;
  params.zeroing_greedy_lookahead = lookahead;
  params.new_zeroing_model = new_model;
  guetzli::ButteraugliComparator c3(w, h, &rgb, target, &stats);
  proc.params_ = params;
  proc.comparator_ = &c3;
  proc.stats_ = &stats;
  c3.StartBlockComparisons();
  const int bw = (w + 7) / 8, bh = (h + 7) / 8;
  std::vector<guetzli::CoeffData> out(bw * bh * 192);
  memset(out.data(), 0, out.size() * sizeof(out[0]));
  for (int by = 0, bix = 0; by < bh; ++by)
    for (int bx = 0; bx < bw; ++bx, ++bix) {
      guetzli::coeff_t block[192] = {0}, orig_block[192] = {0};
      for (int c = 0; c < 3; ++c) {
        if (!(comp_mask & (1 << c))) continue;
        img->component(c).GetCoeffBlock(bx, by, &block[c * 64]);
        const auto& comp = jpg.components[c];
        memcpy(&orig_block[c * 64], &comp.coeffs[(by * comp.width_in_blocks + bx) * 64],
               64 * sizeof(guetzli::coeff_t));
      }
      std::vector<guetzli::CoeffData> order;
      proc.ComputeBlockZeroingOrder(block, orig_block, bx, by, 1, 1,
                                    static_cast<uint8_t>(comp_mask), img, &order);
      for (size_t i = 0; i < order.size(); ++i) out[bix * 192 + i] = order[i];
    }
  c3.FinishBlockComparisons();
  return out;
}

// Candidate image of the stage fixtures: EncodeRGBToJpeg -> remove quant ->
// copy -> global quantization (processor.cc:1160-1163, 94-107, 310-317).
bool StageCandidate(const std::vector<uint8_t>& rgb, int w, int h, int qseed,
                    guetzli::JPEGData* jpg, guetzli::OutputImage* img, int q[3][64]) {
  if (!guetzli::EncodeRGBToJpeg(rgb, w, h, jpg)) return false;
  int q_in[3][64];
  guetzli::RemoveOriginalQuantization(jpg, q_in);
  MakeQ(qseed, q);
  img->CopyFromJpegData(*jpg);
  img->ApplyGlobalQuantization(q);
  return true;
}

// Zeroing-order variants of a stage fixture: lookahead 1 and 2, comp_mask 1
// (Y only) and 6 (Cb+Cr), and the old zeroing model (new_zeroing_model =
// false, processor.cc:400-405) -> OUTDIR/zero_order_la<L>_m<M>_nm<N>.bin.
int ZeroVariants(int argc, char** argv) {
  if (argc < 7) return 1;
  std::vector<uint8_t> rgb = ReadAll(argv[2]);
  const int w = atoi(argv[3]), h = atoi(argv[4]), qseed = atoi(argv[5]);
  const std::string dir = argv[6];
  g_mathMode = MODE_CPU_OPT;
  const float target = static_cast<float>(guetzli::ButteraugliScoreForQuality(95));
  guetzli::JPEGData jpg;
  guetzli::OutputImage img(w, h);
  int q[3][64];
  if (!StageCandidate(rgb, w, h, qseed, &jpg, &img, q)) return 4;
  static const int kVariants[][3] = {{1, 7, 1}, {2, 7, 1}, {3, 1, 1}, {3, 6, 1}, {3, 7, 0}, {2, 6, 0}};
  for (const auto& v : kVariants) {
    std::vector<guetzli::CoeffData> out = ZeroOrders(rgb, w, h, target, jpg, &img, v[0], v[1], v[2] != 0);
    char name[96];
    snprintf(name, sizeof(name), "/zero_order_la%d_m%d_nm%d.bin", v[0], v[1], v[2]);
    WriteAll(dir + name, out.data(), out.size() * sizeof(out[0]));
  }
  return 0;
}

int Stages(int argc, char** argv) {
  if (argc < 7) return 1;
  std::vector<uint8_t> rgb = ReadAll(argv[2]);
  const int w = atoi(argv[3]), h = atoi(argv[4]), qseed = atoi(argv[5]);
  const std::string dir = argv[6];
  g_mathMode = MODE_CPU_OPT;
  const float target = static_cast<float>(guetzli::ButteraugliScoreForQuality(95));

  // Candidate image: EncodeRGBToJpeg -> remove quant -> copy -> global quantization
  // (processor.cc:1160-1163, 94-107, 310-317).
  guetzli::JPEGData jpg;
  if (!guetzli::EncodeRGBToJpeg(rgb, w, h, &jpg)) return 4;
  int q_in[3][64];
  guetzli::RemoveOriginalQuantization(&jpg, q_in);
  int q[3][64];
  MakeQ(qseed, q);
  guetzli::OutputImage img(w, h);
  img.CopyFromJpegData(jpg);
  img.ApplyGlobalQuantization(q);

  FILE* meta = fopen((dir + "/meta.txt").c_str(), "w");
  fprintf(meta, "w %d\nh %d\nqseed %d\ntarget %.9g\n", w, h, qseed, target);
  WriteAll(dir + "/q.i32", &q[0][0], sizeof(q));
  {
    std::vector<int16_t> orig;
    for (int c = 0; c < 3; ++c)
      orig.insert(orig.end(), jpg.components[c].coeffs.begin(), jpg.components[c].coeffs.end());
    WriteAll(dir + "/orig_coeffs.i16", orig.data(), orig.size() * 2);
    std::vector<int16_t> cur;
    for (int c = 0; c < 3; ++c) {
      const auto& comp = img.component(c);
      cur.insert(cur.end(), comp.coeffs(), comp.coeffs() + comp.width_in_blocks() * comp.height_in_blocks() * 64);
    }
    WriteAll(dir + "/cand_coeffs.i16", cur.data(), cur.size() * 2);
    std::vector<uint8_t> srgb = img.ToSRGB();
    WriteAll(dir + "/cand_srgb.u8", srgb.data(), srgb.size());
  }

  // Reference XYB (butteraugli_comparator.cc:31-46).
  std::vector<std::vector<float> > ref = guetzli::ComputeOpsinDynamicsImage(w, h, rgb);
  DumpPlanes(dir + "/ref_xyb.f32", ref);
  // Candidate linear RGB and XYB (butteraugli_comparator.cc:63-65).
  std::vector<std::vector<float> > cand(3, std::vector<float>(w * h));
  img.ToLinearRGB(&cand);
  DumpPlanes(dir + "/cand_linear.f32", cand);
  butteraugli::OpsinDynamicsImage(w, h, cand);
  DumpPlanes(dir + "/cand_xyb.f32", cand);

  // Stage-by-stage DiffmapOpsinDynamicsImageOpt (clbutter_comparator.cpp:1387-1417).
  if (w >= 8 && h >= 8) {
    butteraugli::clButteraugliComparator cmp(w, h, 3);
    const size_t rx = (w + 2) / 3, ry = (h + 2) / 3;
    std::vector<std::vector<float> > xyb0 = ref, xyb1 = cand;
    {
      auto c0 = xyb0, c1 = xyb1;
      butteraugli::MaskHighIntensityChangeOpt(w, h, c0, c1, xyb0, xyb1);
    }
    DumpPlanes(dir + "/mhic0.f32", xyb0);
    DumpPlanes(dir + "/mhic1.f32", xyb1);
    std::vector<float> edge(3 * rx * ry), dc(3 * rx * ry), ac(3 * rx * ry);
    cmp.EdgeDetectorMapOpt(xyb0, xyb1, &edge);
    WriteAll(dir + "/edge.f32", edge.data(), edge.size() * 4);
    cmp.BlockDiffMapOpt(xyb0, xyb1, &dc, &ac);
    WriteAll(dir + "/block_dc.f32", dc.data(), dc.size() * 4);
    WriteAll(dir + "/block_ac.f32", ac.data(), ac.size() * 4);
    cmp.EdgeDetectorLowFreqOpt(xyb0, xyb1, &ac);
    WriteAll(dir + "/block_ac_lf.f32", ac.data(), ac.size() * 4);
    std::vector<std::vector<float> > mask, mask_dc;
    butteraugli::MaskOpt(xyb0, xyb1, w, h, &mask, &mask_dc);
    DumpPlanes(dir + "/mask.f32", mask);
    DumpPlanes(dir + "/mask_dc.f32", mask_dc);
    std::vector<float> res;
    cmp.CombineChannelsOpt(mask, mask_dc, dc, ac, edge, &res);
    WriteAll(dir + "/combined.f32", res.data(), res.size() * 4);
    butteraugli::CalculateDiffmapOpt(w, h, 3, &res);
    WriteAll(dir + "/diffmap_stagewise.f32", res.data(), res.size() * 4);
    fprintf(meta, "res_w %zu\nres_h %zu\n", rx, ry);
  }

  // Full comparator path (butteraugli_comparator.cc:60-70) and weights (:169-233).
  guetzli::ButteraugliComparator comparator(w, h, &rgb, target, nullptr);
  guetzli::ProcessStats stats;
  if (w >= 8 && h >= 8) {
    // Compare() logs through GUETZLI_LOG, which needs a stats object.
    guetzli::ButteraugliComparator c2(w, h, &rgb, target, &stats);
    c2.Compare(img);
    std::vector<float> dm = c2.distmap();
    WriteAll(dir + "/distmap.f32", dm.data(), dm.size() * 4);
    fprintf(meta, "distance %.9g\n", c2.distmap_aggregate());
    for (int dir_ = -1; dir_ <= 1; dir_ += 2)
      for (int rb = 1; rb <= 4; ++rb) {
        const int bw = (w + 7) / 8, bh = (h + 7) / 8;
        std::vector<float> wgt(bw * bh);
        c2.ComputeBlockErrorAdjustmentWeights(dir_, rb, 1.0, 1, 1, dm, &wgt);
        char name[64];
        snprintf(name, sizeof(name), "/weights_d%+d_r%d.f32", dir_, rb);
        WriteAll(dir + name, wgt.data(), wgt.size() * 4);
      }
  }

  // Activity mask of the reference against itself (butteraugli_comparator.cc:72-79).
  {
    std::vector<std::vector<float> > mask_xyz, dummy(3);
    butteraugli::Mask(ref, ref, w, h, &mask_xyz, &dummy);
    DumpPlanes(dir + "/ref_mask.f32", mask_xyz);
  }

  // Per-block greedy zeroing order, CPU_OPT loop of SelectFrequencyMasking
  // (processor.cc:641-672) with comp_mask 7, factor 1 (argv[7] "nozero":
  // skipped -- the frame-size stage hashes, tests/golden/make_stage_hashes.py).
  if (!(argc > 7 && !strcmp(argv[7], "nozero"))) {
    std::vector<guetzli::CoeffData> out = ZeroOrders(rgb, w, h, target, jpg, &img, 3, 7, true);
    WriteAll(dir + "/zero_order.bin", out.data(), out.size() * sizeof(out[0]));
  }
  fclose(meta);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 2 && !strcmp(argv[1], "encode")) return Encode(argc, argv);
  if (argc >= 2 && !strcmp(argv[1], "stages")) return Stages(argc, argv);
  if (argc >= 2 && !strcmp(argv[1], "zero_variants")) return ZeroVariants(argc, argv);
  if (argc >= 2 && !strcmp(argv[1], "encode_jpeg")) return EncodeJpeg(argc, argv);
  if (argc >= 2 && !strcmp(argv[1], "decode")) return Decode(argc, argv);
  fprintf(stderr,
          "usage: guetzli_ref encode RGB W H QUALITY OUT.jpg [c|cpu]\n"
          "       guetzli_ref stages RGB W H QSEED OUTDIR\n");
  return 1;
}
