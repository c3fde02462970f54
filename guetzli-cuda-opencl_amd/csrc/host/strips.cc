// Row-strip decomposition of one frame over the ranks of a job; see strips.h.
#include "host/strips.h"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "host/jpeg_encode.h"
#include "host/thread_pool.h"
#include "../../include/guetzli_hip.h"

namespace gz {

namespace {
using Clock = std::chrono::steady_clock;
inline double Since(Clock::time_point t0) {
  return std::chrono::duration<double>(Clock::now() - t0).count();
}
inline int BitLength(int v) { return v ? 32 - __builtin_clz(static_cast<uint32_t>(v)) : 0; }

int CountFfBytes(uint32_t memory_order_word, int nbytes) {
  int n = 0;
  for (int q = 0; q < nbytes; ++q) n += ((memory_order_word >> (8 * q)) & 0xff) == 0xff;
  return n;
}

template <class T>
void Put(std::vector<uint8_t>* b, const T& v) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(&v);
  b->insert(b->end(), p, p + sizeof(T));
}
template <class T>
T Get(const uint8_t*& p) {
  T v;
  std::memcpy(&v, p, sizeof(T));
  p += sizeof(T);
  return v;
}
}  // namespace

StripLayout StripLayout::Make(int width, int height, int world) {
  StripLayout L;
  L.width = width;
  L.height = height;
  L.world = world;
  const int per = (height + world - 1) / world;
  const int step = (per + kStripAlign - 1) / kStripAlign * kStripAlign;
  for (int r = 0; r < world; ++r) {
    const int y0 = std::min(height, r * step), y1 = std::min(height, (r + 1) * step);
    L.y0.push_back(y0);
    L.y1.push_back(y1);
    L.e0.push_back(y0 == y1 ? y0 : std::max(0, y0 - kStripHalo));
    L.e1.push_back(y0 == y1 ? y1 : std::min(height, y1 + kStripHalo));
  }
  return L;
}

bool Collectives::AllGatherV(const std::vector<uint8_t>& send,
                             std::vector<std::vector<uint8_t>>* out) {
  const int n = world();
  const uint64_t mine = send.size();
  std::vector<uint64_t> sizes(n);
  if (!AllGather(&mine, sizeof(mine), sizes.data())) return false;
  const uint64_t cap = std::max<uint64_t>(1, *std::max_element(sizes.begin(), sizes.end()));
  std::vector<uint8_t> padded(cap, 0), all(cap * n);
  if (!send.empty()) std::memcpy(padded.data(), send.data(), send.size());
  if (!AllGather(padded.data(), cap, all.data())) return false;
  out->resize(n);
  for (int r = 0; r < n; ++r)
    (*out)[r].assign(all.begin() + r * cap, all.begin() + r * cap + sizes[r]);
  return true;
}

Partition Partition::Make(const StripLayout& L, Collectives* coll) {
  Partition p;
  p.coll = coll;
  p.world = coll->world();
  p.rank = coll->rank();
  p.width = L.width;
  p.height = L.height;
  p.bw = (L.width + 7) / 8;
  p.bh = (L.height + 7) / 8;
  p.lb0 = L.e0[p.rank] / 8;
  p.lb1 = (L.e1[p.rank] + 7) / 8;
  p.ob0 = L.y0[p.rank] / 8;
  p.ob1 = (L.y1[p.rank] + 7) / 8;
  for (int r = 0; r < p.world; ++r) p.row0.push_back(L.y0[r] / 8);
  p.row0.push_back(p.bh);
  return p;
}

bool Partition::SumAll(int64_t* v, int n) {
  if (world == 1) return true;
  std::vector<int64_t> all(static_cast<size_t>(n) * world);
  if (!coll->AllGather(v, n * sizeof(int64_t), all.data())) return false;
  for (int i = 0; i < n; ++i) {
    int64_t s = 0;
    for (int r = 0; r < world; ++r) s += all[static_cast<size_t>(r) * n + i];
    v[i] = s;
  }
  return true;
}

// ---------------------------------------------------------------------------
// The strip's entropy coder: histograms of the owned MCUs, then their part of
// the scan at a frame-wide bit offset (Engine::JpegStage/ScanRange on the
// device; the same on the host for comparators without a device).
// ---------------------------------------------------------------------------

class PartitionComparator::Coder {
 public:
  virtual ~Coder() {}
  virtual bool StageStart(const CoeffImage& img, int m0, int m1) = 0;
  // hist: [2c + {0: DC, 1: AC}][256] plain counts; chroma: non-zero chroma
  // coefficients of the staged blocks
  virtual bool StageWait(uint32_t* hist, uint64_t* chroma) = 0;
  virtual bool CompareStart(const CoeffImage& img) = 0;
  virtual bool ScanStart(int ncomp, const JpegCodeTables& codes, int m0, int m1, uint64_t base,
                         bool pad_end) = 0;
  // after everything started: the Compare's block maxima (local blocks) and
  // the scan part
  virtual bool Finish(std::vector<float>* block_max, Part* part) = 0;
  virtual void Keep() = 0;
  // the kept part's stored words (memory byte order, words[0] = frame word
  // base >> 5, shared words zero)
  virtual bool FetchKept(std::vector<uint32_t>* words, Part* part) = 0;
  std::string err;
};

namespace {

PartitionComparator::Part FromScanPart(const Engine::ScanPart& s) {
  PartitionComparator::Part p;
  p.base = s.base;
  p.bits = s.bits;
  p.ff = s.ff;
  p.first_word = s.first_word;
  p.last_word = s.last_word;
  p.first_shared = s.first_shared;
  p.last_open = s.last_open;
  return p;
}

class EngineCoder : public PartitionComparator::Coder {
 public:
  explicit EngineCoder(HipButteraugliComparator* hip) : hip_(hip), e_(hip->engine()) {}
  bool StageStart(const CoeffImage& img, int m0, int m1) override {
    if (!hip_->Sync(img) || !e_->JpegStageEnqueueRange(img.quant, m0, m1)) return Fail();
    std::memcpy(quant_, img.quant, sizeof(quant_));  // (the scan's)
    return true;
  }
  bool StageWait(uint32_t* hist, uint64_t* chroma) override {
    return e_->JpegStageWait(hist, chroma) || Fail();
  }
  bool CompareStart(const CoeffImage& img) override {
    compare_ = true;
    return (hip_->Sync(img) && e_->CompareEnqueue()) || Fail();
  }
  bool ScanStart(int ncomp, const JpegCodeTables& codes, int m0, int m1, uint64_t base,
                 bool pad_end) override {
    return e_->JpegScanEnqueueRange(ncomp, quant_, codes, m0, m1, base, pad_end) || Fail();
  }
  bool Finish(std::vector<float>* block_max, PartitionComparator::Part* part) override {
    if (!e_->Sync()) return Fail();
    if (compare_) {
      float d = 0.0f;
      block_max->resize(e_->blocks());
      if (!e_->CompareFinish(&d, block_max->data())) return Fail();
      compare_ = false;
    }
    if (part) {
      Engine::ScanPart s;
      if (!e_->JpegScanFinishPart(&s)) return Fail();
      *part = FromScanPart(s);
    }
    return true;
  }
  void Keep() override { e_->JpegKeep(); }
  bool FetchKept(std::vector<uint32_t>* words, PartitionComparator::Part* part) override {
    Engine::ScanPart s;
    if (!e_->JpegFetchPart(true, words, &s)) return Fail();
    *part = FromScanPart(s);
    return true;
  }

 private:
  bool Fail() {
    err = e_->error().empty() ? hip_->error() : e_->error();
    return false;
  }
  HipButteraugliComparator* hip_;
  Engine* e_;
  bool compare_ = false;
  int quant_[3][64] = {};
};

// SaveToJpegData + EncodeScan (jpeg_data_writer.cc:447-538) of blocks
// [m0, m1) on the host: the same parts as the device coder (test comparators
// without a device; no performance claim).
class HostCoder : public PartitionComparator::Coder {
 public:
  explicit HostCoder(Comparator* inner) : inner_(inner) {}
  bool StageStart(const CoeffImage& img, int m0, int m1) override {
    img_ = &img;
    std::memset(hist_, 0, sizeof(hist_));
    chroma_ = 0;
    for (int c = 0; c < 3; ++c)
      for (int b = m0; b < m1; ++b) {
        int z[64];
        Quantized(img, c, b, z);
        const int last = b > 0 ? QuantizedDc(img, c, b - 1) : 0;
        const int d = z[0] - last;
        ++hist_[2 * c][BitLength(std::abs(d))];
        int run = 0;
        for (int k = 1; k < 64; ++k) {
          if (!z[k]) {
            ++run;
            continue;
          }
          for (; run > 15; run -= 16) ++hist_[2 * c + 1][0xf0];
          ++hist_[2 * c + 1][(run << 4) + BitLength(std::abs(z[k]))];
          run = 0;
        }
        if (run > 0) ++hist_[2 * c + 1][0];
        if (c > 0)
          for (int k = 0; k < 64; ++k) chroma_ += img.block(c, b)[k] != 0;
      }
    return true;
  }
  bool StageWait(uint32_t* hist, uint64_t* chroma) override {
    std::memcpy(hist, hist_, sizeof(hist_));
    *chroma = chroma_;
    return true;
  }
  bool CompareStart(const CoeffImage& img) override {
    if (!inner_->Compare(img)) {
      err = inner_->error();
      return false;
    }
    compared_ = true;
    return true;
  }
  bool ScanStart(int ncomp, const JpegCodeTables& codes, int m0, int m1, uint64_t base,
                 bool pad_end) override {
    const CoeffImage& img = *img_;
    std::vector<uint32_t> w(1, 0u);  // stream order (MSB first)
    uint64_t pos = base & 31;
    auto put = [&](int n, uint32_t v) {
      for (int i = n - 1; i >= 0; --i, ++pos) {
        if ((pos >> 5) >= w.size()) w.push_back(0u);
        if ((v >> i) & 1) w[pos >> 5] |= 0x80000000u >> (pos & 31);
      }
    };
    for (int b = m0; b < m1; ++b)
      for (int c = 0; c < ncomp; ++c) {
        int z[64];
        Quantized(img, c, b, z);
        const int last = b > 0 ? QuantizedDc(img, c, b - 1) : 0;
        int diff = z[0] - last, bits = diff;
        if (diff < 0) {
          diff = -diff;
          bits -= 1;
        }
        const int nd = BitLength(diff);
        put(codes.dc_len[c][nd], codes.dc_code[c][nd]);
        if (nd) put(nd, static_cast<uint32_t>(bits) & ((1u << nd) - 1));
        int run = 0;
        for (int k = 1; k < 64; ++k) {
          int v = z[k];
          if (!v) {
            ++run;
            continue;
          }
          int vb = v;
          if (v < 0) {
            v = -v;
            vb = ~v;
          }
          for (; run > 15; run -= 16) put(codes.ac_len[c][0xf0], codes.ac_code[c][0xf0]);
          const int nb = BitLength(v);
          const int sym = (run << 4) + nb;
          put(codes.ac_len[c][sym], codes.ac_code[c][sym]);
          put(nb, static_cast<uint32_t>(vb) & ((1u << nb) - 1));
          run = 0;
        }
        if (run > 0) put(codes.ac_len[c][0], codes.ac_code[c][0]);
      }
    const uint64_t bits = pos - (base & 31);
    const uint64_t end = base + bits;
    if (pad_end && (pos & 7)) put(8 - static_cast<int>(pos & 7), 0xffu);
    PartitionComparator::Part& p = part_[slot_];
    p = PartitionComparator::Part();
    p.base = base;
    p.bits = bits;
    const size_t nw = static_cast<size_t>(((base & 31) + bits + 31) / 32);
    w.resize(nw);
    p.first_shared = (base & 31) != 0;
    p.last_open = !pad_end && (end & 31) != 0;
    if (p.first_shared && nw == 1 && p.last_open) {
      err = "HostCoder: a part under one word";
      return false;
    }
    const uint64_t end_bytes = (end + 7) / 8;
    for (size_t i = 0; i < nw; ++i) {
      w[i] = __builtin_bswap32(w[i]);
      if (i == 0 && p.first_shared) {
        p.first_word = w[i];
        w[i] = 0;
      } else if (i + 1 == nw && p.last_open) {
        p.last_word = w[i];
        w[i] = 0;
      } else {
        const uint64_t wi = (base >> 5) + i;
        const int nbytes = static_cast<int>(std::min<uint64_t>(4, end_bytes - 4 * wi));
        p.ff += CountFfBytes(w[i], nbytes);
      }
    }
    words_[slot_] = w;
    return true;
  }
  bool Finish(std::vector<float>* block_max, PartitionComparator::Part* part) override {
    if (compared_) {
      *block_max = inner_->block_max_distance();
      compared_ = false;
    }
    if (part) *part = part_[slot_];
    return true;
  }
  void Keep() override { slot_ ^= 1; }
  bool FetchKept(std::vector<uint32_t>* words, PartitionComparator::Part* part) override {
    *words = words_[slot_ ^ 1];
    *part = part_[slot_ ^ 1];
    return true;
  }

 private:
  static void Quantized(const CoeffImage& img, int c, int b, int z[64]) {
    const coeff_t* blk = img.block(c, b);
    for (int k = 0; k < 64; ++k) {
      const int n = kJPEGNaturalOrder[k];
      z[k] = blk[n] / img.quant[c][n];
    }
  }
  static int QuantizedDc(const CoeffImage& img, int c, int b) {
    return img.block(c, b)[0] / img.quant[c][0];
  }
  Comparator* inner_;
  const CoeffImage* img_ = nullptr;
  uint32_t hist_[6][256];
  uint64_t chroma_ = 0;
  bool compared_ = false;
  std::vector<uint32_t> words_[2];
  PartitionComparator::Part part_[2];
  int slot_ = 0;
};

}  // namespace

// ---------------------------------------------------------------------------
// PartitionComparator
// ---------------------------------------------------------------------------

PartitionComparator::PartitionComparator(Partition* part, std::unique_ptr<Comparator> inner,
                                         float target)
    : part_(part), inner_(std::move(inner)), target_(target) {
  local_blocks_ = (part_->lb1 - part_->lb0) * part_->bw;
  block_max_.assign(local_blocks_, 0.0f);
  if (auto* hip = dynamic_cast<HipButteraugliComparator*>(inner_.get()))
    coder_.reset(new EngineCoder(hip));
  else
    coder_.reset(new HostCoder(inner_.get()));
}

PartitionComparator::~PartitionComparator() = default;

bool PartitionComparator::Fail(const std::string& what) {
  err_ = what;
  return false;
}

// Every exchange message starts with a status word, and a rank whose local
// step failed still takes part in the exchange: all ranks then see the
// failure in the same collective and fail together instead of leaving the
// others blocked in the next one.
bool PartitionComparator::Exchange(bool ok, const std::string& local_err,
                                   const std::vector<uint8_t>& send,
                                   std::vector<std::vector<uint8_t>>* all) {
  if (part_->world == 1) {
    if (!ok) return Fail(local_err);
    all->assign(1, send);
    return true;
  }
  std::vector<uint8_t> msg;
  Put(&msg, static_cast<uint32_t>(ok ? 0 : 1));
  if (ok) msg.insert(msg.end(), send.begin(), send.end());
  const auto t0 = Clock::now();
  const bool sent = part_->coll->AllGatherV(msg, all);
  seconds_exchange += Since(t0);
  if (!sent) return Fail("strip exchange: all-gather failed");
  for (int r = 0; r < part_->world; ++r) {
    std::vector<uint8_t>& m = (*all)[r];
    uint32_t st = 1;
    if (m.size() >= 4) std::memcpy(&st, m.data(), 4);
    if (st == 0) continue;
    if (r == part_->rank) return Fail(local_err);
    return Fail("strip exchange: rank " + std::to_string(r) + " failed");
  }
  for (auto& m : *all) m.erase(m.begin(), m.begin() + 4);
  return true;
}

// The owned coefficients changed since the last exchange in the rows other
// ranks' halos cover (within kStripHalo rows of the owned rows' edges) go
// out; the neighbours' ones inside this strip's halo come in, written into
// the search image (whose halo rows the search loop never edits) and its
// journal, so every mirror of it (the device copy) follows.
bool PartitionComparator::SyncHalo(const CoeffImage& img) {
  if (part_->world == 1) return true;  // (no halo rows)
  const auto t0 = Clock::now();
  const Partition& P = *part_;
  const int halo_rows = kStripHalo / 8;
  std::vector<uint8_t> send;
  if (halo_.CanReplay(img)) {
    const size_t per = static_cast<size_t>(img.blocks) * 64;
    for (size_t i = halo_.pos; i < img.changed.size(); ++i) {
      const uint32_t idx = img.changed[i];
      const int c = static_cast<int>(idx / per);
      const size_t off = idx - c * per;
      const int lb = static_cast<int>(off / 64);
      const int row = lb / P.bw + P.lb0;
      if (!P.OwnsRow(row) || (row >= P.ob0 + halo_rows && row < P.ob1 - halo_rows)) continue;
      Put(&send, static_cast<uint32_t>(c));
      Put(&send, static_cast<uint32_t>((lb + P.LocalBase()) * 64 + off % 64));
      Put(&send, img.coeffs[idx]);
    }
  }
  // (not replayable: a bulk rewrite -- quantization of the originals --
  // which every rank applied to its halo rows too)
  std::vector<std::vector<uint8_t>> all;
  if (!Exchange(true, "", send, &all)) return false;
  CoeffImage& m = const_cast<CoeffImage&>(img);
  constexpr size_t kRec = 4 + 4 + sizeof(coeff_t);
  for (int r = 0; r < P.world; ++r) {
    if (r == P.rank) continue;
    const uint8_t* p = all[r].data();
    for (size_t n = all[r].size() / kRec; n > 0; --n) {
      const int c = static_cast<int>(Get<uint32_t>(p));
      const uint32_t g = Get<uint32_t>(p);
      const coeff_t v = Get<coeff_t>(p);
      const int gb = static_cast<int>(g / 64), row = gb / P.bw;
      if (row < P.lb0 || row >= P.lb1 || P.OwnsRow(row)) continue;
      const int lb = gb - P.LocalBase();
      m.block(c, lb)[g % 64] = v;
      m.MarkChanged(c, lb, static_cast<int>(g % 64));
    }
  }
  halo_.Set(m);
  seconds_halo += Since(t0);
  return true;
}

// The block rows of rank q's owned rows that another rank's back end reads:
// the change order's block weights look kBlockMaxReach block rows past the
// owned rows (ComputeBlockErrorAdjustmentWeights, radius <= 4: a block's
// weight reads the activity of blocks up to 4 away, each of which reads the
// maxima up to 4 further; butteraugli_comparator.cc:169-233), so each rank
// sends those of its rows within that reach of another rank's owned rows.
constexpr int kBlockMaxReach = 8;
static std::vector<int> EdgeRows(const Partition& P, int q) {
  std::vector<int> rows;
  for (int y = P.row0[q]; y < P.row0[q + 1]; ++y)
    for (int r = 0; r < P.world; ++r)
      if (r != q && y >= P.row0[r] - kBlockMaxReach && y < P.row0[r + 1] + kBlockMaxReach) {
        rows.push_back(y);
        break;
      }
  return rows;
}

// This rank's part of a Compare's exchange: the maximum of its owned block
// maxima (the frame's distance is the maximum of the ranks') and its edge
// rows (EdgeRows); round 5 sent every owned block (4 MB per Compare at
// 8192^2).  Appended to *send.
void PartitionComparator::PackBlockMax(const std::vector<float>& bmax, std::vector<uint8_t>* send) const {
  const Partition& P = *part_;
  float own_max = 0.0f;
  for (int b = P.OwnLo(); b < P.OwnHi(); ++b) own_max = std::max(own_max, bmax[b]);
  const std::vector<int> rows = EdgeRows(P, P.rank);
  const size_t at = send->size();
  send->resize(at + (1 + rows.size() * P.bw) * sizeof(float));
  std::memcpy(send->data() + at, &own_max, sizeof(float));
  for (size_t k = 0; k < rows.size(); ++k)
    std::memcpy(send->data() + at + (1 + k * P.bw) * sizeof(float), bmax.data() + (rows[k] * P.bw - P.LocalBase()),
                P.bw * sizeof(float));
}

// Every rank's part (all[r] from byte `skip` on) into block_max_ and the
// distance; own: this rank's maxima.  False: a malformed part.
bool PartitionComparator::UnpackBlockMax(const std::vector<float>& own,
                                         const std::vector<std::vector<uint8_t>>& all, size_t skip) {
  const Partition& P = *part_;
  for (int b = P.OwnLo(); b < P.OwnHi(); ++b) block_max_[b] = own[b];
  float d = 0.0f;
  for (int r = 0; r < P.world; ++r) {
    const std::vector<int> rows = EdgeRows(P, r);
    if (all[r].size() != skip + (1 + rows.size() * P.bw) * sizeof(float)) return false;
    const float* v = reinterpret_cast<const float*>(all[r].data() + skip);
    d = std::max(d, v[0]);
    if (r == P.rank) continue;
    for (size_t k = 0; k < rows.size(); ++k) {
      const int lb0 = rows[k] * P.bw - P.LocalBase();
      if (lb0 < 0 || lb0 + P.bw > local_blocks_) continue;
      std::memcpy(block_max_.data() + lb0, v + 1 + k * P.bw, P.bw * sizeof(float));
    }
  }
  // ButteraugliScoreFromDiffmap (butteraugli.cc:1233-1240): the maximum of
  // the map is the maximum of its block maxima
  distance_ = d;
  return true;
}

bool PartitionComparator::Compare(const CoeffImage& img) {
  if (!SyncHalo(img)) return false;
  std::vector<float> bmax;
  const bool ok = coder_->CompareStart(img) && coder_->Finish(&bmax, nullptr);
  std::vector<uint8_t> send;
  if (ok) PackBlockMax(bmax, &send);
  std::vector<std::vector<uint8_t>> all;
  if (!Exchange(ok, coder_->err, send, &all)) return false;
  return UnpackBlockMax(bmax, all, 0) || Fail("strip exchange: block maxima");
}

// A local step's outcome agreed on by every rank (one small all-gather), so
// that a failing rank does not leave the others in the next exchange.
bool PartitionComparator::Agree(bool ok, const std::string& local_err) {
  if (part_->world == 1) return ok || Fail(local_err);
  const uint32_t mine = ok ? 0u : 1u;
  std::vector<uint32_t> st(part_->world);
  if (!part_->coll->AllGather(&mine, sizeof(mine), st.data()))
    return Fail("strip exchange: all-gather failed");
  for (int r = 0; r < part_->world; ++r) {
    if (st[r] == 0) continue;
    if (r == part_->rank) return Fail(local_err);
    return Fail("strip exchange: rank " + std::to_string(r) + " failed");
  }
  return true;
}

bool StripDeviceOrder() {
  static const bool host = getenv("GZ_STRIP_HOST_ORDER") && atoi(getenv("GZ_STRIP_HOST_ORDER")) != 0;
  return !host;
}

bool PartitionComparator::DeviceOrderReset(bool* available) {
  *available = false;
  if (part_->world == 1) return inner_->DeviceOrderReset(available) || Fail(inner_->error());
  if (!StripDeviceOrder()) return true;
  inner_->SetDeviceOrderScope(part_->OwnLo(), part_->OwnHi(), part_->LocalBase(), this);
  const bool ok = inner_->DeviceOrderReset(available);
  // agreed by every rank: a failure fails all; a rank whose buffers could
  // not be allocated sends every rank to the host order
  int64_t st[2] = {ok ? 0 : 1, ok && *available ? 1 : 0};
  if (!part_->SumAll(st, 2)) return Fail("strip exchange: all-gather failed");
  if (st[0]) return Fail(ok ? "strip exchange: a rank's device order failed" : inner_->error());
  if (st[1] != part_->world) {
    *available = false;
    inner_->SetDeviceOrderScope(0, 0, 0, nullptr);
  }
  return true;
}

// Engine::OrderExchange: in-place sums (values as signed 32-bit: counts and
// histogram deltas), the rank's status summed beside them
bool PartitionComparator::SumU32(bool ok, uint32_t* v, int n) {
  std::vector<int64_t> t(static_cast<size_t>(n) + 1);
  for (int i = 0; i < n; ++i) t[i] = ok ? static_cast<int32_t>(v[i]) : 0;
  t[n] = ok ? 0 : 1;
  const auto t0 = Clock::now();
  const bool sent = part_->SumAll(t.data(), n + 1);
  seconds_exchange += Since(t0);
  if (!sent || t[n]) return false;
  for (int i = 0; i < n; ++i) v[i] = static_cast<uint32_t>(t[i]);
  return true;
}

bool PartitionComparator::Gather(bool ok, const std::vector<unsigned long long>& mine,
                                 std::vector<unsigned long long>* all) {
  std::vector<uint8_t> send(mine.size() * 8);
  if (!mine.empty()) std::memcpy(send.data(), mine.data(), send.size());
  std::vector<std::vector<uint8_t>> got;
  if (!Exchange(ok, "order selection", send, &got)) return false;
  all->clear();
  for (const auto& m : got) {
    const size_t k = all->size();
    all->resize(k + m.size() / 8);
    if (!m.empty()) std::memcpy(all->data() + k, m.data(), m.size() / 8 * 8);
  }
  return true;
}

bool PartitionComparator::StartBlockComparisons() {
  const bool ok = inner_->StartBlockComparisons();
  return Agree(ok, ok ? "" : inner_->error());
}

void PartitionComparator::FinishBlockComparisons() { inner_->FinishBlockComparisons(); }

bool PartitionComparator::BlockZeroingOrders(const CoeffImage& img, const JpegData& orig_jpg,
                                             int comp_mask, int lookahead, bool new_model,
                                             std::vector<CoeffData>* out) {
  if (!SyncHalo(img)) return false;
  const bool ok = inner_->BlockZeroingOrders(img, orig_jpg, comp_mask, lookahead, new_model, out);
  return Agree(ok, ok ? "" : inner_->error());
}

bool PartitionComparator::BlockZeroingCandidates(const CoeffImage& img, const JpegData& orig_jpg,
                                                 int comp_mask, int lookahead, bool new_model,
                                                 std::vector<int>* offsets,
                                                 std::vector<uint8_t>* idx,
                                                 std::vector<float>* err) {
  // (the search reads the entries of owned blocks only; no exchange)
  if (!SyncHalo(img)) return false;
  const bool ok = inner_->BlockZeroingCandidates(img, orig_jpg, comp_mask, lookahead, new_model,
                                                 offsets, idx, err);
  return Agree(ok, ok ? "" : inner_->error());
}

bool PartitionComparator::QuantizeFromOriginal(const int q[3][kDCTBlockSize], CoeffImage* img,
                                               bool need_host) {
  // every rank quantizes its whole strip, halo rows included: the halo then
  // holds exactly its owners' values
  const bool host_coder = dynamic_cast<HipButteraugliComparator*>(inner_.get()) == nullptr;
  const bool ok = inner_->QuantizeFromOriginal(q, img, need_host || host_coder);
  if (!Agree(ok, ok ? "" : inner_->error())) return false;
  halo_.Set(*img);
  return true;
}

bool PartitionComparator::SetOriginalCoeffs(const JpegData& jpg) {
  const bool ok = inner_->SetOriginalCoeffs(jpg);
  return Agree(ok, ok ? "" : inner_->error());
}

void PartitionComparator::ComputeBlockErrorAdjustmentWeights(
    int direction, int max_block_dist, double target_mul, int factor_x, int factor_y,
    const std::vector<float>& max_dist_per_block, std::vector<float>* block_weight) {
  // over the strip image: a block's weight reads the maxima within
  // max_block_dist (<= 4) blocks, inside the halo for every owned block
  const int local_h = std::min(part_->height, 8 * part_->lb1) - 8 * part_->lb0;
  BlockErrorAdjustmentWeights(part_->width, local_h, target_, direction, max_block_dist, target_mul,
                              factor_x, factor_y, max_dist_per_block, block_weight);
}

int PartitionComparator::DeviceHistograms(const CoeffImage& img, JpegHistogram dc[3],
                                          JpegHistogram ac[3]) {
  if (!SyncHalo(img)) return -1;
  uint32_t hist[6 * 256];
  uint64_t chroma = 0;
  const bool ok = coder_->StageStart(img, part_->OwnLo(), part_->OwnHi()) &&
                  coder_->StageWait(hist, &chroma);
  std::vector<uint8_t> send;
  if (ok) {
    send.resize(sizeof(hist));
    std::memcpy(send.data(), hist, sizeof(hist));
    Put(&send, chroma);
  }
  std::vector<std::vector<uint8_t>> all;
  if (!Exchange(ok, coder_->err, send, &all)) return -1;
  std::vector<uint32_t> sum(6 * 256, 0);
  uint64_t csum = 0;
  for (int r = 0; r < part_->world; ++r) {
    const uint8_t* p = all[r].data();
    for (int i = 0; i < 6 * 256; ++i) sum[i] += Get<uint32_t>(p);
    csum += Get<uint64_t>(p);
  }
  return HistogramsFromStage(sum.data(), csum, dc, ac);
}

bool PartitionComparator::DeviceEncodeAndCompare(const CoeffImage& img, const JpegData& meta,
                                                 bool strip_metadata, size_t* size) {
  return CodeAndCompare(img, meta, nullptr, strip_metadata, size);
}

bool PartitionComparator::DeviceEncodeOriginalAndCompare(const CoeffImage& img,
                                                         const JpegData& jpg_in,
                                                         bool strip_metadata, size_t* size,
                                                         bool* used) {
  JpegData hdr;
  JpegHeaderOf(jpg_in, &hdr);
  hdr.width = part_->width;
  hdr.height = part_->height;
  hdr.mcu_cols = part_->bw;
  hdr.mcu_rows = part_->bh;
  for (JpegComponent& c : hdr.components) {
    c.width_in_blocks = part_->bw;
    c.height_in_blocks = part_->bh;
  }
  *used = true;
  return CodeAndCompare(img, jpg_in, &hdr, strip_metadata, size);
}

bool PartitionComparator::DeviceEncodeAndCompareKnown(const CoeffImage& img, const JpegData& meta,
                                                      bool strip_metadata, const JpegHistogram dc[3],
                                                      const JpegHistogram ac[3], int ncomp, double best_score,
                                                      size_t* size, bool* skipped) {
  // The Compare first (its exchange gives every rank the frame's distance);
  // the frame's codes from the back end's tracked histograms bound the
  // scan's size from below (ScanBits: the exact bit count without the
  // stuffing), so a candidate that cannot become the output (MaybeOutput,
  // processor.cc:151-160: ScoreJPEG grows with the distance and the size)
  // is not coded -- the same decision on every rank, from frame-wide values.
  // A candidate that can is coded as DeviceEncodeAndCompare codes it (each
  // rank's part offset needs its own histograms: the stage pass).
  *skipped = false;
  const Partition& P = *part_;
  JpegHistogram dc_h[3], ac_h[3];
  for (int c = 0; c < ncomp; ++c) {
    dc_h[c] = dc[c];
    ac_h[c] = ac[c];
  }
  std::string prologue;
  JpegCodeTables codes;
  if (!PrepareScan(P.width, P.height, img.quant, meta, strip_metadata, ncomp, dc_h, ac_h, &prologue, &codes))
    return Fail("strip coder: jpeg header");
  const size_t size_lb = prologue.size() + static_cast<size_t>((ScanBits(dc, ac, ncomp, codes) + 7) / 8) + 2;
  if (!Compare(img)) return false;
  if (best_score >= 0 && scan_bound_mismatches == 0 && ScoreJPEG(distance_, static_cast<int>(size_lb), target_) >= best_score) {
    *skipped = true;
    ++scans_skipped;
    return true;
  }
  if (!CodeAndCompare(img, meta, nullptr, strip_metadata, size, /*compare=*/false)) return false;
  // (the coded scan's bits are the histograms'; a mismatch would make the
  // bound unsafe: later candidates are then always coded)
  if (cur_size_ < size_lb) ++scan_bound_mismatches;
  return true;
}

bool PartitionComparator::CodeAndCompare(const CoeffImage& img, const JpegData& meta,
                                         const JpegData* hdr, bool strip_metadata, size_t* size,
                                         bool compare) {
  // one stream order per rank: histogram stage, Compare pass; the
  // histograms' exchange and the codes while the pass runs; the scan part at
  // this rank's offset; then the maxima and the parts' seams.  (compare
  // false: the Compare of img has been done; the scan alone.)
  if (!SyncHalo(img)) return false;
  const Partition& P = *part_;
  const int m0 = P.OwnLo(), m1 = P.OwnHi();
  uint32_t hist[6 * 256];
  uint64_t chroma = 0;
  bool ok = coder_->StageStart(img, m0, m1) && (!compare || coder_->CompareStart(img)) &&
            coder_->StageWait(hist, &chroma);
  std::vector<uint8_t> send;
  if (ok) {
    send.resize(sizeof(hist));
    std::memcpy(send.data(), hist, sizeof(hist));
    Put(&send, chroma);
  }
  std::vector<std::vector<uint8_t>> all;
  if (!Exchange(ok, coder_->err, send, &all)) return false;
  // the frame's histograms, codes and headers (the same on every rank)
  std::vector<uint32_t> sum(6 * 256, 0);
  uint64_t csum = 0;
  for (int r = 0; r < P.world; ++r) {
    const uint8_t* p = all[r].data();
    for (int i = 0; i < 6 * 256; ++i) sum[i] += Get<uint32_t>(p);
    csum += Get<uint64_t>(p);
  }
  JpegHistogram dc_h[3], ac_h[3];
  const int ncomp = HistogramsFromStage(sum.data(), csum, dc_h, ac_h);
  if (hdr && static_cast<int>(hdr->components.size()) != ncomp) {
    std::vector<float> unused;
    coder_->Finish(&unused, nullptr);
    return Fail("strip coder: an original without chroma is not supported");
  }
  JpegCodeTables codes;
  if (!(hdr ? PrepareScanFor(*hdr, strip_metadata, ncomp, dc_h, ac_h, &cur_prologue_, &codes)
            : PrepareScan(P.width, P.height, img.quant, meta, strip_metadata, ncomp, dc_h, ac_h,
                          &cur_prologue_, &codes))) {
    std::vector<float> unused;
    coder_->Finish(&unused, nullptr);
    return Fail("strip coder: jpeg header");
  }
  // every rank's bit count from its own histograms: each symbol is its code
  // and its magnitude bits (the DC symbol is its bit count, an AC symbol's
  // low nibble), so the parts' offsets need no further exchange
  std::vector<uint64_t> bits(P.world, 0);
  for (int r = 0; r < P.world; ++r) {
    const uint32_t* h = reinterpret_cast<const uint32_t*>(all[r].data());
    uint64_t b = 0;
    for (int c = 0; c < ncomp; ++c)
      for (int i = 0; i < 256; ++i) {
        b += static_cast<uint64_t>(h[(2 * c) * 256 + i]) * (codes.dc_len[c][i] + i);
        b += static_cast<uint64_t>(h[(2 * c + 1) * 256 + i]) * (codes.ac_len[c][i] + (i & 15));
      }
    bits[r] = b;
  }
  uint64_t base = 0, total = 0;
  for (int r = 0; r < P.world; ++r) {
    if (r < P.rank) base += bits[r];
    total += bits[r];
  }
  Part part;
  std::vector<float> bmax;
  ok = coder_->ScanStart(ncomp, codes, m0, m1, base, P.rank == P.world - 1) &&
       coder_->Finish(&bmax, &part);
  if (ok && part.bits != bits[P.rank]) {
    ok = false;
    coder_->err = "strip coder: scan bits differ from the histogram count";
  }
  send.clear();
  if (ok) {
    Put(&send, part.ff);
    Put(&send, part.first_word);
    Put(&send, part.last_word);
    Put(&send, static_cast<uint32_t>((part.first_shared ? 1 : 0) | (part.last_open ? 2 : 0)));
    if (compare) PackBlockMax(bmax, &send);
  }
  if (!Exchange(ok, coder_->err, send, &all)) return false;
  uint64_t ff = 0;
  uint32_t prev_last = 0;
  for (int r = 0; r < P.world; ++r) {
    const uint8_t* p = all[r].data();
    if (all[r].size() < 20) return Fail("strip exchange: scan parts");
    ff += Get<uint64_t>(p);
    const uint32_t first = Get<uint32_t>(p), last = Get<uint32_t>(p), flags = Get<uint32_t>(p);
    // a word two parts share: complete once both halves are in
    if (flags & 1) ff += CountFfBytes(prev_last | first, 4);
    prev_last = last;
  }
  if (compare && !UnpackBlockMax(bmax, all, 20)) return Fail("strip exchange: block maxima");
  // prologue + scan bytes (padded) + a stuffed 0x00 per 0xff + EOI
  cur_size_ = cur_prologue_.size() + static_cast<size_t>((total + 7) / 8 + ff) + 2;
  *size = cur_size_;
  return true;
}

void PartitionComparator::DeviceKeepEncoded() {
  coder_->Keep();
  kept_prologue_ = cur_prologue_;
  kept_size_ = cur_size_;
}

bool PartitionComparator::DeviceFetchKept(std::string* out) {
  // every rank's part of the kept scan, assembled in rank order
  std::vector<uint32_t> words;
  Part part;
  const bool ok = coder_->FetchKept(&words, &part);
  std::vector<uint8_t> send;
  if (ok) {
    Put(&send, part.base);
    Put(&send, part.bits);
    Put(&send, part.first_word);
    Put(&send, part.last_word);
    Put(&send, static_cast<uint32_t>((part.first_shared ? 1 : 0) | (part.last_open ? 2 : 0)));
    const size_t at = send.size();
    send.resize(at + words.size() * 4);
    std::memcpy(send.data() + at, words.data(), words.size() * 4);
  }
  std::vector<std::vector<uint8_t>> all;
  if (!Exchange(ok, coder_->err, send, &all)) return false;
  uint64_t total = 0;
  for (int r = 0; r < part_->world; ++r) {
    const uint8_t* p = all[r].data();
    const uint64_t base = Get<uint64_t>(p), bits = Get<uint64_t>(p);
    total = std::max(total, base + bits);
  }
  std::vector<uint32_t> stream((total + 31) / 32 + 1, 0u);
  for (int r = 0; r < part_->world; ++r) {
    const uint8_t* p = all[r].data();
    const uint64_t base = Get<uint64_t>(p), bits = Get<uint64_t>(p);
    const uint32_t first = Get<uint32_t>(p), last = Get<uint32_t>(p), flags = Get<uint32_t>(p);
    const size_t n = (all[r].size() - 28) / 4;
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
    const size_t w0 = static_cast<size_t>(base >> 5);
    for (size_t i = 0; i < n; ++i) stream[w0 + i] |= w[i];
    if (flags & 1) stream[w0] |= first;
    if (flags & 2) stream[static_cast<size_t>((base + bits) >> 5)] |= last;
  }
  *out = kept_prologue_;
  AppendStuffedScan(reinterpret_cast<const uint8_t*>(stream.data()), total, out);
  if (out->size() != kept_size_) return Fail("strip coder: assembled size differs from the scored size");
  return true;
}

int ProcessStrips(int device, const ProcessParams& params, const uint8_t* rgb, int w, int h,
                  Collectives* coll, ProcessResult* result, std::string* err) {
  const auto t0 = Clock::now();
  if (w <= 0 || h <= 0 || w >= (1 << 16) || h >= (1 << 16)) {
    if (err) *err = "Could not create jpg data from rgb pixels";
    return GZ_ERR_INVALID_ARG;
  }
  if (params.butteraugli_target > 2.0f) {
    if (err) *err = "butteraugli target above 2.0 (quality below 84) is not supported";
    return GZ_ERR_INVALID_ARG;
  }
  // One rank: its strip is the frame and there is nothing to exchange -- the
  // single-engine search, whose bytes the split reproduces (its device
  // order, known-histogram coding and skipped scans; the strip machinery at
  // world 1 took 1.28 s for configs[4] against the engine's 1.14).
  // GZ_STRIP_FORCE=1 keeps the strip machinery, for its tests.
  static const bool force = getenv("GZ_STRIP_FORCE") && atoi(getenv("GZ_STRIP_FORCE")) != 0;
  if (coll->world() == 1 && !force) {
    const int rc = Process(device, params, rgb, false, w, h, result, err);
    result->detail["strip_single_engine"] = 1;
    return rc;
  }
  const StripLayout L = StripLayout::Make(w, h, coll->world());
  for (int r = 0; r < coll->world(); ++r)
    if (L.y1[r] <= L.y0[r]) {
      if (err) *err = "strips: every rank must own rows (height >= 24 x ranks)";
      return GZ_ERR_INVALID_ARG;
    }
  if (w < 32 || h < 32) {
    // no Butteraugli below 32 px (processor.cc:1170-1181): one rank's work
    JpegData jpg;
    EncodeRGBToJpegData(rgb, w, h, &jpg);
    result->seconds_setup = Since(t0);
    return ProcessJpegData(params, jpg, nullptr, result, err);
  }
  Partition part = Partition::Make(L, coll);
  const int r = coll->rank();
  std::string e;
  auto hip = HipButteraugliComparator::Create(device, w, L.e1[r] - L.e0[r],
                                              rgb + static_cast<size_t>(3) * w * L.e0[r], false,
                                              params.butteraugli_target, &e);
  JpegData jpg;  // the strip's q=1 coefficients (device FDCT of its rows)
  if (hip && !hip->OriginalJpegData(&jpg)) {
    e = hip->error();
    hip.reset();
  }
  // every rank reports whether its device comparator came up before any
  // rank enters the search (a rank that returned here alone would leave the
  // others waiting in the first exchange)
  const uint32_t mine = hip ? 0u : 1u;
  std::vector<uint32_t> status(coll->world());
  if (!coll->AllGather(&mine, sizeof(mine), status.data())) {
    if (err) *err = "strip setup: status all-gather failed";
    return GZ_ERR_INTERNAL;
  }
  for (int q = 0; q < coll->world(); ++q) {
    if (status[q] == 0) continue;
    if (err) *err = q == r ? e : "strip setup: rank " + std::to_string(q) + " failed";
    return GZ_ERR_DEVICE;
  }
  HipButteraugliComparator* hp = hip.get();
  PartitionComparator cmp(&part, std::move(hip), params.butteraugli_target);
  result->seconds_setup = Since(t0);
  const int rc = ProcessJpegData(params, jpg, &cmp, result, err, &part);
  result->compares = hp->compares;
  result->seconds_compare = hp->seconds_compare;
  result->seconds_zeroing = hp->seconds_zeroing;
  result->detail["strip_exchange_s"] = cmp.seconds_exchange;
  result->detail["strip_halo_s"] = cmp.seconds_halo;
  result->seconds_total = Since(t0);
  return rc;
}

}  // namespace gz
