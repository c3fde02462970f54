// Portions restate Guetzli (Copyright 2016 Google Inc., Apache License 2.0,
// http://www.apache.org/licenses/LICENSE-2.0) as modified in
// yyamamoto79/guetzli-cuda-opencl: jpeg_data_writer.cc and entropy_encode.cc (SetDepth /
// ClusterHistograms / the Huffman code construction).
// Byte-exact output forces their operation order and constants; the
// code around them is this repository's own.
#include "host/jpeg_writer.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "host/thread_pool.h"

#include <emmintrin.h>

namespace gz {

namespace {

inline int Log2FloorNonZero(uint32_t n) { return 31 ^ __builtin_clz(n); }
inline int Log2Floor(uint32_t n) { return n == 0 ? -1 : Log2FloorNonZero(n); }

struct TreeNode {
  uint32_t total;
  int16_t left;
  int16_t right_or_value;
};

// Assigns each leaf its depth; false if the tree is deeper than max_depth
// (SetDepth, entropy_encode.cc:26-45).
bool AssignDepths(int root, const TreeNode* pool, uint8_t* depth, int max_depth) {
  int stack[17];
  int level = 0;
  int p = root;
  stack[0] = -1;
  for (;;) {
    if (pool[p].left >= 0) {
      ++level;
      if (level > max_depth) return false;
      stack[level] = pool[p].right_or_value;
      p = pool[p].left;
      continue;
    }
    depth[pool[p].right_or_value] = static_cast<uint8_t>(level);
    while (level >= 0 && stack[level] == -1) --level;
    if (level < 0) return true;
    p = stack[level];
    stack[level] = -1;
  }
}

// Bit packer with 0xff byte stuffing (jpeg_bit_writer.h).
class BitSink {
 public:
  explicit BitSink(std::string* out) : out_(out) {}
  void Put(int nbits, uint64_t bits) {
    free_ -= nbits;
    acc_ |= bits << free_;
    if (free_ <= 16) {
      for (int s = 56; s >= 16; s -= 8) Emit(static_cast<int>((acc_ >> s) & 0xff));
      acc_ <<= 48;
      free_ += 48;
    }
  }
  void Flush() {
    while (free_ <= 56) {
      Emit(static_cast<int>((acc_ >> 56) & 0xff));
      acc_ <<= 8;
      free_ += 8;
    }
    if (free_ < 64) {
      const int pad = 0xff >> (64 - free_);
      Emit(static_cast<int>(((acc_ >> 56) & ~pad) | pad));
    }
    acc_ = 0;
    free_ = 64;
  }

 private:
  void Emit(int byte) {
    out_->push_back(static_cast<char>(byte));
    if (byte == 0xff) out_->push_back(0);
  }
  std::string* out_;
  uint64_t acc_ = 0;
  int free_ = 64;
};

using HuffTable = HuffCodeTable;

void BuildCodeCounts(const uint8_t* depth, int* counts, int* values) {
  // BuildHuffmanCode, jpeg_data_writer.cc:138-153
  for (int i = 0; i < JpegHistogram::kSize; ++i)
    if (depth[i] > 0) ++counts[depth[i]];
  int offset[17] = {0};
  for (int i = 1; i <= 16; ++i) offset[i] = offset[i - 1] + counts[i - 1];
  for (int i = 0; i < JpegHistogram::kSize; ++i)
    if (depth[i] > 0) values[offset[depth[i]]++] = i;
}

void BuildCodeTable(const int* counts, const int* values, HuffTable* t) {
  // canonical code assignment, BuildHuffmanCodeTable jpeg_data_writer.cc:155-186;
  // the last (fake) symbol is dropped.
  int sizes[258];
  int codes[258];
  int p = 0;
  for (int l = 1; l <= 16; ++l)
    for (int i = counts[l]; i > 0; --i) sizes[p++] = l;
  if (p == 0) return;
  sizes[p - 1] = 0;
  const int lastp = p - 1;
  int code = 0, si = sizes[0];
  p = 0;
  while (sizes[p]) {
    while (sizes[p] == si) codes[p++] = code++;
    code <<= 1;
    ++si;
  }
  for (p = 0; p < lastp; ++p) {
    t->depth[values[p]] = static_cast<uint8_t>(sizes[p]);
    t->code[values[p]] = codes[p];
  }
}

void UpdateACHistogramForBlock(const coeff_t* c, JpegHistogram* h) {
  int r = 0;
  for (int k = 1; k < 64; ++k) {
    const coeff_t v = c[kJPEGNaturalOrder[k]];
    if (v == 0) {
      ++r;
      continue;
    }
    while (r > 15) {
      h->Add(0xf0);
      r -= 16;
    }
    h->Add((r << 4) + Log2FloorNonZero(std::abs(v)) + 1);
    r = 0;
  }
  if (r > 0) h->Add(0);
}

void Put16(std::string* out, size_t v) {
  out->push_back(static_cast<char>((v >> 8) & 0xff));
  out->push_back(static_cast<char>(v & 0xff));
}

}  // namespace

void JpegHistogram::Clear() {
  std::memset(counts, 0, sizeof(counts));
  counts[kSize - 1] = 1;
}

void JpegHistogram::AddHistogram(const JpegHistogram& other) {
  for (int i = 0; i + 1 < kSize; ++i) counts[i] += other.counts[i];
  counts[kSize - 1] = 1;
}

int JpegHistogram::NumSymbols() const {
  int n = 0;
  for (int i = 0; i + 1 < kSize; ++i) n += counts[i] > 0 ? 1 : 0;
  return n;
}

namespace {
void HuffmanCodeLengthsUncached(const uint32_t* data, int length, int max_depth, uint8_t* depth);

// The back end rebuilds its entropy codes every 10 coefficient changes; most
// rebuilds leave some component histograms (and their merged pair) as they
// were, so the last few results are kept per thread and reused when the
// counts are identical (checked in full; the function is pure).
struct CodeLengthCache {
  static constexpr int kSlots = 8;
  struct Slot {
    uint64_t hash = 0;
    int length = -1, max_depth = 0;
    uint32_t counts[JpegHistogram::kSize];
    uint8_t depth[JpegHistogram::kSize];
  };
  Slot slot[kSlots];
  int next = 0;
};
}  // namespace

void HuffmanCodeLengths(const uint32_t* data, int length, int max_depth, uint8_t* depth) {
  if (length > JpegHistogram::kSize) {
    HuffmanCodeLengthsUncached(data, length, max_depth, depth);
    return;
  }
  static thread_local CodeLengthCache cache;
  // (four independent multiply chains: a quarter of FNV's dependent latency;
  // a match is confirmed by comparing the counts anyway)
  uint64_t h4[4] = {1469598103934665603ull, 0x9e3779b97f4a7c15ull, 0xc2b2ae3d27d4eb4full, 0x165667b19e3779f9ull};
  int i = 0;
  for (; i + 4 <= length; i += 4)
    for (int k = 0; k < 4; ++k) h4[k] = (h4[k] ^ data[i + k]) * 1099511628211ull;
  for (; i < length; ++i) h4[0] = (h4[0] ^ data[i]) * 1099511628211ull;
  const uint64_t hsh = h4[0] ^ (h4[1] * 31) ^ (h4[2] * 131) ^ (h4[3] * 1031);
  for (CodeLengthCache::Slot& e : cache.slot)
    if (e.hash == hsh && e.length == length && e.max_depth == max_depth &&
        std::memcmp(e.counts, data, length * sizeof(uint32_t)) == 0) {
      // (depth[] of the symbols the tree does not cover is left as the
      // caller set it, as the uncached call does)
      for (int i = 0; i < length; ++i)
        if (data[i]) depth[i] = e.depth[i];
      return;
    }
  CodeLengthCache::Slot& e = cache.slot[cache.next];
  cache.next = (cache.next + 1) % CodeLengthCache::kSlots;
  std::memset(e.depth, 0, sizeof(e.depth));
  HuffmanCodeLengthsUncached(data, length, max_depth, e.depth);
  e.hash = hsh;
  e.length = length;
  e.max_depth = max_depth;
  std::memcpy(e.counts, data, length * sizeof(uint32_t));
  for (int i = 0; i < length; ++i)
    if (data[i]) depth[i] = e.depth[i];
}

namespace {
// Sorts the n leaf keys (count << 16 | 0xffff - symbol: distinct, so the
// sorted order is unique).  The back end asks for the codes of slowly
// changing histograms, so the last few sorted symbol orders are kept per
// thread; when one of them, re-keyed with the new counts, is nearly sorted
// it is finished by insertion sort (linear plus the few inversions),
// otherwise std::sort.
void SortLeaves(uint64_t* keys, int n, const uint32_t* data, int length) {
  struct Orders {
    int n[2] = {0, 0};
    uint16_t sym[2][JpegHistogram::kSize];
    int next = 0;
  };
  static thread_local Orders cache;
  uint64_t seq[JpegHistogram::kSize];
  int best = -1, best_desc = n / 8 + 1;
  if (length <= JpegHistogram::kSize) {
    for (int o = 0; o < 2; ++o) {
      if (cache.n[o] < 2) continue;
      int m = 0, desc = 0;
      uint64_t prev = 0;
      for (int k = 0; k < cache.n[o]; ++k) {
        const int sy = cache.sym[o][k];
        if (sy >= length || !data[sy]) continue;
        const uint64_t key = (static_cast<uint64_t>(data[sy]) << 16) | (0xffff - sy);
        desc += m > 0 && prev > key ? 1 : 0;
        prev = key;
        ++m;
      }
      desc += n - m;  // leaves the order lacks (appended below)
      if (desc < best_desc) {
        best_desc = desc;
        best = o;
      }
    }
  }
  if (best < 0) {
    std::sort(keys, keys + n);
  } else {
    bool in[JpegHistogram::kSize] = {false};
    int m = 0;
    for (int k = 0; k < cache.n[best]; ++k) {
      const int sy = cache.sym[best][k];
      if (sy >= length || !data[sy]) continue;
      seq[m++] = (static_cast<uint64_t>(data[sy]) << 16) | (0xffff - sy);
      in[sy] = true;
    }
    for (int k = 0; k < n; ++k)
      if (!in[0xffff - (keys[k] & 0xffff)]) seq[m++] = keys[k];
    for (int i = 1; i < m; ++i) {  // insertion sort
      const uint64_t v = seq[i];
      int j = i;
      for (; j > 0 && seq[j - 1] > v; --j) seq[j] = seq[j - 1];
      seq[j] = v;
    }
    std::copy(seq, seq + n, keys);
  }
  if (length <= JpegHistogram::kSize) {
    Orders& c = cache;
    c.n[c.next] = n;
    for (int k = 0; k < n; ++k) c.sym[c.next][k] = static_cast<uint16_t>(0xffff - (keys[k] & 0xffff));
    c.next ^= 1;
  }
}

void HuffmanCodeLengthsUncached(const uint32_t* data, int length, int max_depth, uint8_t* depth) {
  // Huffman tree with iterative count flattening until it fits max_depth
  // (CreateHuffmanTree, entropy_encode.cc:65-145).  Leaves sorted by
  // (count asc, symbol desc): a total order, so any correct sort agrees --
  // here a sort of packed 64-bit keys.  Each retry raises every count below
  // count_limit to it: the leaves with count <= count_limit (a prefix of the
  // first attempt's order) become one group ordered by symbol alone, the
  // rest keep their order, so a retry re-sorts only that prefix.  A try's
  // tree height is tracked while it is built; depths are assigned only for
  // the tree that fits -- the same tree, leaf order and merges as the
  // reference's loop, so the same depths.
  TreeNode tree[2 * JpegHistogram::kSize + 2];
  uint8_t height[2 * JpegHistogram::kSize + 2];
  uint64_t base[JpegHistogram::kSize], bysym[JpegHistogram::kSize], keys[JpegHistogram::kSize];
  int n = 0;
  for (int i = length - 1; i >= 0; --i)
    if (data[i]) base[n++] = (static_cast<uint64_t>(data[i]) << 16) | (0xffff - i);
  if (n == 0) return;
  if (n == 1) {
    depth[0xffff - (base[0] & 0xffff)] = 1;
    return;
  }
  std::copy(base, base + n, bysym);  // (filled by descending symbol)
  SortLeaves(base, n, data, length);
  for (uint32_t count_limit = 1;; count_limit *= 2) {
    // leaves with count <= count_limit: key (count_limit, symbol), i.e.
    // ordered by descending symbol -- bysym's order, filtered (no sort)
    int low = 0;
    while (low < n && (base[low] >> 16) <= count_limit) ++low;
    int m = 0;
    for (int k = 0; k < n && m < low; ++k)
      if ((bysym[k] >> 16) <= count_limit) keys[m++] = (static_cast<uint64_t>(count_limit) << 16) | (bysym[k] & 0xffff);
    std::copy(base + low, base + n, keys + low);
    for (int k = 0; k < n; ++k) {
      tree[k] = TreeNode{static_cast<uint32_t>(keys[k] >> 16), -1,
                         static_cast<int16_t>(0xffff - (keys[k] & 0xffff))};
      height[k] = 0;
    }
    const TreeNode sentinel{~0u, -1, -1};
    tree[n] = sentinel;
    tree[n + 1] = sentinel;
    int i = 0, j = n + 1;
    for (int k = n - 1; k != 0; --k) {
      int left, right;
      if (tree[i].total <= tree[j].total) left = i++; else left = j++;
      if (tree[i].total <= tree[j].total) right = i++; else right = j++;
      const int parent = 2 * n - k;
      tree[parent].total = tree[left].total + tree[right].total;
      tree[parent].left = static_cast<int16_t>(left);
      tree[parent].right_or_value = static_cast<int16_t>(right);
      height[parent] = static_cast<uint8_t>(1 + std::max(height[left], height[right]));
      tree[parent + 1] = sentinel;
    }
    if (height[2 * n - 1] <= max_depth && AssignDepths(2 * n - 1, tree, depth, max_depth)) break;
  }
}

}  // namespace

size_t HistogramHeaderCost(const JpegHistogram& h) {
  size_t bits = 17 * 8;
  for (int i = 0; i + 1 < JpegHistogram::kSize; ++i)
    if (h.counts[i] > 0) bits += 8;
  return bits;
}

size_t HistogramEntropyCost(const JpegHistogram& h, const uint8_t depths[256]) {
  size_t bits = 0;
  for (int i = 0; i + 1 < JpegHistogram::kSize; ++i)
    bits += (h.counts[i] / 2) * (depths[i] + (i & 0xf));
  bits += (bits * 3 + 512) >> 10;
  return bits;
}

void BuildDCHistograms(const JpegData& jpg, JpegHistogram* histo) {
  for (size_t i = 0; i < jpg.components.size(); ++i) {
    const JpegComponent& c = jpg.components[i];
    coeff_t last = 0;
    for (int my = 0; my < jpg.mcu_rows; ++my)
      for (int mx = 0; mx < jpg.mcu_cols; ++mx)
        for (int iy = 0; iy < c.v_samp_factor; ++iy)
          for (int ix = 0; ix < c.h_samp_factor; ++ix) {
            const int bidx = (my * c.v_samp_factor + iy) * c.width_in_blocks + mx * c.h_samp_factor + ix;
            const coeff_t dc = c.coeffs[static_cast<size_t>(bidx) << 6];
            histo[i].Add(Log2Floor(std::abs(dc - last)) + 1);
            last = dc;
          }
  }
}

void BuildACHistograms(const JpegData& jpg, JpegHistogram* histo) {
  for (size_t i = 0; i < jpg.components.size(); ++i) {
    const JpegComponent& c = jpg.components[i];
    for (size_t j = 0; j < c.coeffs.size(); j += 64) UpdateACHistogramForBlock(&c.coeffs[j], &histo[i]);
  }
}

size_t JpegHeaderSize(const JpegData& jpg, bool strip_metadata) {
  size_t n = 2;  // SOI
  if (strip_metadata) {
    n += 18;
  } else {
    for (const std::string& a : jpg.app_data) n += 1 + a.size();
    for (const std::string& c : jpg.com_data) n += 2 + c.size();
  }
  n += 4;  // DQT
  for (const QuantTable& q : jpg.quant) n += 1 + (q.precision ? 2 : 1) * 64;
  n += 10 + 3 * jpg.components.size();  // SOF
  n += 4;                                // DHT header
  n += 8 + 2 * jpg.components.size();   // SOS
  n += 2;                                // EOI
  return n;
}

size_t ClusterHistograms(JpegHistogram* histo, size_t* num, int* idx, uint8_t* depth) {
  // greedy merge of the last two histograms while it saves bits
  // (ClusterHistograms, jpeg_data_writer.cc:298-342)
  std::memset(depth, 0, *num * JpegHistogram::kSize);
  size_t costs[4];
  for (size_t i = 0; i < *num; ++i) {
    idx[i] = static_cast<int>(i);
    uint8_t* d = &depth[i * JpegHistogram::kSize];
    HuffmanCodeLengths(histo[i].counts, JpegHistogram::kSize, 16, d);
    costs[i] = HistogramHeaderCost(histo[i]) + HistogramEntropyCost(histo[i], d);
  }
  const size_t orig = *num;
  while (*num > 1) {
    const size_t last = *num - 1, second = *num - 2;
    JpegHistogram combined(histo[last]);
    combined.AddHistogram(histo[second]);
    uint8_t dc[JpegHistogram::kSize] = {0};
    HuffmanCodeLengths(combined.counts, JpegHistogram::kSize, 16, dc);
    const size_t cost = HistogramHeaderCost(combined) + HistogramEntropyCost(combined, dc);
    if (cost < costs[last] + costs[second]) {
      histo[second] = combined;
      histo[last] = JpegHistogram();
      costs[second] = cost;
      std::memcpy(&depth[second * JpegHistogram::kSize], dc, sizeof(dc));
      for (size_t i = 0; i < orig; ++i)
        if (idx[i] == static_cast<int>(last)) idx[i] = static_cast<int>(second);
      --*num;
    } else {
      break;
    }
  }
  size_t total = 0;
  for (size_t i = 0; i < *num; ++i) total += costs[i];
  return (total + 7) / 8;
}

namespace {

// SOI, metadata, DQT and SOF1 (jpeg_data_writer.cc:53-128).
bool WriteHeaderSegments(const JpegData& jpg, bool strip_metadata, std::string* out) {
  const int ncomps = static_cast<int>(jpg.components.size());
  out->append("\xff\xd8", 2);
  if (strip_metadata) {
    static const unsigned char kApp0[] = {0xff, 0xe0, 0x00, 0x10, 0x4a, 0x46, 0x49, 0x46, 0x00,
                                          0x01, 0x01, 0x00, 0x00, 0x01, 0x00, 0x01, 0x00, 0x00};
    out->append(reinterpret_cast<const char*>(kApp0), sizeof(kApp0));
  } else {
    for (const std::string& a : jpg.app_data) {
      out->push_back('\xff');
      out->append(a);
    }
    for (const std::string& c : jpg.com_data) {
      out->append("\xff\xfe", 2);
      out->append(c);
    }
  }
  {
    size_t len = 2;
    for (const QuantTable& q : jpg.quant) len += 1 + (q.precision ? 2 : 1) * 64;
    out->append("\xff\xdb", 2);
    Put16(out, len);
    for (const QuantTable& q : jpg.quant) {
      out->push_back(static_cast<char>((q.precision << 4) + q.index));
      for (int k = 0; k < 64; ++k) {
        const int v = q.values[kJPEGNaturalOrder[k]];
        if (q.precision) out->push_back(static_cast<char>(v >> 8));
        out->push_back(static_cast<char>(v & 0xff));
      }
    }
  }
  out->append("\xff\xc1", 2);
  Put16(out, 8 + 3 * ncomps);
  out->push_back(8);
  Put16(out, jpg.height);
  Put16(out, jpg.width);
  out->push_back(static_cast<char>(ncomps));
  for (const JpegComponent& c : jpg.components) {
    if (c.quant_idx < 0 || static_cast<size_t>(c.quant_idx) >= jpg.quant.size()) return false;
    out->push_back(static_cast<char>(c.id));
    out->push_back(static_cast<char>((c.h_samp_factor << 4) | c.v_samp_factor));
    out->push_back(static_cast<char>(jpg.quant[c.quant_idx].index));
  }
  return true;
}

// DHT + SOS from the per-component DC/AC histograms (ncomps entries each;
// clobbered by clustering) -- BuildAndEncodeHuffmanCodes,
// jpeg_data_writer.cc:361-445.
void WriteHuffmanSegments(const JpegData& jpg, JpegHistogram* dc_h, JpegHistogram* ac_h,
                          HuffTable* dc_tab, HuffTable* ac_tab, std::string* out) {
  const int ncomps = static_cast<int>(jpg.components.size());
  std::vector<JpegHistogram> histo(dc_h, dc_h + ncomps);
  size_t num_dc = ncomps;
  int dc_idx[4], ac_idx[4];
  std::vector<uint8_t> depths(ncomps * JpegHistogram::kSize);
  ClusterHistograms(histo.data(), &num_dc, dc_idx, depths.data());
  histo.resize(num_dc);
  histo.insert(histo.end(), ac_h, ac_h + ncomps);
  depths.resize((num_dc + ncomps) * JpegHistogram::kSize);
  size_t num_ac = ncomps;
  ClusterHistograms(&histo[num_dc], &num_ac, ac_idx, &depths[num_dc * JpegHistogram::kSize]);
  const size_t num_histo = num_dc + num_ac;
  histo.resize(num_histo);
  size_t total_symbols = 0;
  for (const JpegHistogram& h : histo) total_symbols += h.NumSymbols();
  out->append("\xff\xc4", 2);
  Put16(out, 2 + num_histo * 17 + total_symbols);
  for (size_t i = 0; i < num_histo; ++i) {
    const bool is_dc = i < num_dc;
    const int id = static_cast<int>(is_dc ? i : i - num_dc);
    int counts[17] = {0};
    int values[JpegHistogram::kSize] = {0};
    BuildCodeCounts(&depths[i * JpegHistogram::kSize], counts, values);
    HuffTable t;
    std::memset(t.depth, 255, sizeof(t.depth));
    std::memset(t.code, 0, sizeof(t.code));
    BuildCodeTable(counts, values, &t);
    for (int c = 0; c < ncomps; ++c) {
      if (is_dc && dc_idx[c] == id) dc_tab[c] = t;
      if (!is_dc && ac_idx[c] == id) ac_tab[c] = t;
    }
    int max_len = 16;
    while (max_len > 0 && counts[max_len] == 0) --max_len;
    --counts[max_len];
    int nsym = 0;
    for (int j = 0; j <= max_len; ++j) nsym += counts[j];
    out->push_back(static_cast<char>(is_dc ? i : i - num_dc + 0x10));
    for (int j = 1; j <= 16; ++j) out->push_back(static_cast<char>(counts[j]));
    for (int j = 0; j < nsym; ++j) out->push_back(static_cast<char>(values[j]));
  }
  out->append("\xff\xda", 2);
  Put16(out, 6 + 2 * ncomps);
  out->push_back(static_cast<char>(ncomps));
  for (int c = 0; c < ncomps; ++c) {
    out->push_back(static_cast<char>(jpg.components[c].id));
    out->push_back(static_cast<char>((dc_idx[c] << 4) | ac_idx[c]));
  }
  out->push_back(0);
  out->push_back(63);
  out->push_back(0);
}

// One block of the sequential scan (EncodeDCTBlockSequential,
// jpeg_data_writer.cc:447-500).  `at(k)` yields the coefficient at zigzag
// position k.
template <class Sink, class At>
inline void EncodeBlock(Sink& bw, const At& at, coeff_t* last_dc, const HuffTable& dct,
                        const HuffTable& act) {
  const coeff_t dc = at(0);
  coeff_t diff = static_cast<coeff_t>(dc - *last_dc);
  *last_dc = dc;
  coeff_t bits = diff;
  if (diff < 0) {
    diff = static_cast<coeff_t>(-diff);
    --bits;
  }
  const int nb = Log2Floor(static_cast<uint32_t>(static_cast<int>(diff))) + 1;
  bw.Put(dct.depth[nb], static_cast<uint64_t>(dct.code[nb]));
  if (nb > 0) bw.Put(nb, static_cast<uint64_t>(bits & ((1 << nb) - 1)));
  int r = 0;
  for (int k = 1; k < 64; ++k) {
    coeff_t v = at(k);
    if (v == 0) {
      ++r;
      continue;
    }
    coeff_t vb;
    if (v < 0) {
      v = static_cast<coeff_t>(-v);
      vb = static_cast<coeff_t>(~v);
    } else {
      vb = v;
    }
    while (r > 15) {
      bw.Put(act.depth[0xf0], static_cast<uint64_t>(act.code[0xf0]));
      r -= 16;
    }
    const int nbits = Log2FloorNonZero(static_cast<uint32_t>(static_cast<int>(v))) + 1;
    const int sym = (r << 4) + nbits;
    bw.Put(act.depth[sym], static_cast<uint64_t>(act.code[sym]));
    bw.Put(nbits, static_cast<uint64_t>(vb & ((1 << nbits) - 1)));
    r = 0;
  }
  if (r > 0) bw.Put(act.depth[0], static_cast<uint64_t>(act.code[0]));
}

// EncodeBlock for a zigzag block with its non-zero mask: the same symbols,
// visiting only the non-zero coefficients.
template <class Sink>
inline void EncodeBlockMasked(Sink& bw, const coeff_t* zz, uint64_t mask, coeff_t* last_dc,
                              const HuffTable& dct, const HuffTable& act) {
  const coeff_t dc = zz[0];
  coeff_t diff = static_cast<coeff_t>(dc - *last_dc);
  *last_dc = dc;
  coeff_t bits = diff;
  if (diff < 0) {
    diff = static_cast<coeff_t>(-diff);
    --bits;
  }
  const int nb = Log2Floor(static_cast<uint32_t>(static_cast<int>(diff))) + 1;
  bw.Put(dct.depth[nb], static_cast<uint64_t>(dct.code[nb]));
  if (nb > 0) bw.Put(nb, static_cast<uint64_t>(bits & ((1 << nb) - 1)));
  uint64_t m = mask & ~1ull;
  int last = 0;
  while (m) {
    const int k = __builtin_ctzll(m);
    int r = k - last - 1;
    coeff_t v = zz[k];
    coeff_t vb;
    if (v < 0) {
      v = static_cast<coeff_t>(-v);
      vb = static_cast<coeff_t>(~v);
    } else {
      vb = v;
    }
    while (r > 15) {
      bw.Put(act.depth[0xf0], static_cast<uint64_t>(act.code[0xf0]));
      r -= 16;
    }
    const int nbits = Log2FloorNonZero(static_cast<uint32_t>(static_cast<int>(v))) + 1;
    const int sym = (r << 4) + nbits;
    bw.Put(act.depth[sym], static_cast<uint64_t>(act.code[sym]));
    bw.Put(nbits, static_cast<uint64_t>(vb & ((1 << nbits) - 1)));
    last = k;
    m &= m - 1;
  }
  if (last < 63) bw.Put(act.depth[0], static_cast<uint64_t>(act.code[0]));
}

// Unstuffed MSB-first bit buffer: chunks of the scan are encoded into these
// in parallel and concatenated afterwards.
struct RawBits {
  std::vector<uint64_t> words;
  uint64_t acc = 0;
  int used = 0;
  void Clear() {
    words.clear();
    acc = 0;
    used = 0;
  }
  void Put(int n, uint64_t bits) {  // 0 <= n <= 64, bits < 2^n
    if (n == 0) return;
    const int free = 64 - used;
    if (n < free) {
      acc |= bits << (free - n);
      used += n;
    } else {
      const int rem = n - free;
      acc |= bits >> rem;
      words.push_back(acc);
      acc = rem ? (bits << (64 - rem)) : 0;
      used = rem;
    }
  }
  uint64_t bit_count() const { return 64 * static_cast<uint64_t>(words.size()) + used; }
};

// Appends the concatenation of `parts`, padded with one bits to a byte
// boundary and 0xff-stuffed (BitWriter::JumpToByteBoundary + EmitByte).
void EmitStuffed(const std::vector<RawBits>& parts, int nparts, std::string* out) {
  RawBits all;
  uint64_t total = 0;
  for (int i = 0; i < nparts; ++i) total += parts[i].bit_count();
  all.words.reserve(total / 64 + 2);
  for (int i = 0; i < nparts; ++i) {
    const RawBits& p = parts[i];
    if (all.used == 0) {
      all.words.insert(all.words.end(), p.words.begin(), p.words.end());
    } else {
      for (uint64_t w : p.words) all.Put(64, w);
    }
    if (p.used) all.Put(p.used, p.acc >> (64 - p.used));
  }
  if (all.used & 7) all.Put(8 - (all.used & 7), (1u << (8 - (all.used & 7))) - 1);
  const size_t nbytes = all.words.size() * 8 + all.used / 8;
  out->reserve(out->size() + nbytes + nbytes / 128 + 16);
  auto emit = [out](uint8_t b) {
    out->push_back(static_cast<char>(b));
    if (b == 0xff) out->push_back(0);
  };
  for (uint64_t w : all.words)
    for (int s = 56; s >= 0; s -= 8) emit(static_cast<uint8_t>(w >> s));
  for (int s = 56; s > 56 - all.used; s -= 8) emit(static_cast<uint8_t>(all.acc >> s));
}

}  // namespace

// ---------------------------------------------------------------------------
// Staged, multithreaded encode (one-block-per-MCU, i.e. 4:4:4, layouts; any
// other layout takes the serial writer).
//
// Stage: the quantized coefficients in zigzag order, a non-zero bit mask per
// block and the DC / AC symbol histograms.  A full stage runs over chunks of
// blocks on the pool; for a CoeffImage the stage is kept between calls and
// later brought up to date from the image's change journal -- the search
// loop edits a few 10k of millions of coefficients per iteration, so only
// the touched blocks are re-quantized and their symbols swapped in the
// histograms (histograms are counts: the result equals a full recount).
//
// Encode: cluster + Huffman tables (serial, tiny), scan chunks into raw bit
// buffers (parallel), then concatenate + pad + 0xff-stuff (serial, bytes of
// output).
// ---------------------------------------------------------------------------

struct ScanScratch {
  int blocks = 0, stored = 0, ncomp = 0, chunks = 0, per_chunk = 0;
  std::vector<coeff_t> zz;        // [stored][blocks][64] quantized, zigzag order
  std::vector<uint64_t> mask;     // [stored][blocks] bit k <=> zz[k] != 0
  std::vector<uint8_t> stored_nz; // [stored][blocks] non-zero pre-division coefficients
  int64_t chroma_nz = 0;          // sum of stored_nz over components 1..2
  std::vector<RawBits> parts;
  std::vector<JpegHistogram> dc, ac;  // [chunk][4] during a full stage
  std::vector<int64_t> chunk_nz;      // [chunk] chroma non-zeros during a full stage
  JpegHistogram dc_all[4], ac_all[4]; // totals per stored component
  JpegData hdr;                       // the staged image without coefficients
  CoeffCursor cursor;                 // CoeffImage state the stage reflects
  std::vector<uint32_t> stamp;        // [stored * blocks] touched-block marks
  uint32_t stamp_id = 0;
  std::vector<uint32_t> touched;
};

ScanScratch* NewScanScratch() { return new ScanScratch; }
void FreeScanScratch(ScanScratch* s) { delete s; }

namespace {

inline uint64_t NonzeroMask(const coeff_t* zz) {
  uint64_t m = 0;
  const __m128i zero = _mm_setzero_si128();
  for (int i = 0; i < 4; ++i) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(zz + 16 * i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(zz + 16 * i + 8));
    const __m128i z = _mm_packs_epi16(_mm_cmpeq_epi16(a, zero), _mm_cmpeq_epi16(b, zero));
    m |= static_cast<uint64_t>(static_cast<uint16_t>(~_mm_movemask_epi8(z))) << (16 * i);
  }
  return m;
}

// The AC symbols of a block (processor.cc:491-515 / jpeg_data_writer.cc
// BuildACHistograms) from its zigzag values and non-zero mask.
inline void AddAcSymbols(const coeff_t* zz, uint64_t mask, int weight, JpegHistogram* h) {
  uint64_t m = mask & ~1ull;
  int last = 0;
  while (m) {
    const int k = __builtin_ctzll(m);
    int r = k - last - 1;
    while (r > 15) {
      h->Add(0xf0, weight);
      r -= 16;
    }
    h->Add((r << 4) + Log2FloorNonZero(std::abs(zz[k])) + 1, weight);
    last = k;
    m &= m - 1;
  }
  if (last < 63) h->Add(0, weight);
}

inline int DcSymbol(coeff_t dc, coeff_t last) { return Log2Floor(std::abs(dc - last)) + 1; }

void Partition(int blocks, ScanScratch* s) {
  const int target_chunks = 4 * HostThreads();
  s->per_chunk = std::max(64, (blocks + target_chunks - 1) / target_chunks);
  s->chunks = (blocks + s->per_chunk - 1) / s->per_chunk;
}

// Full stage.  load(c, b, zz) writes block b of component c in zigzag order
// and returns the number of non-zero stored (pre-division) coefficients.
template <class Load>
void StageAll(int blocks, int stored, ScanScratch* s, const Load& load) {
  s->blocks = blocks;
  s->stored = stored;
  s->zz.resize(static_cast<size_t>(blocks) * 64 * stored);
  s->mask.resize(static_cast<size_t>(blocks) * stored);
  s->stored_nz.resize(static_cast<size_t>(blocks) * stored);
  Partition(blocks, s);
  s->dc.assign(static_cast<size_t>(s->chunks) * 4, JpegHistogram());
  s->ac.assign(static_cast<size_t>(s->chunks) * 4, JpegHistogram());
  s->chunk_nz.assign(s->chunks, 0);
  ParallelFor(s->chunks, [&](int ch) {
    const int b0 = ch * s->per_chunk, b1 = std::min(blocks, b0 + s->per_chunk);
    int64_t nz = 0;
    coeff_t prev[64];
    for (int c = 0; c < stored; ++c) {
      JpegHistogram& hdc = s->dc[ch * 4 + c];
      JpegHistogram& hac = s->ac[ch * 4 + c];
      coeff_t last = 0;
      if (b0 > 0) {
        load(c, b0 - 1, prev);
        last = prev[0];
      }
      for (int b = b0; b < b1; ++b) {
        const size_t bi = static_cast<size_t>(c) * blocks + b;
        coeff_t* dst = &s->zz[bi * 64];
        const int snz = load(c, b, dst);
        s->stored_nz[bi] = static_cast<uint8_t>(snz);
        if (c > 0) nz += snz;
        const uint64_t m = NonzeroMask(dst);
        s->mask[bi] = m;
        hdc.Add(DcSymbol(dst[0], last));
        last = dst[0];
        AddAcSymbols(dst, m, 1, &hac);
      }
    }
    s->chunk_nz[ch] = nz;
  });
  s->chroma_nz = 0;
  for (int ch = 0; ch < s->chunks; ++ch) s->chroma_nz += s->chunk_nz[ch];
  for (int c = 0; c < 4; ++c) {
    s->dc_all[c].Clear();
    s->ac_all[c].Clear();
    if (c >= stored) continue;
    for (int ch = 0; ch < s->chunks; ++ch) {
      s->dc_all[c].AddHistogram(s->dc[ch * 4 + c]);
      s->ac_all[c].AddHistogram(s->ac[ch * 4 + c]);
    }
  }
  s->stamp.assign(static_cast<size_t>(blocks) * stored, 0);
  s->stamp_id = 0;
}

// Quantization as SaveToJpegData divides (output_image.cc:618-626).
// |stored| <= 2^15 and q < 2^24: the correctly rounded f32 quotient
// truncates to the exact integer quotient (an inexact quotient is at least
// 1/q from an integer, the rounding error below 2^-9/q; checked exhaustively
// for q < 2^16).
struct CoeffImageLoader {
  const CoeffImage& img;
  float qz[3][64];
  explicit CoeffImageLoader(const CoeffImage& im) : img(im) {
    for (int c = 0; c < 3; ++c)
      for (int k = 0; k < 64; ++k) qz[c][k] = static_cast<float>(img.quant[c][kJPEGNaturalOrder[k]]);
  }
  int operator()(int c, int b, coeff_t* dst) const {
    const coeff_t* src = img.block(c, b);
    int nz = 0;
    for (int k = 0; k < 64; ++k) {
      const coeff_t v = src[kJPEGNaturalOrder[k]];
      dst[k] = static_cast<coeff_t>(static_cast<int>(static_cast<float>(v) / qz[c][k]));
      nz += v != 0;
    }
    return nz;
  }
};

// Brings a CoeffImage stage up to date from the image's change journal.
void StageIncremental(const CoeffImage& img, ScanScratch* s) {
  const CoeffImageLoader load(img);
  const int blocks = s->blocks;
  if (++s->stamp_id == 0) {
    std::fill(s->stamp.begin(), s->stamp.end(), 0);
    s->stamp_id = 1;
  }
  s->touched.clear();
  for (size_t i = s->cursor.pos; i < img.changed.size(); ++i) {
    const uint32_t bi = img.changed[i] >> 6;  // c * blocks + b
    if (s->stamp[bi] != s->stamp_id) {
      s->stamp[bi] = s->stamp_id;
      s->touched.push_back(bi);
    }
  }
  // touched blocks in parallel chunks, each with its own histogram deltas
  // (uint32 counts wrap, so negative deltas sum exactly)
  const int nt = static_cast<int>(s->touched.size());
  const int per = 256;
  const int nchunks = (nt + per - 1) / per;
  struct Delta {
    JpegHistogram ac[3];
    int64_t chroma_nz = 0;
    bool dc_moved[3] = {false, false, false};
  };
  std::vector<Delta> deltas(nchunks);
  ParallelFor(nchunks, [&](int ch) {
    Delta& d = deltas[ch];
    for (int c = 0; c < 3; ++c) std::memset(d.ac[c].counts, 0, sizeof(d.ac[c].counts));
    const int t1 = std::min(nt, (ch + 1) * per);
    for (int t = ch * per; t < t1; ++t) {
      const uint32_t bi = s->touched[t];
      const int c = static_cast<int>(bi / blocks), b = static_cast<int>(bi % blocks);
      coeff_t* zz = &s->zz[static_cast<size_t>(bi) * 64];
      AddAcSymbols(zz, s->mask[bi], -1, &d.ac[c]);
      const coeff_t old_dc = zz[0];
      const int snz = load(c, b, zz);
      if (c > 0) d.chroma_nz += snz - s->stored_nz[bi];
      s->stored_nz[bi] = static_cast<uint8_t>(snz);
      s->mask[bi] = NonzeroMask(zz);
      AddAcSymbols(zz, s->mask[bi], 1, &d.ac[c]);
      if (zz[0] != old_dc) d.dc_moved[c] = true;
    }
  });
  bool dc_moved[3] = {false, false, false};
  for (const Delta& d : deltas) {
    for (int c = 0; c < 3; ++c) {
      for (int i = 0; i + 1 < JpegHistogram::kSize; ++i) s->ac_all[c].counts[i] += d.ac[c].counts[i];
      dc_moved[c] = dc_moved[c] || d.dc_moved[c];
    }
    s->chroma_nz += d.chroma_nz;
  }
  for (int c = 0; c < 3; ++c) {
    if (!dc_moved[c]) continue;  // the search loop never edits DC; recount if it did
    s->dc_all[c].Clear();
    coeff_t last = 0;
    for (int b = 0; b < blocks; ++b) {
      const coeff_t dc = s->zz[(static_cast<size_t>(c) * blocks + b) * 64];
      s->dc_all[c].Add(DcSymbol(dc, last));
      last = dc;
    }
  }
}

bool IsOneBlockPerMcu(const JpegData& jpg) {
  const int n = static_cast<int>(jpg.components.size());
  if (n < 1 || n > 4) return false;
  const size_t blocks = static_cast<size_t>(jpg.mcu_cols) * jpg.mcu_rows;
  for (const JpegComponent& c : jpg.components)
    if (c.h_samp_factor != 1 || c.v_samp_factor != 1 || c.width_in_blocks != jpg.mcu_cols ||
        c.coeffs.size() < blocks * 64)
      return false;
  return true;
}

bool WriteJpegSerial(const JpegData& jpg, bool strip_metadata, std::string* out) {
  const int ncomps = static_cast<int>(jpg.components.size());
  if (ncomps < 1 || ncomps > 4) return false;
  if (!WriteHeaderSegments(jpg, strip_metadata, out)) return false;
  std::vector<HuffTable> dc_tab(ncomps), ac_tab(ncomps);
  {
    std::vector<JpegHistogram> dc_h(ncomps), ac_h(ncomps);
    BuildDCHistograms(jpg, dc_h.data());
    BuildACHistograms(jpg, ac_h.data());
    WriteHuffmanSegments(jpg, dc_h.data(), ac_h.data(), dc_tab.data(), ac_tab.data(), out);
  }
  // entropy-coded scan (EncodeScan, jpeg_data_writer.cc:502-538)
  BitSink bw(out);
  coeff_t last_dc[4] = {0, 0, 0, 0};
  for (int my = 0; my < jpg.mcu_rows; ++my)
    for (int mx = 0; mx < jpg.mcu_cols; ++mx)
      for (int ci = 0; ci < ncomps; ++ci) {
        const JpegComponent& c = jpg.components[ci];
        for (int iy = 0; iy < c.v_samp_factor; ++iy)
          for (int ix = 0; ix < c.h_samp_factor; ++ix) {
            const int bidx = (my * c.v_samp_factor + iy) * c.width_in_blocks + mx * c.h_samp_factor + ix;
            const coeff_t* co = &c.coeffs[static_cast<size_t>(bidx) << 6];
            EncodeBlock(bw, [co](int k) { return co[kJPEGNaturalOrder[k]]; }, &last_dc[ci],
                        dc_tab[ci], ac_tab[ci]);
          }
      }
  bw.Flush();
  out->append("\xff\xd9", 2);
  return true;
}

// WriteJpegSerial's output for any sampling layout (4:2:0 MCUs of 2x2 Y
// blocks + Cb + Cr), the work split over MCU ranges on the host pool: the
// histograms per range (each range's DC predictor is the component's last
// block before it, so the differences are the serial pass's), then the scan
// per range into raw bit buffers, concatenated and stuffed.
bool WriteJpegParallel(const JpegData& jpg, bool strip_metadata, std::string* out) {
  const int ncomps = static_cast<int>(jpg.components.size());
  if (ncomps < 1 || ncomps > 4) return false;
  const int mcus = jpg.mcu_rows * jpg.mcu_cols;
  const int target = 4 * HostThreads();
  const int per = std::max(64, (mcus + target - 1) / target);
  const int chunks = (mcus + per - 1) / per;
  bool grid = chunks > 1;
  for (const JpegComponent& c : jpg.components)
    grid = grid && c.width_in_blocks == jpg.mcu_cols * c.h_samp_factor &&
           c.height_in_blocks == jpg.mcu_rows * c.v_samp_factor &&
           c.coeffs.size() == static_cast<size_t>(c.width_in_blocks) * c.height_in_blocks * 64;
  if (!grid) return WriteJpegSerial(jpg, strip_metadata, out);
  auto block_of = [&](const JpegComponent& c, int m, int iy, int ix) {
    const int my = m / jpg.mcu_cols, mx = m % jpg.mcu_cols;
    return &c.coeffs[static_cast<size_t>((my * c.v_samp_factor + iy) * c.width_in_blocks +
                                         mx * c.h_samp_factor + ix) << 6];
  };
  // the DC predictor of each component at the start of MCU m0
  auto start_dc = [&](int ci, int m0) -> coeff_t {
    if (m0 == 0) return 0;
    const JpegComponent& c = jpg.components[ci];
    return block_of(c, m0 - 1, c.v_samp_factor - 1, c.h_samp_factor - 1)[0];
  };
  if (!WriteHeaderSegments(jpg, strip_metadata, out)) return false;
  std::vector<HuffTable> dc_tab(ncomps), ac_tab(ncomps);
  {
    std::vector<JpegHistogram> dc_c(static_cast<size_t>(chunks) * ncomps), ac_c(static_cast<size_t>(chunks) * ncomps);
    ParallelFor(chunks, [&](int ch) {
      const int m0 = ch * per, m1 = std::min(mcus, m0 + per);
      for (int ci = 0; ci < ncomps; ++ci) {
        const JpegComponent& c = jpg.components[ci];
        JpegHistogram& dh = dc_c[static_cast<size_t>(ch) * ncomps + ci];
        JpegHistogram& ah = ac_c[static_cast<size_t>(ch) * ncomps + ci];
        coeff_t last = start_dc(ci, m0);
        for (int m = m0; m < m1; ++m)
          for (int iy = 0; iy < c.v_samp_factor; ++iy)
            for (int ix = 0; ix < c.h_samp_factor; ++ix) {
              const coeff_t* co = block_of(c, m, iy, ix);
              dh.Add(Log2Floor(std::abs(co[0] - last)) + 1);
              last = co[0];
              UpdateACHistogramForBlock(co, &ah);
            }
      }
    });
    // (the MCU grid is every block of each component: BuildACHistograms'
    // counts)
    std::vector<JpegHistogram> dc_h(ncomps), ac_h(ncomps);
    for (int ch = 0; ch < chunks; ++ch)
      for (int ci = 0; ci < ncomps; ++ci) {
        for (int k = 0; k + 1 < JpegHistogram::kSize; ++k) {
          dc_h[ci].counts[k] += dc_c[static_cast<size_t>(ch) * ncomps + ci].counts[k];
          ac_h[ci].counts[k] += ac_c[static_cast<size_t>(ch) * ncomps + ci].counts[k];
        }
      }
    WriteHuffmanSegments(jpg, dc_h.data(), ac_h.data(), dc_tab.data(), ac_tab.data(), out);
  }
  std::vector<RawBits> parts(chunks);
  ParallelFor(chunks, [&](int ch) {
    const int m0 = ch * per, m1 = std::min(mcus, m0 + per);
    RawBits& bw = parts[ch];
    bw.Clear();
    coeff_t last_dc[4];
    for (int ci = 0; ci < ncomps; ++ci) last_dc[ci] = start_dc(ci, m0);
    for (int m = m0; m < m1; ++m)
      for (int ci = 0; ci < ncomps; ++ci) {
        const JpegComponent& c = jpg.components[ci];
        for (int iy = 0; iy < c.v_samp_factor; ++iy)
          for (int ix = 0; ix < c.h_samp_factor; ++ix) {
            const coeff_t* co = block_of(c, m, iy, ix);
            EncodeBlock(bw, [co](int k) { return co[kJPEGNaturalOrder[k]]; }, &last_dc[ci], dc_tab[ci],
                        ac_tab[ci]);
          }
      }
  });
  EmitStuffed(parts, chunks, out);
  out->append("\xff\xd9", 2);
  return true;
}

}  // namespace

int StageCoeffImage(const CoeffImage& img, const JpegData& meta, ScanScratch* s) {
  const bool replay = s->stored == 3 && s->blocks == img.blocks && s->cursor.CanReplay(img) &&
                      img.changed.size() - s->cursor.pos < static_cast<size_t>(img.blocks) * 8;
  if (replay) {
    StageIncremental(img, s);
  } else {
    StageAll(img.blocks, 3, s, CoeffImageLoader(img));
  }
  s->cursor.Set(img);
  s->ncomp = s->chroma_nz > 0 ? 3 : 1;  // SaveToJpegData drops all-zero chroma
  s->hdr.app_data = meta.app_data;
  s->hdr.com_data = meta.com_data;
  img.SaveHeaderToJpegData(s->ncomp, &s->hdr);
  return s->ncomp;
}

bool EncodeStaged(ScanScratch* s, bool strip_metadata, std::string* out) {
  const JpegData& hdr = s->hdr;
  const int ncomps = s->ncomp;
  if (!WriteHeaderSegments(hdr, strip_metadata, out)) return false;
  HuffTable dc_tab[4], ac_tab[4];
  JpegHistogram dc_h[4], ac_h[4];
  for (int c = 0; c < ncomps; ++c) {
    dc_h[c] = s->dc_all[c];
    ac_h[c] = s->ac_all[c];
  }
  WriteHuffmanSegments(hdr, dc_h, ac_h, dc_tab, ac_tab, out);
  const int blocks = s->blocks;
  Partition(blocks, s);
  s->parts.resize(s->chunks);
  ParallelFor(s->chunks, [&](int ch) {
    RawBits& bw = s->parts[ch];
    bw.Clear();
    const int b0 = ch * s->per_chunk, b1 = std::min(blocks, b0 + s->per_chunk);
    coeff_t last_dc[4];
    for (int c = 0; c < ncomps; ++c)
      last_dc[c] = b0 > 0 ? s->zz[(static_cast<size_t>(c) * blocks + b0 - 1) * 64] : 0;
    for (int b = b0; b < b1; ++b)
      for (int c = 0; c < ncomps; ++c) {
        const size_t bi = static_cast<size_t>(c) * blocks + b;
        EncodeBlockMasked(bw, &s->zz[bi * 64], s->mask[bi], &last_dc[c], dc_tab[c], ac_tab[c]);
      }
  });
  EmitStuffed(s->parts, s->chunks, out);
  out->append("\xff\xd9", 2);
  return true;
}

int CoeffImageHistograms(const CoeffImage& img, ScanScratch* s, JpegHistogram dc[3],
                         JpegHistogram ac[3]) {
  JpegData none;
  const int n = StageCoeffImage(img, none, s);
  for (int c = 0; c < 3; ++c) {
    dc[c].Clear();
    ac[c].Clear();
    if (c < n) {
      dc[c] = s->dc_all[c];
      ac[c] = s->ac_all[c];
    }
  }
  return n;
}

bool WriteCoeffImageJpeg(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                         ScanScratch* s, std::string* out) {
  StageCoeffImage(img, meta, s);
  return EncodeStaged(s, strip_metadata, out);
}

bool WriteJpeg(const JpegData& jpg, bool strip_metadata, std::string* out) {
  // WriteJpeg (jpeg_data_writer.cc:540-553)
  if (!IsOneBlockPerMcu(jpg)) return WriteJpegParallel(jpg, strip_metadata, out);
  ScanScratch s;
  const int ncomp = static_cast<int>(jpg.components.size());
  StageAll(jpg.mcu_cols * jpg.mcu_rows, ncomp, &s, [&](int c, int b, coeff_t* dst) {
    const coeff_t* src = &jpg.components[c].coeffs[static_cast<size_t>(b) * 64];
    for (int k = 0; k < 64; ++k) dst[k] = src[kJPEGNaturalOrder[k]];
    return 0;
  });
  s.ncomp = ncomp;
  JpegHeaderOf(jpg, &s.hdr);
  return EncodeStaged(&s, strip_metadata, out);
}

bool WriteJpegReference(const JpegData& jpg, bool strip_metadata, std::string* out) {
  return WriteJpegSerial(jpg, strip_metadata, out);
}

bool WriteJpegPrologue(const JpegData& hdr, bool strip_metadata, JpegHistogram* dc_h,
                       JpegHistogram* ac_h, HuffCodeTable* dc_tab, HuffCodeTable* ac_tab,
                       std::string* out) {
  if (!WriteHeaderSegments(hdr, strip_metadata, out)) return false;
  WriteHuffmanSegments(hdr, dc_h, ac_h, dc_tab, ac_tab, out);
  return true;
}

void AppendStuffedScan(const uint8_t* bits_be, uint64_t nbits, std::string* out) {
  // pad the last byte with one bits, 0xff -> 0xff 0x00 (BitWriter::
  // JumpToByteBoundary / EmitByte, jpeg_bit_writer.h), then EOI
  const uint64_t full = nbits / 8;
  const int rem = static_cast<int>(nbits % 8);
  out->reserve(out->size() + full + full / 128 + 8);
  const uint8_t* p = bits_be;
  const uint8_t* end = bits_be + full;
  while (p < end) {
    const uint8_t* ff = static_cast<const uint8_t*>(std::memchr(p, 0xff, end - p));
    if (!ff) {
      out->append(reinterpret_cast<const char*>(p), end - p);
      break;
    }
    out->append(reinterpret_cast<const char*>(p), ff + 1 - p);
    out->push_back(0);
    p = ff + 1;
  }
  if (rem) {
    const uint8_t b = static_cast<uint8_t>(bits_be[full] | (0xff >> rem));
    out->push_back(static_cast<char>(b));
    if (b == 0xff) out->push_back(0);
  }
  out->append("\xff\xd9", 2);
}

}  // namespace gz
