#include "host/jpeg_writer.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

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

struct HuffTable {
  uint8_t depth[256];
  int code[256];
};

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

void HuffmanCodeLengths(const uint32_t* data, int length, int max_depth, uint8_t* depth) {
  // Huffman tree with iterative count flattening until it fits max_depth
  // (CreateHuffmanTree, entropy_encode.cc:65-145).  Leaves sorted by
  // (count asc, symbol desc): a total order, so any correct sort agrees.
  std::vector<TreeNode> tree(2 * length + 1);
  for (uint32_t count_limit = 1;; count_limit *= 2) {
    int n = 0;
    for (int i = length - 1; i >= 0; --i) {
      if (data[i]) {
        tree[n++] = TreeNode{std::max(data[i], count_limit), -1, static_cast<int16_t>(i)};
      }
    }
    if (n == 1) {
      depth[tree[0].right_or_value] = 1;
      break;
    }
    std::sort(tree.begin(), tree.begin() + n, [](const TreeNode& a, const TreeNode& b) {
      return a.total != b.total ? a.total < b.total : a.right_or_value > b.right_or_value;
    });
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
      tree[parent + 1] = sentinel;
    }
    if (AssignDepths(2 * n - 1, tree.data(), depth, max_depth)) break;
  }
}

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

bool WriteJpeg(const JpegData& jpg, bool strip_metadata, std::string* out) {
  const int ncomps = static_cast<int>(jpg.components.size());
  if (ncomps < 1 || ncomps > 4) return false;
  // SOI + metadata (EncodeMetadata, jpeg_data_writer.cc:53-75)
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
  // DQT (jpeg_data_writer.cc:77-100)
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
  // SOF1 (jpeg_data_writer.cc:102-128)
  {
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
  }
  // DHT + SOS (BuildAndEncodeHuffmanCodes, jpeg_data_writer.cc:361-445)
  std::vector<HuffTable> dc_tab(ncomps), ac_tab(ncomps);
  {
    std::vector<JpegHistogram> histo(ncomps);
    BuildDCHistograms(jpg, histo.data());
    size_t num_dc = ncomps;
    int dc_idx[4], ac_idx[4];
    std::vector<uint8_t> depths(ncomps * JpegHistogram::kSize);
    ClusterHistograms(histo.data(), &num_dc, dc_idx, depths.data());
    histo.resize(num_dc + ncomps);
    depths.resize((num_dc + ncomps) * JpegHistogram::kSize);
    BuildACHistograms(jpg, &histo[num_dc]);
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
  // entropy-coded scan (EncodeScan / EncodeDCTBlockSequential, :447-538)
  {
    BitSink bw(out);
    coeff_t last_dc[4] = {0, 0, 0, 0};
    for (int my = 0; my < jpg.mcu_rows; ++my)
      for (int mx = 0; mx < jpg.mcu_cols; ++mx)
        for (int ci = 0; ci < ncomps; ++ci) {
          const JpegComponent& c = jpg.components[ci];
          const HuffTable& dct = dc_tab[ci];
          const HuffTable& act = ac_tab[ci];
          for (int iy = 0; iy < c.v_samp_factor; ++iy)
            for (int ix = 0; ix < c.h_samp_factor; ++ix) {
              const int bidx = (my * c.v_samp_factor + iy) * c.width_in_blocks + mx * c.h_samp_factor + ix;
              const coeff_t* co = &c.coeffs[static_cast<size_t>(bidx) << 6];
              coeff_t diff = static_cast<coeff_t>(co[0] - last_dc[ci]);
              last_dc[ci] = co[0];
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
                coeff_t v = co[kJPEGNaturalOrder[k]];
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
        }
    bw.Flush();
  }
  out->append("\xff\xd9", 2);
  return true;
}

}  // namespace gz
