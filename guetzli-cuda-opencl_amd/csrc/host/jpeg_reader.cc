// JPEG reader / decoder for the JPEG-input entry point (see
// jpeg_reader.h).  Clean-room: the marker grammar and entropy decoding are
// those of ITU-T T.81 (sequential Huffman: F.2.2; progressive: G.1.2), with
// the container conventions of guetzli::ReadJpeg that the rest of the
// search depends on -- APPn strings keep their marker byte and length
// (jpeg_data_reader.cc:395-407), COM strings their length (:410-421),
// quantization tables in order of appearance with natural-order values
// (:350-375) and components' quant_idx re-pointed at them (:888-906),
// coefficient arrays over the MCU-padded block grid (:140-152).
#include "host/jpeg_reader.h"

#include "host/image420.h"

#include <string.h>

#include <algorithm>

namespace gz {
namespace {

struct Huffman {
  bool defined = false;
  int maxcode[18];   // largest code of each length (-1: none)
  int valptr[17];    // index into vals of the first code of each length
  int mincode[17];
  uint8_t vals[256];
};

bool BuildHuffman(const uint8_t counts[17], const uint8_t* vals, int nvals, Huffman* h) {
  int code = 0, k = 0;
  for (int l = 1; l <= 16; ++l) {
    h->valptr[l] = k;
    h->mincode[l] = code;
    code += counts[l];
    k += counts[l];
    h->maxcode[l] = counts[l] ? code - 1 : -1;
    if (code > (1 << l)) return false;  // over-subscribed
    code <<= 1;
  }
  h->maxcode[17] = 0x7fffffff;
  if (k != nvals) return false;
  memcpy(h->vals, vals, nvals);
  h->defined = true;
  return true;
}

// Bits of one entropy-coded interval (stuffing already removed); zeros past
// its end, as a decoder sees at a marker.
struct Bits {
  const uint8_t* p = nullptr;
  size_t n = 0, pos = 0;
  uint32_t acc = 0;
  int nbits = 0;
  int Get(int k) {  // k <= 16
    while (nbits < k) {
      acc = (acc << 8) | (pos < n ? p[pos] : 0);
      ++pos;
      nbits += 8;
    }
    nbits -= k;
    return static_cast<int>((acc >> nbits) & ((1u << k) - 1));
  }
  int Decode(const Huffman& h) {
    int code = 0;
    for (int l = 1; l <= 16; ++l) {
      code = (code << 1) | Get(1);
      if (code <= h.maxcode[l]) return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
    return -1;
  }
};

inline int Extend(int v, int s) { return s == 0 ? 0 : (v < (1 << (s - 1)) ? v - (1 << s) + 1 : v); }

struct Reader {
  const uint8_t* d;
  size_t len, pos = 0;
  JpegData* jpg;
  std::string* err;
  Huffman dc[4], ac[4];
  int restart_interval = 0;
  bool progressive = false, found_sof = false;

  bool Fail(const char* m) {
    if (err) *err = m;
    return false;
  }
  bool Need(size_t k) { return pos + k <= len; }
  int U8() { return d[pos++]; }
  int U16() {
    const int v = (d[pos] << 8) | d[pos + 1];
    pos += 2;
    return v;
  }

  bool SOF(int marker) {
    if (found_sof) return Fail("duplicate SOF");
    found_sof = true;
    progressive = marker == 0xc2;
    if (!Need(2)) return Fail("truncated SOF");
    const size_t start = pos, mlen = U16();
    if (mlen < 8 || !Need(mlen - 2)) return Fail("bad SOF length");
    if (U8() != 8) return Fail("only 8-bit precision is supported");
    jpg->height = U16();
    jpg->width = U16();
    const int nc = U8();
    if (jpg->width <= 0 || jpg->height <= 0) return Fail("bad image size");
    if (nc < 1 || nc > 4 || mlen != 8 + 3 * static_cast<size_t>(nc)) return Fail("bad component count");
    jpg->components.assign(nc, JpegComponent());
    jpg->max_h_samp_factor = jpg->max_v_samp_factor = 1;
    for (int i = 0; i < nc; ++i) {
      JpegComponent& c = jpg->components[i];
      c.id = U8();
      for (int j = 0; j < i; ++j)
        if (jpg->components[j].id == c.id) return Fail("duplicate component id");
      const int hv = U8();
      c.h_samp_factor = hv >> 4;
      c.v_samp_factor = hv & 15;
      if (c.h_samp_factor < 1 || c.h_samp_factor > 15 || c.v_samp_factor < 1 || c.v_samp_factor > 15)
        return Fail("bad sampling factor");
      c.quant_idx = U8();
      jpg->max_h_samp_factor = std::max(jpg->max_h_samp_factor, c.h_samp_factor);
      jpg->max_v_samp_factor = std::max(jpg->max_v_samp_factor, c.v_samp_factor);
    }
    jpg->mcu_cols = (jpg->width + 8 * jpg->max_h_samp_factor - 1) / (8 * jpg->max_h_samp_factor);
    jpg->mcu_rows = (jpg->height + 8 * jpg->max_v_samp_factor - 1) / (8 * jpg->max_v_samp_factor);
    for (JpegComponent& c : jpg->components) {
      if (jpg->max_h_samp_factor % c.h_samp_factor || jpg->max_v_samp_factor % c.v_samp_factor)
        return Fail("non-integral subsampling ratio");
      c.width_in_blocks = jpg->mcu_cols * c.h_samp_factor;
      c.height_in_blocks = jpg->mcu_rows * c.v_samp_factor;
      const uint64_t nb = static_cast<uint64_t>(c.width_in_blocks) * c.height_in_blocks;
      // JPEG_IMAGE_TOO_LARGE above 2M blocks per component, as the reference
      // (jpeg_data_reader.cc:151-158): checked before any allocation
      if (nb > (1ull << 21)) return Fail("image too large");
      c.coeffs.assign(nb * 64, 0);
    }
    return pos == start + mlen || Fail("bad SOF length");
  }

  bool DHT() {
    if (!Need(2)) return Fail("truncated DHT");
    const size_t start = pos, mlen = U16();
    if (mlen < 2 || !Need(mlen - 2)) return Fail("bad DHT length");
    while (pos < start + mlen) {
      if (!Need(17)) return Fail("truncated DHT");
      const int tc = U8();
      const int cls = tc >> 4, id = tc & 15;
      if (cls > 1 || id > 3) return Fail("bad Huffman table class / index");
      uint8_t counts[17] = {0};
      int total = 0;
      for (int l = 1; l <= 16; ++l) total += counts[l] = static_cast<uint8_t>(U8());
      if (total == 0 || total > 256 || pos + total > start + mlen) return Fail("bad Huffman table");
      if (!BuildHuffman(counts, d + pos, total, cls ? &ac[id] : &dc[id])) return Fail("bad Huffman code");
      pos += total;
    }
    return pos == start + mlen || Fail("bad DHT length");
  }

  bool DQT() {
    if (!Need(2)) return Fail("truncated DQT");
    const size_t start = pos, mlen = U16();
    if (mlen < 2 || !Need(mlen - 2)) return Fail("bad DQT length");
    while (pos < start + mlen) {
      const int pq = U8();
      QuantTable t;
      t.index = pq & 15;
      t.precision = pq >> 4;
      if (t.index > 3 || t.precision > 1) return Fail("bad quantization table index / precision");
      if (pos + (t.precision ? 128 : 64) > start + mlen) return Fail("truncated DQT");
      for (int k = 0; k < 64; ++k) {
        const int v = t.precision ? U16() : U8();
        if (v < 1) return Fail("zero quantization value");
        t.values[kJPEGNaturalOrder[k]] = v;
      }
      jpg->quant.push_back(t);
    }
    return pos == start + mlen || Fail("bad DQT length");
  }

  bool DRI() {
    if (!Need(4)) return Fail("truncated DRI");
    if (U16() != 4) return Fail("bad DRI length");
    restart_interval = U16();
    return true;
  }

  bool APP(int marker) {
    if (!Need(2)) return Fail("truncated APP");
    const size_t mlen = (d[pos] << 8) | d[pos + 1];
    if (mlen < 2 || !Need(mlen)) return Fail("bad APP length");
    // marker byte + length + payload, as guetzli stores it
    jpg->app_data.emplace_back(reinterpret_cast<const char*>(d + pos - 1), mlen + 1);
    (void)marker;
    pos += mlen;
    return true;
  }

  bool COM() {
    if (!Need(2)) return Fail("truncated COM");
    const size_t mlen = (d[pos] << 8) | d[pos + 1];
    if (mlen < 2 || !Need(mlen)) return Fail("bad COM length");
    jpg->com_data.emplace_back(reinterpret_cast<const char*>(d + pos), mlen);
    pos += mlen;
    return true;
  }

  bool Skip() {
    if (!Need(2)) return Fail("truncated marker segment");
    const size_t mlen = (d[pos] << 8) | d[pos + 1];
    if (mlen < 2 || !Need(mlen)) return Fail("bad marker length");
    pos += mlen;
    return true;
  }

  // The entropy-coded data after an SOS header, split at RSTn markers and
  // de-stuffed; pos is left at the marker that ends the scan.
  void ScanIntervals(std::vector<std::vector<uint8_t>>* iv) {
    iv->assign(1, std::vector<uint8_t>());
    while (pos < len) {
      const uint8_t b = d[pos];
      if (b != 0xff) {
        iv->back().push_back(b);
        ++pos;
        continue;
      }
      if (pos + 1 >= len) break;
      const uint8_t m = d[pos + 1];
      if (m == 0x00) {
        iv->back().push_back(0xff);
        pos += 2;
      } else if (m >= 0xd0 && m <= 0xd7) {
        iv->emplace_back();
        pos += 2;
      } else if (m == 0xff) {
        ++pos;  // fill byte
      } else {
        break;  // a marker: end of the scan
      }
    }
  }

  bool SOS() {
    if (!found_sof) return Fail("SOS before SOF");
    if (!Need(2)) return Fail("truncated SOS");
    const size_t start = pos, mlen = U16();
    if (!Need(mlen - 2) || mlen < 6) return Fail("bad SOS length");
    const int ns = U8();
    if (ns < 1 || ns > 4 || mlen != 6 + 2 * static_cast<size_t>(ns)) return Fail("bad SOS component count");
    int ci[4], td[4], ta[4];
    for (int i = 0; i < ns; ++i) {
      const int id = U8(), t = U8();
      ci[i] = -1;
      for (size_t j = 0; j < jpg->components.size(); ++j)
        if (jpg->components[j].id == id) ci[i] = static_cast<int>(j);
      if (ci[i] < 0) return Fail("SOS references an unknown component");
      for (int j = 0; j < i; ++j)
        if (ci[j] == ci[i]) return Fail("duplicate component in SOS");
      td[i] = t >> 4;
      ta[i] = t & 15;
      if (td[i] > 3 || ta[i] > 3) return Fail("bad Huffman table selector");
    }
    const int ss = U8(), se = U8(), a = U8();
    const int ah = a >> 4, al = a & 15;
    if (pos != start + mlen) return Fail("bad SOS length");
    if (progressive) {
      if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || al > 13 || ah > 13)
        return Fail("bad progressive scan parameters");
    } else if (ss != 0 || se != 63 || ah != 0 || al != 0) {
      return Fail("bad sequential scan parameters");
    }
    const bool dc_scan = ss == 0;
    for (int i = 0; i < ns; ++i) {
      if (dc_scan && ah == 0 && !dc[td[i]].defined) return Fail("undefined DC Huffman table");
      if (!dc_scan && !ac[ta[i]].defined) return Fail("undefined AC Huffman table");
      if (!progressive && !ac[ta[i]].defined) return Fail("undefined AC Huffman table");
    }
    std::vector<std::vector<uint8_t>> iv;
    ScanIntervals(&iv);

    // units: MCUs of the interleaved scan, or blocks of the one component
    int units_w, units_h;
    if (ns == 1) {
      const JpegComponent& c = jpg->components[ci[0]];
      const int cw = (jpg->width * c.h_samp_factor + jpg->max_h_samp_factor - 1) / jpg->max_h_samp_factor;
      const int ch = (jpg->height * c.v_samp_factor + jpg->max_v_samp_factor - 1) / jpg->max_v_samp_factor;
      units_w = (cw + 7) / 8;
      units_h = (ch + 7) / 8;
    } else {
      units_w = jpg->mcu_cols;
      units_h = jpg->mcu_rows;
    }
    const long units = static_cast<long>(units_w) * units_h;
    int pred[4] = {0, 0, 0, 0};
    int eobrun = 0;
    size_t seg = 0;
    Bits bits;
    bits.p = iv[0].data();
    bits.n = iv[0].size();
    for (long u = 0; u < units; ++u) {
      if (restart_interval > 0 && u > 0 && u % restart_interval == 0) {
        if (++seg >= iv.size()) return Fail("missing restart marker");
        bits = Bits();
        bits.p = iv[seg].data();
        bits.n = iv[seg].size();
        pred[0] = pred[1] = pred[2] = pred[3] = 0;
        eobrun = 0;
      }
      const int ux = static_cast<int>(u % units_w), uy = static_cast<int>(u / units_w);
      for (int i = 0; i < ns; ++i) {
        JpegComponent& c = jpg->components[ci[i]];
        const int nh = ns == 1 ? 1 : c.h_samp_factor, nv = ns == 1 ? 1 : c.v_samp_factor;
        for (int v = 0; v < nv; ++v)
          for (int hh = 0; hh < nh; ++hh) {
            const int bx = ux * nh + hh, by = uy * nv + v;
            coeff_t* blk = &c.coeffs[(static_cast<size_t>(by) * c.width_in_blocks + bx) * 64];
            bool ok;
            if (!progressive)
              ok = Sequential(&bits, dc[td[i]], ac[ta[i]], &pred[i], blk);
            else if (dc_scan)
              ok = ah == 0 ? DcFirst(&bits, dc[td[i]], al, &pred[i], blk) : DcRefine(&bits, al, blk);
            else
              ok = ah == 0 ? AcFirst(&bits, ac[ta[i]], ss, se, al, &eobrun, blk)
                           : AcRefine(&bits, ac[ta[i]], ss, se, al, &eobrun, blk);
            if (!ok) return Fail("corrupt entropy-coded data");
          }
      }
    }
    return true;
  }

  static bool Sequential(Bits* b, const Huffman& dch, const Huffman& ach, int* pred, coeff_t* blk) {
    const int t = b->Decode(dch);
    if (t < 0 || t > 11) return false;
    *pred += Extend(t ? b->Get(t) : 0, t);
    blk[0] = static_cast<coeff_t>(*pred);
    for (int k = 1; k <= 63; ++k) {
      const int rs = b->Decode(ach);
      if (rs < 0) return false;
      const int r = rs >> 4, s = rs & 15;
      if (s == 0) {
        if (r != 15) break;
        k += 15;
        continue;
      }
      k += r;
      if (k > 63) return false;
      blk[kJPEGNaturalOrder[k]] = static_cast<coeff_t>(Extend(b->Get(s), s));
    }
    return true;
  }
  static bool DcFirst(Bits* b, const Huffman& dch, int al, int* pred, coeff_t* blk) {
    const int t = b->Decode(dch);
    if (t < 0 || t > 11) return false;
    *pred += Extend(t ? b->Get(t) : 0, t);
    blk[0] = static_cast<coeff_t>(*pred * (1 << al));
    return true;
  }
  static bool DcRefine(Bits* b, int al, coeff_t* blk) {
    if (b->Get(1)) blk[0] = static_cast<coeff_t>(blk[0] | (1 << al));
    return true;
  }
  static bool AcFirst(Bits* b, const Huffman& ach, int ss, int se, int al, int* eobrun, coeff_t* blk) {
    if (*eobrun > 0) {
      --*eobrun;
      return true;
    }
    for (int k = ss; k <= se; ++k) {
      const int rs = b->Decode(ach);
      if (rs < 0) return false;
      const int r = rs >> 4, s = rs & 15;
      if (s == 0) {
        if (r < 15) {
          *eobrun = (1 << r) - 1;
          if (r) *eobrun += b->Get(r);
          break;
        }
        k += 15;
        continue;
      }
      k += r;
      if (k > se) return false;
      blk[kJPEGNaturalOrder[k]] = static_cast<coeff_t>(Extend(b->Get(s), s) * (1 << al));
    }
    return true;
  }
  // Successive-approximation refinement of AC coefficients (G.1.2.3): a
  // correction bit for every already-nonzero coefficient passed over, and
  // new coefficients of magnitude 1 << al placed after r zero-history ones.
  static bool AcRefine(Bits* b, const Huffman& ach, int ss, int se, int al, int* eobrun, coeff_t* blk) {
    const int p1 = 1 << al, m1 = -(1 << al);
    auto refine = [&](coeff_t* c) {
      if (b->Get(1) && (*c & p1) == 0) *c = static_cast<coeff_t>(*c >= 0 ? *c + p1 : *c + m1);
    };
    int k = ss;
    if (*eobrun == 0) {
      for (; k <= se; ++k) {
        const int rs = b->Decode(ach);
        if (rs < 0) return false;
        int r = rs >> 4, s = rs & 15;
        int val = 0;
        if (s) {
          if (s != 1) return false;
          val = b->Get(1) ? p1 : m1;
        } else if (r != 15) {
          *eobrun = 1 << r;
          if (r) *eobrun += b->Get(r);
          break;
        }
        while (k <= se) {
          coeff_t* c = &blk[kJPEGNaturalOrder[k]];
          if (*c != 0) {
            refine(c);
          } else {
            if (r == 0) break;
            --r;
          }
          ++k;
        }
        if (val) {
          if (k > se) return false;
          blk[kJPEGNaturalOrder[k]] = static_cast<coeff_t>(val);
        }
      }
    }
    if (*eobrun > 0) {
      for (; k <= se; ++k) {
        coeff_t* c = &blk[kJPEGNaturalOrder[k]];
        if (*c != 0) refine(c);
      }
      --*eobrun;
    }
    return true;
  }

  bool Run() {
    if (len < 2 || d[0] != 0xff || d[1] != 0xd8) return Fail("not a JPEG (no SOI)");
    pos = 2;
    for (;;) {
      // next marker (fill bytes allowed)
      if (!Need(2)) return Fail("truncated file (no EOI)");
      if (d[pos] != 0xff) return Fail("marker expected");
      while (pos < len && d[pos] == 0xff) ++pos;
      if (pos >= len) return Fail("truncated file (no EOI)");
      const int m = d[pos++];
      bool ok;
      if (m == 0xd9) break;  // EOI
      if (m == 0xc0 || m == 0xc1 || m == 0xc2) ok = SOF(m);
      else if (m == 0xc4) ok = DHT();
      else if (m == 0xdb) ok = DQT();
      else if (m == 0xdd) ok = DRI();
      else if (m == 0xda) ok = SOS();
      else if (m >= 0xe0 && m <= 0xef) ok = APP(m);
      else if (m == 0xfe) ok = COM();
      else if ((m >= 0xc3 && m <= 0xcf) || m == 0xdc || m == 0xde || m == 0xdf)
        return Fail("unsupported JPEG process (arithmetic, lossless, hierarchical or DNL)");
      else if (m >= 0xd0 && m <= 0xd7)
        ok = true;  // stray restart marker
      else
        ok = Skip();
      if (!ok) return false;
    }
    if (!found_sof) return Fail("missing SOF marker");
    // FixupIndexes: quant_idx -> position of the first table with that index
    for (JpegComponent& c : jpg->components) {
      int found = -1;
      for (size_t j = 0; j < jpg->quant.size() && found < 0; ++j)
        if (jpg->quant[j].index == c.quant_idx) found = static_cast<int>(j);
      if (found < 0) return Fail("quantization table not found");
      c.quant_idx = found;
    }
    return true;
  }
};

inline int Clamp255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
inline int Fix16(double x) { return static_cast<int>(x * 65536.0 + 0.5); }

}  // namespace

bool ReadJpeg(const uint8_t* data, size_t len, JpegData* jpg, std::string* err) {
  *jpg = JpegData();
  Reader r{data, len, 0, jpg, err};
  return r.Run();
}

bool JpegIs444(const JpegData& jpg) {
  if (jpg.components.size() != 3 || jpg.max_h_samp_factor != 1 || jpg.max_v_samp_factor != 1) return false;
  for (const JpegComponent& c : jpg.components)
    if (c.h_samp_factor != 1 || c.v_samp_factor != 1) return false;
  return true;
}

bool JpegIs420(const JpegData& jpg) {
  if (jpg.components.size() != 3 || jpg.max_h_samp_factor != 2 || jpg.max_v_samp_factor != 2) return false;
  const JpegComponent* c = jpg.components.data();
  return c[0].h_samp_factor == 2 && c[0].v_samp_factor == 2 && c[1].h_samp_factor == 1 &&
         c[1].v_samp_factor == 1 && c[2].h_samp_factor == 1 && c[2].v_samp_factor == 1;
}

bool HasYCbCrColorSpace(const JpegData& jpg) {
  bool adobe = false;
  uint8_t transform = 0;
  for (const std::string& app : jpg.app_data) {
    if (static_cast<uint8_t>(app[0]) == 0xe0) return true;
    if (static_cast<uint8_t>(app[0]) == 0xee && app.size() >= 15) {
      adobe = true;
      transform = static_cast<uint8_t>(app[14]);
    }
  }
  if (adobe) return transform != 0;
  if (jpg.components.size() < 3) return false;
  return jpg.components[0].id != 'R' || jpg.components[1].id != 'G' || jpg.components[2].id != 'B';
}

bool CheckJpegSanity(const JpegData& jpg) {
  for (const JpegComponent& c : jpg.components) {
    const int* q = jpg.quant[c.quant_idx].values;
    for (size_t i = 0; i < c.coeffs.size(); ++i)
      if (std::abs(static_cast<int64_t>(c.coeffs[i]) * q[i % 64]) > (1 << 12)) return false;
  }
  return true;
}

bool DecodeJpegToRGB(const JpegData& jpg, std::vector<uint8_t>* rgb) {
  if (!(JpegIs444(jpg) || JpegIs420(jpg)) || !HasYCbCrColorSpace(jpg)) return false;
  const int w = jpg.width, h = jpg.height;
  SubsampledPlane plane[3];
  for (int c = 0; c < 3; ++c) {
    const JpegComponent& comp = jpg.components[c];
    const int* q = jpg.quant[comp.quant_idx].values;
    SubsampledPlane& P = plane[c];
    // (4:4:4 or 4:2:0: both directions share the factor)
    P.Reset(w, h, jpg.max_h_samp_factor / comp.h_samp_factor);
    // CopyFromJpegData: blocks in raster order (the factor-2 update reads the
    // pixels of blocks already set), coeff * quant stored as coeff_t
    for (int by = 0; by < P.hib; ++by)
      for (int bx = 0; bx < P.wib; ++bx) {
        const coeff_t* src = &comp.coeffs[(static_cast<size_t>(by) * comp.width_in_blocks + bx) * 64];
        coeff_t deq[64];
        for (int k = 0; k < 64; ++k) deq[k] = static_cast<coeff_t>(src[k] * q[k]);
        uint8_t idct[64];
        BlockIdctBytes(deq, idct);
        P.Update(bx, by, idct);
      }
  }
  // ToSRGB: ToPixels' rounding (output_image.cc:68-98), then
  // ColorTransformYCbCrToRGB with libjpeg's build_ycc_rgb_table
  // (color_transform.h:211-218)
  int cr_r[256], cb_b[256], cr_g[256], cb_g[256];
  for (int i = 0; i < 256; ++i) {
    const int x = i - 128;
    cr_r[i] = (Fix16(1.40200) * x + 32768) >> 16;
    cb_b[i] = (Fix16(1.77200) * x + 32768) >> 16;
    cr_g[i] = -Fix16(0.71414) * x;
    cb_g[i] = -Fix16(0.34414) * x + 32768;
  }
  rgb->resize(static_cast<size_t>(3) * w * h);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const size_t p = static_cast<size_t>(y) * w + x;
      int v[3];
      for (int c = 0; c < 3; ++c) v[c] = PixelByte(plane[c].px[p], x);
      (*rgb)[3 * p] = static_cast<uint8_t>(Clamp255(v[0] + cr_r[v[2]]));
      (*rgb)[3 * p + 1] = static_cast<uint8_t>(Clamp255(v[0] + ((cr_g[v[2]] + cb_g[v[1]]) >> 16)));
      (*rgb)[3 * p + 2] = static_cast<uint8_t>(Clamp255(v[0] + cb_b[v[1]]));
    }
  return true;
}

}  // namespace gz
