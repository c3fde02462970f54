// PNG reader mirroring the reference CLI's ReadPNG (guetzli/guetzli.cc:
// 51-156).  See png_reader.h.  The libpng transforms it asks for are
// restated here: PACKING + EXPAND (palette -> RGB, gray below 8 bits ->
// 8 bits, tRNS -> an alpha channel) + STRIP_16 (keep the high byte), then
// ReadPNG's own step: gray / gray+alpha / RGB / RGBA -> RGB with alpha
// blended on black, (v * a + 128) / 255.
#include "host/png_reader.h"

#include <string.h>
#include <zlib.h>

#include <algorithm>

namespace gz {

namespace {

uint32_t Be32(const uint8_t* p) {
  return (static_cast<uint32_t>(p[0]) << 24) | (static_cast<uint32_t>(p[1]) << 16) |
         (static_cast<uint32_t>(p[2]) << 8) | p[3];
}

struct Header {
  uint32_t w = 0, h = 0;
  int depth = 0, color = 0, interlace = 0;
  int channels = 0;  // samples per pixel in the file
};

constexpr int kAdam7[7][4] = {  // x0, y0, dx, dy
    {0, 0, 8, 8}, {4, 0, 8, 8}, {0, 4, 4, 8}, {2, 0, 4, 4}, {0, 2, 2, 4}, {1, 0, 2, 2}, {0, 1, 1, 2}};

bool Fail(std::string* err, const char* msg) {
  if (err) *err = msg;
  return false;
}

// Inflates the concatenated IDAT data into exactly `need` bytes, then runs
// the stream to its end (its Adler-32 is checked, as libpng does); data past
// the end of the image is tolerated (libpng: a warning).
bool Inflate(const std::vector<uint8_t>& z, size_t need, std::vector<uint8_t>* out) {
  out->assign(need, 0);
  z_stream s;
  memset(&s, 0, sizeof(s));
  if (inflateInit(&s) != Z_OK) return false;
  s.next_in = const_cast<Bytef*>(z.data());
  s.avail_in = static_cast<uInt>(z.size());
  size_t done = 0;
  int rc = Z_OK;
  while (done < need) {
    const size_t chunk = std::min<size_t>(need - done, 1u << 30);
    s.next_out = out->data() + done;
    s.avail_out = static_cast<uInt>(chunk);
    rc = inflate(&s, Z_NO_FLUSH);
    done += chunk - s.avail_out;
    if (rc == Z_STREAM_END) break;
    if (rc != Z_OK) {
      inflateEnd(&s);
      return false;
    }
    if (s.avail_in == 0 && s.avail_out != 0) {  // input exhausted: not enough image data
      inflateEnd(&s);
      return false;
    }
  }
  if (done < need) {
    inflateEnd(&s);
    return false;
  }
  uint8_t scratch[4096];
  while (rc != Z_STREAM_END) {
    s.next_out = scratch;
    s.avail_out = sizeof(scratch);
    rc = inflate(&s, Z_NO_FLUSH);
    if (rc != Z_OK && rc != Z_STREAM_END) {
      inflateEnd(&s);
      return false;
    }
    if (rc == Z_OK && s.avail_in == 0 && s.avail_out != 0) {
      inflateEnd(&s);
      return false;  // the stream ends early: its end (and checksum) never arrives
    }
  }
  inflateEnd(&s);
  return true;
}

// Reverses one row's filter in place (PNG filter method 0).
bool Unfilter(int type, uint8_t* row, const uint8_t* prev, size_t n, size_t bpp) {
  switch (type) {
    case 0:
      return true;
    case 1:
      for (size_t i = bpp; i < n; ++i) row[i] = static_cast<uint8_t>(row[i] + row[i - bpp]);
      return true;
    case 2:
      if (prev)
        for (size_t i = 0; i < n; ++i) row[i] = static_cast<uint8_t>(row[i] + prev[i]);
      return true;
    case 3:
      for (size_t i = 0; i < n; ++i) {
        const int a = i >= bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
        row[i] = static_cast<uint8_t>(row[i] + ((a + b) >> 1));
      }
      return true;
    case 4:
      for (size_t i = 0; i < n; ++i) {
        const int a = i >= bpp ? row[i - bpp] : 0, b = prev ? prev[i] : 0;
        const int c = prev && i >= bpp ? prev[i - bpp] : 0;
        const int p = a + b - c;
        const int pa = abs(p - a), pb = abs(p - b), pc = abs(p - c);
        const int pred = (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
        row[i] = static_cast<uint8_t>(row[i] + pred);
      }
      return true;
    default:
      return false;
  }
}

// Sample i of a row packed at `depth` bits.
inline uint32_t Sample(const uint8_t* row, size_t i, int depth) {
  switch (depth) {
    case 16: return (static_cast<uint32_t>(row[2 * i]) << 8) | row[2 * i + 1];
    case 8: return row[i];
    default: {
      const size_t bit = i * depth;
      return (row[bit >> 3] >> (8 - depth - (bit & 7))) & ((1u << depth) - 1);
    }
  }
}

inline uint8_t BlendOnBlack(uint8_t v, uint8_t a) {  // guetzli.cc:47-49
  return static_cast<uint8_t>((static_cast<int>(v) * static_cast<int>(a) + 128) / 255);
}

}  // namespace

bool ReadPng(const uint8_t* data, size_t size, int* width, int* height, std::vector<uint8_t>* rgb,
             std::string* err) {
  static const uint8_t kSig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
  if (!data || size < 8 || memcmp(data, kSig, 8) != 0) return Fail(err, "not a PNG file");
  Header hd;
  bool have_ihdr = false, have_plte = false, seen_idat = false, ended = false;
  std::vector<uint8_t> plte;   // RGB triplets
  std::vector<uint8_t> trns;   // raw tRNS payload
  std::vector<uint8_t> z;      // concatenated IDAT
  size_t pos = 8;
  while (!ended) {
    if (size - pos < 12) return Fail(err, "truncated PNG");
    const uint32_t len = Be32(data + pos);
    if (len > 0x7fffffffu || size - pos - 12 < len) return Fail(err, "truncated PNG chunk");
    const uint8_t* type = data + pos + 4;
    const uint8_t* body = data + pos + 8;
    const bool critical = !(type[0] & 0x20);
    const uint32_t crc = Be32(body + len);
    const bool crc_ok = (crc32(crc32(0L, Z_NULL, 0), type, 4 + len) & 0xffffffffu) == crc;
    pos += 12 + static_cast<size_t>(len);
    if (!crc_ok) {
      if (critical) return Fail(err, "PNG chunk CRC error");
      continue;  // ancillary: dropped (libpng's default)
    }
    if (!memcmp(type, "IHDR", 4)) {
      if (have_ihdr || len != 13) return Fail(err, "bad IHDR");
      hd.w = Be32(body);
      hd.h = Be32(body + 4);
      hd.depth = body[8];
      hd.color = body[9];
      hd.interlace = body[12];
      if (body[10] != 0 || body[11] != 0 || hd.interlace > 1) return Fail(err, "unsupported PNG header");
      // libpng's default user limits: at most 1,000,000 columns and rows
      if (hd.w == 0 || hd.h == 0 || hd.w > 1000000u || hd.h > 1000000u)
        return Fail(err, "PNG image size out of range");
      const int d = hd.depth;
      switch (hd.color) {
        case 0: hd.channels = 1; if (d != 1 && d != 2 && d != 4 && d != 8 && d != 16) return Fail(err, "bad bit depth"); break;
        case 2: hd.channels = 3; if (d != 8 && d != 16) return Fail(err, "bad bit depth"); break;
        case 3: hd.channels = 1; if (d != 1 && d != 2 && d != 4 && d != 8) return Fail(err, "bad bit depth"); break;
        case 4: hd.channels = 2; if (d != 8 && d != 16) return Fail(err, "bad bit depth"); break;
        case 6: hd.channels = 4; if (d != 8 && d != 16) return Fail(err, "bad bit depth"); break;
        default: return Fail(err, "bad color type");
      }
      have_ihdr = true;
    } else if (!have_ihdr) {
      return Fail(err, "PNG chunk before IHDR");
    } else if (!memcmp(type, "PLTE", 4)) {
      if (hd.color == 0 || hd.color == 4) continue;  // ignored in gray images
      if (have_plte || seen_idat || len % 3 != 0 || len == 0 || len > 768) {
        if (hd.color == 3) return Fail(err, "bad PLTE");
        continue;  // a suggested palette of an RGB image: not used
      }
      plte.assign(body, body + len);
      have_plte = true;
    } else if (!memcmp(type, "tRNS", 4)) {
      if (seen_idat) continue;
      if ((hd.color == 0 && len == 2) || (hd.color == 2 && len == 6) ||
          (hd.color == 3 && have_plte && len >= 1 && len <= plte.size() / 3))
        trns.assign(body, body + len);
      // (other combinations: libpng warns and ignores the chunk)
    } else if (!memcmp(type, "IDAT", 4)) {
      if (hd.color == 3 && !have_plte) return Fail(err, "PNG palette missing");
      seen_idat = true;
      z.insert(z.end(), body, body + len);
    } else if (!memcmp(type, "IEND", 4)) {
      ended = true;
    } else if (critical) {
      return Fail(err, "unknown critical PNG chunk");
    }
  }
  if (!have_ihdr || !seen_idat) return Fail(err, "PNG without image data");
  const size_t w = hd.w, h = hd.h;
  const int ch = hd.channels, depth = hd.depth;
  const size_t bpp = std::max<size_t>(1, static_cast<size_t>(ch) * depth / 8);
  struct Pass {
    size_t x0, y0, dx, dy, pw, ph, stride;
  };
  std::vector<Pass> passes;
  for (int p = 0; p < (hd.interlace ? 7 : 1); ++p) {
    Pass ps;
    if (hd.interlace) {
      ps.x0 = kAdam7[p][0]; ps.y0 = kAdam7[p][1]; ps.dx = kAdam7[p][2]; ps.dy = kAdam7[p][3];
    } else {
      ps.x0 = ps.y0 = 0; ps.dx = ps.dy = 1;
    }
    ps.pw = w > ps.x0 ? (w - ps.x0 + ps.dx - 1) / ps.dx : 0;
    ps.ph = h > ps.y0 ? (h - ps.y0 + ps.dy - 1) / ps.dy : 0;
    ps.stride = (ps.pw * ch * depth + 7) / 8;
    if (ps.pw && ps.ph) passes.push_back(ps);
  }
  size_t need = 0;
  for (const Pass& ps : passes) need += ps.ph * (1 + ps.stride);
  // deflate expands at most 1032:1 (258-byte matches coded in 2 bits), so a
  // header promising more than that cannot be backed by this IDAT data:
  // libpng ends such a file with "not enough image data"; failing before
  // allocating keeps a tiny file from asking for terabytes
  if (need / 1032 > z.size() + 64) return Fail(err, "PNG image data error");
  std::vector<uint8_t> raw;
  if (!Inflate(z, need, &raw)) return Fail(err, "PNG image data error");
  // samples after EXPAND / STRIP_16: out_ch 8-bit values per pixel
  const bool palette = hd.color == 3;
  const bool alpha_from_trns = !trns.empty();
  const int out_ch = palette ? (alpha_from_trns ? 4 : 3)
                             : ch + ((hd.color == 0 || hd.color == 2) && alpha_from_trns ? 1 : 0);
  std::vector<uint8_t> px(w * h * out_ch);
  uint32_t key[3] = {0, 0, 0};
  if (alpha_from_trns && (hd.color == 0 || hd.color == 2)) {
    for (int c = 0; c < ch; ++c) {
      uint32_t v = (static_cast<uint32_t>(trns[2 * c]) << 8) | trns[2 * c + 1];
      v = depth == 16 ? v : (depth == 8 ? (v & 0xffu) : (v & ((1u << depth) - 1)));
      key[c] = v;
    }
  }
  size_t off = 0;
  for (const Pass& ps : passes) {
    const uint8_t* prev = nullptr;
    for (size_t r = 0; r < ps.ph; ++r) {
      uint8_t* row = raw.data() + off + 1;
      if (!Unfilter(raw[off], row, prev, ps.stride, bpp)) return Fail(err, "bad PNG row filter");
      const size_t y = ps.y0 + r * ps.dy;
      for (size_t i = 0; i < ps.pw; ++i) {
        const size_t x = ps.x0 + i * ps.dx;
        uint8_t* o = px.data() + (y * w + x) * out_ch;
        if (palette) {
          const uint32_t idx = Sample(row, i, depth);
          const bool in = 3 * idx + 2 < plte.size();
          o[0] = in ? plte[3 * idx] : 0;
          o[1] = in ? plte[3 * idx + 1] : 0;
          o[2] = in ? plte[3 * idx + 2] : 0;
          if (alpha_from_trns) o[3] = idx < trns.size() ? trns[idx] : 255;
          continue;
        }
        bool is_key = alpha_from_trns;
        for (int c = 0; c < ch; ++c) {
          const uint32_t v = Sample(row, i * ch + c, depth);
          if (c < 3 && alpha_from_trns && v != key[c]) is_key = false;
          uint8_t b;
          switch (depth) {
            case 16: b = static_cast<uint8_t>(v >> 8); break;
            case 8: b = static_cast<uint8_t>(v); break;
            case 4: b = static_cast<uint8_t>(v * 0x11); break;
            case 2: b = static_cast<uint8_t>(v * 0x55); break;
            default: b = static_cast<uint8_t>(v * 0xff); break;
          }
          o[c] = b;
        }
        if (alpha_from_trns) o[ch] = is_key ? 0 : 255;
      }
      prev = row;
      off += 1 + ps.stride;
    }
  }
  // ReadPNG: 1 gray, 2 gray + alpha, 3 RGB, 4 RGBA -> RGB on black
  rgb->resize(3 * w * h);
  for (size_t i = 0; i < w * h; ++i) {
    const uint8_t* s = px.data() + i * out_ch;
    uint8_t* d = rgb->data() + 3 * i;
    switch (out_ch) {
      case 1: d[0] = d[1] = d[2] = s[0]; break;
      case 2: d[0] = d[1] = d[2] = BlendOnBlack(s[0], s[1]); break;
      case 3: d[0] = s[0]; d[1] = s[1]; d[2] = s[2]; break;
      default:
        d[0] = BlendOnBlack(s[0], s[3]);
        d[1] = BlendOnBlack(s[1], s[3]);
        d[2] = BlendOnBlack(s[2], s[3]);
        break;
    }
  }
  *width = static_cast<int>(w);
  *height = static_cast<int>(h);
  return true;
}

}  // namespace gz
