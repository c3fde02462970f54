// PNG input: the reference CLI's reader (ReadPNG, guetzli/guetzli.cc:51-156:
// libpng with PNG_TRANSFORM_PACKING | EXPAND | STRIP_16, then alpha blended
// on black) as a clean-room decoder over zlib's inflate.  Host only; the
// decoded RGB8 goes to the same encode as any RGB input.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

namespace gz {

// Decodes a PNG file into interleaved RGB8.  Returns false (with *err) for
// anything libpng's read would reject: bad signature or chunk order, a bad
// CRC on a critical chunk (ancillary chunks with a bad CRC are dropped, as
// libpng's default does), unsupported header fields, short or damaged image
// data, a missing IEND.
bool ReadPng(const uint8_t* data, size_t size, int* width, int* height, std::vector<uint8_t>* rgb,
             std::string* err);

}  // namespace gz
