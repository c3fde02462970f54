// Baseline Huffman JPEG serializer and the entropy-size estimator used by the
// search loop (guetzli/jpeg_data_writer.cc, entropy_encode.cc,
// jpeg_bit_writer.h).  Output bytes are identical to the reference writer.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "host/jpeg_model.h"

namespace gz {

// Symbol histogram; every symbol is counted twice and a fake symbol 256 with
// count 1 guarantees it gets the all-ones code (jpeg_data_writer.h:63-92).
struct JpegHistogram {
  static const int kSize = 257;
  uint32_t counts[kSize];
  JpegHistogram() { Clear(); }
  void Clear();
  void Add(int symbol) { counts[symbol] += 2; }
  void Add(int symbol, int weight) { counts[symbol] += 2 * weight; }
  void AddHistogram(const JpegHistogram& other);
  int NumSymbols() const;
};

// A component's Huffman code: bit length and code of each symbol.
struct HuffCodeTable {
  uint8_t depth[256];
  int code[256];
};

// Length-limited Huffman code lengths (CreateHuffmanTree, entropy_encode.cc:65-145).
void HuffmanCodeLengths(const uint32_t* counts, int length, int max_depth, uint8_t* depth);

size_t HistogramHeaderCost(const JpegHistogram& h);
size_t HistogramEntropyCost(const JpegHistogram& h, const uint8_t depths[256]);
void BuildDCHistograms(const JpegData& jpg, JpegHistogram* histo);
void BuildACHistograms(const JpegData& jpg, JpegHistogram* histo);
size_t JpegHeaderSize(const JpegData& jpg, bool strip_metadata);
size_t ClusterHistograms(JpegHistogram* histo, size_t* num, int* histo_indexes, uint8_t* depths);

// WriteJpeg (jpeg_data_writer.cc:540-553).  Appends to *out.  4:4:4 input
// takes the staged multithreaded encoder, anything else the serial one.
bool WriteJpeg(const JpegData& jpg, bool strip_metadata, std::string* out);
// The serial writer, always (test comparison baseline).
bool WriteJpegReference(const JpegData& jpg, bool strip_metadata, std::string* out);

// Everything before the entropy-coded scan for the component histograms
// dc_h / ac_h (clobbered): SOI, metadata, DQT, SOF1, DHT, SOS; fills the
// per-component code tables the scan is encoded with.
bool WriteJpegPrologue(const JpegData& hdr, bool strip_metadata, JpegHistogram* dc_h,
                       JpegHistogram* ac_h, HuffCodeTable* dc_tab, HuffCodeTable* ac_tab,
                       std::string* out);
// Appends an unstuffed scan bitstream (MSB-first bytes, nbits bits): pads
// the last byte with ones, byte-stuffs 0xff, appends EOI.
void AppendStuffedScan(const uint8_t* bits_be, uint64_t nbits, std::string* out);

// Reusable scratch of the staged encoder.
struct ScanScratch;
ScanScratch* NewScanScratch();
void FreeScanScratch(ScanScratch* s);

// Stage 1 of encoding { JpegData j = meta; img.SaveToJpegData(&j); } --
// quantization and symbol counts, parallel.  After it returns img is no longer
// referenced (the search may keep editing it while EncodeStaged runs).
// Returns the component count SaveToJpegData keeps (1 if chroma is all zero).
int StageCoeffImage(const CoeffImage& img, const JpegData& meta, ScanScratch* s);
// Stage 2: WriteJpeg of the staged image; appends to *out.
bool EncodeStaged(ScanScratch* s, bool strip_metadata, std::string* out);

// DC / AC histograms of img as SaveToJpegData would store it (components at
// or above the returned count are cleared); returns that count.
int CoeffImageHistograms(const CoeffImage& img, ScanScratch* s, JpegHistogram dc[3],
                         JpegHistogram ac[3]);

// StageCoeffImage + EncodeStaged: byte-identical to SaveToJpegData + WriteJpeg.
bool WriteCoeffImageJpeg(const CoeffImage& img, const JpegData& meta, bool strip_metadata,
                         ScanScratch* s, std::string* out);

}  // namespace gz
