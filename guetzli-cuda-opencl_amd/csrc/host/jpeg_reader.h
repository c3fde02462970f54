// JPEG input side of guetzli::Process(params, stats, jpeg_bytes, out)
// (guetzli/processor.cc:1029-1066): the reader (ReadJpeg with
// JPEG_READ_ALL, guetzli/jpeg_data_reader.cc:931-1079), the checks the
// entry point applies to its result, and DecodeJpegToRGB for 4:4:4 inputs
// (guetzli/jpeg_data_decoder.cc:45-55).  Host code: it runs once per input
// file, before the search loop.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "host/jpeg_model.h"

namespace gz {

// Baseline, extended (SOF1) and progressive Huffman JPEGs, any sampling
// factors, restart intervals.  jpg->components[i].coeffs are the QUANTIZED
// coefficients in natural order over the MCU-padded block grid, quant_idx
// indexes jpg->quant (FixupIndexes, jpeg_data_reader.cc:888-906).
bool ReadJpeg(const uint8_t* data, size_t len, JpegData* jpg, std::string* err);

bool JpegIs444(const JpegData& jpg);  // JPEGData::Is444, jpeg_data.cc:36-46
bool JpegIs420(const JpegData& jpg);  // JPEGData::Is420, jpeg_data.cc:24-34
// jpeg_data_decoder.cc:25-43 (JFIF APP0, Adobe transform, or non-RGB ids)
bool HasYCbCrColorSpace(const JpegData& jpg);
// CheckJpegSanity, processor.cc:118-131: |coeff * quant| <= 4096
bool CheckJpegSanity(const JpegData& jpg);

// DecodeJpegToRGB (jpeg_data_decoder.cc:45-55) for 3-component YCbCr 4:4:4
// and 4:2:0 images: OutputImage::CopyFromJpegData (dequantize, the integer
// IDCT of idct.cc:139-161, the fancy upsampler of output_image.cc:135-205 for
// the subsampled chroma) + ToSRGB.  False for any other layout (the reference
// returns an empty image there).
bool DecodeJpegToRGB(const JpegData& jpg, std::vector<uint8_t>* rgb);

}  // namespace gz
