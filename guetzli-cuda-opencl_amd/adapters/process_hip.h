// Whole-encode drop-in for the reference tree: guetzli::Process
// (guetzli/processor.h:44-46 and :62-64) over libguetzli_hip's C ABI
// (gz_process_rgb / gz_process_jpeg, include/guetzli_hip.h).  Same contract as
// the reference: false on bad input or parameters -- and, new, on a device
// error (there is no silent CPU fallback).  Compiled against the reference's
// guetzli/processor.h and guetzli/stats.h only.
#ifndef GUETZLI_HIP_ADAPTER_PROCESS_HIP_H_
#define GUETZLI_HIP_ADAPTER_PROCESS_HIP_H_

#include <stdint.h>

#include <string>
#include <vector>

#include "guetzli/processor.h"
#include "guetzli/stats.h"

namespace guetzli {

// Process(params, stats, rgb, w, h, out) (processor.cc:1157-1185).
bool ProcessHip(const Params& params, ProcessStats* stats, const std::vector<uint8_t>& rgb,
                int w, int h, std::string* jpg_out, int device = 0);
// Process(params, stats, jpeg_bytes, out) (processor.cc:1029-1066).
bool ProcessHip(const Params& params, ProcessStats* stats, const std::string& data,
                std::string* jpg_out, int device = 0);

}  // namespace guetzli

#endif  // GUETZLI_HIP_ADAPTER_PROCESS_HIP_H_
