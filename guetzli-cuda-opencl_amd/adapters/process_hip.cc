// guetzli::Process over libguetzli_hip -- see process_hip.h.
#include "process_hip.h"

#include <stdio.h>

#include "guetzli_hip.h"

namespace guetzli {

namespace {

gz_params ToGz(const Params& params) {
  gz_params p;
  gz_params_init(&p);
  p.butteraugli_target = params.butteraugli_target;
  p.clear_metadata = params.clear_metadata ? 1 : 0;
  p.try_420 = params.try_420 ? 1 : 0;
  p.force_420 = params.force_420 ? 1 : 0;
  p.use_silver_screen = params.use_silver_screen ? 1 : 0;
  p.zeroing_greedy_lookahead = params.zeroing_greedy_lookahead;
  p.new_zeroing_model = params.new_zeroing_model ? 1 : 0;
  return p;
}

bool Finish(gz_status st, ProcessStats* stats, const gz_process_stats& gs, uint8_t* jpeg,
            size_t size, std::string* out) {
  if (st != GZ_OK) {
    fprintf(stderr, "guetzli (hip): %s\n", gz_last_error());
    if (stats && stats->debug_output) {
      *stats->debug_output += gz_last_error();
      *stats->debug_output += "\n";
    }
    return false;
  }
  out->assign(reinterpret_cast<const char*>(jpeg), size);
  gz_free(jpeg);
  if (stats) {  // the counters Processor keeps (stats.h:29-31)
    stats->counters[kNumItersCnt] += gs.iterations;
    stats->counters[kNumItersUpCnt] += gs.iterations_up;
    stats->counters[kNumItersDownCnt] += gs.iterations_down;
  }
  return true;
}

}  // namespace

bool ProcessHip(const Params& params, ProcessStats* stats, const std::vector<uint8_t>& rgb,
                int w, int h, std::string* jpg_out, int device) {
  if (w <= 0 || h <= 0 || rgb.size() != 3u * static_cast<size_t>(w) * h) return false;
  const gz_params p = ToGz(params);
  uint8_t* jpeg = nullptr;
  size_t size = 0;
  gz_process_stats gs = {};
  const gz_status st = gz_process_rgb(device, &p, rgb.data(), w, h, &jpeg, &size, &gs);
  return Finish(st, stats, gs, jpeg, size, jpg_out);
}

bool ProcessHip(const Params& params, ProcessStats* stats, const std::string& data,
                std::string* jpg_out, int device) {
  const gz_params p = ToGz(params);
  uint8_t* jpeg = nullptr;
  size_t size = 0;
  gz_process_stats gs = {};
  const gz_status st = gz_process_jpeg(device, &p, reinterpret_cast<const uint8_t*>(data.data()),
                                       data.size(), &jpeg, &size, &gs);
  return Finish(st, stats, gs, jpeg, size, jpg_out);
}

}  // namespace guetzli
