// CPU end-to-end check of the row-strip decomposition (host/strips.h): WORLD
// ranks run as threads, each with the product's partitioned search loop and
// PartitionComparator over a CPU-oracle comparator of its strip (rows +
// halo; the strip's entropy coding then runs on the host) and an in-process
// all-gather; every rank must produce the reference bytes.  Test
// infrastructure only.
//
//   strips_oracle_e2e RGB W H QUALITY WORLD OUT.jpg [FAIL_RANK compare|zeroing N]
//
// With a failure injected into one rank's comparator (its N-th Compare or
// zeroing call), every rank must return an error (exit 5) -- none may block.
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "host/strips.h"
#include "oracle_comparator.h"

namespace {

// Equal-size all-gather among threads: the last rank to arrive publishes
// the concatenation of the generation's blocks.
struct Exchange {
  explicit Exchange(int world) : world(world), slots(world) {}
  int world;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<std::vector<uint8_t>> slots;
  std::vector<uint8_t> result;
  int arrived = 0;
  unsigned long gen = 0;
};

class ThreadCollectives : public gz::Collectives {
 public:
  ThreadCollectives(Exchange* x, int rank) : x_(x), rank_(rank) {}
  int rank() const override { return rank_; }
  int world() const override { return x_->world; }
  bool AllGather(const void* send, size_t bytes, void* recv) override {
    std::unique_lock<std::mutex> lk(x_->mu);
    const auto* p = static_cast<const uint8_t*>(send);
    x_->slots[rank_].assign(p, p + bytes);
    const unsigned long g = x_->gen;
    if (++x_->arrived == x_->world) {
      x_->result.clear();
      for (auto& s : x_->slots) {
        if (s.size() != bytes) return false;
        x_->result.insert(x_->result.end(), s.begin(), s.end());
      }
      x_->arrived = 0;
      ++x_->gen;
      x_->cv.notify_all();
    } else {
      x_->cv.wait(lk, [&] { return x_->gen != g; });
    }
    std::memcpy(recv, x_->result.data(), bytes * x_->world);
    return true;
  }

 private:
  Exchange* x_;
  int rank_;
};

}  // namespace

int main(int argc, char** argv) {
  if (argc < 7) {
    fprintf(stderr, "usage: strips_oracle_e2e RGB W H QUALITY WORLD OUT.jpg\n");
    return 1;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  const int w = atoi(argv[2]), h = atoi(argv[3]), q = atoi(argv[4]), world = atoi(argv[5]);
  std::vector<uint8_t> rgb(3 * static_cast<size_t>(w) * h);
  if (fread(rgb.data(), 1, rgb.size(), f) != rgb.size()) return 2;
  fclose(f);
  gz::ProcessParams params;
  params.butteraugli_target = static_cast<float>(gz::ButteraugliScoreForQuality(q));
  const gz::StripLayout L = gz::StripLayout::Make(w, h, world);
  const int fail_rank = argc >= 10 ? atoi(argv[7]) : -1;
  const std::string fail_kind = argc >= 10 ? argv[8] : "";
  const int fail_at = argc >= 10 ? atoi(argv[9]) : -1;
  Exchange x(world);
  std::vector<std::string> out(world), errs(world);
  std::vector<int> rc(world, -1), iters(world, 0);
  std::vector<double> fast_iters(world, 0.0), fallbacks(world, 0.0);
  std::vector<std::thread> ranks;
  for (int r = 0; r < world; ++r) {
    ranks.emplace_back([&, r] {
      ThreadCollectives coll(&x, r);
      // this rank's strip (owned rows + halo): its q=1 coefficients, an
      // oracle comparator of its rows, the product's partitioned search
      const int e0 = L.e0[r], hs = L.e1[r] - L.e0[r];
      const uint8_t* srgb = rgb.data() + static_cast<size_t>(3) * w * e0;
      gz::JpegData jpg;
      gz::EncodeRGBToJpegData(srgb, w, hs, &jpg);
      auto* oc = new gz_test::OracleComparator(w, hs, srgb, params.butteraugli_target);
      if (r == fail_rank) (fail_kind == "compare" ? oc->fail_compare_at : oc->fail_zeroing_at) = fail_at;
      gz::Partition part = gz::Partition::Make(L, &coll);
      gz::PartitionComparator cmp(&part, std::unique_ptr<gz::Comparator>(oc), params.butteraugli_target);
      gz::ProcessResult res;
      rc[r] = gz::ProcessJpegData(params, jpg, &cmp, &res, &errs[r], &part);
      out[r] = res.jpeg;
      iters[r] = res.iterations;
      fast_iters[r] = res.detail["strip_order_fast_iters"];
      fallbacks[r] = res.detail["strip_order_fallbacks"];
    });
  }
  for (auto& t : ranks) t.join();
  if (fail_rank >= 0) {
    for (int r = 0; r < world; ++r) {
      printf("rank %d rc %d: %s\n", r, rc[r], errs[r].c_str());
      if (rc[r] == 0) return 6;  // a rank missed the injected failure
    }
    return 5;
  }
  for (int r = 0; r < world; ++r) {
    if (rc[r] != 0) {
      fprintf(stderr, "rank %d failed: %d %s\n", r, rc[r], errs[r].c_str());
      return 3;
    }
    if (out[r] != out[0]) {
      fprintf(stderr, "rank %d bytes differ from rank 0\n", r);
      return 4;
    }
  }
  FILE* o = fopen(argv[6], "wb");
  fwrite(out[0].data(), 1, out[0].size(), o);
  fclose(o);
  // (the back end's iterations whose order came from the ranks' own entries
  // alone, and those that fell back to the exact order: host/processor.cc
  // StripOrder)
  printf("{\"bytes\": %zu, \"iters\": %d, \"world\": %d, \"strip_order_fast_iters\": %d, "
         "\"strip_order_fallbacks\": %d}\n",
         out[0].size(), iters[0], world, static_cast<int>(fast_iters[0]), static_cast<int>(fallbacks[0]));
  return 0;
}
