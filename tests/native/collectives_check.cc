// StagedAllGather's buffer handling (host/rccl_collectives.h) on the CPU:
// the RCCL transport replaced by a host-memory one, ranks as threads that
// meet at each all-gather.  Checks the rank-ordered result of every
// exchange over a run of sizes (zero bytes included; growing, then smaller
// again), that the buffers grow only past their capacity, that the
// variable-size gather built on it (Collectives::AllGatherV) holds, and that
// every allocation is released.  Prints "ok ..." or a failure.
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "host/rccl_collectives.h"
#include "host/strips.h"

namespace {

// A reusable barrier for `n` threads.
class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void Wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const long gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen; });
    }
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  long gen_ = 0;
};

struct Bus {
  explicit Bus(int world) : world(world), sends(world), barrier(world) {}
  int world;
  std::vector<const void*> sends;
  Barrier barrier;
  std::atomic<long> live{0};      // bytes allocated and not freed
  std::atomic<long> gathers{0};
};

class HostTransport : public gz::StagedAllGather::Transport {
 public:
  HostTransport(Bus* bus, int rank) : bus_(bus), rank_(rank) {}
  bool DeviceAlloc(size_t bytes, void** p) override { return Alloc(bytes, p); }
  void DeviceFree(void* p) override { Free(p); }
  bool HostAlloc(size_t bytes, void** p) override { return Alloc(bytes, p); }
  void HostFree(void* p) override { Free(p); }
  bool CopyToDevice(void* dev, const void* host, size_t bytes) override {
    std::memcpy(dev, host, bytes);
    return true;
  }
  bool CopyToHost(void* host, const void* dev, size_t bytes) override {
    std::memcpy(host, dev, bytes);
    return true;
  }
  bool AllGather(const void* dev_send, void* dev_recv, size_t bytes) override {
    bus_->sends[rank_] = dev_send;
    bus_->barrier.Wait();
    for (int r = 0; r < bus_->world; ++r)
      std::memcpy(static_cast<char*>(dev_recv) + r * bytes, bus_->sends[r], bytes);
    bus_->barrier.Wait();  // (no rank reuses its send buffer before all have read it)
    if (rank_ == 0) ++bus_->gathers;
    return true;
  }
  bool Wait() override { return true; }
  std::string Error() const override { return "host transport"; }

 private:
  bool Alloc(size_t bytes, void** p) {
    char* q = static_cast<char*>(std::malloc(bytes + 16));
    if (!q) return false;
    std::memcpy(q, &bytes, sizeof(bytes));
    bus_->live += static_cast<long>(bytes);
    std::memset(q + 16, 0xcd, bytes);  // (stale bytes must never reach a result)
    *p = q + 16;
    return true;
  }
  void Free(void* p) {
    char* q = static_cast<char*>(p) - 16;
    size_t bytes;
    std::memcpy(&bytes, q, sizeof(bytes));
    bus_->live -= static_cast<long>(bytes);
    std::free(q);
  }
  Bus* bus_;
  int rank_;
};

// The library's Collectives (equal-size + the variable-size form on top) over one StagedAllGather.
class StagedCollectives : public gz::Collectives {
 public:
  explicit StagedCollectives(gz::StagedAllGather* g) : g_(g) {}
  int rank() const override { return g_->rank(); }
  int world() const override { return g_->world(); }
  bool AllGather(const void* send, size_t bytes, void* recv) override { return g_->Run(send, bytes, recv); }

 private:
  gz::StagedAllGather* g_;
};

uint8_t Pattern(int rank, size_t i, int iter) { return static_cast<uint8_t>(rank * 31 + i * 7 + iter * 13 + 1); }

}  // namespace

int main() {
  const int world = 3;
  Bus bus(world);
  const size_t sizes[] = {5, 0, 70000, 3, 200000, 0, 1, 65536, 150000, 9};
  std::atomic<int> bad{0};
  std::vector<size_t> grows(world), caps(world);
  std::vector<std::thread> th;
  for (int r = 0; r < world; ++r)
    th.emplace_back([&, r] {
      HostTransport t(&bus, r);
      {
        gz::StagedAllGather g(&t, r, world);
        int iter = 0;
        for (size_t n : sizes) {
          std::vector<uint8_t> send(n), recv(n * world + 1, 0x5a);
          for (size_t i = 0; i < n; ++i) send[i] = Pattern(r, i, iter);
          if (!g.Run(send.data(), n, recv.data())) ++bad;
          for (int q = 0; q < world; ++q)
            for (size_t i = 0; i < n; ++i)
              if (recv[q * n + i] != Pattern(q, i, iter)) {
                ++bad;
                break;
              }
          if (recv[n * world] != 0x5a) ++bad;  // nothing past the result
          ++iter;
        }
        StagedCollectives coll(&g);
        for (int round = 0; round < 3; ++round) {
          std::vector<uint8_t> mine(r * 1000 + round * 77 + 1, static_cast<uint8_t>(r + round));
          std::vector<std::vector<uint8_t>> all;
          if (!coll.AllGatherV(mine, &all) || static_cast<int>(all.size()) != world) {
            ++bad;
            continue;
          }
          for (int q = 0; q < world; ++q)
            if (all[q] != std::vector<uint8_t>(q * 1000 + round * 77 + 1, static_cast<uint8_t>(q + round))) ++bad;
        }
        grows[r] = g.grows();
        caps[r] = g.capacity();
      }
    });
  for (auto& x : th) x.join();
  // 5 -> 64 KiB, 70000 -> 105000, 200000 -> 300000: three allocations, none after
  for (int r = 0; r < world; ++r)
    if (grows[r] != 3 || caps[r] < 200000) {
      printf("BAD grows %zu cap %zu on rank %d\n", grows[r], caps[r], r);
      return 1;
    }
  if (bad) {
    printf("BAD %d mismatches\n", bad.load());
    return 1;
  }
  if (bus.live != 0) {
    printf("BAD %ld bytes not freed\n", bus.live.load());
    return 1;
  }
  printf("ok %ld gathers\n", bus.gathers.load());
  return 0;
}
