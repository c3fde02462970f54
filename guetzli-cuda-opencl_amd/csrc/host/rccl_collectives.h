// The exchange a frame split over GPUs needs (gz_collectives: an equal-size
// all-gather of host buffers, host/strips.h) implemented natively over RCCL
// (NCCL's API on ROCm; over xGMI between the GPUs of a node), for C++
// callers that run one process per GPU without torch.distributed
// (INTEGRATION.md §6).  The reference has no collectives at all
// (single process, device 0); this is north_star's "RCCL over
// xGMI" for the drop-in's multi-GPU entry gz_process_rgb_strips.
//
// StagedAllGather holds the buffer handling -- device send / receive
// buffers and pinned host staging that grow to the largest exchange and are
// reused, zero-byte exchanges, the rank-ordered layout of the result --
// over a Transport that does the device work.  RcclTransport is the real
// one: its own HIP stream on the rank's GPU and an ncclComm_t, RCCL loaded
// with dlopen on first use (a library that never gathers does not map it).
// tests/native/collectives_check.cc drives StagedAllGather over a
// host-memory transport (ranks as threads) on the CPU.
//
// Failure behaviour: a rank whose local step fails (a staging allocation
// or copy) returns false before it enters ncclAllGather, and its peers stay
// blocked there -- RCCL has no timeout.  The strips' exchanges
// (PartitionComparator::Exchange) carry a status word so that a failed
// *search* step fails every rank in the same all-gather; a failure of the
// transport itself leaves the job to the caller's own watchdog (as for any
// RCCL program).  Staging buffers are allocated on the communicator's
// device whatever device the calling thread has current.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>

namespace gz {

class StagedAllGather {
 public:
  // The device side of one rank: asynchronous copies and the all-gather on
  // one stream, Wait() for all of them.
  struct Transport {
    virtual ~Transport() {}
    virtual bool DeviceAlloc(size_t bytes, void** p) = 0;
    virtual void DeviceFree(void* p) = 0;
    virtual bool HostAlloc(size_t bytes, void** p) = 0;  // pinned
    virtual void HostFree(void* p) = 0;
    virtual bool CopyToDevice(void* dev, const void* host, size_t bytes) = 0;
    virtual bool CopyToHost(void* host, const void* dev, size_t bytes) = 0;
    // dev_recv[r * bytes .. (r + 1) * bytes) := rank r's dev_send
    virtual bool AllGather(const void* dev_send, void* dev_recv, size_t bytes) = 0;
    virtual bool Wait() = 0;
    virtual std::string Error() const = 0;
  };

  StagedAllGather(Transport* t, int rank, int world) : t_(t), rank_(rank), world_(world) {}
  ~StagedAllGather();
  StagedAllGather(const StagedAllGather&) = delete;
  StagedAllGather& operator=(const StagedAllGather&) = delete;

  // recv[r * bytes .. (r + 1) * bytes) := rank r's send (every rank the same
  // bytes); false with error() on a failure.
  bool Run(const void* send, size_t bytes, void* recv);
  int rank() const { return rank_; }
  int world() const { return world_; }
  size_t capacity() const { return cap_; }
  size_t grows() const { return grows_; }
  const std::string& error() const { return err_; }

 private:
  bool Reserve(size_t bytes);
  Transport* t_;
  int rank_, world_;
  size_t cap_ = 0;     // bytes per rank the buffers hold
  size_t grows_ = 0;   // reallocations so far
  void* d_send_ = nullptr;
  void* d_recv_ = nullptr;  // world * cap_
  void* h_stage_ = nullptr; // pinned, world * cap_ (the send block first, then the result)
  std::string err_;
};

}  // namespace gz

namespace gz {

// RCCL communicators for gz_collectives (C ABI: gz_rccl_* in
// include/guetzli_hip.h).  RcclUniqueId: ncclGetUniqueId (one rank calls it
// and hands the 128 bytes to the others by its own means).  RcclCreate:
// ncclCommInitRank of (rank, world) on `device` -- every rank calls it, it
// returns when all have.  RcclAllGather has gz_collectives' callback shape
// (ctx = the RcclComm).
struct RcclComm;
constexpr int kRcclIdBytes = 128;
bool RcclUniqueId(uint8_t id[kRcclIdBytes], std::string* err);
RcclComm* RcclCreate(int device, int rank, int world, const uint8_t id[kRcclIdBytes], std::string* err);
void RcclDestroy(RcclComm* c);
int RcclAllGather(void* ctx, const void* send, size_t bytes, void* recv);
const std::string& RcclError(const RcclComm* c);
// The librccl the communicators use (loaded on first use; empty if none).
const std::string& RcclLibraryPath();

}  // namespace gz
