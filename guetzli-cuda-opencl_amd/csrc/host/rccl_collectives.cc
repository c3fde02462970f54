#include "host/rccl_collectives.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <mutex>

namespace gz {

StagedAllGather::~StagedAllGather() {
  if (d_send_) t_->DeviceFree(d_send_);
  if (d_recv_) t_->DeviceFree(d_recv_);
  if (h_stage_) t_->HostFree(h_stage_);
}

// Grow-only: the buffers of the largest exchange so far (at least 64 KiB
// per rank, then 1.5x the request), so a run of exchanges of similar sizes
// allocates once.
bool StagedAllGather::Reserve(size_t bytes) {
  if (bytes <= cap_) return true;
  if (d_send_) t_->DeviceFree(d_send_);
  if (d_recv_) t_->DeviceFree(d_recv_);
  if (h_stage_) t_->HostFree(h_stage_);
  d_send_ = d_recv_ = h_stage_ = nullptr;
  cap_ = 0;
  size_t cap = bytes + bytes / 2;
  if (cap < (size_t{1} << 16)) cap = size_t{1} << 16;
  const size_t all = cap * static_cast<size_t>(world_);
  if (!t_->DeviceAlloc(cap, &d_send_) || !t_->DeviceAlloc(all, &d_recv_) || !t_->HostAlloc(all, &h_stage_)) {
    err_ = "all-gather staging: " + t_->Error();
    if (d_send_) t_->DeviceFree(d_send_);
    if (d_recv_) t_->DeviceFree(d_recv_);
    if (h_stage_) t_->HostFree(h_stage_);
    d_send_ = d_recv_ = h_stage_ = nullptr;
    return false;
  }
  cap_ = cap;
  ++grows_;
  return true;
}

bool StagedAllGather::Run(const void* send, size_t bytes, void* recv) {
  // (every rank makes the same call: a zero-byte exchange is one on every
  // rank, and skipping it everywhere keeps them in step)
  if (bytes == 0) return true;
  if (!Reserve(bytes)) return false;
  const size_t all = bytes * static_cast<size_t>(world_);
  // the caller's (pageable) block through the pinned staging: one DMA each way
  std::memcpy(h_stage_, send, bytes);
  if (!t_->CopyToDevice(d_send_, h_stage_, bytes) || !t_->AllGather(d_send_, d_recv_, bytes) ||
      !t_->CopyToHost(h_stage_, d_recv_, all) || !t_->Wait()) {
    err_ = "all-gather: " + t_->Error();
    return false;
  }
  std::memcpy(recv, h_stage_, all);
  return true;
}

namespace {

// The few RCCL entry points used, resolved once from librccl.  The types are
// RCCL's (rccl.h) restated: opaque handles, an int result, the 128-byte id.
//
// Which librccl: the one beside the HIP runtime this process already uses.
// The library's own libamdhip64.so.7 dependency binds to whatever runtime of
// that soname is mapped first -- in a process that imported torch, the one
// torch bundles (torch/lib).  The system RCCL (/opt/rocm) against that
// runtime fails in ncclCommInitRank (hipGetDeviceCount), so the RCCL built
// with the mapped runtime -- torch's own librccl.so beside it, or ROCm's in
// /opt/rocm/lib for a plain C++ caller -- is tried first.
struct RcclApi {
  using Comm = void*;
  struct UniqueId {
    char internal[kRcclIdBytes];
  };
  int (*GetUniqueId)(UniqueId*) = nullptr;
  int (*CommInitRank)(Comm*, int, UniqueId, int) = nullptr;
  int (*AllGather)(const void*, void*, size_t, int, Comm, hipStream_t) = nullptr;
  int (*CommDestroy)(Comm) = nullptr;
  const char* (*GetErrorString)(int) = nullptr;
  std::string err;
  std::string path;  // the librccl loaded
  bool ok = false;
};
constexpr int kRcclUint8 = 1;  // ncclUint8 (ncclDataType_t)

const RcclApi& Api() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    std::string tried;
    Dl_info info{};
    if (dladdr(reinterpret_cast<void*>(&hipGetDeviceCount), &info) && info.dli_fname) {
      std::string dir = info.dli_fname;
      const size_t slash = dir.rfind('/');
      dir = slash == std::string::npos ? std::string(".") : dir.substr(0, slash);
      for (const char* name : {"/librccl.so.1", "/librccl.so"}) {
        const std::string path = dir + name;
        h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
        if (h) {
          api.path = path;
          break;
        }
        tried += path + " ";
      }
    }
    if (!h && (h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL))) api.path = "librccl.so.1";
    if (!h && (h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL))) api.path = "/opt/rocm/lib/librccl.so.1";
    if (!h) {
      const char* e = dlerror();
      api.err = std::string("librccl not loadable (") + tried + "librccl.so.1): " + (e ? e : "?");
      return;
    }
    api.GetUniqueId = reinterpret_cast<decltype(api.GetUniqueId)>(dlsym(h, "ncclGetUniqueId"));
    api.CommInitRank = reinterpret_cast<decltype(api.CommInitRank)>(dlsym(h, "ncclCommInitRank"));
    api.AllGather = reinterpret_cast<decltype(api.AllGather)>(dlsym(h, "ncclAllGather"));
    api.CommDestroy = reinterpret_cast<decltype(api.CommDestroy)>(dlsym(h, "ncclCommDestroy"));
    api.GetErrorString = reinterpret_cast<decltype(api.GetErrorString)>(dlsym(h, "ncclGetErrorString"));
    api.ok = api.GetUniqueId && api.CommInitRank && api.AllGather && api.CommDestroy && api.GetErrorString;
    if (!api.ok) api.err = "librccl lacks an entry point";
  });
  return api;
}

std::string RcclMessage(const char* what, int r) {
  const RcclApi& a = Api();
  return std::string(what) + ": " + (a.GetErrorString ? a.GetErrorString(r) : "error");
}

// HIP + RCCL on the rank's device: its own non-blocking stream.
class RcclTransport : public StagedAllGather::Transport {
 public:
  RcclTransport(int device, RcclApi::Comm comm, hipStream_t s) : device_(device), comm_(comm), s_(s) {}
  // (staging buffers on the communicator's device, whatever device the
  // calling thread had current)
  bool DeviceAlloc(size_t bytes, void** p) override {
    return Hip(hipSetDevice(device_), "hipSetDevice") && Hip(hipMalloc(p, bytes), "hipMalloc");
  }
  void DeviceFree(void* p) override { (void)hipFree(p); }
  bool HostAlloc(size_t bytes, void** p) override { return Hip(hipHostMalloc(p, bytes), "hipHostMalloc"); }
  void HostFree(void* p) override { (void)hipHostFree(p); }
  bool CopyToDevice(void* dev, const void* host, size_t bytes) override {
    return Hip(hipSetDevice(device_), "hipSetDevice") &&
           Hip(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s_), "H2D");
  }
  bool CopyToHost(void* host, const void* dev, size_t bytes) override {
    return Hip(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, s_), "D2H");
  }
  bool AllGather(const void* dev_send, void* dev_recv, size_t bytes) override {
    const int r = Api().AllGather(dev_send, dev_recv, bytes, kRcclUint8, comm_, s_);
    if (r != 0) err_ = RcclMessage("ncclAllGather", r);
    return r == 0;
  }
  bool Wait() override { return Hip(hipStreamSynchronize(s_), "hipStreamSynchronize"); }
  std::string Error() const override { return err_; }

 private:
  bool Hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    err_ = std::string(what) + ": " + hipGetErrorString(e);
    return false;
  }
  int device_;
  RcclApi::Comm comm_;
  hipStream_t s_;
  std::string err_;
};

}  // namespace

struct RcclComm {
  int device = 0;
  RcclApi::Comm comm = nullptr;
  hipStream_t stream = nullptr;
  RcclTransport* transport = nullptr;
  StagedAllGather* gather = nullptr;
  std::string err;
};

bool RcclUniqueId(uint8_t id[kRcclIdBytes], std::string* err) {
  const RcclApi& a = Api();
  if (!a.ok) {
    *err = a.err;
    return false;
  }
  RcclApi::UniqueId u;
  const int r = a.GetUniqueId(&u);
  if (r != 0) {
    *err = RcclMessage("ncclGetUniqueId", r);
    return false;
  }
  std::memcpy(id, u.internal, kRcclIdBytes);
  return true;
}

RcclComm* RcclCreate(int device, int rank, int world, const uint8_t id[kRcclIdBytes], std::string* err) {
  const RcclApi& a = Api();
  if (!a.ok) {
    *err = a.err;
    return nullptr;
  }
  if (hipSetDevice(device) != hipSuccess) {
    *err = "hipSetDevice failed";
    return nullptr;
  }
  RcclApi::UniqueId u;
  std::memcpy(u.internal, id, kRcclIdBytes);
  RcclComm* c = new RcclComm;
  c->device = device;
  int r = a.CommInitRank(&c->comm, world, u, rank);
  if (r != 0) {
    *err = RcclMessage("ncclCommInitRank", r);
    delete c;
    return nullptr;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    *err = "hipStreamCreate failed";
    a.CommDestroy(c->comm);
    delete c;
    return nullptr;
  }
  c->transport = new RcclTransport(device, c->comm, c->stream);
  c->gather = new StagedAllGather(c->transport, rank, world);
  return c;
}

void RcclDestroy(RcclComm* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  delete c->gather;  // (frees its buffers through the transport)
  delete c->transport;
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->comm) Api().CommDestroy(c->comm);
  delete c;
}

int RcclAllGather(void* ctx, const void* send, size_t bytes, void* recv) {
  RcclComm* c = static_cast<RcclComm*>(ctx);
  if (!c->gather->Run(send, bytes, recv)) {
    c->err = c->gather->error();
    return 1;
  }
  return 0;
}

const std::string& RcclError(const RcclComm* c) { return c->err; }

const std::string& RcclLibraryPath() { return Api().path; }

}  // namespace gz
