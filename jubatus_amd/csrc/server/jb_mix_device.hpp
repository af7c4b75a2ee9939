// Device planes of the native MIX (the Plane interface of
// csrc/native/jb_mix_group.hpp over HBM tables):
//
// * RcclPlane: one RCCL communicator per group epoch (the unique id travels
//   over the group's control plane), collectives on the server's MIX stream,
//   non-blocking communicator so that a stuck peer can be aborted: every wait
//   polls the stream against the interconnect deadline and calls
//   ncclCommAbort when it passes (reference: the interconnect timeout of
//   server-to-server calls, server_util.cpp:184-194).
// * StagedPlane: device -> pinned host -> control-plane reduction -> device,
//   for members that share one GPU (RCCL needs one rank per device) or when
//   JUBATUS_MIX_PLANE=host asks for it.
#pragma once
#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <string>
#include <vector>

#include "jb_mix_group.hpp"
#include "jb_roctx.hpp"

// csrc/hip/mix.hip
extern "C" int jb_mix_pair_sum(float* p, const float* q, int64_t n, hipStream_t st);
extern "C" int jb_mix_pair_max(uint8_t* p, const uint8_t* q, int64_t n, hipStream_t st);

namespace jb {
namespace mix {

inline void hipchk(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// poll `stream` until idle or the deadline (then Timeout)
inline void wait_stream(hipStream_t st, double dl) {
  int spin = 0;
  for (;;) {
    const hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) hipchk(e, "MIX stream");
    if (now_s() > dl) throw Timeout("MIX collective exceeded the interconnect timeout");
    if (++spin > 100) std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
}

class RcclPlane : public Plane {
 public:
  RcclPlane(Star& star, int device, hipStream_t st, double dl) : st_(st) {
    ncclUniqueId id;
    if (star.rank() == 0 && ncclGetUniqueId(&id) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
    star.bcast(0, &id, sizeof id, dl);
    hipchk(hipSetDevice(device), "hipSetDevice");
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclResult_t r = ncclCommInitRankConfig(&comm_, star.world(), id, star.rank(), &cfg);
    if (r != ncclSuccess && r != ncclInProgress)
      throw std::runtime_error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    settle(dl, "ncclCommInitRank");
  }
  ~RcclPlane() override {
    if (dbuf_ && !aborted_) { (void)hipStreamSynchronize(st_); (void)hipFree(dbuf_); }
    if (comm_) {
      if (aborted_) return;
      (void)hipStreamSynchronize(st_);
      ncclCommDestroy(comm_);
    }
  }
  const char* name() const override { return "rccl"; }

  void allreduce_sum(float* p, size_t n, double dl) override {
    if (!n) return;
    jb::tx::Range tr("rccl.allreduce_sum_f32");
    check(ncclAllReduce(p, p, n, ncclFloat32, ncclSum, comm_, st_), dl, "ncclAllReduce");
    wait_stream(st_, dl);
  }
  void allreduce_max(uint8_t* p, size_t n, double dl) override {
    if (!n) return;
    jb::tx::Range tr("rccl.allreduce_max_u8");
    check(ncclAllReduce(p, p, n, ncclUint8, ncclMax, comm_, st_), dl, "ncclAllReduce");
    wait_stream(st_, dl);
  }
  bool allreduce_sum_bf16(uint16_t* p, size_t n, double dl) override {
    if (!n) return true;
    jb::tx::Range tr("rccl.allreduce_sum_bf16");
    check(ncclAllReduce(p, p, n, ncclBfloat16, ncclSum, comm_, st_), dl, "ncclAllReduce");
    wait_stream(st_, dl);
    return true;
  }
  void bcast(void* p, size_t bytes, int root, double dl) override {
    if (!bytes) return;
    jb::tx::Range tr("rccl.broadcast");
    check(ncclBroadcast(p, p, bytes, ncclUint8, root, comm_, st_), dl, "ncclBroadcast");
    wait_stream(st_, dl);
  }
  // the payload over RCCL (padded to the largest rank's), the sizes over
  // the control plane
  std::vector<std::string> allgather_bytes(Star& s, const std::string& mine, double dl) override {
    const std::vector<std::string> sz = s.allgather(std::to_string(mine.size()), dl);
    size_t mx = 1;
    for (const auto& x : sz) mx = std::max<size_t>(mx, (size_t)std::stoull(x));
    const int w = s.world();
    uint8_t* d = dev_bytes(mx * (size_t)(w + 1));
    hipchk(hipMemsetAsync(d, 0, mx, st_), "MIX memset");
    if (!mine.empty()) hipchk(hipMemcpyAsync(d, mine.data(), mine.size(), hipMemcpyHostToDevice, st_), "MIX H2D");
    jb::tx::Range tr("rccl.allgather_bytes");
    check(ncclAllGather(d, d + mx, mx, ncclUint8, comm_, st_), dl, "ncclAllGather");
    std::string all(mx * (size_t)w, '\0');
    hipchk(hipMemcpyAsync(&all[0], d + mx, all.size(), hipMemcpyDeviceToHost, st_), "MIX D2H");
    wait_stream(st_, dl);
    std::vector<std::string> out((size_t)w);
    for (int r = 0; r < w; ++r) out[(size_t)r] = all.substr((size_t)r * mx, (size_t)std::stoull(sz[(size_t)r]));
    return out;
  }
  std::string bcast_bytes(Star& s, int root, const std::string& b, double dl) override {
    uint64_t n = b.size();
    s.bcast(root, &n, 8, dl);
    if (n == 0) return std::string();
    uint8_t* d = dev_bytes((size_t)n);
    if (s.rank() == root) hipchk(hipMemcpyAsync(d, b.data(), n, hipMemcpyHostToDevice, st_), "MIX H2D");
    check(ncclBroadcast(d, d, n, ncclUint8, root, comm_, st_), dl, "ncclBroadcast");
    std::string out((size_t)n, '\0');
    hipchk(hipMemcpyAsync(&out[0], d, n, hipMemcpyDeviceToHost, st_), "MIX D2H");
    wait_stream(st_, dl);
    return out;
  }

  // pair rounds: send / receive with the peer only (RCCL point-to-point over
  // xGMI), then fold what arrived; a rank without a peer does nothing
  void pair_sum(Star&, float* p, size_t n, int peer, double dl) override {
    if (peer < 0 || n == 0) return;
    float* q = (float*)dev_bytes(n * 4);
    pair_xfer(p, q, n * 4, peer, dl);
    hipchk((hipError_t)jb_mix_pair_sum(p, q, (int64_t)n, st_), "jb_mix_pair_sum");
    wait_stream(st_, dl);
  }
  void pair_max(Star&, uint8_t* p, size_t n, int peer, double dl) override {
    if (peer < 0 || n == 0) return;
    uint8_t* q = dev_bytes(n);
    pair_xfer(p, q, n, peer, dl);
    hipchk((hipError_t)jb_mix_pair_max(p, q, (int64_t)n, st_), "jb_mix_pair_max");
    wait_stream(st_, dl);
  }

  void abort() override {
    if (comm_ && !aborted_) {
      aborted_ = true;
      ncclCommAbort(comm_);
    }
  }

 private:
  // a non-blocking communicator: wait until the call settled
  void settle(double dl, const char* what) {
    for (;;) {
      ncclResult_t st = ncclSuccess;
      ncclCommGetAsyncError(comm_, &st);
      if (st == ncclSuccess) return;
      if (st != ncclInProgress) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(st));
      if (now_s() > dl) throw Timeout(std::string(what) + " exceeded the interconnect timeout");
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
  }
  void check(ncclResult_t r, double dl, const char* what) {
    if (r == ncclInProgress) { settle(dl, what); return; }
    if (r != ncclSuccess) throw std::runtime_error(std::string(what) + ": " + ncclGetErrorString(r));
  }

  void pair_xfer(const void* send, void* recv, size_t bytes, int peer, double dl) {
    check(ncclGroupStart(), dl, "ncclGroupStart");
    check(ncclSend(send, bytes, ncclUint8, peer, comm_, st_), dl, "ncclSend");
    check(ncclRecv(recv, bytes, ncclUint8, peer, comm_, st_), dl, "ncclRecv");
    check(ncclGroupEnd(), dl, "ncclGroupEnd");
  }

  uint8_t* dev_bytes(size_t n) {
    if (n > dcap_) {
      if (dbuf_) { (void)hipStreamSynchronize(st_); (void)hipFree(dbuf_); }
      dbuf_ = nullptr;
      hipchk(hipMalloc((void**)&dbuf_, n), "hipMalloc");
      dcap_ = n;
    }
    return dbuf_;
  }

  hipStream_t st_;
  ncclComm_t comm_ = nullptr;
  bool aborted_ = false;
  uint8_t* dbuf_ = nullptr;   // byte collectives (row diffs, model hand-over)
  size_t dcap_ = 0;
};

class StagedPlane : public Plane {
 public:
  StagedPlane(Star& star, hipStream_t st) : host_(&star), st_(st) {}
  ~StagedPlane() override {
    if (buf_) (void)hipHostFree(buf_);
  }
  const char* name() const override { return "host"; }

  void allreduce_sum(float* p, size_t n, double dl) override {
    float* h = (float*)stage(p, n * 4, dl);
    host_.allreduce_sum(h, n, dl);
    unstage(p, n * 4, dl);
  }
  void allreduce_max(uint8_t* p, size_t n, double dl) override {
    uint8_t* h = (uint8_t*)stage(p, n, dl);
    host_.allreduce_max(h, n, dl);
    unstage(p, n, dl);
  }
  void bcast(void* p, size_t bytes, int root, double dl) override {
    void* h = stage(p, bytes, dl);
    host_.bcast(h, bytes, root, dl);
    unstage(p, bytes, dl);
  }
  void pair_sum(Star& s, float* p, size_t n, int peer, double dl) override {
    float* h = peer >= 0 ? (float*)stage(p, n * 4, dl) : nullptr;
    host_.pair_sum(s, h, peer >= 0 ? n : 0, peer, dl);
    if (peer >= 0) unstage(p, n * 4, dl);
  }
  void pair_max(Star& s, uint8_t* p, size_t n, int peer, double dl) override {
    uint8_t* h = peer >= 0 ? (uint8_t*)stage(p, n, dl) : nullptr;
    host_.pair_max(s, h, peer >= 0 ? n : 0, peer, dl);
    if (peer >= 0) unstage(p, n, dl);
  }

 private:
  void* stage(const void* d, size_t bytes, double dl) {
    if (bytes > cap_) {
      if (buf_) hipchk(hipHostFree(buf_), "hipHostFree");
      buf_ = nullptr;
      hipchk(hipHostMalloc(&buf_, bytes, hipHostMallocDefault), "hipHostMalloc");
      cap_ = bytes;
    }
    hipchk(hipMemcpyAsync(buf_, d, bytes, hipMemcpyDeviceToHost, st_), "MIX D2H");
    wait_stream(st_, dl);
    return buf_;
  }
  void unstage(void* d, size_t bytes, double dl) {
    hipchk(hipMemcpyAsync(d, buf_, bytes, hipMemcpyHostToDevice, st_), "MIX H2D");
    wait_stream(st_, dl);
  }
  HostPlane host_;
  hipStream_t st_;
  void* buf_ = nullptr;
  size_t cap_ = 0;
};

// RCCL unless the members share a device (or JUBATUS_MIX_PLANE=host): the
// members exchange their devices' PCI bus ids over the control plane
inline std::unique_ptr<Plane> make_device_plane(Star& star, int device, hipStream_t st, double dl) {
  const char* want = getenv("JUBATUS_MIX_PLANE");
  char bus[64] = {0};
  hipchk(hipDeviceGetPCIBusId(bus, sizeof bus - 1, device), "hipDeviceGetPCIBusId");
  const auto all = star.allgather(std::string(bus), dl);
  bool shared = false;
  for (size_t i = 0; i < all.size(); ++i)
    for (size_t j = i + 1; j < all.size(); ++j) shared |= all[i] == all[j];
  int64_t host[1] = {(shared || (want && std::string(want) == "host")) ? 1 : 0};
  star.allreduce_max(host, 1, dl);   // every member picks the same plane
  const bool force_rccl = want && std::string(want) == "rccl";   // (also for a single rank: checks)
  if (host[0] || (star.world() == 1 && !force_rccl)) return std::unique_ptr<Plane>(new StagedPlane(star, st));
  return std::unique_ptr<Plane>(new RcclPlane(star, device, st, dl));
}

}  // namespace mix
}  // namespace jb
