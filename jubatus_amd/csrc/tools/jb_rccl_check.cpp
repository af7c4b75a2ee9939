// jb_rccl_check: the RCCL data plane of the native MIX (jb_mix_device.hpp
// RcclPlane) on this process's GPU as a one-rank group: communicator setup
// through the control plane, SUM / MAX all-reduce and broadcast of device
// buffers on a stream, the deadline wait, and the abort path. Prints one
// JSON line; exit 0 when every check passed (tests/test_native_dist_gpu.py).
#include <hip/hip_runtime_api.h>
#include <stdio.h>

#include <vector>

#include "jb_mix_device.hpp"

int main() {
  using namespace jb::mix;
  hipchk(hipSetDevice(0), "hipSetDevice");
  hipStream_t st;
  hipchk(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "stream");
  Star star(0, 1);
  const double dl = now_s() + 60;
  bool ok = true;
  double t_init = now_s();
  std::unique_ptr<Plane> pl(new RcclPlane(star, 0, st, dl));
  t_init = now_s() - t_init;
  const size_t n = 1 << 20;
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)(i % 97) * 0.5f;
  float* d = nullptr;
  uint8_t* m = nullptr;
  hipchk(hipMalloc((void**)&d, n * 4), "hipMalloc");
  hipchk(hipMalloc((void**)&m, n), "hipMalloc");
  hipchk(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice), "H2D");
  hipchk(hipMemset(m, 3, n), "memset");
  double t_ar = now_s();
  pl->allreduce_sum(d, n, now_s() + 30);
  t_ar = now_s() - t_ar;
  pl->allreduce_max(m, n, now_s() + 30);
  pl->bcast(d, n * 4, 0, now_s() + 30);
  std::vector<float> back(n);
  std::vector<uint8_t> mb(n);
  hipchk(hipMemcpy(back.data(), d, n * 4, hipMemcpyDeviceToHost), "D2H");
  hipchk(hipMemcpy(mb.data(), m, n, hipMemcpyDeviceToHost), "D2H");
  for (size_t i = 0; i < n; ++i) ok = ok && back[i] == h[i] && mb[i] == 3;
  pl->abort();   // the watchdog path: the communicator is torn down without a hang
  pl.reset();
  printf("{\"plane\": \"rccl\", \"ok\": %s, \"init_s\": %.3f, \"allreduce_4MiB_ms\": %.3f}\n", ok ? "true" : "false",
         t_init, t_ar * 1e3);
  return ok ? 0 : 1;
}
