// Latency of publishing a small result to fine-grained host memory with a
// completion flag the host spins on, by publish method:
//   0  system-scope fence (writes back the L2) then the flag
//   1  wait for this thread's stores to complete, block barrier, then the
//      flag as a system-scope relaxed atomic store (no L2 write-back)
// with the L2 clean or dirtied by a preceding kernel that writes `dirty` MiB
// of device memory (the score vector / candidates of a top-k chain).
// Build: hipcc --offload-arch=gfx950 -O3 -o fence_bench tools/fence_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

__global__ void dirty_kernel(float* p, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    p[i] = v + (float)i;
}

template <int METHOD>
__global__ void publish_kernel(float* out, volatile uint32_t* done, uint32_t seq, int k) {
  const int t = threadIdx.x;
  if (t < k) out[t] = (float)seq + t;
  if (METHOD == 0) {
    __threadfence_system();
    __syncthreads();
    if (t == 0) done[0] = seq;
  } else {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t == 0)
      __hip_atomic_store((uint32_t*)done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  float* dev;
  const size_t dirty_elems = (size_t)64 << 20 >> 2;    // up to 64 MiB
  CK(hipMalloc(&dev, dirty_elems * 4));
  float* out;
  uint32_t* done;
  CK(hipHostMalloc((void**)&out, 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&done, 64, hipHostMallocMapped | hipHostMallocCoherent));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint32_t seq = 0;
  const int dirty_mib[] = {0, 4, 32};
  for (int method = 0; method < 2; ++method) {
    for (int dm : dirty_mib) {
      std::vector<double> lat;
      int bad = 0;
      for (int it = 0; it < iters; ++it) {
        if (dm > 0) {
          dirty_kernel<<<1024, 256, 0, st>>>(dev, (size_t)dm << 20 >> 2, (float)it);
          CK(hipStreamSynchronize(st));
        }
        ++seq;
        const auto t0 = std::chrono::steady_clock::now();
        if (method == 0)
          publish_kernel<0><<<1, 64, 0, st>>>(out, done, seq, 10);
        else
          publish_kernel<1><<<1, 64, 0, st>>>(out, done, seq, 10);
        while (__atomic_load_n((volatile uint32_t*)done, __ATOMIC_ACQUIRE) != seq) {
        }
        const auto t1 = std::chrono::steady_clock::now();
        for (int j = 0; j < 10; ++j)
          if (((volatile float*)out)[j] != (float)seq + j) ++bad;
        lat.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        CK(hipStreamSynchronize(st));
      }
      std::sort(lat.begin(), lat.end());
      printf("{\"method\": %d, \"dirty_mib\": %d, \"p50_us\": %.2f, \"p90_us\": %.2f, "
             "\"p99_us\": %.2f, \"stale_reads\": %d}\n",
             method, dm, lat[lat.size() / 2], lat[lat.size() * 9 / 10], lat[lat.size() * 99 / 100],
             bad);
      fflush(stdout);
    }
  }
  CK(hipFree(dev));
  CK(hipHostFree(out));
  CK(hipHostFree(done));
  return 0;
}
