// Shared pieces of the linear-model kernels: agent-scope loads, the lane
// layout over label columns and the all-label score of one sample.
// Used by linear.hip (train/classify) and classify_direct.hip.
#pragma once
#include "jb_device.hpp"

namespace jb {

__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int LC>
struct Lanes {
  static constexpr int LW = LC >= 64 ? 64 : LC;  // lanes per feature group
  static constexpr int G = 64 / LW;              // feature groups per pass
  static constexpr int K = LC >= 64 ? LC / 64 : 1;  // labels per lane
};

// scores of all LC labels of one sample; acc[k] = score of label (lane%LW)+64k
template <int LC>
__device__ __forceinline__ void sample_scores(const int32_t* __restrict__ fidx,
                                              const float* __restrict__ fval, int64_t beg,
                                              int n, const float* W, int lane, float (&acc)[Lanes<LC>::K]) {
  using L = Lanes<LC>;
  const int g = lane / L::LW;
  const int l0 = lane % L::LW;
#pragma unroll
  for (int k = 0; k < L::K; ++k) acc[k] = 0.f;
  for (int j = g; j < n; j += L::G) {
    const int32_t idx = fidx[beg + j];
    const float x = fval[beg + j];
    if (idx >= 0) {
      const float* wr = W + (int64_t)idx * LC + l0;
#pragma unroll
      for (int k = 0; k < L::K; ++k) acc[k] += x * ld_agent(wr + 64 * k);
    }
  }
#pragma unroll
  for (int off = L::LW; off < 64; off <<= 1) {
#pragma unroll
    for (int k = 0; k < L::K; ++k) acc[k] += __shfl_xor(acc[k], off, 64);
  }
}

}  // namespace jb

// label-capacity template dispatch (LC is a power of two, 8..1024)
#define JB_LC_DISPATCH(LCV, CALL) \
  switch (LCV) {                  \
    case 8: CALL(8); break;       \
    case 16: CALL(16); break;     \
    case 32: CALL(32); break;     \
    case 64: CALL(64); break;     \
    case 128: CALL(128); break;   \
    case 256: CALL(256); break;   \
    case 512: CALL(512); break;   \
    case 1024: CALL(1024); break; \
    default: return -1;           \
  }
