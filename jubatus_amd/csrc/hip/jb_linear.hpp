// Shared pieces of the linear-model kernels: agent-scope loads, the lane
// layout over label columns and the all-label score of one sample.
// Used by linear.hip (train/classify) and classify_direct.hip.
#pragma once
#include "jb_device.hpp"

namespace jb {

__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

enum Method : int { PERCEPTRON = 0, PA = 1, PA1 = 2, PA2 = 3, CW = 4, AROW = 5, NHERD = 6 };
// kSerial: several streams with the result of applying them one after the
// other (serial.hip: speculative scoring + an ordered committer)
enum UpdateMode : int { kExact = 0, kAtomic = 1, kHogwild = 2, kSerial = 3 };

// step sizes of one update; returns false when the sample causes no update.
// W += tau * (S) * x ; precision increments use beta (see header).
__device__ __forceinline__ bool step_coeffs(int method, float margin, float var, float nrm,
                                            bool has_l, float C, float* tau, float* beta) {
  switch (method) {
    case PERCEPTRON:
      if (margin <= 0.f) { *tau = 1.f; *beta = 0.f; return true; }
      return false;
    case PA: case PA1: case PA2: {
      const float loss = 1.f - margin;
      if (!(loss > 0.f && nrm > 0.f)) return false;
      const float sq = (has_l ? 2.f : 1.f) * nrm;
      if (method == PA) *tau = loss / sq;
      else if (method == PA1) *tau = fminf(C, loss / sq);
      else *tau = loss / (sq + 0.5f / C);
      *beta = 0.f;
      return true;
    }
    case CW: {
      if (!(var > 0.f)) return false;
      const float phi = C;
      const float b = 1.f + 2.f * phi * margin;
      const float disc = b * b - 8.f * phi * (margin - phi * var);
      const float gamma = (-b + sqrtf(fmaxf(disc, 0.f))) / (4.f * phi * var);
      if (!(gamma > 0.f)) return false;
      *tau = gamma; *beta = 2.f * gamma * phi;
      return true;
    }
    case AROW:
      if (!(margin < 1.f)) return false;
      *beta = 1.f / (var + 1.f / C);
      *tau = (1.f - margin) * *beta;
      return true;
    case NHERD: {
      if (!(margin < 1.f)) return false;
      *tau = (1.f - margin) / (var + 1.f / C);
      const float cv = 1.f + C * var;
      *beta = (C * C * var + 2.f * C) / (cv * cv);
      return true;
    }
    default: return false;
  }
}

// precision increment for one (feature, label): s = 1/P before the update
__device__ __forceinline__ float dprec(int method, float beta, float x, float s) {
  const float bx2 = beta * x * x;
  return method == CW ? bx2 : bx2 / (1.f - bx2 * s);
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

// best wrong label among the lanes of one feature group (lowest index on ties)
template <int LW>
__device__ __forceinline__ void argmax_wrong(float& best, int& bl) {
#pragma unroll
  for (int off = 1; off < LW; off <<= 1) {
    const float ob = __shfl_xor(best, off, 64);
    const int ol = __shfl_xor(bl, off, 64);
    if (ol >= 0 && (bl < 0 || ob > best || (ob == best && ol < bl))) { best = ob; bl = ol; }
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
