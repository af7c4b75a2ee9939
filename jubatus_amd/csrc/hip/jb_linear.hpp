// Shared pieces of the linear-model kernels: agent-scope loads, the lane
// layout over label columns and the all-label score of one sample.
// Used by linear.hip (train/classify) and classify_direct.hip.
#pragma once
#include "jb_device.hpp"

namespace jb {

__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------
// W storage type. fp32 (float) or bf16 (uint16_t bit pattern, the upper half
// of the fp32 value): the bf16 table halves W's HBM footprint and gather
// bytes; arithmetic stays fp32 (loads widen, the precision table P stays
// fp32). A bf16 store rounds stochastically - the increment of an online
// update is often far below half a bf16 ulp of the weight, and
// round-to-nearest would drop it every time; stochastic rounding keeps the
// expected value of the stored weight equal to the fp32 sum. The random bits
// come from a hash of (element address, sample), so a run is reproducible.
using bf16_t = uint16_t;

__device__ __forceinline__ uint32_t jb_mix32(uint32_t a, uint32_t b) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u;
  h ^= h >> 15;
  h *= 0x2C1B3C6Du;
  h ^= h >> 12;
  h *= 0x297A2D39u;
  h ^= h >> 15;
  return h;
}

__device__ __forceinline__ float bf16_f(uint32_t b) { return __uint_as_float(b << 16); }

// fp32 -> bf16 with stochastic rounding (r: 32 random bits; the low 16 are
// used). Adding r to the magnitude's discarded bits carries into the kept
// part with probability (discarded / 2^16). Inf stays inf; NaN stays NaN.
__device__ __forceinline__ uint32_t f_bf16_sr(float v, uint32_t r) {
  const uint32_t u = __float_as_uint(v);
  if ((u & 0x7f800000u) == 0x7f800000u) return (u >> 16) | ((u & 0xffffu) ? 0x40u : 0u);
  const uint32_t t = u + (r & 0xffffu);
  // rounding up past the largest finite value gives inf (as RNE would)
  return t >> 16;
}

// W element access, overloaded on the storage type. ldw: agent-scope load
// (a stream sees other streams' updates in L2, not a stale L1 line; bf16
// loads the aligned 32-bit word and takes its half). stw: plain store.
// addw: memory-side add that no concurrent add loses (bf16: a CAS loop on the
// word; under contention it retries, the fp32 table takes a float atomic).
__device__ __forceinline__ float ldw(const float* p) { return ld_agent(p); }
__device__ __forceinline__ float ldw(const bf16_t* p) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3);
  const uint32_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ((uintptr_t)p & 2) ? __uint_as_float(v & 0xffff0000u) : __uint_as_float(v << 16);
}
__device__ __forceinline__ void stw(float* p, float v, uint32_t) { *p = v; }
__device__ __forceinline__ void stw(bf16_t* p, float v, uint32_t r) { *p = (bf16_t)f_bf16_sr(v, r); }
__device__ __forceinline__ void addw(float* p, float d, uint32_t) { atomicAdd(p, d); }
__device__ __forceinline__ void addw(bf16_t* p, float d, uint32_t r) {
  uint32_t* w = reinterpret_cast<uint32_t*>((uintptr_t)p & ~(uintptr_t)3);
  const int sh = ((uintptr_t)p & 2) ? 16 : 0;
  uint32_t old = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    const float cur = bf16_f((old >> sh) & 0xffffu);
    const uint32_t nb = f_bf16_sr(cur + d, r);
    const uint32_t nw = (old & ~(0xffffu << sh)) | (nb << sh);
    if (nw == old) return;                     // the rounded sum equals the stored value
    const uint32_t seen = atomicCAS(w, old, nw);
    if (seen == old) return;
    old = seen;
    r = jb_mix32(r, seen);                     // fresh bits for the retry
  }
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
template <int LC, typename WT>
__device__ __forceinline__ void sample_scores(const int32_t* __restrict__ fidx,
                                              const float* __restrict__ fval, int64_t beg,
                                              int n, const WT* W, int lane, float (&acc)[Lanes<LC>::K]) {
  using L = Lanes<LC>;
  const int g = lane / L::LW;
  const int l0 = lane % L::LW;
#pragma unroll
  for (int k = 0; k < L::K; ++k) acc[k] = 0.f;
  for (int j = g; j < n; j += L::G) {
    const int32_t idx = fidx[beg + j];
    const float x = fval[beg + j];
    if (idx >= 0) {
      const WT* wr = W + (int64_t)idx * LC + l0;
#pragma unroll
      for (int k = 0; k < L::K; ++k) acc[k] += x * ldw(wr + 64 * k);
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

// apply the update of one feature (lane-per-feature form)
template <int LC, int MODE, typename WT>
__device__ __forceinline__ void apply_feature(WT* W, float* P, int32_t idx, float x, int y,
                                              int lstar, bool use_s, int method, float tau,
                                              float beta, float a, float b, float wy, float wl,
                                              uint32_t rnd) {
  const int64_t row = (int64_t)idx * LC;
  const float dwy = use_s ? tau * a * x : tau * x;
  const float dwl = use_s ? -tau * b * x : -tau * x;
  if (MODE == kAtomic) {
    addw(W + row + y, dwy, jb_mix32((uint32_t)(row + y), rnd));
    if (lstar >= 0) addw(W + row + lstar, dwl, jb_mix32((uint32_t)(row + lstar), rnd));
    if (use_s) {
      atomicAdd(P + row + y, dprec(method, beta, x, a));
      if (lstar >= 0) atomicAdd(P + row + lstar, dprec(method, beta, x, b));
    }
  } else {
    stw(W + row + y, wy + dwy, jb_mix32((uint32_t)(row + y), rnd));
    if (lstar >= 0) stw(W + row + lstar, wl + dwl, jb_mix32((uint32_t)(row + lstar), rnd));
    if (use_s) {
      P[row + y] = 1.f / a + dprec(method, beta, x, a);
      if (lstar >= 0) P[row + lstar] = 1.f / b + dprec(method, beta, x, b);
    }
  }
}

// One sample on the direct path: gathers straight from W / P (any feature
// count, any label capacity) and applies the update. Used for samples wider
// than the pipelined window and for label capacities above 64. Returns
// whether the sample updated. The increments are applied with float atomics
// in every mode: a row repeated inside the sample then counts every time
// (as in the reference's per-feature loop), and in exact mode (one stream)
// nothing else touches the table, so the result is the same as plain stores.
template <int LC, int MODE, typename WT>
__device__ __forceinline__ bool general_sample(const int32_t* __restrict__ fidx,
                                               const float* __restrict__ fval, int64_t beg, int n,
                                               int y, WT* W, float* P, const bool (&act)[Lanes<LC>::K],
                                               int lane, int method, float C,
                                               uint8_t* __restrict__ touched) {
  using L = Lanes<LC>;
  const int l0 = lane % L::LW;
  const bool use_s = method >= CW;
  float acc[L::K];
  sample_scores<LC>(fidx, fval, beg, n, W, lane, acc);
  float sy = 0.f, best = -INFINITY;
  int bl = -1;
#pragma unroll
  for (int k = 0; k < L::K; ++k) {
    const int l = l0 + 64 * k;
    if (l == y) sy = acc[k];
    if (act[k] && l != y && acc[k] > best) { best = acc[k]; bl = l; }
  }
  sy = __shfl(sy, y % L::LW, 64);
  argmax_wrong<L::LW>(best, bl);
  const int lstar = bl;
  const float margin = sy - (lstar >= 0 ? best : 0.f);
  float var = 0.f, nrm = 0.f;
  for (int base = 0; base < n; base += 64) {
    const int j = base + lane;
    if (j < n) {
      const int32_t idx = fidx[beg + j];
      const float x = fval[beg + j];
      if (idx >= 0) {
        const int64_t row = (int64_t)idx * LC;
        nrm += x * x;
        if (use_s) {
          const float a = 1.f / ld_agent(P + row + y);
          const float b = lstar >= 0 ? 1.f / ld_agent(P + row + lstar) : 0.f;
          var += x * x * (a + b);
        }
      }
    }
  }
  var = wave_sum(var);
  nrm = wave_sum(nrm);
  float tau = 0.f, beta = 0.f;
  if (!step_coeffs(method, margin, var, nrm, lstar >= 0, C, &tau, &beta)) return false;
  for (int base = 0; base < n; base += 64) {
    const int j = base + lane;
    if (j >= n) continue;
    const int32_t idx = fidx[beg + j];
    if (idx < 0) continue;
    const float x = fval[beg + j];
    const int64_t row = (int64_t)idx * LC;
    const float a = use_s ? 1.f / ld_agent(P + row + y) : 1.f;
    const float b = (use_s && lstar >= 0) ? 1.f / ld_agent(P + row + lstar) : 1.f;
    apply_feature<LC, kAtomic>(W, P, idx, x, y, lstar, use_s, method, tau, beta, a, b, 0.f, 0.f,
                               (uint32_t)beg);
    if (touched != nullptr) touched[idx] = 1;
  }
  return true;
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
