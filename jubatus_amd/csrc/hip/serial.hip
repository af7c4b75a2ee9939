// Serial-equivalent training of many concurrent train requests (update mode
// kSerial): the result is exactly that of applying the batch's samples one
// after the other in request order - request 0's samples, then request 1's,
// ... - i.e. one valid serialization of concurrent train RPCs against the
// reference's classifier, whose driver applies every sample to the model
// left by the previous one (jubatus/server/server/classifier_serv.cpp:138-144).
//
// Online updates are sequential, but on a trained model most samples do not
// update it (their margin clears the loss threshold), and a sample that does
// not update leaves the model unchanged. So:
//
//   1. serial_score_kernel (whole GPU, one wave per sample): every sample is
//      scored against the model at the start of the batch (M0) and gets its
//      *slack*: how far its margin is from the update threshold of the method
//      (< 0: it would update under M0).
//   2. serial_commit_kernel (one 1024-thread workgroup) walks the batch in
//      order, 1024 samples per round. It keeps, in LDS, D[f] = the summed
//      magnitude of every increment the batch has applied to row f so far.
//      A sample j's margin can have moved by at most 2 * sum_f |x_jf| D[f]
//      since M0 (each label score moves by at most sum_f |x_jf| D[f]), so if
//      that bound is below its slack its decision under the current model is
//      the one it had under M0 - no update - and it is settled without
//      touching the table. The first sample of the round that is not settled
//      this way is applied *exactly* (one wave rescoring it against the live
//      table, as the single-stream path would), D grows by its increments,
//      and the rest of the round is re-checked against the new D.
//   3. When the batch updates too much for this to pay (a round with many
//      exact steps, or the D table full), the committer stops and the rest of
//      the batch runs through the single-stream exact pipelined kernel
//      (linear.hip, kExact) - the plain sequential update.
//
// Rounding: the M0 margin and the exact rescoring sum in different orders, so
// the slack keeps a relative guard band (kSlackGuard) - a sample within it of
// the threshold always takes the exact step.
#include "jb_linear.hpp"
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <unordered_map>

namespace jb {

constexpr int kCommitThreads = 512;
constexpr int kDBits = 14;
constexpr int kDCap = 1 << kDBits;   // D table slots (LDS hash, power of two)
constexpr int kDProbe = 32;          // linear-probe limit (a miss past it saturates)
constexpr int kDFull = kDCap * 5 / 8;
constexpr int kBloomBits = 16;       // filter bits (8 KB of LDS)
constexpr int kSerialNF = 16;        // features of a sample kept in registers
constexpr float kSlackGuard = 1e-4f; // relative guard band of the slack
constexpr int kStepBits = 8;
constexpr int kStepCap = 1 << kStepBits;  // step table slots
constexpr int kStepList = 64;        // distinct rows of one step the table holds
// why a committer stopped (tail[kTailReason]): the batch is done, the D
// table saturated (a new segment re-scores the rest against the current
// model with an empty table), or too many updates per round (the rest goes
// to the sequential kernel)
constexpr int kTailReason = 20;
// kStopRescore: the segment's exact steps that did not update passed
// rescore_waste - the bound, grown by every step since the segment's scores,
// no longer settles samples that would not update; scoring the rest of the
// batch again against the live model (whole GPU, ~tens of us) is cheaper than
// more wasted single-wave steps (~3.4 us each, profiles/r03_serial_v5_segments.jsonl)
constexpr int64_t kStopDone = 0, kStopSaturated = 1, kStopDense = 2, kStopRescore = 3;
constexpr int kSerialSegments = 4;       // segments of a small batch
constexpr int kSerialSegmentsBig = 48;   // of a batch of >= kSerialBigBatch samples
constexpr int64_t kSerialBigBatch = 16384;
constexpr int kDeltaSegmentsMin = 8;     // delta committer segments of a big batch
constexpr int kDeltaSegmentsMax = 512;
// verified committer windows of a big batch (vcommit.hip); a segment costs
// ~20 us, a sequential tail ~2 us per sample
constexpr int kVerifiedSegmentsMax = 2048;
constexpr int kRescoreWaste = 16;        // wasted exact steps that end a segment
constexpr int kScoreMaxBlocks = 8192;    // serial_score_kernel grid cap (grid-stride)
// committer phase timings (tail[4..19]): shader-clock reads in the step loop
// cost more than the phases they measure, so they are compiled in only for
// diagnosis (JB_SERIAL_TIMING=1 at build time)
#ifndef JB_SERIAL_TIMING
#define JB_SERIAL_TIMING 0
#endif
constexpr bool kSerialTiming = JB_SERIAL_TIMING != 0;
__device__ __forceinline__ uint64_t stamp() { return kSerialTiming ? clock64() : 0; }

// scores of all labels of one sample with plain (L1-cached) loads: the
// score pass reads a table nothing writes during the kernel
template <int LC>
__device__ __forceinline__ void sample_scores_ro(const int32_t* __restrict__ fidx,
                                                 const float* __restrict__ fval, int64_t beg, int n,
                                                 const float* __restrict__ W, int lane,
                                                 float (&acc)[Lanes<LC>::K]) {
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
      for (int k = 0; k < L::K; ++k) acc[k] += x * wr[64 * k];
    }
  }
#pragma unroll
  for (int off = L::LW; off < 64; off <<= 1) {
#pragma unroll
    for (int k = 0; k < L::K; ++k) acc[k] += __shfl_xor(acc[k], off, 64);
  }
}

// margin = score(y) - best wrong active label (0 when there is none);
// every lane gets the result
template <int LC>
__device__ __forceinline__ float margin_of(const float (&acc)[Lanes<LC>::K], int y,
                                           const bool (&act)[Lanes<LC>::K], int lane, int* lstar,
                                           float* sy_out, float* best_out) {
  using L = Lanes<LC>;
  const int l0 = lane % L::LW;
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
  *lstar = bl;
  *sy_out = sy;
  *best_out = bl >= 0 ? best : 0.f;
  return sy - (bl >= 0 ? best : 0.f);
}

// Slack of one sample's decision (see header): >= 0 how far its margin may
// move before its update decision changes, < 0 it updates under this model,
// +inf it can never update (no features), NaN: not a trainable sample.
__device__ __forceinline__ float decision_slack(int method, float margin, float nrm, bool has_l,
                                                float C, float sy, float best) {
  float s;
  switch (method) {
    case PERCEPTRON: s = margin; break;               // updates iff margin <= 0
    case PA: case PA1: case PA2:
      if (!(nrm > 0.f)) return INFINITY;
      s = margin - 1.f;                               // updates iff margin < 1
      break;
    case CW: {
      // updates iff margin < phi * var; var <= (2 or 1) * |x|^2 since P >= 1
      if (!(nrm > 0.f)) return INFINITY;
      s = margin - C * (has_l ? 2.f : 1.f) * nrm;
      break;
    }
    default:                                          // AROW, NHERD: margin < 1
      s = margin - 1.f;
      break;
  }
  const float guard = kSlackGuard * (1.f + fabsf(sy) + fabsf(best));
  if (method == PERCEPTRON ? !(s > guard) : !(s >= guard)) return -1.f;
  return s - guard;
}

template <int LC>
__global__ __launch_bounds__(256) void serial_score_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, const float* __restrict__ W,
    const int32_t* __restrict__ active, int method, float C, float* __restrict__ slack,
    float* __restrict__ l1n, const int64_t* __restrict__ reason) {
  using L = Lanes<LC>;
  const int lane = threadIdx.x & 63;
  // the batch went sequential, or the previous segment finished it
  if (reason != nullptr && (*reason == kStopDense || *reason == kStopDone)) return;
  const int64_t beg = stream_ptr[0];
  const int64_t cnt = stream_ptr[nstreams] - beg;
  bool act[L::K];
#pragma unroll
  for (int k = 0; k < L::K; ++k) act[k] = active[lane % L::LW + 64 * k] != 0;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; wid < cnt;
       wid += nwaves) {
  const int64_t s = beg + wid;
  const int y = labels[s];
  if (y < 0 || y >= LC) {
    if (lane == 0) slack[wid] = NAN;
    continue;
  }
  const int64_t fb = row_ptr[s];
  const int n = (int)(row_ptr[s + 1] - fb);
  float acc[L::K];
  sample_scores_ro<LC>(fidx, fval, fb, n, W, lane, acc);
  int lstar;
  float sy, best;
  const float margin = margin_of<LC>(acc, y, act, lane, &lstar, &sy, &best);
  float nrm = 0.f, l1 = 0.f;
  for (int j = lane; j < n; j += 64) {
    const float x = fval[fb + j];
    if (fidx[fb + j] >= 0) {
      nrm += x * x;
      l1 += fabsf(x);
    }
  }
  nrm = wave_sum(nrm);
  l1 = wave_sum(l1);
  if (lane == 0) {
    slack[wid] = decision_slack(method, margin, nrm, lstar >= 0, C, sy, best);
    l1n[wid] = l1;
  }
  }
}

// ------------------------------------------------------------ D table (LDS)
// D[f] per row the batch has written, keyed (open addressing over kDCap
// slots) behind a one-hash Bloom filter: the common lookup - a row nothing
// wrote - is one LDS read of the filter. Keys past kDFull (or a probe run
// past kDProbe) saturate the table: every later sample is then unsafe and
// the committer hands the batch to the sequential kernel.
struct DTable {
  int32_t* key;
  float* val;
  uint32_t* bloom;
  int* nkeys;
  int* sat;
  // the current exact step's increments (row -> summed |increment|): a
  // small keyed table the other threads read to grow their bounds
  // incrementally after the step (cleared by wave 0 before the next one)
  int32_t* skey;
  float* sval;
  int32_t* slist;
  int* sn;
  float* dmax;      // max_f D[f] (the cheap bound 2 |x|_1 Dmax)

  __device__ __forceinline__ static uint32_t slot(int32_t idx) {
    return ((uint32_t)idx * 0x9E3779B1u) >> (32 - kDBits);
  }
  __device__ __forceinline__ static uint32_t fbit(int32_t idx) {
    return ((uint32_t)idx * 0x85EBCA77u) >> (32 - kBloomBits);
  }
  __device__ __forceinline__ static uint32_t sslot(int32_t idx) {
    return ((uint32_t)idx * 0x9E3779B1u) >> (32 - kStepBits);
  }
  __device__ __forceinline__ bool maybe(int32_t idx) const {
    const uint32_t b = fbit(idx);
    return (bloom[b >> 5] >> (b & 31)) & 1u;
  }
  // (static: a member taking `this` would force the LDS pointer table into
  // memory)
  __device__ __attribute__((noinline)) static float probe_at(const int32_t* key, const float* val,
                                                             int32_t idx) {
    uint32_t h = slot(idx);
    for (int p = 0; p < kDProbe; ++p) {
      const int32_t k = key[h];
      if (k == idx) return val[h];
      if (k < 0) return 0.f;
      h = (h + 1) & (kDCap - 1);
    }
    return 0.f;   // never inserted past the probe limit (that saturates instead)
  }
  __device__ __forceinline__ float probe(int32_t idx) const { return probe_at(key, val, idx); }
  __device__ __forceinline__ float get(int32_t idx) const { return maybe(idx) ? probe(idx) : 0.f; }
  // increment of row idx in the last step (valid while *sn <= kStepList)
  __device__ __forceinline__ float step_get(int32_t idx) const {
    uint32_t h = sslot(idx);
    for (int p = 0; p < kStepCap; ++p) {
      const int32_t k = skey[h];
      if (k == idx) return sval[h];
      if (k < 0) return 0.f;
      h = (h + 1) & (kStepCap - 1);
    }
    return 0.f;
  }
  __device__ void add(int32_t idx, float v) {
    const uint32_t b = fbit(idx);
    atomicOr(&bloom[b >> 5], 1u << (b & 31));
    uint32_t h = slot(idx);
    bool done = false;
    for (int p = 0; p < kDProbe; ++p) {
      const int32_t old = atomicCAS(&key[h], -1, idx);
      if (old == -1 || old == idx) {
        const float prev = atomicAdd(&val[h], v);
        atomicMax((int*)dmax, __float_as_int(prev + v));   // non-negative floats order as ints
        if (old == -1 && atomicAdd(nkeys, 1) + 1 >= kDFull) *sat = 1;
        done = true;
        break;
      }
      h = (h + 1) & (kDCap - 1);
    }
    if (!done) {
    *sat = 1;
    atomicMax((int*)dmax, __float_as_int(INFINITY));
  }
    // the step table (past kStepList distinct rows the readers recompute
    // their bounds from the D table instead)
    if (*sn > kStepList) return;
    h = sslot(idx);
    for (int p = 0; p < kStepCap; ++p) {
      const int32_t old = atomicCAS(&skey[h], -1, idx);
      if (old == -1 || old == idx) {
        atomicAdd(&sval[h], v);
        if (old == -1) {
          const int n = atomicAdd(sn, 1);
          if (n < kStepList) slist[n] = (int32_t)h;
          else *sn = kStepList + 1;
        }
        return;
      }
      h = (h + 1) & (kStepCap - 1);
    }
    *sn = kStepList + 1;
  }
  // sum_u |x_u| D[idx_u] over a sample's first NF features: the filter
  // words and first probe slots of all features are read together (one LDS
  // round trip), the rare longer probe chains after
  // (in chunks of 8 features: fewer live registers)
  template <int NF>
  __device__ __forceinline__ float bound(const int32_t (&ix)[NF], const float (&xv)[NF]) const {
    constexpr int B = 8;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < NF; c += B) {
      uint32_t bw[B];
      int32_t k0[B];
      float v0[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int32_t idx = ix[c + u] >= 0 ? ix[c + u] : 0;
        const uint32_t b = fbit(idx);
        const uint32_t h = slot(idx);
        bw[u] = (bloom[b >> 5] >> (b & 31)) & 1u;
        k0[u] = key[h];
        v0[u] = val[h];
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int32_t idx = ix[c + u];
        if (idx < 0 || !bw[u] || k0[u] < 0) continue;
        acc += fabsf(xv[c + u]) * (k0[u] == idx ? v0[u] : probe(idx));
      }
    }
    return acc;
  }
  // the same over the step table (the increments of the last exact step)
  template <int NF>
  __device__ __forceinline__ float step_bound(const int32_t (&ix)[NF], const float (&xv)[NF]) const {
    constexpr int B = 8;
    float acc = 0.f;
#pragma unroll
    for (int c = 0; c < NF; c += B) {
      int32_t k0[B];
      float v0[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const uint32_t h = sslot(ix[c + u] >= 0 ? ix[c + u] : 0);
        k0[u] = skey[h];
        v0[u] = sval[h];
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const int32_t idx = ix[c + u];
        if (idx < 0 || k0[u] < 0) continue;
        acc += fabsf(xv[c + u]) * (k0[u] == idx ? v0[u] : step_get(idx));
      }
    }
    return acc;
  }
  // wave 0, before a step: empty the step table
  __device__ void step_clear(int lane) {
    const int n = *sn;
    if (n > kStepList) {
      for (int i = lane; i < kStepCap; i += 64) { skey[i] = -1; sval[i] = 0.f; }
    } else {
      for (int i = lane; i < n; i += 64) { skey[slist[i]] = -1; sval[slist[i]] = 0.f; }
    }
  }
};

// Exact step of one sample against the live table (one wave; the committer
// is the only writer while it runs). The single-stream semantics of
// linear.hip's direct path, plus the increment magnitudes into D. Returns
// whether the sample updated.
template <int LC>
__device__ bool commit_sample(const int32_t* __restrict__ fidx, const float* __restrict__ fval,
                              int64_t beg, int n, int y, float* W, float* P,
                              const bool (&act)[Lanes<LC>::K], int lane, int method, float C,
                              uint8_t* __restrict__ touched, DTable& d) {
  const bool use_s = method >= CW;
  float acc[Lanes<LC>::K];
  sample_scores<LC>(fidx, fval, beg, n, W, lane, acc);     // agent-scope loads
  int lstar;
  float sy, best;
  const float margin = margin_of<LC>(acc, y, act, lane, &lstar, &sy, &best);
  float var = 0.f, nrm = 0.f;
  for (int j = lane; j < n; j += 64) {
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
  var = wave_sum(var);
  nrm = wave_sum(nrm);
  float tau = 0.f, beta = 0.f;
  if (!step_coeffs(method, margin, var, nrm, lstar >= 0, C, &tau, &beta)) return false;
  for (int j = lane; j < n; j += 64) {
    const int32_t idx = fidx[beg + j];
    if (idx < 0) continue;
    const float x = fval[beg + j];
    const int64_t row = (int64_t)idx * LC;
    const float a = use_s ? 1.f / ld_agent(P + row + y) : 1.f;
    const float b = (use_s && lstar >= 0) ? 1.f / ld_agent(P + row + lstar) : 1.f;
    const float dwy = tau * a * x;
    const float dwl = lstar >= 0 ? -tau * b * x : 0.f;
    // atomics: a row repeated inside the sample counts every time, each
    // occurrence against the pre-sample state (as the other paths)
    atomicAdd(W + row + y, dwy);
    if (lstar >= 0) atomicAdd(W + row + lstar, dwl);
    if (use_s) {
      atomicAdd(P + row + y, dprec(method, beta, x, a));
      if (lstar >= 0) atomicAdd(P + row + lstar, dprec(method, beta, x, b));
    }
    if (touched != nullptr) touched[idx] = 1;
    d.add(idx, fabsf(dwy) + fabsf(dwl));
  }
  return true;
}

// Exact step of one sample whose features sit in LDS (the owning thread
// staged them), LC <= 64: every W / P element of the sample is gathered in
// ONE round trip (lane (g, l0) loads features g, g + G, ... of label l0),
// then the margin, the confidence of y / l* and the update follow from
// registers. Same semantics as commit_sample.
template <int LC>
__device__ bool commit_staged(const int32_t* sI, const float* sX, int n, int y, float* W, float* P,
                              bool act, int lane, int method, float C,
                              uint8_t* __restrict__ touched, DTable& d) {
  constexpr int G = 64 / LC;
  constexpr int U = (kSerialNF + G - 1) / G;
  const bool use_s = method >= CW;
  const int g = lane / LC;
  const int l0 = lane % LC;
  int32_t ix[U];
  float xv[U], w[U], pv[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int j = u * G + g;
    ix[u] = j < n ? sI[j] : -1;
    xv[u] = j < n ? sX[j] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t row = (int64_t)(ix[u] >= 0 ? ix[u] : 0) * LC + l0;
    w[u] = ld_agent(W + row);
    pv[u] = use_s ? ld_agent(P + row) : 1.f;
  }
  float acc = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (ix[u] >= 0) acc += xv[u] * w[u];
#pragma unroll
  for (int off = LC; off < 64; off <<= 1) acc += __shfl_xor(acc, off, 64);
  const float sy = __shfl(acc, y, 64);
  float best = (act && l0 != y) ? acc : -INFINITY;
  int bl = (act && l0 != y) ? l0 : -1;
  argmax_wrong<LC>(best, bl);
  const int lstar = __builtin_amdgcn_readfirstlane(bl);
  best = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(best)));
  const float margin = sy - (lstar >= 0 ? best : 0.f);
  float v = 0.f, q = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    if (ix[u] < 0) continue;
    const float x2 = xv[u] * xv[u];
    if (l0 == 0) q += x2;
    if (use_s && (l0 == y || (lstar >= 0 && l0 == lstar))) v += x2 * (1.f / pv[u]);
  }
  const float var = use_s ? wave_sum(v) : 0.f;
  const float nrm = wave_sum(q);
  float tau = 0.f, beta = 0.f;
  if (!step_coeffs(method, margin, var, nrm, lstar >= 0, C, &tau, &beta)) return false;
  const bool mine = l0 == y || (lstar >= 0 && l0 == lstar);
  // Plain read-modify-write stores unless a row repeats inside the sample:
  // this wave is the table's only writer while the committer runs, and a
  // plain store keeps the line in the XCD's L2 for the next step's loads (a
  // float atomic executes at the memory side and drops it)
  bool dup = false;
  if (lane < n)
    for (int j = lane + 1; j < n; ++j) dup |= sI[j] == sI[lane] && sI[lane] >= 0;
  const bool plain = __builtin_amdgcn_ballot_w64(dup) == 0;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    float mag = 0.f;
    if (ix[u] >= 0 && mine) {
      const int64_t row = (int64_t)ix[u] * LC + l0;
      const float a = use_s ? 1.f / pv[u] : 1.f;
      const float dw = (l0 == y ? tau : -tau) * a * xv[u];
      if (plain) {
        W[row] = w[u] + dw;
        if (use_s) P[row] = pv[u] + dprec(method, beta, xv[u], a);
      } else {
        atomicAdd(W + row, dw);
        if (use_s) atomicAdd(P + row, dprec(method, beta, xv[u], a));
      }
      if (touched != nullptr && l0 == y) touched[ix[u]] = 1;
      mag = fabsf(dw);
    }
    // the y lane adds the feature's two increments to D in one go
    const float other = __shfl(mag, g * LC + (lstar >= 0 ? lstar : y), 64);
    if (ix[u] >= 0 && l0 == y) d.add(ix[u], mag + (lstar >= 0 ? other : 0.f));
  }
  return true;
}

// Workgroup barrier over LDS only: the committer's waves exchange state
// through LDS alone (only wave 0 touches W / P, and it drains its own stores
// before it reads them again), so outstanding global loads - the next
// round's prefetched descriptors, wave 0's atomics - stay in flight across
// it (__syncthreads() would wait for every one of them: vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// a sample's first NF features into registers
template <int NF>
__device__ __forceinline__ void load_features(int32_t (&fi)[NF], float (&fx)[NF], bool live, int nf, int64_t fb,
                                              const int32_t* __restrict__ fidx, const float* __restrict__ fval) {
#pragma unroll
  for (int u = 0; u < NF; ++u) {
    const bool v = live && u < nf;
    fi[u] = v ? fidx[fb + u] : -1;
    fx[u] = v ? fval[fb + u] : 0.f;
  }
}

// The ordered committer (see header). One workgroup of 1024 threads; thread t
// owns sample p + t of the round starting at p, with the sample's slack,
// label and features in registers (prefetched a round ahead: one load round
// trip per round). The owner of the first unsettled sample stages it in LDS
// for wave 0's exact step. tail[0] receives the first sample it did not
// settle (the end of the batch when it finished), tail[1] the end of the
// batch: the exact single-stream kernel runs [tail[0], tail[1]).
template <int LC>
__global__ __launch_bounds__(kCommitThreads) void serial_commit_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, float* W, float* P,
    const int32_t* __restrict__ active, int method, float C, const float* __restrict__ slack,
    const float* __restrict__ l1n, unsigned long long* __restrict__ stats, uint8_t* __restrict__ touched,
    int64_t* __restrict__ tail, int bail_after, int seg, int rescore_waste) {
  using L = Lanes<LC>;
  constexpr int T = kCommitThreads;
  // a later segment runs only when the previous one stopped early for a re-score
  if (seg > 0 && (tail[kTailReason] == kStopDense || tail[kTailReason] == kStopDone)) return;
  constexpr int NF = kSerialNF;
  constexpr bool kStaged = LC <= 32;   // (LC 64: 16 features per lane would spill)
  __shared__ int32_t s_key[kDCap];
  __shared__ float s_val[kDCap];
  __shared__ uint32_t s_bloom[(1 << kBloomBits) / 32];
  __shared__ int32_t s_skey[kStepCap];
  __shared__ float s_sval[kStepCap];
  __shared__ int32_t s_slist[kStepList];
  __shared__ int s_sn;
  __shared__ float s_dmax;
  __shared__ int s_first[2];
  __shared__ int s_sat, s_nkeys, s_waste;
  __shared__ unsigned s_valid;
  __shared__ int32_t s_fi[NF];
  __shared__ float s_fx[NF];
  __shared__ int s_n, s_y;
  __shared__ int64_t s_fb;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  for (int i = tid; i < kDCap; i += T) {
    s_key[i] = -1;
    s_val[i] = 0.f;
  }
  for (int i = tid; i < (1 << kBloomBits) / 32; i += T) s_bloom[i] = 0u;
  for (int i = tid; i < kStepCap; i += T) {
    s_skey[i] = -1;
    s_sval[i] = 0.f;
  }
  if (tid == 0) {
    s_sn = 0;
    s_dmax = 0.f;
    s_valid = 0;
    s_sat = 0;
    s_nkeys = 0;
    s_waste = 0;
    s_first[0] = s_first[1] = INT_MAX;
  }
  DTable d{s_key, s_val, s_bloom, &s_nkeys, &s_sat, s_skey, s_sval, s_slist, &s_sn, &s_dmax};
  bool act[L::K];
#pragma unroll
  for (int k = 0; k < L::K; ++k) act[k] = active[lane % L::LW + 64 * k] != 0;
  const int64_t beg = stream_ptr[0];
  const int64_t end = stream_ptr[nstreams];
  // round descriptors of the next round (prefetched)
  float n_sl = NAN, n_l1 = 0.f;
  int64_t n_fb = 0, n_fe = 0;
  int n_y = -1;
  if (beg + tid < end) {
    n_sl = slack[tid];
    n_l1 = l1n[tid];
    n_fb = row_ptr[beg + tid];
    n_fe = row_ptr[beg + tid + 1];
    n_y = labels[beg + tid];
  }
  __syncthreads();
  unsigned n_upd = 0;
  int n_waste = 0;         // wave 0: exact steps of this segment that did not update
  int64_t stop = end;
  int64_t why = kStopDone;
  int iter = 0;
  int64_t n_steps = 0, n_rounds = 0;
  // diagnostics: shader-clock cycles thread 0 spends per phase (bound
  // checks, barrier A, staging + B1, the exact step, B2, round setup)
  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
  uint64_t wwork = 0, tw = stamp();   // per wave: cycles from B2 to the next ballot
  const uint64_t w0 = kSerialTiming ? wall_clock64() : 0;
  uint64_t tc = stamp();
  for (int64_t p = beg; p < end; p += T) {
    const int64_t j = p + tid;
    const bool live = j < end;
    const float sl = n_sl;
    const float l1 = n_l1;
    const int64_t fb = n_fb;
    const int nf = (int)(n_fe - n_fb);
    const int yl = n_y;
    // features are loaded only by samples the cheap bound 2 |x|_1 Dmax does
    // not settle (most samples of a trained model never read them)
    int32_t fi[NF];
    float fx[NF];
#pragma unroll
    for (int u = 0; u < NF; ++u) {
      fi[u] = -1;
      fx[u] = 0.f;
    }
    bool loaded = false;
    // the next round's descriptors go in flight
    const int64_t jn = j + T;
    n_sl = NAN;
    n_l1 = 0.f;
    n_fb = n_fe = 0;
    n_y = -1;
    if (jn < end) {
      n_sl = slack[jn - beg];
      n_l1 = l1n[jn - beg];
      n_fb = row_ptr[jn];
      n_fe = row_ptr[jn + 1];
      n_y = labels[jn];
    }
    // only finite, non-negative slacks can be settled by the bound
    const bool open = live && !(sl != sl) && sl < INFINITY;
    int lim = -1;          // round offsets <= lim are settled
    int steps = 0;
    // the sample's bound 2 * sum_f |x_f| D_f: from the D table once per
    // round, then grown by each exact step's increments (step table)
    auto full_bound = [&]() {
      float b = d.bound<NF>(fi, fx);
      for (int u = NF; u < nf; ++u) {
        const int32_t idx = fidx[fb + u];
        if (idx >= 0) b += fabsf(fval[fb + u]) * d.get(idx);
      }
      return b;
    };
    tw = stamp();
    float bnd = 0.f;
    if (open && (sl < 0.f || 2.f * l1 * s_dmax >= sl)) {
      load_features<NF>(fi, fx, live, nf, fb, fidx, fval);
      loaded = true;
      if (sl >= 0.f && !s_sat) bnd = full_bound();
    }
    { const uint64_t t = stamp(); ph[5] += t - tc; tc = t; }
    for (;;) {
      if (open && tid > lim && sl >= 0.f && !loaded && 2.f * l1 * s_dmax >= sl) {
        load_features<NF>(fi, fx, live, nf, fb, fidx, fval);   // Dmax grew past the cheap test
        loaded = true;
        bnd = full_bound();
      }
      const bool unsafe = open && tid > lim && (sl < 0.f || s_sat || (loaded && 2.f * bnd >= sl));
      wwork += stamp() - tw;
      const uint64_t m = __builtin_amdgcn_ballot_w64(unsafe);
      if (lane == 0 && m != 0) atomicMin(&s_first[iter & 1], wv * 64 + (int)__builtin_ctzll(m));
      { const uint64_t t = stamp(); ph[0] += t - tc; tc = t; }
      lds_barrier();       // A: the first unsettled sample of the round is known
      { const uint64_t t = stamp(); ph[1] += t - tc; tc = t; }
      const int k = s_first[iter & 1];
      if (tid == 0) s_first[(iter + 1) & 1] = INT_MAX;
      ++iter;
      if (k == INT_MAX) break;
      if (tid == k) {      // the owner stages its sample for wave 0
        if (!loaded) load_features<NF>(fi, fx, live, nf, fb, fidx, fval);
        s_n = nf;
        s_y = yl;
        s_fb = fb;
        if (nf <= NF)
          for (int u = 0; u < nf; ++u) { s_fi[u] = fi[u]; s_fx[u] = fx[u]; }
      }
      if (wv == 0) {       // nobody reads the previous step's table past barrier A
        d.step_clear(lane);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) s_sn = 0;
      }
      lds_barrier();       // B1
      { const uint64_t t = stamp(); ph[2] += t - tc; tc = t; }
      if (wv == 0) {
        // this step reads what the previous one wrote (its atomics drained
        // meanwhile, behind barriers A / B1)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int n = s_n;
        bool up;
        if (kStaged && n <= NF)
          up = commit_staged<(LC <= 32 ? LC : 32)>(s_fi, s_fx, n, s_y, W, P, act[0], lane, method, C,
                                                   touched, d);
        else
          up = commit_sample<LC>(fidx, fval, s_fb, n, s_y, W, P, act, lane, method, C, touched, d);
        if (up) ++n_upd; else ++n_waste;
        if (lane == 0) s_waste = n_waste;
      }
      lim = k;
      ++steps;
      ++n_steps;
      { const uint64_t t = stamp(); ph[3] += t - tc; tc = t; }
      lds_barrier();       // B2: D / the step table / s_sat visible to every wave
      { const uint64_t t = stamp(); ph[4] += t - tc; tc = t; }
      tw = stamp();
      if (s_sat || steps > bail_after || (rescore_waste > 0 && s_waste > rescore_waste)) {
        stop = p + k + 1;
        why = s_sat ? kStopSaturated : steps > bail_after ? kStopDense : kStopRescore;
        break;
      }
      if (loaded && open && tid > k && sl >= 0.f) {
        if (s_sn > kStepList || nf > NF) {
          bnd = full_bound();
        } else {
          bnd += d.step_bound<NF>(fi, fx);
        }
      }
    }
    ++n_rounds;
    // samples of this round settled here (valid label)
    const bool counted = live && !(sl != sl) && j < stop;
    const uint64_t cm = __builtin_amdgcn_ballot_w64(counted);
    if (lane == 0 && cm != 0) atomicAdd(&s_valid, (unsigned)__popcll(cm));
    if (stop != end) break;
  }
  __syncthreads();
  // diagnostics of the batch: the first segment sets them, later ones add
  auto put = [&](int i, int64_t v) { tail[i] = seg == 0 ? v : tail[i] + v; };
  if (lane == 0) put(12 + wv, (int64_t)wwork);
  if (tid == 0) {
    tail[0] = stop;
    tail[1] = end;
    tail[kTailReason] = why;
    put(2, n_steps);        // exact steps, rounds
    put(3, n_rounds);
    put(21, 1);             // segments
    for (int i = 0; i < 6; ++i) put(4 + i, (int64_t)ph[i]);
    put(10, kSerialTiming ? (int64_t)(wall_clock64() - w0) : 0);    // 100 MHz ticks
    put(11, (int64_t)(stamp() - tc) + (int64_t)(ph[0] + ph[1] + ph[2] + ph[3] + ph[4] + ph[5]));
    if (stats != nullptr && s_valid > 0) atomicAdd(stats + 1, (unsigned long long)s_valid);
  }
  if (tid == 0 && stats != nullptr && n_upd > 0) atomicAdd(stats, (unsigned long long)n_upd);
}

}  // namespace jb

// commit.hip: per-sample scratch bytes of the delta committer
extern "C" int64_t jb_delta_scratch_per_sample();

// bytes of the kSerial scratch for batches of up to n_max samples:
// [tail int64 x 32 = 256 B][per sample: the delta committer's S0 scores,
// precisions and best wrong label (commit.hip, LC <= 64) or this file's
// slack + |x|_1 (LC > 64)]; n_max bounds the batch's sample count
// stream_ptr[nstreams] - stream_ptr[0]
extern "C" int64_t jb_vcommit_fixed_bytes();
extern "C" int64_t jb_serial_scratch_bytes(int64_t n_max) {
  const int64_t n = n_max > 0 ? n_max : 1;
  // vcommit.hip: the slack of every sample (4 B) after the records, then its
  // 256-aligned fixed region (state, candidate bits, staged store)
  return 256 + ((jb_delta_scratch_per_sample() + 4) * n + 255) / 256 * 256 + jb_vcommit_fixed_bytes();
}

// the scratch a label capacity needs: past 64 labels only the bound
// committer runs (tail words, slack and |x|_1 per sample: 8 B a sample)
extern "C" int64_t jb_serial_scratch_bytes_lc(int64_t n_max, int LC) {
  const int64_t n = n_max > 0 ? n_max : 1;
  if (LC > 64) return 256 + (8 * n + 255) / 256 * 256;
  return jb_serial_scratch_bytes(n_max);
}

// commit.hip: the delta committer (label capacities <= 64)
extern "C" int jb_delta_prepare(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                                int64_t n_max, float* W, float* S, const int32_t* active, int LC,
                                int method, float C, unsigned long long* stats, uint8_t* touched,
                                void* scratch, int nseg, hipStream_t stream);

// pinned host words per scratch buffer: the last delta batch's final stop
// reason and segment count (tail[20], tail[21])
static std::mutex& delta_seen_mu() {
  static std::mutex mu;
  return mu;
}
static std::unordered_map<void*, int64_t*>& delta_seen_map() {
  static std::unordered_map<void*, int64_t*> seen;
  return seen;
}
static int64_t* delta_segments_seen(void* scratch) {
  std::lock_guard<std::mutex> g(delta_seen_mu());
  auto& seen = delta_seen_map();
  auto it = seen.find(scratch);
  if (it != seen.end()) return it->second;
  int64_t* p = nullptr;
  if (hipHostMalloc((void**)&p, 4 * sizeof(int64_t), hipHostMallocDefault) != hipSuccess) return nullptr;
  // until the first batch reports: done in 128 segments (a host running
  // batches ahead of the device must not read "unknown" as "short": every
  // batch would get all 512 and pay ~12 us per empty one; a young model's
  // first batches need ~100-300, so 2 x 128 + 4 keeps them whole - with 2 x
  // 64 + 4 the first ones handed a sequential tail on: 86 vs 45 ms for
  // batches 0-5, profiles/serial_exact_r4_prof_switch.jsonl)
  p[0] = jb::kStopDone;
  p[1] = 128;
  p[2] = 0;   // (verified committer) segment estimate with its stepper chunks
  seen[scratch] = p;
  return p;
}

// vcommit.hip: the verified committer (label capacities <= 64)
extern "C" int jb_vcommit_prepare(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                  const int32_t* labels, const int64_t* stream_ptr, int nstreams, int64_t n_max,
                                  float* W, float* S, const int32_t* active, int LC, int method, float C,
                                  unsigned long long* stats, uint8_t* touched, void* scratch, int nseg,
                                  hipStream_t stream);

// a scratch buffer's owner (re)allocated it: the pinned words of a freed
// buffer that had the same address must not carry its segment history over
extern "C" int jb_serial_scratch_forget(void* scratch) {
  std::lock_guard<std::mutex> g(delta_seen_mu());
  auto& seen = delta_seen_map();
  auto it = seen.find(scratch);
  if (it == seen.end()) return 0;
  (void)hipHostFree(it->second);
  seen.erase(it);
  return 1;
}

// committer of LC <= 64: 2 = verified (vcommit.hip, default), 1 = delta
// (commit.hip, JB_SERIAL_COMMITTER=delta), 0 = this file's bound committer
// (JB_SERIAL_COMMITTER=bound); the last two for A/B runs
static int serial_committer() {
  static const int v = [] {
    const char* e = getenv("JB_SERIAL_COMMITTER");
    if (e != nullptr && strcmp(e, "bound") == 0) return 0;
    if (e != nullptr && strcmp(e, "delta") == 0) return 1;
    return 2;
  }();
  return v;
}

// Steps 1-2 of a kSerial batch (score, commit); the caller then runs the
// exact single-stream kernel over stream_ptr = (int64_t*)scratch (step 3).
// bail_after: exact steps per 1024-sample round past which the committer
// hands the rest of the batch to the sequential kernel.
extern "C" int jb_serial_prepare(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                 const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                                 int64_t n_max, float* W, float* S, const int32_t* active, int LC,
                                 int method, float C, unsigned long long* stats, uint8_t* touched,
                                 void* scratch, int64_t scratch_bytes, int bail_after,
                                 hipStream_t stream) {
  if (nstreams <= 0 || n_max <= 0) return 0;
  if (scratch == nullptr || scratch_bytes < jb_serial_scratch_bytes_lc(n_max, LC)) return -3;
  if (method >= jb::CW && S == nullptr) return -4;
  if (LC <= 64 && serial_committer() == 2) {
    // verified committer: a segment is one window (score, gather, commit,
    // verify); a window that fails verification runs again. The count follows
    // the segments the previous batch on this scratch used (pinned readback,
    // one batch late at worst); the rest of a batch that runs out of them goes
    // to the sequential kernel.
    int nseg = jb::kSerialSegments;
    int64_t* seen = delta_segments_seen(scratch);
    if (n_max >= jb::kSerialBigBatch) {
      const int64_t why = seen != nullptr ? ((volatile int64_t*)seen)[0] : 0;
      // (with the windows the previous batch's stepper chunks stood in for -
      // vcommit.hip seg_estimate: a batch that is sparse again after a dense
      // one must not run out of segments)
      const int64_t est = seen != nullptr ? ((volatile int64_t*)seen)[2] : 0;
      const int64_t prev = std::max<int64_t>(seen != nullptr ? ((volatile int64_t*)seen)[1] : 0, est);
      const bool short_of = why != jb::kStopDone && why != jb::kStopDense;
      // slack over the previous batch's count: prev / 2 + 8 by default
      // (JB_VC_SEG_SLACK = d,c: prev / d + c, an A/B knob)
      static const std::pair<int, int> slack = [] {
        const char* e = getenv("JB_VC_SEG_SLACK");
        int d = 2, c = 8;
        if (e != nullptr && sscanf(e, "%d,%d", &d, &c) != 2) { d = 2; c = 8; }
        return std::make_pair(d > 0 ? d : 2, c >= 0 ? c : 8);
      }();
      nseg = short_of ? jb::kVerifiedSegmentsMax
                      : (int)std::min<int64_t>(jb::kVerifiedSegmentsMax,
                                               std::max<int64_t>(jb::kDeltaSegmentsMin,
                                                                 prev + prev / slack.first + slack.second));
    } else {
      nseg = 8;
    }
    const int rc = jb_vcommit_prepare(row_ptr, fidx, fval, labels, stream_ptr, nstreams, n_max, W, S, active,
                                      LC, method, C, stats, touched, scratch, nseg, stream);
    if (rc == 0 && seen != nullptr) {
      (void)hipMemcpyAsync(seen, (int64_t*)scratch + 20, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, stream);
      (void)hipMemcpyAsync(seen + 2, (int64_t*)scratch + 18, sizeof(int64_t), hipMemcpyDeviceToHost, stream);
    }
    return rc;
  }
  if (LC <= 64 && serial_committer() == 1) {
    // delta committer: segments end only when the LDS row store fills. A
    // segment that finds the batch done costs two empty launches (~4 us), a
    // batch that runs out of segments hands its rest to the sequential kernel:
    // the count follows the segments the previous batch on this scratch used
    // (read back asynchronously into pinned memory, one batch late at worst)
    // A batch after one that ran out of segments (its last stop reason is
    // not done / dense: the rest went to the sequential kernel, ~100x slower
    // per sample) gets every segment.
    int nseg = jb::kSerialSegments;
    int64_t* seen = delta_segments_seen(scratch);
    if (n_max >= jb::kSerialBigBatch) {
      const int64_t why = seen != nullptr ? ((volatile int64_t*)seen)[0] : 0;
      const int64_t prev = seen != nullptr ? ((volatile int64_t*)seen)[1] : 0;
      const bool short_of = why != jb::kStopDone && why != jb::kStopDense;
      nseg = short_of ? jb::kDeltaSegmentsMax
                      : (int)std::min<int64_t>(jb::kDeltaSegmentsMax,
                                               std::max<int64_t>(jb::kDeltaSegmentsMin, 2 * prev + 4));
    }
    const int rc = jb_delta_prepare(row_ptr, fidx, fval, labels, stream_ptr, nstreams, n_max, W, S, active,
                                    LC, method, C, stats, touched, scratch, nseg, stream);
    if (rc == 0 && seen != nullptr)
      (void)hipMemcpyAsync(seen, (int64_t*)scratch + 20, 2 * sizeof(int64_t), hipMemcpyDeviceToHost, stream);
    return rc;
  }
  int64_t* tail = (int64_t*)scratch;
  float* slack = (float*)((uint8_t*)scratch + 256);
  float* l1n = slack + n_max;     // |x|_1 of each sample
  // (slack[i] belongs to sample stream_ptr[0] + i)
  const int64_t blocks = std::min<int64_t>((n_max * 64 + 255) / 256, jb::kScoreMaxBlocks);
  // a big batch that updates often re-scores its rest many times (kStopRescore);
  // the last segment never stops for that (its rest would go sequential)
  const int nseg = n_max >= jb::kSerialBigBatch ? jb::kSerialSegmentsBig : jb::kSerialSegments;
  // segments: a committer that saturated its D table hands [tail[0], end)
  // to the next segment (score + commit against the model as it is then);
  // the range lives in tail[0..1] on the device, so no host round trip
  for (int seg = 0; seg < nseg; ++seg) {
    const int waste = seg + 1 < nseg ? jb::kRescoreWaste : 0;
    const int64_t* sp = seg == 0 ? stream_ptr : tail;
    const int ns = seg == 0 ? nstreams : 1;
    const int64_t* why = seg == 0 ? nullptr : tail + jb::kTailReason;
#define JB_SERIAL(L)                                                                              \
  hipLaunchKernelGGL((jb::serial_score_kernel<L>), dim3((unsigned)blocks), dim3(256), 0, stream,  \
                     row_ptr, fidx, fval, labels, sp, ns, W, active, method, C, slack, l1n, why); \
  hipLaunchKernelGGL((jb::serial_commit_kernel<L>), dim3(1), dim3(jb::kCommitThreads), 0, stream, \
                     row_ptr, fidx, fval, labels, sp, ns, W, S, active, method, C, slack, l1n,    \
                     stats,                                                                       \
                     touched, tail, bail_after, seg, waste);
    JB_LC_DISPATCH(LC, JB_SERIAL)
#undef JB_SERIAL
  }
  return (int)hipGetLastError();
}
