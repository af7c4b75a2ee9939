// Online linear classifiers (perceptron, PA, PA1, PA2, CW, AROW, NHERD) on a
// hashed weight table resident in HBM.
//
// Reference: the classifier engine's train/classify hot loops,
// jubatus/server/server/classifier_serv.cpp:128-173, which call jubatus_core's
// linear classifiers (EXTERNAL). Update rules are the published ones
// (Crammer et al. JMLR 2006; Dredze et al. ICML 2008; Crammer et al. NIPS
// 2009; Crammer & Lee NIPS 2010) in the multi-class "correct label vs best
// wrong label" form; the exact formulas are spelled out in
// jubatus_amd/models/linear_oracle.py, which is the numerical oracle for this
// file.
//
// Storage: W[H][LC] and P[H][LC] (fp32), LC = label capacity (power of two).
// P is the diagonal *precision* 1/S of the confidence methods (init 1). Every
// covariance update of CW/AROW/NHERD is an additive precision update
//     CW:         P += beta x^2
//     AROW/NHERD: P += beta x^2 / (1 - beta s x^2)   (s = 1/P)
// which is algebraically the reference form S -= beta S^2 x^2 but stays
// positive and commutes, so concurrent streams can apply it with float
// atomics. One feature row of W is LC*4 contiguous bytes, so the score gather
// of one feature is one coalesced segment.
//
// Execution model (MI355X): one wave64 owns one *stream* (a contiguous run of
// samples that must be applied in order, e.g. one train RPC). Inside a sample
// the wave is parallel over (feature, label) for the scores and over features
// for the variance/update; samples of one stream run back to back, so the
// result of a single stream is exactly the sequential online update.
// Different streams (concurrent train requests) update the shared table
// lock-free - the GPU analogue of the reference's giant-lock-free classifier
// (ChangeLog.rst:152). Update modes (template MODE):
//   kExact   one stream: plain stores, drained before the next sample
//   kAtomic  concurrent streams, memory-side float atomics: no update is lost
//   kHogwild concurrent streams, plain stores of (read value + increment):
//            racing updates of a hot row may be lost (Hogwild), but the
//            precision form keeps every P positive
// Loads use the agent-scope (sc1) path so a stream sees the latest L2
// contents instead of a stale L1 line.
#include "jb_linear.hpp"

namespace jb {

enum Method : int { PERCEPTRON = 0, PA = 1, PA1 = 2, PA2 = 3, CW = 4, AROW = 5, NHERD = 6 };
enum UpdateMode : int { kExact = 0, kAtomic = 1, kHogwild = 2 };

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

// apply the update of one feature (lane-per-feature form)
template <int LC, int MODE>
__device__ __forceinline__ void apply_feature(float* W, float* P, int32_t idx, float x, int y,
                                              int lstar, bool use_s, int method, float tau,
                                              float beta, float a, float b, float wy, float wl) {
  const int64_t row = (int64_t)idx * LC;
  const float dwy = use_s ? tau * a * x : tau * x;
  const float dwl = use_s ? -tau * b * x : -tau * x;
  if (MODE == kAtomic) {
    atomicAdd(W + row + y, dwy);
    if (lstar >= 0) atomicAdd(W + row + lstar, dwl);
    if (use_s) {
      atomicAdd(P + row + y, dprec(method, beta, x, a));
      if (lstar >= 0) atomicAdd(P + row + lstar, dprec(method, beta, x, b));
    }
  } else {
    W[row + y] = wy + dwy;
    if (lstar >= 0) W[row + lstar] = wl + dwl;
    if (use_s) {
      P[row + y] = 1.f / a + dprec(method, beta, x, a);
      if (lstar >= 0) P[row + lstar] = 1.f / b + dprec(method, beta, x, b);
    }
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

// One sample on the direct path: gathers straight from W / P (any feature
// count, any label capacity) and applies the update. Used for samples wider
// than the pipelined window and for label capacities above 64.
template <int LC, int MODE>
__device__ __forceinline__ void general_sample(const int32_t* __restrict__ fidx,
                                               const float* __restrict__ fval, int64_t beg, int n,
                                               int y, float* W, float* P, const bool (&act)[Lanes<LC>::K],
                                               int lane, int method, float C) {
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
  if (!step_coeffs(method, margin, var, nrm, lstar >= 0, C, &tau, &beta)) return;
  for (int base = 0; base < n; base += 64) {
    const int j = base + lane;
    if (j >= n) continue;
    const int32_t idx = fidx[beg + j];
    if (idx < 0) continue;
    const float x = fval[beg + j];
    const int64_t row = (int64_t)idx * LC;
    const float a = use_s ? 1.f / ld_agent(P + row + y) : 1.f;
    const float b = (use_s && lstar >= 0) ? 1.f / ld_agent(P + row + lstar) : 1.f;
    float wy = 0.f, wl = 0.f;
    if (MODE != kAtomic) {
      wy = ld_agent(W + row + y);
      wl = lstar >= 0 ? ld_agent(W + row + lstar) : 0.f;
    }
    apply_feature<LC, MODE>(W, P, idx, x, y, lstar, use_s, method, tau, beta, a, b, wy, wl);
  }
}

// Label capacities above 64: every sample on the direct path.
template <int LC, int MODE>
__global__ __launch_bounds__(256) void linear_train_wide_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, float* W, float* P,
    const int32_t* __restrict__ active, int method, float C) {
  using L = Lanes<LC>;
  const int lane = threadIdx.x & 63;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wid >= nstreams) return;
  bool act[L::K];
#pragma unroll
  for (int k = 0; k < L::K; ++k) act[k] = active[lane % L::LW + 64 * k] != 0;
  for (int64_t s = stream_ptr[wid]; s < stream_ptr[wid + 1]; ++s) {
    const int y = labels[s];
    if (y < 0 || y >= LC) continue;
    const int64_t beg = row_ptr[s];
    general_sample<LC, MODE>(fidx, fval, beg, (int)(row_ptr[s + 1] - beg), y, W, P, act, lane,
                             method, C);
    if (MODE == kExact) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// ---------------------------------------------------------------------------
// Pipelined path (LC <= 64). A sample's W / P rows are gathered with every
// load of the sample in flight at once (U unrolled passes of G features),
// staged in LDS, and the gather of sample s+1 is issued *before* sample s is
// reduced and applied, so its latency hides behind s's arithmetic and the
// in-order vmcnt never makes s+1's data wait for s's atomics. Sample s's own
// increments are forwarded into the staged rows of s+1 (an LDS add wherever
// s+1 reuses one of s's features), so one stream still sees exactly its own
// sequential updates; other streams' updates arrive as the loads observe
// them (the same lock-free semantics as before). Per-sample descriptors
// (row offsets, labels) come from a 64-entry register window refreshed every
// ~60 samples; feature descriptors of s+2 are prefetched during s.
template <int LC>
struct Pipe {
  static_assert(LC <= 64, "pipelined path covers label capacities up to 64");
  static constexpr int G = 64 / LC;              // features per pass
  static constexpr int F = LC <= 32 ? 32 : 16;   // max features of a staged sample
  static constexpr int U = F / G;                // unrolled passes per gather
};

__device__ __forceinline__ int64_t readlane64(int64_t v, int i) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, i);
  const int hi = __builtin_amdgcn_readlane((int)((uint64_t)v >> 32), i);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}

// Issue the gather of one staged sample: lane (g, l0) loads W / P of
// features u*G + g, label l0. Every load is unconditional (invalid slots read
// row 0) and nothing reads the results here, so the whole gather is U (or 2U)
// loads in flight; ``vmask`` bit u marks the valid slots for the commit.
template <int LC>
__device__ __forceinline__ uint32_t gather_issue(const float* W, const float* P, bool use_s,
                                                 const int32_t* sI, int n, int g, int l0,
                                                 float (&gw)[Pipe<LC>::U],
                                                 float (&gp)[Pipe<LC>::U]) {
  using Q = Pipe<LC>;
  int64_t rows[Q::U];
  uint32_t vmask = 0;
#pragma unroll
  for (int u = 0; u < Q::U; ++u) {
    const int j = u * Q::G + g;
    const int32_t idx = sI[j];
    const bool v = j < n && idx >= 0;
    vmask |= (v ? 1u : 0u) << u;
    rows[u] = (int64_t)(v ? idx : 0) * LC + l0;
  }
  if (use_s) {
#pragma unroll
    for (int u = 0; u < Q::U; ++u) {
      gw[u] = ld_agent(W + rows[u]);
      gp[u] = ld_agent(P + rows[u]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < Q::U; ++u) {
      gw[u] = ld_agent(W + rows[u]);
      gp[u] = 1.f;
    }
  }
  return vmask;
}

template <int LC>
__device__ __forceinline__ void gather_commit(float* sW, float* sP, bool use_s, int n, int g,
                                              int l0, uint32_t vmask,
                                              const float (&gw)[Pipe<LC>::U],
                                              const float (&gp)[Pipe<LC>::U]) {
  using Q = Pipe<LC>;
#pragma unroll
  for (int u = 0; u < Q::U; ++u) {
    const int j = u * Q::G + g;
    const bool v = (vmask >> u) & 1u;
    if (j < n) {
      sW[j * LC + l0] = v ? gw[u] : 0.f;
      if (use_s) sP[j * LC + l0] = v ? gp[u] : 1.f;
    }
  }
}

// feature list of a sample into its LDS slot (lane j = feature j)
template <int LC>
__device__ __forceinline__ void put_features(int32_t* sI, float* sX, int32_t idx, float x, int n,
                                             int lane) {
  if (lane < Pipe<LC>::F) {
    const bool v = lane < n && idx >= 0;
    sI[lane] = v ? idx : -1;
    sX[lane] = v ? x : 0.f;
  }
}

// make the compiler wait for these registers here (before later atomics
// enter the in-order vmcnt queue) instead of at their first use
#define JB_CONSUME(r) asm volatile("" ::"v"(r))

// sum of the G lane groups of one label (lanes l0, l0+LC, ...): every lane
// ends with the full score of its label
template <int LC>
__device__ __forceinline__ float group_sum(float v, int lane) {
  if (LC <= 8) v += dpp_f<kDppRowRor8>(v);
  if (LC <= 16) v += partner16_f(v, lane);
  if (LC <= 32) v += partner32_f(v, lane);
  return v;
}

// arg-max over the LC lanes of a label group (ties -> lowest label); every
// group holds the same scores, so every lane ends with the answer
template <int LC>
__device__ __forceinline__ void group_argmax(float& best, int& bl, int lane) {
  auto step = [&](float ob, int ol) {
    if (ol >= 0 && (bl < 0 || ob > best || (ob == best && ol < bl))) { best = ob; bl = ol; }
  };
  step(dpp_f<kDppXor1>(best), dpp_i<kDppXor1>(bl));
  step(dpp_f<kDppXor2>(best), dpp_i<kDppXor2>(bl));
  step(dpp_f<kDppHalfMirror>(best), dpp_i<kDppHalfMirror>(bl));
  if (LC >= 16) step(dpp_f<kDppMirror>(best), dpp_i<kDppMirror>(bl));
  if (LC >= 32) step(partner16_f(best, lane), partner16_i(bl, lane));
  if (LC >= 64) step(partner32_f(best, lane), partner32_i(bl, lane));
}

template <int LC, int MODE>
__global__ __launch_bounds__(256) void linear_train_pipe_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, float* W, float* P,
    const int32_t* __restrict__ active, int method, float C) {
  using Q = Pipe<LC>;
  constexpr int F = Q::F;
  __shared__ float sW[4][2][F * LC];
  __shared__ float sP[4][2][F * LC];
  __shared__ int32_t sI[4][2][F];
  __shared__ float sX[4][2][F];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wid >= nstreams) return;
  const int g = lane / LC;
  const int l0 = lane % LC;
  bool act[1] = {active[l0] != 0};
  const bool use_s = method >= CW;

  const int64_t s_beg = stream_ptr[wid], s_end = stream_ptr[wid + 1];
  if (s_beg >= s_end) return;
  // descriptor window: lane i holds row_ptr[wb + i] and labels[wb + i]
  int64_t wb = s_beg;
  int64_t rp = (wb + lane <= s_end) ? row_ptr[wb + lane] : 0;
  int lab = (wb + lane < s_end) ? labels[wb + lane] : -1;

  // feature descriptors of sample s (current) and s+1, lane j = feature j
  const int64_t beg0 = readlane64(rp, 0);
  int n_s = (int)(readlane64(rp, 1) - beg0);
  int y_s = __builtin_amdgcn_readlane(lab, 0);
  int32_t idx_s = lane < n_s ? fidx[beg0 + lane] : -1;
  float x_s = lane < n_s ? fval[beg0 + lane] : 0.f;
  int n1 = 0, y1 = -1;
  int32_t idx1 = -1;
  float x1 = 0.f;
  if (s_beg + 1 < s_end) {
    const int64_t b1 = readlane64(rp, 1);
    n1 = (int)(readlane64(rp, 2) - b1);
    y1 = __builtin_amdgcn_readlane(lab, 1);
    idx1 = lane < n1 ? fidx[b1 + lane] : -1;
    x1 = lane < n1 ? fval[b1 + lane] : 0.f;
  }
  JB_CONSUME(idx_s);
  JB_CONSUME(x_s);
  JB_CONSUME(idx1);
  JB_CONSUME(x1);
  put_features<LC>(sI[wv][0], sX[wv][0], idx_s, x_s, n_s, lane);
  put_features<LC>(sI[wv][1], sX[wv][1], idx1, x1, n1, lane);
  float gw[Q::U], gp[Q::U];
  uint32_t vmask = 0;
  bool staged = n_s <= F;
  if (staged) {
    vmask = gather_issue<LC>(W, P, use_s, sI[wv][0], n_s, g, l0, gw, gp);
    gather_commit<LC>(sW[wv][0], sP[wv][0], use_s, n_s, g, l0, vmask, gw, gp);
  }

  for (int64_t s = s_beg; s < s_end; ++s) {
    const int c = (int)((s - s_beg) & 1);
    const int c1 = c ^ 1;
    if (s + 3 - wb > 63) {  // slide the descriptor window (every ~60 samples)
      wb = s;
      rp = (wb + lane <= s_end) ? row_ptr[wb + lane] : 0;
      lab = (wb + lane < s_end) ? labels[wb + lane] : -1;
      JB_CONSUME(rp);
      JB_CONSUME(lab);
    }
    const bool valid_s = y_s >= 0 && y_s < LC;
    const bool general_s = valid_s && !staged;
    const bool pipe1 = s + 1 < s_end && n1 <= F;
    const bool early = pipe1 && !general_s;
    // 1. the gather of s+1 goes in flight first
    if (early) vmask = gather_issue<LC>(W, P, use_s, sI[wv][c1], n1, g, l0, gw, gp);
    // 2. feature descriptors of s+2
    int n2 = 0, y2 = -1;
    int32_t idx2 = -1;
    float x2 = 0.f;
    if (s + 2 < s_end) {
      const int i2 = (int)(s + 2 - wb);
      const int64_t b2 = readlane64(rp, i2);
      n2 = (int)(readlane64(rp, i2 + 1) - b2);
      y2 = __builtin_amdgcn_readlane(lab, i2);
      idx2 = lane < n2 ? fidx[b2 + lane] : -1;
      x2 = lane < n2 ? fval[b2 + lane] : 0.f;
    }
    // 3. sample s (LDS + registers only while the loads above are in flight)
    bool upd = false;
    int lstar = -1;
    float dwy = 0.f, dwl = 0.f, dpy = 0.f, dpl = 0.f, py = 1.f, pl = 1.f, wy = 0.f, wl = 0.f;
    const bool mine = lane < n_s && idx_s >= 0;
    if (general_s) {
      const int i = (int)(s - wb);
      const int64_t b0 = readlane64(rp, i);
      general_sample<LC, MODE>(fidx, fval, b0, (int)(readlane64(rp, i + 1) - b0), y_s, W, P, act,
                               lane, method, C);
    } else if (valid_s) {
      const float* cw = sW[wv][c];
      const float* cp = sP[wv][c];
      const float* cx = sX[wv][c];
      float acc = 0.f;
#pragma unroll
      for (int u = 0; u < Q::U; ++u) {
        const int j = u * Q::G + g;
        if (j < n_s) acc += cx[j] * cw[j * LC + l0];
      }
      acc = group_sum<LC>(acc, lane);
      const float sy = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(acc), y_s));
      float best = (act[0] && l0 != y_s) ? acc : -INFINITY;
      int bl = (act[0] && l0 != y_s) ? l0 : -1;
      group_argmax<LC>(best, bl, lane);
      lstar = __builtin_amdgcn_readfirstlane(bl);
      best = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(best)));
      const float margin = sy - (lstar >= 0 ? best : 0.f);
      float a = 1.f, b = 1.f, x2s = 0.f;
      if (mine) {
        x2s = x_s * x_s;
        if (use_s) {
          py = cp[lane * LC + y_s];
          pl = lstar >= 0 ? cp[lane * LC + lstar] : 1.f;
          a = 1.f / py;
          b = lstar >= 0 ? 1.f / pl : 0.f;
        }
        wy = cw[lane * LC + y_s];
        wl = lstar >= 0 ? cw[lane * LC + lstar] : 0.f;
      }
      const float var = use_s ? wave_sum_fast(x2s * (a + b), lane) : 0.f;
      const float nrm = wave_sum_fast(x2s, lane);
      float tau = 0.f, beta = 0.f;
      upd = step_coeffs(method, margin, var, nrm, lstar >= 0, C, &tau, &beta);
      if (upd && mine) {
        dwy = use_s ? tau * a * x_s : tau * x_s;
        dwl = use_s ? -tau * b * x_s : -tau * x_s;
        if (use_s) {
          dpy = dprec(method, beta, x_s, a);
          dpl = lstar >= 0 ? dprec(method, beta, x_s, b) : 0.f;
        }
      }
    }
    // 4. stage s+1 and forward s's own increments into it: lane k (feature k
    //    of s+1) scans s's features through readlane (registers only)
    if (early) {
      gather_commit<LC>(sW[wv][c1], sP[wv][c1], use_s, n1, g, l0, vmask, gw, gp);
      if (upd) {
        float fwy = 0.f, fwl = 0.f, fpy = 0.f, fpl = 0.f;
        const bool kv = lane < n1 && idx1 >= 0;
        for (int j = 0; j < n_s; ++j) {
          const int32_t ij = __builtin_amdgcn_readlane(idx_s, j);
          const bool hit = kv && ij == idx1;
          if (__builtin_amdgcn_ballot_w64(hit)) {
            const float ay = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dwy), j));
            const float al = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dwl), j));
            const float by = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dpy), j));
            const float bq = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dpl), j));
            if (hit) { fwy += ay; fwl += al; fpy += by; fpl += bq; }
          }
        }
        __builtin_amdgcn_wave_barrier();
        if (kv && (fwy != 0.f || fwl != 0.f || fpy != 0.f || fpl != 0.f)) {
          float* nw = sW[wv][c1] + lane * LC;
          float* np = sP[wv][c1] + lane * LC;
          nw[y_s] += fwy;
          if (lstar >= 0) nw[lstar] += fwl;
          if (use_s) {
            np[y_s] += fpy;
            if (lstar >= 0) np[lstar] += fpl;
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    JB_CONSUME(idx2);
    JB_CONSUME(x2);
    // 5. apply s to the table
    if (upd && mine) {
      const int64_t row = (int64_t)idx_s * LC;
      if (MODE == kAtomic) {
        atomicAdd(W + row + y_s, dwy);
        if (lstar >= 0) atomicAdd(W + row + lstar, dwl);
        if (use_s) {
          atomicAdd(P + row + y_s, dpy);
          if (lstar >= 0) atomicAdd(P + row + lstar, dpl);
        }
      } else {
        W[row + y_s] = wy + dwy;
        if (lstar >= 0) W[row + lstar] = wl + dwl;
        if (use_s) {
          P[row + y_s] = py + dpy;
          if (lstar >= 0) P[row + lstar] = pl + dpl;
        }
      }
    }
    if (MODE == kExact && (upd || general_s)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // 6. s+1 not prefetched (s took the direct path): stage it now that s landed
    if (pipe1 && !early) {
      if (MODE != kExact) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      vmask = gather_issue<LC>(W, P, use_s, sI[wv][c1], n1, g, l0, gw, gp);
      gather_commit<LC>(sW[wv][c1], sP[wv][c1], use_s, n1, g, l0, vmask, gw, gp);
    }
    // slot c is free again: it receives the features of s+2
    put_features<LC>(sI[wv][c], sX[wv][c], idx2, x2, n2, lane);
    __builtin_amdgcn_wave_barrier();
    staged = pipe1;
    idx_s = idx1; x_s = x1; n_s = n1; y_s = y1;
    idx1 = idx2; x1 = x2; n1 = n2; y1 = y2;
  }
}

template <int LC>
__global__ __launch_bounds__(256) void linear_classify_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, int n_samples, const float* W, float* __restrict__ out) {
  using L = Lanes<LC>;
  const int lane = threadIdx.x & 63;
  const int s = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (s >= n_samples) return;
  const int64_t beg = row_ptr[s];
  const int n = (int)(row_ptr[s + 1] - beg);
  float acc[L::K];
  sample_scores<LC>(fidx, fval, beg, n, W, lane, acc);
  if (lane < L::LW) {
#pragma unroll
    for (int k = 0; k < L::K; ++k) out[(int64_t)s * LC + lane + 64 * k] = acc[k];
  }
}

// Model averaging after an all-reduce(sum): W = W_sum * inv_n (one fused pass)
__global__ void scale_kernel(float* __restrict__ p, int64_t n, float a) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  const int64_t n4 = n & ~(int64_t)3;
  for (int64_t i = tid * 4; i < n4; i += stride) {
    float4 v = *reinterpret_cast<float4*>(p + i);
    v.x *= a; v.y *= a; v.z *= a; v.w *= a;
    *reinterpret_cast<float4*>(p + i) = v;
  }
  if (tid < n - n4) p[n4 + tid] *= a;  // tail (n % 4 elements)
}

// Overlapped MIX finish: W += red * inv_n - loc (red = cluster sum of the
// snapshot, loc = this rank's snapshot; updates made since the snapshot are
// kept). One fused pass, float4 when the three pointers are 16-B aligned.
__global__ void mix_apply_kernel(float* __restrict__ w, const float* __restrict__ red,
                                 const float* __restrict__ loc, int64_t n, float inv_n) {
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t n4 = n >> 2;
  float4* w4 = reinterpret_cast<float4*>(w);
  const float4* r4 = reinterpret_cast<const float4*>(red);
  const float4* l4 = reinterpret_cast<const float4*>(loc);
  for (int64_t i = tid; i < n4; i += stride) {
    float4 a = w4[i];
    const float4 r = r4[i], l = l4[i];
    a.x += r.x * inv_n - l.x; a.y += r.y * inv_n - l.y;
    a.z += r.z * inv_n - l.z; a.w += r.w * inv_n - l.w;
    w4[i] = a;
  }
  for (int64_t i = (n4 << 2) + tid; i < n; i += stride) w[i] += red[i] * inv_n - loc[i];
}

}  // namespace jb

extern "C" int jb_linear_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                               const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                               float* W, float* S, const int32_t* active, int LC, int method,
                               float C, int mode, hipStream_t stream) {
  if (nstreams <= 0) return 0;
  const int threads = 256;
  const int blocks = (nstreams * 64 + threads - 1) / threads;
#define JB_TRAIN_M(L, M)                                                                      \
  if (L <= 64)                                                                                \
    hipLaunchKernelGGL((jb::linear_train_pipe_kernel<(L <= 64 ? L : 64), M>), dim3(blocks),    \
                       dim3(threads), 0, stream, row_ptr, fidx, fval, labels, stream_ptr,      \
                       nstreams, W, S, active, method, C);                                    \
  else                                                                                        \
    hipLaunchKernelGGL((jb::linear_train_wide_kernel<L, M>), dim3(blocks), dim3(threads), 0,  \
                       stream, row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S,       \
                       active, method, C);
#define JB_TRAIN(L)                                        \
  if (mode == jb::kAtomic) { JB_TRAIN_M(L, jb::kAtomic) }  \
  else if (mode == jb::kHogwild) { JB_TRAIN_M(L, jb::kHogwild) } \
  else { JB_TRAIN_M(L, jb::kExact) }
  JB_LC_DISPATCH(LC, JB_TRAIN)
#undef JB_TRAIN
#undef JB_TRAIN_M
  return (int)hipGetLastError();
}

extern "C" int jb_linear_classify(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                  int n_samples, const float* W, int LC, float* out,
                                  hipStream_t stream) {
  if (n_samples <= 0) return 0;
  const int threads = 256;
  const int blocks = (n_samples * 64 + threads - 1) / threads;
#define JB_CLS(L)                                                                       \
  hipLaunchKernelGGL((jb::linear_classify_kernel<L>), dim3(blocks), dim3(threads), 0, \
                     stream, row_ptr, fidx, fval, n_samples, W, out);
  JB_LC_DISPATCH(LC, JB_CLS)
#undef JB_CLS
  return (int)hipGetLastError();
}

extern "C" int jb_scale(float* p, int64_t n, float a, hipStream_t stream) {
  if (n <= 0) return 0;
  const int threads = 256;
  int64_t blocks = (n / 4 + threads - 1) / threads;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(jb::scale_kernel, dim3((unsigned)blocks), dim3(threads), 0, stream, p, n, a);
  return (int)hipGetLastError();
}

extern "C" int jb_mix_apply(float* w, const float* red, const float* loc, int64_t n, float inv_n,
                            hipStream_t stream) {
  if (n <= 0) return 0;
  if (((uintptr_t)w | (uintptr_t)red | (uintptr_t)loc) & 15) return -2;
  const int threads = 256;
  int64_t blocks = (n / 4 + threads - 1) / threads;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(jb::mix_apply_kernel, dim3((unsigned)blocks), dim3(threads), 0, stream, w, red,
                     loc, n, inv_n);
  return (int)hipGetLastError();
}
