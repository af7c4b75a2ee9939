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
#include "jb_device.hpp"

namespace jb {

enum Method : int { PERCEPTRON = 0, PA = 1, PA1 = 2, PA2 = 3, CW = 4, AROW = 5, NHERD = 6 };
enum UpdateMode : int { kExact = 0, kAtomic = 1, kHogwild = 2 };

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

// Staged-row capacity of the fast path: NMAX features x LC labels per wave.
template <int LC>
struct Stage {
  static constexpr int NMAX = LC <= 64 ? 1024 / LC : 0;
};

template <int LC, int MODE>
__global__ __launch_bounds__(256) void linear_train_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, float* W, float* P,
    const int32_t* __restrict__ active, int method, float C) {
  using L = Lanes<LC>;
  constexpr int NMAX = Stage<LC>::NMAX;
  // per-wave LDS image of the gathered W / P rows of the current sample
  __shared__ float sW[4][NMAX > 0 ? NMAX * LC : 1];
  __shared__ float sP[4][NMAX > 0 ? NMAX * LC : 1];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wid >= nstreams) return;
  const int g = lane / L::LW;
  const int l0 = lane % L::LW;
  bool act[L::K];
#pragma unroll
  for (int k = 0; k < L::K; ++k) act[k] = active[l0 + 64 * k] != 0;
  const bool use_s = method >= CW;

  const int64_t s_beg = stream_ptr[wid], s_end = stream_ptr[wid + 1];
  // software prefetch of the next sample's (idx, x) for lane j = feature j
  int64_t nb = s_beg < s_end ? row_ptr[s_beg] : 0;
  int nn = s_beg < s_end ? (int)(row_ptr[s_beg + 1] - nb) : 0;
  int32_t pidx = (lane < nn) ? fidx[nb + lane] : -1;
  float px = (lane < nn) ? fval[nb + lane] : 0.f;
  int py = s_beg < s_end ? labels[s_beg] : -1;

  for (int64_t s = s_beg; s < s_end; ++s) {
    const int64_t beg = nb;
    const int n = nn;
    const int y = py;
    const int32_t my_idx = pidx;
    const float my_x = px;
    if (s + 1 < s_end) {  // issue next sample's descriptor loads now
      nb = row_ptr[s + 1];
      nn = (int)(row_ptr[s + 2] - nb);
      pidx = (lane < nn) ? fidx[nb + lane] : -1;
      px = (lane < nn) ? fval[nb + lane] : 0.f;
      py = labels[s + 1];
    }
    if (y < 0 || y >= LC) continue;

    if (NMAX > 0 && n <= NMAX && n <= 64) {
      // ---------------- fast path: one gather round trip, rows staged in LDS
      float acc = 0.f;
      // wave-uniform trip count: every lane takes part in each shuffle
      for (int j0 = 0; j0 < n; j0 += L::G) {
        const int j = j0 + g;
        const int src = j < 64 ? j : 63;
        const int32_t idx = __shfl(my_idx, src, 64);
        const float x = __shfl(my_x, src, 64);
        if (j < n) {
          float w = 0.f, pr = 1.f;
          if (idx >= 0) {
            const int64_t row = (int64_t)idx * LC + l0;
            w = ld_agent(W + row);
            if (use_s) pr = ld_agent(P + row);
            acc += x * w;
          }
          sW[wv][j * LC + l0] = w;
          if (use_s) sP[wv][j * LC + l0] = pr;
        }
      }
#pragma unroll
      for (int off = L::LW; off < 64; off <<= 1) acc += __shfl_xor(acc, off, 64);
      const float sy = __shfl(acc, y % L::LW, 64);
      float best = (act[0] && l0 != y) ? acc : -INFINITY;
      int bl = (act[0] && l0 != y) ? l0 : -1;
      argmax_wrong<L::LW>(best, bl);
      const int lstar = bl;
      const float margin = sy - (lstar >= 0 ? best : 0.f);
      __builtin_amdgcn_wave_barrier();
      // lane-per-feature: staged values of feature `lane`
      float a = 1.f, b = 1.f, wy = 0.f, wl = 0.f, x2 = 0.f;
      const bool mine = lane < n && my_idx >= 0;
      if (mine) {
        x2 = my_x * my_x;
        if (use_s) {
          a = 1.f / sP[wv][lane * LC + y];
          b = lstar >= 0 ? 1.f / sP[wv][lane * LC + lstar] : 0.f;
        }
        if (MODE != kAtomic) {
          wy = sW[wv][lane * LC + y];
          wl = lstar >= 0 ? sW[wv][lane * LC + lstar] : 0.f;
        }
      }
      const float var = wave_sum(use_s ? x2 * (a + b) : 0.f);
      const float nrm = wave_sum(x2);
      float tau = 0.f, beta = 0.f;
      if (step_coeffs(method, margin, var, nrm, lstar >= 0, C, &tau, &beta)) {
        if (mine)
          apply_feature<LC, MODE>(W, P, my_idx, my_x, y, lstar, use_s, method, tau, beta, a, b,
                                  wy, wl);
        // the next sample of this stream must observe these stores
        if (MODE == kExact) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_wave_barrier();
      continue;
    }

    // ---------------- general path (many features or > 64 labels)
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
    if (!step_coeffs(method, margin, var, nrm, lstar >= 0, C, &tau, &beta)) continue;
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
    if (MODE == kExact) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
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

}  // namespace jb

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

extern "C" int jb_linear_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                               const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                               float* W, float* S, const int32_t* active, int LC, int method,
                               float C, int mode, hipStream_t stream) {
  if (nstreams <= 0) return 0;
  const int threads = 256;
  const int blocks = (nstreams * 64 + threads - 1) / threads;
#define JB_TRAIN_M(L, M)                                                                     \
  hipLaunchKernelGGL((jb::linear_train_kernel<L, M>), dim3(blocks), dim3(threads), 0, stream,  \
                     row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S, active, method, C);
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
