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
// (ChangeLog.rst:152) - using memory-side float atomics so that no update is
// lost. Loads use the agent-scope (sc1) path so a stream always sees the
// latest L2 contents instead of a stale L1 line.
#include "jb_device.hpp"

namespace jb {

enum Method : int { PERCEPTRON = 0, PA = 1, PA1 = 2, PA2 = 3, CW = 4, AROW = 5, NHERD = 6 };

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

template <int LC, bool CONC>
__global__ __launch_bounds__(256) void linear_train_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, float* W, float* S,
    const int32_t* __restrict__ active, int method, float C) {
  using L = Lanes<LC>;
  const int lane = threadIdx.x & 63;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wid >= nstreams) return;
  const int l0 = lane % L::LW;
  bool act[L::K];
#pragma unroll
  for (int k = 0; k < L::K; ++k) act[k] = active[l0 + 64 * k] != 0;
  const bool use_s = method >= CW;

  const int64_t s_beg = stream_ptr[wid], s_end = stream_ptr[wid + 1];
  for (int64_t s = s_beg; s < s_end; ++s) {
    const int64_t beg = row_ptr[s];
    const int n = (int)(row_ptr[s + 1] - beg);
    const int y = labels[s];
    if (y < 0 || y >= LC) continue;
    float acc[L::K];
    sample_scores<LC>(fidx, fval, beg, n, W, lane, acc);

    // correct-label score and best wrong label (lowest index wins ties)
    float sy = 0.f, best = -INFINITY;
    int bl = -1;
#pragma unroll
    for (int k = 0; k < L::K; ++k) {
      const int l = l0 + 64 * k;
      if (l == y) sy = acc[k];
      if (act[k] && l != y && acc[k] > best) { best = acc[k]; bl = l; }
    }
    sy = __shfl(sy, y % L::LW, 64);
#pragma unroll
    for (int off = 1; off < L::LW; off <<= 1) {
      const float ob = __shfl_xor(best, off, 64);
      const int ol = __shfl_xor(bl, off, 64);
      if (ol >= 0 && (bl < 0 || ob > best || (ob == best && ol < bl))) { best = ob; bl = ol; }
    }
    const int lstar = bl;
    const float margin = sy - (lstar >= 0 ? best : 0.f);

    // pass 2: lane-per-feature variance / squared norm (first 64 features kept in registers)
    int32_t idx0 = -1; float x0 = 0.f, sy0 = 1.f, sl0 = 1.f, wy0 = 0.f, wl0 = 0.f;
    float var = 0.f, nrm = 0.f;
    for (int base = 0; base < n; base += 64) {
      const int j = base + lane;
      if (j < n) {
        const int32_t idx = fidx[beg + j];
        const float x = fval[beg + j];
        if (idx >= 0) {
          const int64_t row = (int64_t)idx * LC;
          nrm += x * x;
          float a = 1.f, b = 1.f;
          if (use_s) {
            a = 1.f / ld_agent(S + row + y);
            b = lstar >= 0 ? 1.f / ld_agent(S + row + lstar) : 0.f;
            var += x * x * (a + b);
          }
          if (base == 0) {
            idx0 = idx; x0 = x; sy0 = a; sl0 = b;
            if (!CONC) { wy0 = ld_agent(W + row + y); wl0 = lstar >= 0 ? ld_agent(W + row + lstar) : 0.f; }
          }
        }
      }
    }
    var = wave_sum(var);
    nrm = wave_sum(nrm);

    // step sizes
    float tau = 0.f, beta = 0.f;  // W += tau*(S)*x ; S update uses beta
    bool upd = false;
    switch (method) {
      case PERCEPTRON: if (margin <= 0.f) { tau = 1.f; upd = true; } break;
      case PA: case PA1: case PA2: {
        const float loss = 1.f - margin;
        if (loss > 0.f && nrm > 0.f) {
          const float sq = (lstar >= 0 ? 2.f : 1.f) * nrm;
          if (method == PA) tau = loss / sq;
          else if (method == PA1) tau = fminf(C, loss / sq);
          else tau = loss / (sq + 0.5f / C);
          upd = true;
        }
      } break;
      case CW: {
        if (var > 0.f) {
          const float phi = C;
          const float b = 1.f + 2.f * phi * margin;
          const float disc = b * b - 8.f * phi * (margin - phi * var);
          const float gamma = (-b + sqrtf(fmaxf(disc, 0.f))) / (4.f * phi * var);
          if (gamma > 0.f) { tau = gamma; beta = 2.f * gamma * phi; upd = true; }
        }
      } break;
      case AROW: {
        if (margin < 1.f) {
          beta = 1.f / (var + 1.f / C);
          tau = (1.f - margin) * beta;
          upd = true;
        }
      } break;
      case NHERD: {
        if (margin < 1.f) {
          tau = (1.f - margin) / (var + 1.f / C);
          const float cv = 1.f + C * var;
          beta = (C * C * var + 2.f * C) / (cv * cv);
          upd = true;
        }
      } break;
      default: break;
    }

    if (upd) {
      for (int base = 0; base < n; base += 64) {
        const int j = base + lane;
        if (j >= n) continue;
        int32_t idx; float x, a, b, wy, wl;
        if (base == 0) { idx = idx0; x = x0; a = sy0; b = sl0; wy = wy0; wl = wl0; }
        else {
          idx = fidx[beg + j]; x = fval[beg + j];
          if (idx < 0) continue;
          const int64_t row = (int64_t)idx * LC;
          a = use_s ? 1.f / ld_agent(S + row + y) : 1.f;
          b = (use_s && lstar >= 0) ? 1.f / ld_agent(S + row + lstar) : 1.f;
          if (!CONC) { wy = ld_agent(W + row + y); wl = lstar >= 0 ? ld_agent(W + row + lstar) : 0.f; }
        }
        if (idx < 0) continue;
        const int64_t row = (int64_t)idx * LC;
        const float dwy = use_s ? tau * a * x : tau * x;
        const float dwl = use_s ? -tau * b * x : -tau * x;
        // precision increments (see header)
        float dsy = 0.f, dsl = 0.f;
        if (use_s) {
          const float bx2 = beta * x * x;
          if (method == CW) {
            dsy = bx2;
            dsl = bx2;
          } else {
            dsy = bx2 / (1.f - bx2 * a);
            dsl = bx2 / (1.f - bx2 * b);
          }
        }
        if (CONC) {
          atomicAdd(W + row + y, dwy);
          if (lstar >= 0) atomicAdd(W + row + lstar, dwl);
          if (use_s) {
            atomicAdd(S + row + y, dsy);
            if (lstar >= 0) atomicAdd(S + row + lstar, dsl);
          }
        } else {
          W[row + y] = wy + dwy;
          if (lstar >= 0) W[row + lstar] = wl + dwl;
          if (use_s) {
            S[row + y] = 1.f / a + dsy;
            if (lstar >= 0) S[row + lstar] = 1.f / b + dsl;
          }
        }
      }
      // the next sample of this stream must observe these stores
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
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
                               float C, int concurrent, hipStream_t stream) {
  if (nstreams <= 0) return 0;
  const int threads = 256;
  const int blocks = (nstreams * 64 + threads - 1) / threads;
#define JB_TRAIN(L)                                                                            \
  if (concurrent)                                                                              \
    hipLaunchKernelGGL((jb::linear_train_kernel<L, true>), dim3(blocks), dim3(threads), 0,    \
                       stream, row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S,       \
                       active, method, C);                                                    \
  else                                                                                         \
    hipLaunchKernelGGL((jb::linear_train_kernel<L, false>), dim3(blocks), dim3(threads), 0,   \
                       stream, row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S,       \
                       active, method, C);
  JB_LC_DISPATCH(LC, JB_TRAIN)
#undef JB_TRAIN
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
