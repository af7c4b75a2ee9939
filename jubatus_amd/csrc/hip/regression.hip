// Online passive-aggressive regression on a hashed weight vector in HBM.
//
// Reference: the regression engine's train/estimate loops,
// jubatus/server/server/regression_serv.cpp:123-149, over jubatus_core's PA
// regression (EXTERNAL). Rule (numerical oracle: models/regression.py):
//   running mean / variance of the targets (count, sum, sum of squares)
//   err = y - w.x,  loss = |err| - sensitivity * stddev
//   loss > 0:  w += sign(err) * min(C, loss) / ||x||^2 * x
//
// One wave64 per update stream (see linear.hip for the stream model); the
// lanes own features. Exact mode (one stream): plain stores drained before
// the next sample and the target statistics carried in registers. Concurrent
// streams: float atomics for w and for the statistics deltas.
#include "jb_device.hpp"

namespace jb {

__device__ __forceinline__ float ld_agent_r(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool CONC>
__global__ __launch_bounds__(256) void regression_train_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const float* __restrict__ targets,
    const int64_t* __restrict__ stream_ptr, int nstreams, float* W, float* stats, float C,
    float eps) {
  const int lane = threadIdx.x & 63;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wid >= nstreams) return;
  float sum = stats[0], sq = stats[1], cnt = stats[2];
  float dsum = 0.f, dsq = 0.f, dcnt = 0.f;
  for (int64_t s = stream_ptr[wid]; s < stream_ptr[wid + 1]; ++s) {
    const int64_t beg = row_ptr[s];
    const int n = (int)(row_ptr[s + 1] - beg);
    float dot = 0.f, nrm = 0.f;
    int32_t idx0 = -1;
    float x0 = 0.f, w0 = 0.f;
    for (int base = 0; base < n; base += 64) {
      const int j = base + lane;
      if (j < n) {
        const int32_t idx = fidx[beg + j];
        const float x = fval[beg + j];
        if (idx >= 0) {
          const float w = ld_agent_r(W + idx);
          dot += x * w;
          nrm += x * x;
          if (base == 0) { idx0 = idx; x0 = x; w0 = w; }
        }
      }
    }
    dot = wave_sum(dot);
    nrm = wave_sum(nrm);
    const float y = targets[s];
    sum += y; sq += y * y; cnt += 1.f;
    dsum += y; dsq += y * y; dcnt += 1.f;
    const float avg = sum / cnt;
    const float sd = sqrtf(fmaxf(0.f, sq / cnt - avg * avg));
    const float err = y - dot;
    const float sgn = err > 0.f ? 1.f : -1.f;
    const float loss = sgn * err - eps * sd;
    if (!(loss > 0.f) || !(nrm > 0.f)) continue;
    const float coeff = sgn * fminf(C, loss) / nrm;
    for (int base = 0; base < n; base += 64) {
      const int j = base + lane;
      if (j >= n) continue;
      int32_t idx; float x, w;
      if (base == 0) { idx = idx0; x = x0; w = w0; }
      else {
        idx = fidx[beg + j]; x = fval[beg + j];
        w = idx >= 0 ? ld_agent_r(W + idx) : 0.f;
      }
      if (idx < 0) continue;
      if (CONC) atomicAdd(W + idx, coeff * x);
      else W[idx] = w + coeff * x;
    }
    if (!CONC) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (lane == 0) {
    if (CONC) {
      atomicAdd(stats + 0, dsum);
      atomicAdd(stats + 1, dsq);
      atomicAdd(stats + 2, dcnt);
    } else {
      stats[0] = sum; stats[1] = sq; stats[2] = cnt;
    }
  }
}

// y_hat = w.x per sample (wave per sample)
__global__ __launch_bounds__(256) void regression_estimate_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, int n_samples, const float* W, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int s = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (s >= n_samples) return;
  const int64_t beg = row_ptr[s];
  const int n = (int)(row_ptr[s + 1] - beg);
  float dot = 0.f;
  for (int j = lane; j < n; j += 64) {
    const int32_t idx = fidx[beg + j];
    if (idx >= 0) dot += fval[beg + j] * W[idx];
  }
  dot = wave_sum(dot);
  if (lane == 0) out[s] = dot;
}

}  // namespace jb

extern "C" int jb_regression_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                   const float* targets, const int64_t* stream_ptr, int nstreams,
                                   float* W, float* stats, float C, float eps, int concurrent,
                                   hipStream_t stream) {
  if (nstreams <= 0) return 0;
  const int threads = 256, blocks = (nstreams * 64 + threads - 1) / threads;
  if (concurrent)
    hipLaunchKernelGGL(jb::regression_train_kernel<true>, dim3(blocks), dim3(threads), 0, stream,
                       row_ptr, fidx, fval, targets, stream_ptr, nstreams, W, stats, C, eps);
  else
    hipLaunchKernelGGL(jb::regression_train_kernel<false>, dim3(blocks), dim3(threads), 0, stream,
                       row_ptr, fidx, fval, targets, stream_ptr, nstreams, W, stats, C, eps);
  return (int)hipGetLastError();
}

extern "C" int jb_regression_estimate(const int64_t* row_ptr, const int32_t* fidx,
                                      const float* fval, int n, const float* W, float* out,
                                      hipStream_t stream) {
  if (n <= 0) return 0;
  const int threads = 256, blocks = (n * 64 + threads - 1) / threads;
  hipLaunchKernelGGL(jb::regression_estimate_kernel, dim3(blocks), dim3(threads), 0, stream,
                     row_ptr, fidx, fval, n, W, out);
  return (int)hipGetLastError();
}
