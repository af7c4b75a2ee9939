// Exact sparse similarity index on the device (recommender / anomaly
// methods inverted_index = cosine, inverted_index_euclid = euclidean
// distance; nearest_neighbor-style "similar_row" queries).
//
// Reference: recommender_serv.cpp:136-224 (update_row / similar_row_*) and
// anomaly_serv.cpp:157-244 (LOF over inverted_index_euclid) call
// jubatus_core's inverted index (EXTERNAL). Its contract: exact cosine
// similarity / euclidean distance between the query's sparse feature vector
// and every stored row, then the k best.
//
// Storage (HBM, append-only): every stored row is a sorted run of (feature,
// value) pairs in one pool; per slot: offset, length, squared norm, valid.
// A row update appends a new run and repoints the slot (the old run is
// garbage until the host compacts the pool); a removal clears `valid`. No
// host mirror is rebuilt on a write: an update is one small H2D copy plus
// pool_append_kernel.
//
// Query: pool_scan_kernel scores up to kPoolMaxQ queries in ONE pass over
// the pool (the queries sit in LDS - uploaded CSR, or, for queries that are
// stored rows, copied from the pool by slot; each 16-lane group walks one row's run
// with coalesced loads and binary-searches every entry in each query; the
// group sums with DPP), writing [nq][nrows] scores for the fused top-k
// (topk.hip). For text-like data (n-gram features that most rows share) a
// feature-major postings list would touch most of the pool anyway, and its
// scattered score accumulation costs random atomics; one streaming pass over
// the pool is the bandwidth-optimal plan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jb_device.hpp"

namespace jb {

constexpr int kPoolMaxQ = 8;          // queries per pass
constexpr int kPoolMaxQEntries = 4096;

__global__ __launch_bounds__(256) void pool_scan_kernel(
    const int64_t* __restrict__ qptr, const int32_t* __restrict__ qidx,
    const float* __restrict__ qval, const double* __restrict__ qn2_in,
    const int32_t* __restrict__ qslots, int nq,
    const int64_t* __restrict__ r_off, const int32_t* __restrict__ r_len,
    const double* __restrict__ r_n2, const uint8_t* __restrict__ valid, int64_t nrows,
    const int32_t* __restrict__ p_idx, const float* __restrict__ p_val, int metric,
    float* __restrict__ out) {
  __shared__ int32_t s_idx[kPoolMaxQEntries];
  __shared__ float s_val[kPoolMaxQEntries];
  __shared__ int s_ptr[kPoolMaxQ + 1];
  __shared__ double s_qn2[kPoolMaxQ];
  if (qslots) {
    // queries are stored rows: their runs come straight from the pool
    if (threadIdx.x == 0) {
      int acc = 0;
      for (int q = 0; q < nq; ++q) {
        s_ptr[q] = acc;
        acc += r_len[qslots[q]];
      }
      s_ptr[nq] = acc;
    }
    if (threadIdx.x < (unsigned)nq) s_qn2[threadIdx.x] = r_n2[qslots[threadIdx.x]];
    __syncthreads();
    for (int q = 0; q < nq; ++q) {
      const int64_t o = r_off[qslots[q]];
      const int b = s_ptr[q], len = s_ptr[q + 1] - b;
      for (int i = threadIdx.x; i < len; i += blockDim.x) {
        s_idx[b + i] = p_idx[o + i];
        s_val[b + i] = p_val[o + i];
      }
    }
  } else {
    if (threadIdx.x <= (unsigned)nq) s_ptr[threadIdx.x] = (int)(qptr[threadIdx.x] - qptr[0]);
    if (threadIdx.x < (unsigned)nq) s_qn2[threadIdx.x] = qn2_in[threadIdx.x];
    const int qtot = (int)(qptr[nq] - qptr[0]);
    for (int i = threadIdx.x; i < qtot; i += blockDim.x) {
      s_idx[i] = qidx[qptr[0] + i];
      s_val[i] = qval[qptr[0] + i];
    }
  }
  __syncthreads();
  const double* qn2 = s_qn2;
  const int64_t r = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int l16 = threadIdx.x & 15;
  // dot products and norms in double: the euclidean distance of a row to
  // itself (|q|^2 + |r|^2 - 2 q.r) must cancel to ~0, not to fp32 noise
  double dot[kPoolMaxQ];
#pragma unroll
  for (int q = 0; q < kPoolMaxQ; ++q) dot[q] = 0.0;
  const bool live = r < nrows && valid[r];
  if (live) {
    const int64_t off = r_off[r];
    const int len = r_len[r];
    for (int j = l16; j < len; j += 16) {
      const int32_t f = p_idx[off + j];
      const float v = p_val[off + j];
#pragma unroll
      for (int q = 0; q < kPoolMaxQ; ++q) {
        if (q >= nq) break;
        int lo = s_ptr[q], hi = s_ptr[q + 1] - 1;
        while (lo <= hi) {
          const int mid = (lo + hi) >> 1;
          const int32_t x = s_idx[mid];
          if (x == f) { dot[q] += (double)v * (double)s_val[mid]; break; }
          if (x < f) lo = mid + 1; else hi = mid - 1;
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < kPoolMaxQ; ++q) {
    if (q >= nq) break;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) dot[q] += __shfl_xor(dot[q], off, 64);  // one 16-lane row
  }
  if (l16 != 0 || r >= nrows) return;
  const double b2 = live ? r_n2[r] : 0.0;
  for (int q = 0; q < nq; ++q) {
    float o;
    if (!live) {
      o = metric == 0 ? -INFINITY : INFINITY;
    } else if (metric == 0) {
      const double den = sqrt(qn2[q]) * sqrt(b2);
      o = den > 0.0 ? (float)(dot[q] / den) : 0.f;
    } else {
      o = (float)sqrt(fmax(0.0, qn2[q] + b2 - 2.0 * dot[q]));
    }
    out[(int64_t)q * nrows + r] = o;
  }
}

// Append rows. `pack` (one H2D copy) = int64 meta[4 n] (slot, run length,
// squared norm as double bits, run offset within this append) followed by
// int32 feature indices[nnz] and float values[nnz]; row i's run lands at
// pool position base + meta[4 i + 3] and the slot is repointed to it.
__global__ __launch_bounds__(256) void pool_append_kernel(const uint8_t* __restrict__ pack, int n,
                                                          int64_t nnz, int64_t base,
                                                          int64_t* __restrict__ r_off,
                                                          int32_t* __restrict__ r_len,
                                                          double* __restrict__ r_n2,
                                                          uint8_t* __restrict__ valid,
                                                          int32_t* __restrict__ p_idx,
                                                          float* __restrict__ p_val) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t* meta = reinterpret_cast<const int64_t*>(pack);
  const int32_t* fidx = reinterpret_cast<const int32_t*>(pack + 32 * (int64_t)n);
  const float* fval = reinterpret_cast<const float*>(fidx + nnz);
  if (t < nnz) {
    p_idx[base + t] = fidx[t];
    p_val[base + t] = fval[t];
  }
  if (t < n) {
    const int64_t slot = meta[4 * t];
    r_off[slot] = base + meta[4 * t + 3];
    r_len[slot] = (int32_t)meta[4 * t + 1];
    r_n2[slot] = __longlong_as_double((long long)meta[4 * t + 2]);
    valid[slot] = 1;
  }
}

}  // namespace jb

extern "C" int jb_pool_scan(const int64_t* qptr, const int32_t* qidx, const float* qval,
                            const double* qn2, const int32_t* qslots, int nq,
                            const int64_t* r_off, const int32_t* r_len,
                            const double* r_n2, const uint8_t* valid, int64_t nrows,
                            const int32_t* p_idx, const float* p_val, int metric, float* out,
                            hipStream_t stream) {
  if (nq <= 0 || nrows <= 0) return 0;
  if (nq > jb::kPoolMaxQ) return -2;
  const unsigned blocks = (unsigned)((nrows + 15) / 16);
  hipLaunchKernelGGL(jb::pool_scan_kernel, dim3(blocks), dim3(256), 0, stream, qptr, qidx, qval,
                     qn2, qslots, nq, r_off, r_len, r_n2, valid, nrows, p_idx, p_val, metric, out);
  return (int)hipGetLastError();
}

extern "C" int jb_pool_append(const uint8_t* pack, int n, int64_t nnz, int64_t base,
                              int64_t* r_off, int32_t* r_len, double* r_n2, uint8_t* valid,
                              int32_t* p_idx, float* p_val, hipStream_t stream) {
  const int64_t work = nnz > n ? nnz : n;
  if (work <= 0) return 0;
  const unsigned blocks = (unsigned)((work + 255) / 256);
  hipLaunchKernelGGL(jb::pool_append_kernel, dim3(blocks), dim3(256), 0, stream, pack, n, nnz,
                     base, r_off, r_len, r_n2, valid, p_idx, p_val);
  return (int)hipGetLastError();
}
