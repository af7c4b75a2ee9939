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
// Query: pool_rows_kernel scores up to kPoolMaxQ queries in ONE pass over
// the pool. The queries sit in an LDS hash table (feature -> per-query
// values); LPR lanes walk one row's run (LPR = 1 for the short rows of
// structured data, 4 / 16 for text-like rows; chosen by the host from the
// mean run length), probing the table once per entry and accumulating fp64
// dot products, then reduce with DPP and write the cosine similarity /
// euclidean distance [nq][nrows] for the fused top-k (topk.hip). Loads are
// unpredicated (clamped indices) so every lane's requests are in flight at
// once; no cross-lane traffic at all for LPR = 1. For text-like data (n-gram
// features most rows share) a feature-major postings list would touch most
// of the pool anyway and its scattered accumulation costs random atomics; one
// coalesced pass over the pool is the bandwidth-optimal plan.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "jb_device.hpp"

namespace jb {

constexpr int kPoolMaxQ = 8;          // queries per pass
constexpr int kPoolMaxQEntries = 4096;

constexpr int kRowsMaxBlocks = 4096;

__device__ __forceinline__ uint32_t pool_hash(int32_t f) { return (uint32_t)f * 0x9E3779B1u; }

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffff), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// Query sources of the scan. DevQuery: a device CSR (qptr / qidx / qval /
// qn2) or stored rows (qslots: their runs are read from the pool). ArgQuery:
// the latency path - up to kArgSlots normalized query entries (or up to 8
// stored-row slots) travel in the kernel arguments, so a single query needs
// no H2D copy at all.
constexpr int kArgSlots = 320;
struct alignas(16) PoolQArgs {
  int32_t nq, qtot, by_slot, pad;
  int32_t ptr[kPoolMaxQ + 1];
  int32_t slot[kPoolMaxQ];
  double qn2[kPoolMaxQ];
  int32_t idx[kArgSlots];
  float val[kArgSlots];
};

struct DevQuery {
  const int64_t* qptr;
  const int32_t* qidx;
  const float* qval;
  const double* qn2;
  const int32_t* qslots;
  __device__ bool by_slot() const { return qslots != nullptr; }
  __device__ int32_t slot(int q) const { return qslots[q]; }
  __device__ int64_t start(int q) const { return qptr[q]; }
  __device__ int64_t end(int q) const { return qptr[q + 1]; }
  __device__ int64_t base() const { return qptr[0]; }
  __device__ double norm2(int q) const { return qn2[q]; }
  __device__ int32_t f(int64_t i) const { return qidx[i]; }
  __device__ float v(int64_t i) const { return qval[i]; }
};

struct ArgQuery {
  const PoolQArgs& a;
  __device__ bool by_slot() const { return a.by_slot != 0; }
  __device__ int32_t slot(int q) const { return a.slot[q]; }
  __device__ int64_t start(int q) const { return a.ptr[q]; }
  __device__ int64_t end(int q) const { return a.ptr[q + 1]; }
  __device__ int64_t base() const { return 0; }
  __device__ double norm2(int q) const { return a.qn2[q]; }
  __device__ int32_t f(int64_t i) const { return a.idx[i]; }
  __device__ float v(int64_t i) const { return a.val[i]; }
};

// LDS layout (dynamic): keys[T] int32 (-1 = empty) | uid[T] int32 (0 = not
// yet published, else 1 + unique id) | vals[qtot * QM] float.
// T = power of two >= 2 * query entries.
template <int QM, int LPR, class Q>
__device__ __forceinline__ void pool_rows_body(
    const Q& qs, int nq, int qtot, int tbits,
    const int64_t* __restrict__ r_off, const int32_t* __restrict__ r_len,
    const double* __restrict__ r_n2, const uint8_t* __restrict__ valid, int64_t nrows,
    const int32_t* __restrict__ p_idx, const float* __restrict__ p_val, int metric,
    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t s_dyn[];
  const int T = 1 << tbits;
  int32_t* s_key = reinterpret_cast<int32_t*>(s_dyn);
  int32_t* s_uid = s_key + T;
  float* s_vals = reinterpret_cast<float*>(s_uid + T);
  __shared__ int s_nuniq;
  __shared__ int s_ptr[kPoolMaxQ + 1];
  __shared__ int64_t s_off[kPoolMaxQ];
  __shared__ double s_qn2[kPoolMaxQ];
  for (int i = threadIdx.x; i < T; i += blockDim.x) { s_key[i] = -1; s_uid[i] = 0; }
  for (int i = threadIdx.x; i < qtot * QM; i += blockDim.x) s_vals[i] = 0.f;
  if (threadIdx.x == 0) {
    s_nuniq = 0;
    int a = 0;
    for (int q = 0; q < nq; ++q) {
      s_ptr[q] = a;
      if (qs.by_slot()) {   // queries are stored rows: their runs come straight from the pool
        const int32_t sl = qs.slot(q);
        const int l = r_len[sl];
        s_off[q] = r_off[sl];
        s_qn2[q] = r_n2[sl];
        a += l < qtot - a ? l : qtot - a;       // (clamped to the LDS the host sized)
      } else {
        s_off[q] = qs.start(q);
        s_qn2[q] = qs.norm2(q);
        a = (int)(qs.end(q) - qs.base());
      }
    }
    s_ptr[nq] = a;
  }
  __syncthreads();
  // table build: one thread per query entry inserts (feature -> unique id)
  // and adds its value into that id's row of the value table
  for (int e = threadIdx.x; e < s_ptr[nq]; e += blockDim.x) {
    int q = 0;
    while (q + 1 < nq && e >= s_ptr[q + 1]) ++q;
    const int64_t src = s_off[q] + (e - s_ptr[q]);
    const int32_t f = qs.by_slot() ? p_idx[src] : qs.f(src);
    const float v = qs.by_slot() ? p_val[src] : qs.v(src);
    uint32_t h = pool_hash(f) >> (32 - tbits);
    while (true) {
      const int32_t old = atomicCAS(&s_key[h], -1, f);
      if (old == -1) { __atomic_store_n(&s_uid[h], atomicAdd(&s_nuniq, 1) + 1, __ATOMIC_RELAXED); break; }
      if (old == f) break;
      h = (h + 1) & (T - 1);
    }
    int u;
    while ((u = __atomic_load_n(&s_uid[h], __ATOMIC_RELAXED)) == 0) {}
    atomicAdd(&s_vals[(u - 1) * QM + q], v);
  }
  __syncthreads();
  constexpr int kRowsPerBlock = 256 / LPR;
  const int sub = threadIdx.x % LPR;
  for (int64_t base = (int64_t)blockIdx.x * kRowsPerBlock; base < nrows;
       base += (int64_t)gridDim.x * kRowsPerBlock) {
    const int64_t r = base + threadIdx.x / LPR;
    const int64_t rc = r < nrows ? r : nrows - 1;
    // unpredicated metadata loads (clamped row): issued together
    const uint8_t vld = valid[rc];
    const int64_t off = r_off[rc];
    const int len0 = r_len[rc];
    const double b2 = r_n2[rc];
    const bool live = r < nrows && vld;
    const int len = live ? len0 : 0;
    double dot[QM];
#pragma unroll
    for (int q = 0; q < QM; ++q) dot[q] = 0.0;
    for (int j0 = 0; j0 < len; j0 += 4 * LPR) {
      int32_t f[4];
      float v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int j = j0 + k * LPR + sub;
        const int jc = j < len ? j : len - 1;
        f[k] = p_idx[off + jc];
        v[k] = p_val[off + jc];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (j0 + k * LPR + sub >= len) continue;
        uint32_t h = pool_hash(f[k]) >> (32 - tbits);
        int u = -1;
        while (true) {
          const int32_t key = s_key[h];
          if (key == f[k]) { u = s_uid[h] - 1; break; }
          if (key == -1) break;
          h = (h + 1) & (T - 1);
        }
        if (u >= 0) {
#pragma unroll
          for (int q = 0; q < QM; ++q) dot[q] += (double)v[k] * (double)s_vals[u * QM + q];
        }
      }
    }
    if (LPR > 1) {
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        dot[q] += dpp_d<kDppXor1>(dot[q]);
        dot[q] += dpp_d<kDppXor2>(dot[q]);
        if (LPR > 4) {
          dot[q] += dpp_d<kDppHalfMirror>(dot[q]);
          dot[q] += dpp_d<kDppMirror>(dot[q]);
        }
      }
    }
    if (sub == 0 && r < nrows) {
#pragma unroll
      for (int q = 0; q < QM; ++q) {
        if (q >= nq) break;
        float o;
        if (!live) {
          o = metric == 0 ? -INFINITY : INFINITY;
        } else if (metric == 0) {
          const double den = sqrt(s_qn2[q]) * sqrt(b2);
          o = den > 0.0 ? (float)(dot[q] / den) : 0.f;
        } else {
          // dot products and norms in double: the euclidean distance of a row
          // to itself (|q|^2 + |r|^2 - 2 q.r) must cancel to ~0
          o = (float)sqrt(fmax(0.0, s_qn2[q] + b2 - 2.0 * dot[q]));
        }
        out[(int64_t)q * nrows + r] = o;
      }
    }
  }
}

template <int QM, int LPR>
__global__ __launch_bounds__(256) void pool_rows_kernel(
    DevQuery qs, int nq, int qtot, int tbits, const int64_t* __restrict__ r_off,
    const int32_t* __restrict__ r_len, const double* __restrict__ r_n2,
    const uint8_t* __restrict__ valid, int64_t nrows, const int32_t* __restrict__ p_idx,
    const float* __restrict__ p_val, int metric, float* __restrict__ out) {
  pool_rows_body<QM, LPR>(qs, nq, qtot, tbits, r_off, r_len, r_n2, valid, nrows, p_idx, p_val,
                          metric, out);
}

template <int QM, int LPR>
__global__ __launch_bounds__(256) void pool_rows_args_kernel(
    const PoolQArgs a, int tbits, const int64_t* __restrict__ r_off,
    const int32_t* __restrict__ r_len, const double* __restrict__ r_n2,
    const uint8_t* __restrict__ valid, int64_t nrows, const int32_t* __restrict__ p_idx,
    const float* __restrict__ p_val, int metric, float* __restrict__ out) {
  pool_rows_body<QM, LPR>(ArgQuery{a}, a.nq, a.qtot, tbits, r_off, r_len, r_n2, valid, nrows,
                          p_idx, p_val, metric, out);
}

// Append rows. `pack` (one H2D copy) = int64 meta[4 n] (slot, run length,
// squared norm as double bits, run offset within this append) followed by
// int32 feature indices[nnz] and float values[nnz]; row i's run lands at
// pool position base + meta[4 i + 3] and the slot is repointed to it (the
// run it replaces becomes garbage until the host compacts the pool).
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

namespace {
struct ScanGeom {
  int tbits, QM;
  size_t lds;
  unsigned blocks;
};

int scan_geom(int nq, int qtot, int64_t nrows, int lpr, ScanGeom* g) {
  if (nq <= 0 || nq > jb::kPoolMaxQ || qtot < 0 || qtot > jb::kPoolMaxQEntries) return -2;
  if (lpr != 1 && lpr != 4 && lpr != 16) return -2;
  g->tbits = 4;
  while ((1 << g->tbits) < 2 * qtot) ++g->tbits;
  g->QM = nq == 1 ? 1 : nq == 2 ? 2 : nq <= 4 ? 4 : 8;
  g->lds = (size_t)8 * (1 << g->tbits) + (size_t)4 * (qtot > 0 ? qtot : 1) * g->QM;
  if (g->lds > 160 * 1024) return -3;
  const int64_t rpb = 256 / lpr;
  const int64_t want = (nrows + rpb - 1) / rpb;
  g->blocks = (unsigned)(want < jb::kRowsMaxBlocks ? want : jb::kRowsMaxBlocks);
  return 0;
}

#define JB_POOL_DISPATCH(LAUNCH)                                             \
  switch (g.QM * 100 + lpr) {                                                \
    case 101: LAUNCH(1, 1); break;   case 104: LAUNCH(1, 4); break;          \
    case 116: LAUNCH(1, 16); break;  case 201: LAUNCH(2, 1); break;          \
    case 204: LAUNCH(2, 4); break;   case 216: LAUNCH(2, 16); break;         \
    case 401: LAUNCH(4, 1); break;   case 404: LAUNCH(4, 4); break;          \
    case 416: LAUNCH(4, 16); break;  case 801: LAUNCH(8, 1); break;          \
    case 804: LAUNCH(8, 4); break;   default: LAUNCH(8, 16); break;          \
  }
}  // namespace

// scores [nq][nrows] of nq queries (device CSR + qn2 [nq], or stored rows
// by slot) over the pool; lpr: lanes per row (1, 4 or 16)
extern "C" int jb_pool_scan(const int64_t* qptr, const int32_t* qidx, const float* qval,
                            const double* qn2, const int32_t* qslots, int nq, int qtot,
                            const int64_t* r_off, const int32_t* r_len, const double* r_n2,
                            const uint8_t* valid, int64_t nrows, const int32_t* p_idx,
                            const float* p_val, int metric, int lpr, float* out,
                            hipStream_t stream) {
  if (nq <= 0 || nrows <= 0) return 0;
  ScanGeom g;
  int rc = scan_geom(nq, qtot, nrows, lpr, &g);
  if (rc) return rc;
  jb::DevQuery qs{qptr, qidx, qval, qn2, qslots};
#define JB_LAUNCH_DEV(Q, L)                                                                    \
  hipLaunchKernelGGL((jb::pool_rows_kernel<Q, L>), dim3(g.blocks), dim3(256), g.lds, stream, qs, \
                     nq, qtot, g.tbits, r_off, r_len, r_n2, valid, nrows, p_idx, p_val, metric,  \
                     out)
  JB_POOL_DISPATCH(JB_LAUNCH_DEV)
#undef JB_LAUNCH_DEV
  return (int)hipGetLastError();
}

extern "C" int jb_topk_scores_direct(const float* src_d, int flip, int nq, int64_t nrows, int k,
                                     float* scratch_d, int32_t* scratch_i, float* out_d_host,
                                     int32_t* out_i_host, uint32_t* done_host,
                                     hipStream_t stream);   // topk.hip

// Latency path: nq (<= 8) queries given on the host - a CSR of hashed
// features (any order, repeats, idx < 0 dropped: normalized here) or stored
// rows by slot (qslots != nullptr) - scored with the query in the kernel
// arguments, then the exact top-k lands in pinned host memory (out_d /
// out_i, [nq][k]); returns once it is there. 1: the query does not fit the
// kernel arguments (the caller takes the device-CSR path).
extern "C" int jb_pool_query_direct(const int32_t* idx, const float* val, const int64_t* row_ptr,
                                    const int32_t* qslots, const int64_t* slot_len, int nq,
                                    const int64_t* r_off, const int32_t* r_len,
                                    const double* r_n2, const uint8_t* valid, int64_t nrows,
                                    const int32_t* p_idx, const float* p_val, int metric, int lpr,
                                    int k, float* scores, float* scratch_d, int32_t* scratch_i,
                                    float* out_d_host, int32_t* out_i_host, uint32_t* done_host,
                                    hipStream_t stream) {
  if (nq <= 0 || nrows <= 0 || k <= 0) return 0;
  if (nq > jb::kPoolMaxQ) return 1;
  jb::PoolQArgs a;
  a.nq = nq;
  a.pad = 0;
  if (qslots) {
    a.by_slot = 1;
    int64_t tot = 0;
    for (int q = 0; q < nq; ++q) { a.slot[q] = qslots[q]; tot += slot_len[q]; }
    if (tot > jb::kPoolMaxQEntries) return 1;
    a.qtot = (int32_t)tot;
  } else {
    a.by_slot = 0;
    // per query: drop idx < 0, sort by feature (stable), merge repeats
    // (double sum stored as float), squared norm of the stored floats
    int n = 0;
    struct E { int32_t f; float v; int pos; };
    E tmp[jb::kArgSlots];
    for (int q = 0; q < nq; ++q) {
      a.ptr[q] = n;
      int m = 0;
      for (int64_t j = row_ptr[q]; j < row_ptr[q + 1]; ++j) {
        if (idx[j] < 0) continue;
        if (m >= jb::kArgSlots) return 1;
        tmp[m] = {idx[j], val[j], m};
        ++m;
      }
      std::sort(tmp, tmp + m, [](const E& x, const E& y) {
        return x.f < y.f || (x.f == y.f && x.pos < y.pos);
      });
      double sq = 0.0;
      for (int i = 0; i < m;) {
        const int32_t f = tmp[i].f;
        double acc = 0.0;
        while (i < m && tmp[i].f == f) acc += (double)tmp[i++].v;
        if (n >= jb::kArgSlots) return 1;
        const float v32 = (float)acc;
        a.idx[n] = f;
        a.val[n] = v32;
        sq += (double)v32 * (double)v32;
        ++n;
      }
      a.qn2[q] = sq;
    }
    a.ptr[nq] = n;
    a.qtot = n;
  }
  ScanGeom g;
  int rc = scan_geom(nq, a.qtot, nrows, lpr, &g);
  if (rc) return rc;
#define JB_LAUNCH_ARG(Q, L)                                                                     \
  hipLaunchKernelGGL((jb::pool_rows_args_kernel<Q, L>), dim3(g.blocks), dim3(256), g.lds, stream, \
                     a, g.tbits, r_off, r_len, r_n2, valid, nrows, p_idx, p_val, metric, scores)
  JB_POOL_DISPATCH(JB_LAUNCH_ARG)
#undef JB_LAUNCH_ARG
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return jb_topk_scores_direct(scores, metric == 0 ? 1 : 0, nq, nrows, k, scratch_d, scratch_i,
                               out_d_host, out_i_host, done_host, stream);
}
#undef JB_POOL_DISPATCH

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
