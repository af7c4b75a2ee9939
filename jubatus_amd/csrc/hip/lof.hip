// LOF state on the device (anomaly engine, method lof / light_lof).
//
// Reference: anomaly_serv.cpp:157-244 (add / update / overwrite / calc_score)
// over jubatus_core's lof_storage (EXTERNAL): per stored row its k nearest
// neighbours, k-distance and local reachability density (Breunig et al.,
// SIGMOD 2000), refreshed for the reverse-nearest-neighbour set of every
// changed row. Semantics (models/lof_state.py, which is also the NumPy
// oracle of these kernels):
//   nb[p]      k nearest rows of p (ascending (distance, slot)), -1 padded
//   kdist[p]   distance to the k-th neighbour (ignore_kth_same_point: the
//              last positive distance of the list)
//   lrd[p]     1 / mean_{x in nb[p]} max(kdist[x], d(p, x))
//   LOF(q)     mean_{o in N_k(q)} lrd[o] / lrd(q)
// Insert of p with its rnn-nearest candidates C (ascending): nb[p] = C[:k];
// every o in C with a valid list takes p into its list if p is closer than
// its current k-th neighbour. Every row whose list changed, and every row
// listing one of them, gets lrd_ok = 0 (lof_mark_kernel, one pass over the
// lists). Rows without a valid list (bulk-loaded, or listing a row that
// moved) get one on demand: the score kernel reports them as missing, the
// host queries their neighbours and lof_set_lists_kernel installs them (and
// lof_mark_kernel then marks the rows listing them stale). An lrd counts as
// current only while every row of its list has a valid list.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "jb_device.hpp"
#include "jb_host_wait.hpp"

namespace jb {

constexpr int kLofMaxK = 64;
constexpr int kLofMaxChanged = 1024;

__device__ __forceinline__ float lof_kth(const int32_t* s, const float* d, int k, int ignore_same) {
  float kd = 0.f;
  for (int j = 0; j < k; ++j) {
    if (s[j] < 0) break;
    if (!ignore_same || d[j] > 0.f) kd = d[j];
  }
  return kd;
}

// Candidate / target lists travel in the kernel arguments (latency path:
// no H2D copy): up to kLofArgMax (slot, distance) pairs.
constexpr int kLofArgMax = 128;
struct LofArgs {
  int32_t n, pad;
  int32_t s[kLofArgMax];
  float d[kLofArgMax];
};

// p's list from its candidates; candidates o take p in. One block of 64
// threads; each thread's working copy of a list sits in LDS.
__device__ __forceinline__ void lof_insert_body(
    int p, const int32_t* __restrict__ cs, const float* __restrict__ cd, int nc, int k,
    int ignore_same, int32_t* __restrict__ nb_slot, float* __restrict__ nb_dist,
    float* __restrict__ kdist, uint8_t* __restrict__ ok, uint8_t* __restrict__ lrd_ok,
    int32_t* __restrict__ changed, int32_t* __restrict__ nchanged, bool first = true) {
  __shared__ int n_ch;
  __shared__ int32_t l_s[64][kLofMaxK];
  __shared__ float l_d[64][kLofMaxK];
  if (threadIdx.x == 0 && !first) n_ch = *nchanged;   // a later chunk of candidates: reverse inserts only
  if (threadIdx.x == 0 && first) {
    n_ch = 0;
    int32_t* ps = nb_slot + (int64_t)p * k;
    float* pd = nb_dist + (int64_t)p * k;
    for (int j = 0; j < k; ++j) {
      ps[j] = j < nc ? cs[j] : -1;
      pd[j] = j < nc ? cd[j] : INFINITY;
    }
    kdist[p] = lof_kth(ps, pd, k, ignore_same);
    ok[p] = 1;
    lrd_ok[p] = 0;
    changed[0] = p;
    n_ch = 1;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nc; i += blockDim.x) {
    const int32_t o = cs[i];
    const float d = cd[i];
    if (o < 0 || o == p || !ok[o]) continue;
    int32_t* os = nb_slot + (int64_t)o * k;
    float* od = nb_dist + (int64_t)o * k;
    int32_t* ts = l_s[threadIdx.x];
    float* td = l_d[threadIdx.x];
    int n = 0;
    bool had = false;
    for (int j = 0; j < k; ++j) {            // o's list without p
      if (os[j] < 0) break;
      if (os[j] == p) { had = true; continue; }
      ts[n] = os[j];
      td[n] = od[j];
      ++n;
    }
    const bool full = n == k;
    if (!had && full && !(d < td[k - 1] || (d == td[k - 1] && p < ts[k - 1]))) continue;
    int at = n;                               // insert (d, p) in (distance, slot) order
    while (at > 0 && (td[at - 1] > d || (td[at - 1] == d && ts[at - 1] > p))) --at;
    for (int j = (n < k ? n : k - 1); j > at; --j) { ts[j] = ts[j - 1]; td[j] = td[j - 1]; }
    if (at < k) { ts[at] = p; td[at] = d; }
    const int m = n < k ? n + 1 : k;
    for (int j = 0; j < k; ++j) {
      os[j] = j < m ? ts[j] : -1;
      od[j] = j < m ? td[j] : INFINITY;
    }
    kdist[o] = lof_kth(os, od, k, ignore_same);
    lrd_ok[o] = 0;
    const int w = atomicAdd(&n_ch, 1);
    if (w < kLofMaxChanged) changed[w] = o;
  }
  __syncthreads();
  if (threadIdx.x == 0) *nchanged = n_ch < kLofMaxChanged ? n_ch : kLofMaxChanged;
}

__global__ __launch_bounds__(64) void lof_add_kernel(
    const LofArgs a, int p, int k, int ignore_same, int32_t* __restrict__ nb_slot,
    float* __restrict__ nb_dist, float* __restrict__ kdist, uint8_t* __restrict__ ok,
    uint8_t* __restrict__ lrd_ok, int32_t* __restrict__ changed, int32_t* __restrict__ nchanged,
    int first, const int32_t* __restrict__ abort_flag = nullptr) {
  if (abort_flag != nullptr && *abort_flag != 0) return;   // an earlier add of the batch stopped it
  __shared__ int32_t cs[kLofArgMax];
  __shared__ float cd[kLofArgMax];
  for (int i = threadIdx.x; i < a.n; i += blockDim.x) { cs[i] = a.s[i]; cd[i] = a.d[i]; }
  __syncthreads();
  lof_insert_body(p, cs, cd, a.n, k, ignore_same, nb_slot, nb_dist, kdist, ok, lrd_ok, changed,
                  nchanged, first != 0);
}

// Every row listing a changed row: lrd_ok = 0 (and, clear_ok: ok = 0 -
// its list must be recomputed, e.g. the listed row moved or was removed).
__global__ __launch_bounds__(256) void lof_mark_kernel(int64_t nrows, int k,
                                                       const int32_t* __restrict__ nb_slot,
                                                       const int32_t* __restrict__ changed,
                                                       const int32_t* __restrict__ nchanged,
                                                       int clear_ok, uint8_t* __restrict__ ok,
                                                       uint8_t* __restrict__ lrd_ok,
                                                       const int32_t* __restrict__ abort_flag = nullptr) {
  if (abort_flag != nullptr && *abort_flag != 0) return;
  __shared__ int32_t tab[2 * kLofMaxChanged];
  const int nch = *nchanged;
  for (int i = threadIdx.x; i < 2 * kLofMaxChanged; i += blockDim.x) tab[i] = -1;
  __syncthreads();
  for (int i = threadIdx.x; i < nch; i += blockDim.x) {
    const int32_t c = changed[i];
    uint32_t h = ((uint32_t)c * 0x9E3779B1u) >> 21;
    while (true) {
      const int32_t old = atomicCAS(&tab[h], -1, c);
      if (old == -1 || old == c) break;
      h = (h + 1) & (2 * kLofMaxChanged - 1);
    }
  }
  __syncthreads();
  const int64_t y = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= nrows || !ok[y]) return;
  const int32_t* ys = nb_slot + y * k;
  for (int j = 0; j < k; ++j) {
    const int32_t x = ys[j];
    if (x < 0) break;
    uint32_t h = ((uint32_t)x * 0x9E3779B1u) >> 21;
    bool hit = false;
    while (true) {
      const int32_t t = tab[h];
      if (t == x) { hit = true; break; }
      if (t == -1) break;
      h = (h + 1) & (2 * kLofMaxChanged - 1);
    }
    if (hit) {
      lrd_ok[y] = 0;
      if (clear_ok) ok[y] = 0;
      return;
    }
  }
}

// Install freshly queried neighbour lists (kk candidates per row, ascending,
// may include the row itself). One thread per row.
__global__ __launch_bounds__(256) void lof_set_lists_kernel(
    int n, const int32_t* __restrict__ slots, const int32_t* __restrict__ cs,
    const float* __restrict__ cd, int kk, int k, int ignore_same, int32_t* __restrict__ nb_slot,
    float* __restrict__ nb_dist, float* __restrict__ kdist, uint8_t* __restrict__ ok,
    uint8_t* __restrict__ lrd_ok, int32_t* __restrict__ changed, int32_t* __restrict__ nchanged) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) *nchanged = n < kLofMaxChanged ? n : kLofMaxChanged;
  if (i >= n) return;
  const int32_t s = slots[i];
  int32_t* os = nb_slot + (int64_t)s * k;
  float* od = nb_dist + (int64_t)s * k;
  int m = 0;
  for (int j = 0; j < kk && m < k; ++j) {
    const int32_t o = cs[(int64_t)i * kk + j];
    if (o < 0 || o == s) continue;
    os[m] = o;
    od[m] = cd[(int64_t)i * kk + j];
    ++m;
  }
  for (int j = m; j < k; ++j) { os[j] = -1; od[j] = INFINITY; }
  kdist[s] = lof_kth(os, od, k, ignore_same);
  ok[s] = 1;
  lrd_ok[s] = 0;
  if (i < kLofMaxChanged) changed[i] = s;
}

__device__ __forceinline__ float lof_lrd(const int32_t* s, const float* d, int k,
                                         const float* __restrict__ kdist) {
  float sum = 0.f;
  int n = 0;
  for (int j = 0; j < k; ++j) {
    if (s[j] < 0) break;
    sum += fmaxf(kdist[s[j]], d[j]);
    ++n;
  }
  if (n == 0) return 0.f;
  const float mean = sum / n;
  return mean <= 0.f ? INFINITY : 1.f / mean;
}

// LOF of one point from its neighbours (ts, td: nt entries, ascending):
// refreshes the stale lrd of those neighbours, writes to pinned host memory
// out = [status, score bits, lrd(q) bits, nmissing, missing slots...]:
// (status published last, by system-scope stores) status 1 = done,
// 2 = rows without a valid list (missing) - the host
// installs their lists and runs the kernel again. One block.
__device__ __forceinline__ void lof_score_body(
    const int32_t* __restrict__ ts, const float* __restrict__ td, int nt, int k,
    const int32_t* __restrict__ nb_slot, const float* __restrict__ nb_dist,
    const float* __restrict__ kdist, const uint8_t* __restrict__ ok, float* __restrict__ lrd,
    uint8_t* __restrict__ lrd_ok, int store_slot, uint32_t* __restrict__ out, int max_missing,
    int32_t* __restrict__ abort_flag = nullptr) {
  __shared__ int nmiss;
  if (threadIdx.x == 0) nmiss = 0;
  __syncthreads();
  const int t = threadIdx.x;
  auto miss = [&](int32_t s) {
    const int w = atomicAdd(&nmiss, 1);
    if (w < max_missing) sys_store(out + 4 + w, (uint32_t)s);
  };
  if (t < nt) {
    const int32_t o = ts[t];
    if (!ok[o]) {
      miss(o);
    } else {
      // lrd[o] is current only while every row o lists has a valid list
      const int32_t* os = nb_slot + (int64_t)o * k;
      bool good = true;
      for (int j = 0; j < k; ++j) {
        if (os[j] < 0) break;
        if (!ok[os[j]]) { miss(os[j]); good = false; }
      }
      if (good && !lrd_ok[o]) {
        lrd[o] = lof_lrd(os, nb_dist + (int64_t)o * k, k, kdist);
        lrd_ok[o] = 1;
      }
    }
  }
  // the host reads out[] once out[0] is set: every thread's system-scope
  // stores are acknowledged before the barrier, the status goes last (a
  // system-scope release fence would write back the whole L2 instead)
  sys_stores_block_done();
  if (t != 0) return;
  if (nmiss > 0) {
    // a batch of adds stops here: the host installs the missing lists and
    // scores this add again before the later ones run (sequential order)
    if (abort_flag != nullptr) *abort_flag = 1;
    sys_store(out + 3, (uint32_t)(nmiss < max_missing ? nmiss : max_missing));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sys_store(out, 2u);
    return;
  }
  // lrd of the query point itself (its own neighbours' k-distances)
  float sum = 0.f, lsum = 0.f;
  bool linf = false;
  for (int j = 0; j < nt; ++j) {
    sum += fmaxf(kdist[ts[j]], td[j]);
    const float l = lrd[ts[j]];
    if (isinf(l)) linf = true; else lsum += l;
  }
  float score = 1.f, lp = 0.f;
  if (nt > 0) {
    const float mean = sum / nt;
    lp = mean <= 0.f ? INFINITY : 1.f / mean;
    const float mean_lo = linf ? INFINITY : lsum / nt;
    if (isinf(lp)) score = isinf(mean_lo) ? 1.f : 0.f;
    else if (lp == 0.f) score = INFINITY;
    else if (isinf(mean_lo)) score = INFINITY;
    else score = mean_lo / lp;
  }
  if (store_slot >= 0) { lrd[store_slot] = lp; lrd_ok[store_slot] = 1; }
  sys_store(out + 1, __float_as_uint(score));
  sys_store(out + 2, __float_as_uint(lp));
  sys_store(out + 3, 0u);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sys_store(out, 1u);
}

__global__ __launch_bounds__(64) void lof_score_kernel(
    const LofArgs a, int k, const int32_t* __restrict__ nb_slot,
    const float* __restrict__ nb_dist, const float* __restrict__ kdist,
    const uint8_t* __restrict__ ok, float* __restrict__ lrd, uint8_t* __restrict__ lrd_ok,
    int store_slot, uint32_t* __restrict__ out, int max_missing,
    int32_t* __restrict__ abort_flag = nullptr) {
  if (abort_flag != nullptr && *abort_flag != 0) {   // skipped: an earlier add stopped the batch
    if (threadIdx.x == 0) sys_store(out, 3u);
    return;
  }
  __shared__ int32_t ts[kLofMaxK];
  __shared__ float td[kLofMaxK];
  const int nt = a.n < kLofMaxK ? a.n : kLofMaxK;
  if ((int)threadIdx.x < nt) { ts[threadIdx.x] = a.s[threadIdx.x]; td[threadIdx.x] = a.d[threadIdx.x]; }
  __syncthreads();
  lof_score_body(ts, td, nt, k, nb_slot, nb_dist, kdist, ok, lrd, lrd_ok, store_slot, out,
                 max_missing, abort_flag);
}

}  // namespace jb

extern "C" int jb_lof_mark(int64_t nrows, int k, const int32_t* nb_slot, const int32_t* changed,
                           const int32_t* nchanged, int clear_ok, uint8_t* ok, uint8_t* lrd_ok,
                           hipStream_t stream) {
  if (nrows <= 0) return 0;
  const unsigned blocks = (unsigned)((nrows + 255) / 256);
  hipLaunchKernelGGL(jb::lof_mark_kernel, dim3(blocks), dim3(256), 0, stream, nrows, k, nb_slot,
                     changed, nchanged, clear_ok, ok, lrd_ok);
  return (int)hipGetLastError();
}

extern "C" int jb_lof_set_lists(int n, const int32_t* slots, const int32_t* cs, const float* cd,
                                int kk, int k, int ignore_same, int32_t* nb_slot, float* nb_dist,
                                float* kdist, uint8_t* ok, uint8_t* lrd_ok, int32_t* changed,
                                int32_t* nchanged, hipStream_t stream) {
  if (n <= 0) return 0;
  if (k <= 0 || k > jb::kLofMaxK || n > jb::kLofMaxChanged) return -2;
  hipLaunchKernelGGL(jb::lof_set_lists_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, n,
                     slots, cs, cd, kk, k, ignore_same, nb_slot, nb_dist, kdist, ok, lrd_ok,
                     changed, nchanged);
  return (int)hipGetLastError();
}

namespace {
int fill_args(jb::LofArgs* a, const int32_t* sl, const float* d, int n) {
  if (n < 0 || n > jb::kLofArgMax) return -2;
  a->n = n;
  a->pad = 0;
  for (int i = 0; i < n; ++i) { a->s[i] = sl[i]; a->d[i] = d[i]; }
  return 0;
}
}  // namespace

// One LOF add on the device (latency path): the candidates (rnn nearest of
// p, ascending, p excluded; host arrays) go in the kernel arguments; p's
// list is written and p enters its candidates' lists (lof_add_kernel), the
// rows depending on a changed list are marked (lof_mark_kernel), then p is
// scored from its k nearest (lof_score_kernel, lrd[p] stored). Waits for
// the score; out_host = [status, score, lrd, nmissing, missing...].
extern "C" int jb_lof_add(int p, const int32_t* cs, const float* cd, int nc, int k,
                          int ignore_same, int64_t nrows, int32_t* nb_slot, float* nb_dist,
                          float* kdist, uint8_t* ok, float* lrd, uint8_t* lrd_ok,
                          int32_t* changed, int32_t* nchanged, uint32_t* out_host,
                          int max_missing, hipStream_t stream) {
  if (k <= 0 || k > jb::kLofMaxK || nc < 0) return -2;
  // the candidates travel in the kernel arguments, kLofArgMax per launch: the
  // first launch sets p's own list (its k nearest are the head of the first
  // chunk) and the reverse inserts of that chunk, later ones (a
  // reverse_nearest_neighbor_num above the argument budget) only insert p
  // into their candidates' lists
  jb::LofArgs a;
  for (int c0 = 0; c0 == 0 || c0 < nc; c0 += jb::kLofArgMax) {
    const int cn = nc - c0 < jb::kLofArgMax ? nc - c0 : jb::kLofArgMax;
    int rc = fill_args(&a, cs + c0, cd + c0, cn < 0 ? 0 : cn);
    if (rc) return rc;
    hipLaunchKernelGGL(jb::lof_add_kernel, dim3(1), dim3(64), 0, stream, a, p, k, ignore_same,
                       nb_slot, nb_dist, kdist, ok, lrd_ok, changed, nchanged, c0 == 0 ? 1 : 0);
  }
  int rc = fill_args(&a, cs, cd, nc < jb::kLofArgMax ? nc : jb::kLofArgMax);
  if (rc) return rc;
  const unsigned blocks = (unsigned)((nrows + 255) / 256);
  hipLaunchKernelGGL(jb::lof_mark_kernel, dim3(blocks), dim3(256), 0, stream, nrows, k, nb_slot,
                     changed, nchanged, 0, ok, lrd_ok);
  a.n = nc < k ? nc : k;               // score from the k nearest
  out_host[0] = 0;
  hipLaunchKernelGGL(jb::lof_score_kernel, dim3(1), dim3(64), 0, stream, a, k, nb_slot, nb_dist,
                     kdist, ok, lrd, lrd_ok, p, out_host, max_missing);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return jb::wait_nonzero(out_host, stream);
}

// A batch of adds in arrival order, one wait: add i's kernels (insert,
// mark, score into out_host + i * out_stride) are enqueued behind add i - 1's
// without a host round trip. An add whose score finds rows without a valid
// list sets *abort_dev; every later kernel of the batch then exits (status 3)
// and the host finishes that add (missing lists installed, scored again)
// before it resubmits the rest - the order of the sequential adds.
// cs / cd: [nadd][stride] candidates (ascending, p excluded), nc[i] of them.
extern "C" int jb_lof_add_many(int nadd, const int32_t* ps, const int32_t* cs, const float* cd,
                               const int32_t* nc, int stride, int k, int ignore_same, int64_t nrows,
                               int32_t* nb_slot, float* nb_dist, float* kdist, uint8_t* ok, float* lrd,
                               uint8_t* lrd_ok, int32_t* changed, int32_t* nchanged, uint32_t* out_host,
                               int out_stride, int max_missing, int32_t* abort_dev, hipStream_t stream) {
  if (nadd <= 0) return 0;
  if (k <= 0 || k > jb::kLofMaxK || stride > jb::kLofArgMax) return -2;
  hipError_t e = hipMemsetAsync(abort_dev, 0, sizeof(int32_t), stream);
  if (e != hipSuccess) return (int)e;
  const unsigned blocks = (unsigned)((nrows + 255) / 256);
  for (int i = 0; i < nadd; ++i) out_host[(int64_t)i * out_stride] = 0;
  jb::LofArgs a;
  for (int i = 0; i < nadd; ++i) {
    const int n = nc[i];
    int rc = fill_args(&a, cs + (int64_t)i * stride, cd + (int64_t)i * stride, n < 0 ? 0 : n);
    if (rc) return rc;
    hipLaunchKernelGGL(jb::lof_add_kernel, dim3(1), dim3(64), 0, stream, a, ps[i], k, ignore_same, nb_slot,
                       nb_dist, kdist, ok, lrd_ok, changed, nchanged, 1, (const int32_t*)abort_dev);
    hipLaunchKernelGGL(jb::lof_mark_kernel, dim3(blocks), dim3(256), 0, stream, nrows, k, nb_slot, changed,
                       nchanged, 0, ok, lrd_ok, (const int32_t*)abort_dev);
    a.n = n < k ? n : k;
    hipLaunchKernelGGL(jb::lof_score_kernel, dim3(1), dim3(64), 0, stream, a, k, nb_slot, nb_dist, kdist, ok,
                       lrd, lrd_ok, ps[i], out_host + (int64_t)i * out_stride, max_missing, abort_dev);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return jb::wait_nonzero(out_host + (int64_t)(nadd - 1) * out_stride, stream);
}

// LOF of a point from its nt (<= 64) nearest (host arrays), lrd of the
// targets refreshed; waits; same out_host layout
extern "C" int jb_lof_score(const int32_t* ts, const float* td, int nt, int k,
                            const int32_t* nb_slot, const float* nb_dist, const float* kdist,
                            const uint8_t* ok, float* lrd, uint8_t* lrd_ok, int store_slot,
                            uint32_t* out_host, int max_missing, hipStream_t stream) {
  if (nt > 64 || k > jb::kLofMaxK) return -2;
  jb::LofArgs a;
  int rc = fill_args(&a, ts, td, nt);
  if (rc) return rc;
  out_host[0] = 0;
  hipLaunchKernelGGL(jb::lof_score_kernel, dim3(1), dim3(64), 0, stream, a, k, nb_slot, nb_dist,
                     kdist, ok, lrd, lrd_ok, store_slot, out_host, max_missing);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return jb::wait_nonzero(out_host, stream);
}

namespace jb {
// rows that changed or were removed: their list and lrd are no longer valid
// (models/lof_state.py DeviceLofState.moved: ok[s] = lrd_ok[s] = 0)
__global__ void lof_invalidate_kernel(const int32_t* __restrict__ slots, int n, int64_t nrows,
                                      uint8_t* __restrict__ ok, uint8_t* __restrict__ lrd_ok) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t s = slots[i];
  if (s < 0 || s >= nrows) return;
  ok[s] = 0;
  lrd_ok[s] = 0;
}
}  // namespace jb

extern "C" int jb_lof_invalidate(const int32_t* slots, int n, int64_t nrows, uint8_t* ok,
                                 uint8_t* lrd_ok, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(jb::lof_invalidate_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, slots,
                     n, nrows, ok, lrd_ok);
  return (int)hipGetLastError();
}
