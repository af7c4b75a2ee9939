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
constexpr int kLofU = 8;                // cooperative loads in flight per thread
constexpr int kLofKR = 16;              // k up to this: list edits and scores in registers

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

// LDS of the insert and score bodies (one block of 64 threads; a kernel
// running both shares one copy): per candidate / target row its list, the
// distances, its rows' k-distances and list flags; +1 per row so that the
// 64 threads' rows start on different banks
struct LofLds {
  int32_t s[64][kLofMaxK + 1];
  float d[64][kLofMaxK + 1];
  float kd[64][kLofMaxK + 1];
  uint8_t okb[64][kLofMaxK + 1];
  uint8_t ok1[64], stale[64], lok1[64], chg[64];
  float kd1[64], lrd1[64], lr1[64];
  uint32_t lst[64];
  int n_ch, nmiss;
  bool prof;                      // phase stamps on (lof_add_batch_kernel, prof != nullptr)
  unsigned long long ph[8], tlast;
};

// The insert / score bodies run in one-wave blocks (every launch is 64
// threads): lanes exchange LDS data after their LDS operations complete -
// no barrier, and no wait for the global stores in flight (a __syncthreads
// fence waits for every store's acknowledgement, ~1-2 us after scattered
// row writes). __syncthreads stays where a later global load depends on
// another lane's global store.
__device__ __forceinline__ void lof_lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// e / k for the flattened (row, entry) indices of a round (e < 2^16, k <= 64):
// one multiply-high by ceil(2^32 / k) instead of an integer division's ~25
// instructions (exact while e * k < 2^32)
__device__ __forceinline__ uint32_t lof_kinv(int k) { return (uint32_t)((0x100000000ull + k - 1) / k); }
__device__ __forceinline__ int lof_div(int e, uint32_t kinv) { return (int)__umulhi((uint32_t)e, kinv); }

// phase stamp i (shader cycles since the previous stamp), lane 0, when on
__device__ __forceinline__ void lof_stamp(LofLds& L, int i) {
  if (!L.prof) return;
  const unsigned long long t = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    L.ph[i] += t - L.tlast;
    L.tlast = t;
  }
}

// Staleness stamps (optional, kstamp / lstamp non-null): kstamp[x] = the add
// epoch that last changed x's list / k-distance, lstamp[o] = the epoch lrd[o]
// was computed at; lrd[o] is current only while lrd_ok[o] and every row x it
// lists has kstamp[x] <= lstamp[o]. With stamps an add needs no mark pass over
// every list (lof_add_score_kernel: insert and score in one launch).
// p's list from its candidates; candidates o take p in. One block of 64
// threads. The candidates' lists are fetched cooperatively first (every
// (candidate, entry) load of a round of 64 candidates in flight at once, one
// memory latency instead of k dependent ones per thread), then each thread
// edits its candidate's copy in LDS and writes it back.
__device__ __forceinline__ void lof_insert_body(
    int p, const int32_t* __restrict__ cs, const float* __restrict__ cd, int nc, int k,
    int ignore_same, int32_t* __restrict__ nb_slot, float* __restrict__ nb_dist,
    float* __restrict__ kdist, uint8_t* __restrict__ ok, uint8_t* __restrict__ lrd_ok,
    int32_t* __restrict__ changed, int32_t* __restrict__ nchanged, bool first, LofLds& L,
    uint32_t* __restrict__ kstamp = nullptr, uint32_t epoch = 0, const float* __restrict__ lrd = nullptr,
    const uint32_t* __restrict__ lstamp = nullptr) {
  // fused (lrd non-null, nc <= 64): candidate c's fields the score needs -
  // ok, lrd_ok, lrd, kdist, lstamp, as they stand after this insert - are
  // left in L (ok1, lok1, lr1, kd1, lst) and its list in L.s / L.d[c]: the
  // score of p (its targets are the head of the candidates) reads them there
  const bool fused = lrd != nullptr;
  int& n_ch = L.n_ch;
  auto& l_s = L.s;
  auto& l_d = L.d;
  uint8_t* l_ok = L.ok1;
  const int t = threadIdx.x;
  const uint32_t kinv = lof_kinv(k);
  if (t == 0 && !first) n_ch = *nchanged;   // a later chunk of candidates: reverse inserts only
  if (t == 0 && first) {
    int32_t* ps = nb_slot + (int64_t)p * k;
    float* pd = nb_dist + (int64_t)p * k;
    for (int j = 0; j < k; ++j) {
      ps[j] = j < nc ? cs[j] : -1;
      pd[j] = j < nc ? cd[j] : INFINITY;
    }
    kdist[p] = lof_kth(cs, cd, nc < k ? nc : k, ignore_same);
    ok[p] = 1;
    lrd_ok[p] = 0;
    if (kstamp != nullptr) kstamp[p] = epoch;
    changed[0] = p;
    n_ch = 1;
  }
  for (int c0 = 0; c0 < nc; c0 += 64) {
    const int cn = nc - c0 < 64 ? nc - c0 : 64;
    // the candidate's own flags first (issued with the list loads below)
    uint8_t f_ok = 0, f_lok = 0;
    float f_lr = 0.f, f_kd = 0.f;
    uint32_t f_lst = 0;
    if (t < cn) {
      const int32_t o = cs[c0 + t];
      const int32_t oc = o >= 0 ? o : p;
      f_ok = ok[oc];
      if (fused) {
        f_lok = lrd_ok[oc];
        f_lr = lrd[oc];
        f_kd = kdist[oc];
        f_lst = lstamp != nullptr ? lstamp[oc] : 0u;
      }
      if (o < 0 || o == p) f_ok = 0;
    }
    // kLofU loads of each array in flight per thread before the first LDS
    // store (a load -> store loop waits one memory latency per entry)
    for (int e0 = t; e0 < cn * k; e0 += 64 * kLofU) {
      int32_t vs[kLofU];
      float vd[kLofU];
#pragma unroll
      for (int u = 0; u < kLofU; ++u) {
        const int e = e0 + 64 * u;
        const int c = e < cn * k ? lof_div(e, kinv) : 0, j = e - c * k;
        const int32_t o = cs[c0 + c];
        const int64_t at = (int64_t)(o >= 0 ? o : p) * k + (e < cn * k ? j : 0);
        vs[u] = nb_slot[at];
        vd[u] = nb_dist[at];
      }
#pragma unroll
      for (int u = 0; u < kLofU; ++u) {
        const int e = e0 + 64 * u;
        if (e < cn * k) {
          const int c = lof_div(e, kinv), j = e - c * k;
          l_s[c][j] = vs[u];
          l_d[c][j] = vd[u];
        }
      }
    }
    if (t < cn) {
      L.chg[t] = 0;
      l_ok[t] = f_ok;
      if (fused) { L.lok1[t] = f_lok; L.lr1[t] = f_lr; L.kd1[t] = f_kd; L.lst[t] = f_lst; }
    }
    lof_lds_sync();
    lof_stamp(L, 1);
    if (t < cn && l_ok[t]) {
      const int32_t o = cs[c0 + t];
      const float d = cd[c0 + t];
      int32_t* ts = l_s[t];
      float* td = l_d[t];
      bool upd = false;
      float kd = 0.f;
      if (k <= kLofKR) {
        // in registers (static indices throughout): a list edit of dependent
        // LDS round trips costs ~10 K cycles per add, this ~a few hundred
        int32_t rs[kLofKR];
        float rd[kLofKR];
#pragma unroll
        for (int j = 0; j < kLofKR; ++j) {      // unconditional reads (rows hold kLofMaxK + 1), then masks
          const int32_t vs = ts[j];
          const float vd = td[j];
          rs[j] = j < k ? vs : -1;
          rd[j] = j < k ? vd : INFINITY;
        }
        // o's list without p (lists are sorted, -1 padded at the end)
        bool had = false;
#pragma unroll
        for (int j = 0; j < kLofKR; ++j) {
          had |= rs[j] == p;
          rs[j] = had ? (j + 1 < kLofKR ? rs[j + 1] : -1) : rs[j];
          rd[j] = had ? (j + 1 < kLofKR ? rd[j + 1] : INFINITY) : rd[j];
        }
        int n = 0, at = 0;
        int32_t ls = -1;
        float ld = INFINITY;
#pragma unroll
        for (int j = 0; j < kLofKR; ++j) {
          const bool v = j < k && rs[j] >= 0;
          n += v;
          at += v && (rd[j] < d || (rd[j] == d && rs[j] < p));
          if (j == k - 1) { ls = rs[j]; ld = rd[j]; }
        }
        upd = had || n < k || d < ld || (d == ld && p < ls);
        if (upd) {
          const int m = n < k ? n + 1 : k;
#pragma unroll
          for (int j = kLofKR - 1; j >= 0; --j) {
            // insert (d, p) at `at`: later entries move up one
            const int32_t sj = j < at ? rs[j] : (j == at ? p : (j > 0 ? rs[j - 1] : -1));
            const float dj = j < at ? rd[j] : (j == at ? d : (j > 0 ? rd[j - 1] : INFINITY));
            rs[j] = j < m ? sj : -1;
            rd[j] = j < m ? dj : INFINITY;
          }
#pragma unroll
          for (int j = 0; j < kLofKR; ++j) {
            if (j < k) { ts[j] = rs[j]; td[j] = rd[j]; }
            if (j < k && rs[j] >= 0 && (!ignore_same || rd[j] > 0.f)) kd = rd[j];
          }
        }
      } else {
        int n = 0;
        bool had = false;
        for (int j = 0; j < k; ++j) {          // o's list without p (compacted in place)
          const int32_t x = ts[j];
          if (x < 0) break;
          if (x == p) { had = true; continue; }
          ts[n] = x;
          td[n] = td[j];
          ++n;
        }
        const bool full = n == k;
        upd = had || !full || d < td[k - 1] || (d == td[k - 1] && p < ts[k - 1]);
        if (upd) {
          int at = n;                             // insert (d, p) in (distance, slot) order
          while (at > 0 && (td[at - 1] > d || (td[at - 1] == d && ts[at - 1] > p))) --at;
          for (int j = (n < k ? n : k - 1); j > at; --j) { ts[j] = ts[j - 1]; td[j] = td[j - 1]; }
          if (at < k) { ts[at] = p; td[at] = d; }
          const int m = n < k ? n + 1 : k;
          for (int j = m; j < k; ++j) { ts[j] = -1; td[j] = INFINITY; }
          kd = lof_kth(ts, td, k, ignore_same);
        }
      }
      if (upd) {
        L.chg[t] = 1;                           // written back below, row by row
        kdist[o] = kd;
        lrd_ok[o] = 0;
        if (kstamp != nullptr) kstamp[o] = epoch;
        if (fused) { L.kd1[t] = kd; L.lok1[t] = 0; }
        const int w = atomicAdd(&n_ch, 1);
        if (w < kLofMaxChanged) changed[w] = o;
      }
    }
    lof_lds_sync();
    lof_stamp(L, 2);
    // the changed lists back to HBM, consecutive lanes on consecutive entries
    // of a row (a lane per row would touch 64 rows per store instruction)
    for (int e = t; e < cn * k; e += 64) {
      const int c = lof_div(e, kinv), j = e - c * k;
      if (L.chg[c]) {
        const int64_t at = (int64_t)cs[c0 + c] * k + j;
        nb_slot[at] = l_s[c][j];
        nb_dist[at] = l_d[c][j];
      }
    }
    __syncthreads();
    lof_stamp(L, 3);
  }
  if (t == 0) *nchanged = n_ch < kLofMaxChanged ? n_ch : kLofMaxChanged;
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
  lof_lds_sync();
  __shared__ LofLds L;
  lof_insert_body(p, cs, cd, a.n, k, ignore_same, nb_slot, nb_dist, kdist, ok, lrd_ok, changed,
                  nchanged, first != 0, L);
}

// Every row listing a changed row: lrd_ok = 0 (and, clear_ok: ok = 0 -
// its list must be recomputed, e.g. the listed row moved or was removed).
// The lists are read as one flat array, 8 entries a thread (two 16-byte
// loads, coalesced); the changed rows sit in an LDS hash table sized to
// their count. Rows without a valid list may be marked too: harmless, their
// lrd is not used before their list is installed (which resets both flags).
constexpr int kMarkPer = 8;
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
  int bits = 6;
  while ((1 << bits) < 2 * nch) ++bits;
  const uint32_t mask = (1u << bits) - 1u;
  for (int i = threadIdx.x; i <= (int)mask; i += blockDim.x) tab[i] = -1;
  __syncthreads();
  for (int i = threadIdx.x; i < nch; i += blockDim.x) {
    const int32_t c = changed[i];
    uint32_t h = ((uint32_t)c * 0x9E3779B1u) >> (32 - bits);
    while (true) {
      const int32_t old = atomicCAS(&tab[h], -1, c);
      if (old == -1 || old == c) break;
      h = (h + 1) & mask;
    }
  }
  __syncthreads();
  const int64_t total = nrows * k;
  const int64_t e0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * kMarkPer;
  if (e0 >= total) return;
  int32_t x[kMarkPer];
  if (e0 + kMarkPer <= total) {
    const int4 v0 = *reinterpret_cast<const int4*>(nb_slot + e0);
    const int4 v1 = *reinterpret_cast<const int4*>(nb_slot + e0 + 4);
    x[0] = v0.x; x[1] = v0.y; x[2] = v0.z; x[3] = v0.w;
    x[4] = v1.x; x[5] = v1.y; x[6] = v1.z; x[7] = v1.w;
  } else {
#pragma unroll
    for (int u = 0; u < kMarkPer; ++u) x[u] = e0 + u < total ? nb_slot[e0 + u] : -1;
  }
#pragma unroll
  for (int u = 0; u < kMarkPer; ++u) {
    if (x[u] < 0) continue;
    uint32_t h = ((uint32_t)x[u] * 0x9E3779B1u) >> (32 - bits);
    bool hit = false;
    while (true) {
      const int32_t tv = tab[h];
      if (tv == x[u]) { hit = true; break; }
      if (tv == -1) break;
      h = (h + 1) & mask;
    }
    if (hit) {
      const int64_t y = (e0 + u) / k;
      lrd_ok[y] = 0;
      if (clear_ok) ok[y] = 0;
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
    int32_t* __restrict__ abort_flag, LofLds& L, const uint32_t* __restrict__ kstamp = nullptr,
    uint32_t* __restrict__ lstamp = nullptr, uint32_t epoch = 0, bool defer = false, bool have_lists = false,
    bool no_cache = false) {
  // no_cache: recomputed lrd values are used, not stored (several blocks
  // scoring at once could otherwise see one block's lrd_ok before its lrd)
  // have_lists: the targets' lists and fields are in L already (the fused
  // insert left them there; targets = its candidates' head)
  // defer: out is device scratch the caller copies to the host later - plain
  // stores, no waits for acknowledgements (a batch of adds in one launch)
  auto put = [&](uint32_t* at, uint32_t v) {
    if (defer) *at = v;
    else sys_store(at, v);
  };
  // the targets' lists and their rows' flags / k-distances (and stamps) are
  // fetched in two cooperative rounds (every load of a round in flight at
  // once), then each target's thread works from LDS
  int& nmiss = L.nmiss;
  auto& l_s = L.s;
  auto& l_d = L.d;
  auto& l_kd = L.kd;
  auto& l_ok = L.okb;
  uint8_t* s_ok = L.ok1;
  float* s_kd = L.kd1;
  float* s_lrd = L.lrd1;
  const int t = threadIdx.x;
  const uint32_t kinv = lof_kinv(k);
  if (t == 0) nmiss = 0;
  uint8_t lok = 0;
  float lr = 0.f;
  if (have_lists) {
    if (t < nt) {
      lok = L.lok1[t];
      lr = L.lr1[t];
      L.stale[t] = 0;
    }
  } else if (t < nt) {
    const int32_t o = ts[t];
    s_ok[t] = ok[o];
    lok = lrd_ok[o];
    lr = lrd[o];
    s_kd[t] = kdist[o];
    L.stale[t] = 0;
    if (kstamp != nullptr) L.lst[t] = lstamp[o];
  }
  for (int e0 = t; e0 < (have_lists ? 0 : nt * k); e0 += 64 * kLofU) {
    int32_t vs[kLofU];
    float vd[kLofU];
#pragma unroll
    for (int u = 0; u < kLofU; ++u) {
      const int e = e0 + 64 * u < nt * k ? e0 + 64 * u : 0;
      const int c = lof_div(e, kinv), j = e - c * k;
      const int64_t at = (int64_t)ts[c] * k + j;
      vs[u] = nb_slot[at];
      vd[u] = nb_dist[at];
    }
#pragma unroll
    for (int u = 0; u < kLofU; ++u) {
      const int e = e0 + 64 * u;
      if (e < nt * k) {
        const int c = lof_div(e, kinv), j = e - c * k;
        l_s[c][j] = vs[u];
        l_d[c][j] = vd[u];
      }
    }
  }
  lof_lds_sync();
  for (int e0 = t; e0 < nt * k; e0 += 64 * kLofU) {
    uint8_t vo[kLofU];
    float vk[kLofU];
    uint32_t vt[kLofU];
#pragma unroll
    for (int u = 0; u < kLofU; ++u) {
      const int e = e0 + 64 * u;
      const int c = e < nt * k ? lof_div(e, kinv) : 0, j = e - c * k;
      const int32_t x = e < nt * k ? l_s[c][j] : -1;
      // a list is valid (in range) only while its row is ok
      const int32_t xr = (s_ok[c] && x >= 0) ? x : 0;
      vo[u] = ok[xr];
      vk[u] = kdist[xr];
      vt[u] = kstamp != nullptr ? kstamp[xr] : 0u;
    }
#pragma unroll
    for (int u = 0; u < kLofU; ++u) {
      const int e = e0 + 64 * u;
      if (e < nt * k) {
        const int c = lof_div(e, kinv), j = e - c * k;
        const int32_t x = l_s[c][j];
        if (s_ok[c] && x >= 0) {
          l_ok[c][j] = vo[u];
          l_kd[c][j] = vk[u];
          if (kstamp != nullptr && vt[u] > L.lst[c]) L.stale[c] = 1;
        }
      }
    }
  }
  lof_lds_sync();
  lof_stamp(L, 5);
  auto miss = [&](int32_t s) {
    const int w = atomicAdd(&nmiss, 1);
    if (w < max_missing) put(out + 4 + w, (uint32_t)s);
  };
  if (t < nt) {
    const int32_t o = ts[t];
    if (!s_ok[t]) {
      miss(o);
    } else {
      // lrd[o] is current only while every row o lists has a valid list
      bool good = true;
      int n = 0;
      float sum = 0.f;
      if (k <= kLofKR) {
        // all of the list's LDS reads issued together, then the sum in order
        int32_t xs[kLofKR];
        uint8_t xo[kLofKR];
        float xm[kLofKR];
#pragma unroll
        for (int j = 0; j < kLofKR; ++j) {
          const int32_t vs = l_s[t][j];
          const uint8_t vo = l_ok[t][j];
          const float vm = fmaxf(l_kd[t][j], l_d[t][j]);
          xs[j] = j < k ? vs : -1;
          xo[j] = j < k ? vo : 1;
          xm[j] = j < k ? vm : 0.f;
        }
#pragma unroll
        for (int j = 0; j < kLofKR; ++j) {
          if (xs[j] < 0) continue;              // (-1 entries are a suffix)
          if (!xo[j]) { miss(xs[j]); good = false; }
          sum += xm[j];
          ++n;
        }
      } else {
        for (int j = 0; j < k; ++j) {
          const int32_t x = l_s[t][j];
          if (x < 0) break;
          if (!l_ok[t][j]) { miss(x); good = false; }
          sum += fmaxf(l_kd[t][j], l_d[t][j]);
          ++n;
        }
      }
      if (good && (!lok || L.stale[t])) {
        const float mean = n > 0 ? sum / n : 0.f;
        lr = n == 0 ? 0.f : (mean <= 0.f ? INFINITY : 1.f / mean);
        if (!no_cache) {
          lrd[o] = lr;
          lrd_ok[o] = 1;
          if (lstamp != nullptr) lstamp[o] = epoch;
        }
      }
    }
    s_lrd[t] = lr;
  }
  // the host reads out[] once out[0] is set: every thread's system-scope
  // stores are acknowledged before the barrier, the status goes last (a
  // system-scope release fence would write back the whole L2 instead)
  if (defer) lof_lds_sync();
  else sys_stores_block_done();
  if (t != 0) return;
  if (nmiss > 0) {
    // a batch of adds stops here: the host installs the missing lists and
    // scores this add again before the later ones run (sequential order)
    if (abort_flag != nullptr) *abort_flag = 1;
    put(out + 3, (uint32_t)(nmiss < max_missing ? nmiss : max_missing));
    if (!defer) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    put(out, 2u);
    return;
  }
  // lrd of the query point itself (its own neighbours' k-distances)
  float sum = 0.f, lsum = 0.f;
  bool linf = false;
  for (int j0 = 0; j0 < nt; j0 += 16) {         // 16 LDS reads of each array in flight
    float a[16], l[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {               // (the arrays hold 64: reads in bounds)
      const int jj = (j0 + u) & 63;
      const float va = fmaxf(s_kd[jj], td[jj]);
      const float vl = s_lrd[jj];
      a[u] = j0 + u < nt ? va : 0.f;
      l[u] = j0 + u < nt ? vl : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (j0 + u >= nt) break;
      sum += a[u];
      if (isinf(l[u])) linf = true; else lsum += l[u];
    }
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
  if (store_slot >= 0) {
    lrd[store_slot] = lp;
    lrd_ok[store_slot] = 1;
    if (lstamp != nullptr) lstamp[store_slot] = epoch;
  }
  put(out + 1, __float_as_uint(score));
  put(out + 2, __float_as_uint(lp));
  put(out + 3, 0u);
  if (!defer) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  put(out, 1u);
}

__global__ __launch_bounds__(64) void lof_score_kernel(
    const LofArgs a, int k, const int32_t* __restrict__ nb_slot,
    const float* __restrict__ nb_dist, const float* __restrict__ kdist,
    const uint8_t* __restrict__ ok, float* __restrict__ lrd, uint8_t* __restrict__ lrd_ok,
    int store_slot, uint32_t* __restrict__ out, int max_missing,
    int32_t* __restrict__ abort_flag = nullptr, const uint32_t* __restrict__ kstamp = nullptr,
    uint32_t* __restrict__ lstamp = nullptr, uint32_t epoch = 0) {
  if (abort_flag != nullptr && *abort_flag != 0) {   // skipped: an earlier add stopped the batch
    if (threadIdx.x == 0) sys_store(out, 3u);
    return;
  }
  __shared__ int32_t ts[kLofMaxK];
  __shared__ float td[kLofMaxK];
  __shared__ LofLds L;
  const int nt = a.n < kLofMaxK ? a.n : kLofMaxK;
  if ((int)threadIdx.x < nt) { ts[threadIdx.x] = a.s[threadIdx.x]; td[threadIdx.x] = a.d[threadIdx.x]; }
  lof_lds_sync();
  lof_score_body(ts, td, nt, k, nb_slot, nb_dist, kdist, ok, lrd, lrd_ok, store_slot, out,
                 max_missing, abort_flag, L, kstamp, lstamp, epoch);
}

// Independent scores in one launch, a block each (calc_score of a batch):
// query q's targets ts_h / td_h [q * stride, + nt_h[q]) in pinned host
// memory, its status and score into out + q * out_stride. Reads only: the
// lrd values a block recomputes are not cached.
__global__ __launch_bounds__(64) void lof_score_many_kernel(
    const int32_t* __restrict__ ts_h, const float* __restrict__ td_h, const int32_t* __restrict__ nt_h, int stride,
    int k, const int32_t* __restrict__ nb_slot, const float* __restrict__ nb_dist, const float* __restrict__ kdist,
    const uint8_t* __restrict__ ok, float* __restrict__ lrd, uint8_t* __restrict__ lrd_ok,
    const uint32_t* __restrict__ kstamp, uint32_t* __restrict__ lstamp, uint32_t* __restrict__ out, int out_stride,
    int max_missing) {
  __shared__ int32_t ts[kLofMaxK];
  __shared__ float td[kLofMaxK];
  __shared__ LofLds L;
  const int q = blockIdx.x;
  const int nt0 = nt_h[q];
  const int nt = nt0 < kLofMaxK ? nt0 : kLofMaxK;
  if ((int)threadIdx.x < nt) {
    ts[threadIdx.x] = ts_h[(int64_t)q * stride + threadIdx.x];
    td[threadIdx.x] = td_h[(int64_t)q * stride + threadIdx.x];
  }
  if (threadIdx.x == 0) L.prof = false;
  lof_lds_sync();
  lof_score_body(ts, td, nt, k, nb_slot, nb_dist, kdist, ok, lrd, lrd_ok, -1, out + (int64_t)q * out_stride,
                 max_missing, nullptr, L, kstamp, lstamp, 0u, false, false, true);
}

// One add in one launch (stamps, no mark pass): p's insert (candidates in
// the arguments, all <= kLofArgMax of them), then its score from the k
// nearest, lrd[p] stored; out as lof_score_kernel
__global__ __launch_bounds__(64) void lof_add_score_kernel(
    const LofArgs a, int p, int k, int ignore_same, int32_t* __restrict__ nb_slot,
    float* __restrict__ nb_dist, float* __restrict__ kdist, uint8_t* __restrict__ ok,
    float* __restrict__ lrd, uint8_t* __restrict__ lrd_ok, int32_t* __restrict__ changed,
    int32_t* __restrict__ nchanged, uint32_t* __restrict__ kstamp, uint32_t* __restrict__ lstamp,
    uint32_t epoch, uint32_t* __restrict__ out, int max_missing, int32_t* __restrict__ abort_flag) {
  if (abort_flag != nullptr && *abort_flag != 0) {   // skipped: an earlier add stopped the batch
    if (threadIdx.x == 0) sys_store(out, 3u);
    return;
  }
  __shared__ int32_t cs[kLofArgMax];
  __shared__ float cd[kLofArgMax];
  __shared__ LofLds L;
  for (int i = threadIdx.x; i < a.n; i += blockDim.x) { cs[i] = a.s[i]; cd[i] = a.d[i]; }
  lof_lds_sync();
  const bool fz = a.n <= 64;                         // targets' lists stay in LDS
  lof_insert_body(p, cs, cd, a.n, k, ignore_same, nb_slot, nb_dist, kdist, ok, lrd_ok, changed,
                  nchanged, true, L, kstamp, epoch, fz ? lrd : nullptr, lstamp);
  // the insert's global stores are visible to the block after the barrier
  lof_lds_sync();
  const int nt = a.n < k ? a.n : k;
  lof_score_body(cs, cd, nt, k, nb_slot, nb_dist, kdist, ok, lrd, lrd_ok, p, out, max_missing,
                 abort_flag, L, kstamp, lstamp, epoch, false, fz);
}

// A batch of adds in one launch, in order (one block loops over them: no
// launch or inter-kernel gap per add): add i (epoch epoch0 + i) inserts p =
// ps[i] with its nc[i] candidates, then scores it into out + i * out_stride.
// The candidates are read from pinned host memory once, into cand (device
// scratch, [nadd][stride] slots then distances). An add that meets rows
// without a valid list stops the batch there (status 2); the later ones get
// status 3 (not run) and the host resubmits them after finishing it.
__global__ __launch_bounds__(64) void lof_add_batch_kernel(
    int nadd, const int32_t* __restrict__ ps, const int32_t* __restrict__ nc, const int32_t* __restrict__ cs_h,
    const float* __restrict__ cd_h, int stride, int k, int ignore_same, int32_t* __restrict__ nb_slot,
    float* __restrict__ nb_dist, float* __restrict__ kdist, uint8_t* __restrict__ ok, float* __restrict__ lrd,
    uint8_t* __restrict__ lrd_ok, int32_t* __restrict__ changed, int32_t* __restrict__ nchanged,
    uint32_t* __restrict__ kstamp, uint32_t* __restrict__ lstamp, uint32_t epoch0, int32_t* __restrict__ cand,
    uint32_t* __restrict__ res, uint32_t* __restrict__ out, int out_stride, int max_missing,
    unsigned long long* __restrict__ prof, uint32_t* __restrict__ chain) {
  __shared__ int32_t cs[kLofArgMax];
  __shared__ float cd[kLofArgMax];
  __shared__ int32_t s_p[64], s_n[64];
  __shared__ LofLds L;
  const int t = threadIdx.x;
  // chain (optional): set when a batch stops; a batch queued behind a stopped
  // one does not run (status 3 for every add: the host reruns it after
  // installing the missing lists and clearing the word)
  if (chain != nullptr && chain[0] != 0u) {
    for (int i = t; i < nadd - 1; i += blockDim.x) sys_store(out + (int64_t)i * out_stride, 3u);
    sys_stores_block_done();
    if (t == 0) sys_store(out + (int64_t)(nadd - 1) * out_stride, 3u);
    return;
  }
  const int tot = nadd * stride;
  float* cand_d = reinterpret_cast<float*>(cand + tot);
  for (int e0 = t; e0 < tot; e0 += 64 * kLofU) {  // one pass over host memory, kLofU loads in flight
    int32_t vs[kLofU];
    float vd[kLofU];
#pragma unroll
    for (int u = 0; u < kLofU; ++u) {
      const int e = e0 + 64 * u < tot ? e0 + 64 * u : 0;
      vs[u] = cs_h[e];
      vd[u] = cd_h[e];
    }
#pragma unroll
    for (int u = 0; u < kLofU; ++u)
      if (e0 + 64 * u < tot) { cand[e0 + 64 * u] = vs[u]; cand_d[e0 + 64 * u] = vd[u]; }
  }
  if (t < nadd) { s_p[t] = ps[t]; s_n[t] = nc[t]; }
  if (t < 8) L.ph[t] = 0;
  if (t == 0) {
    L.prof = prof != nullptr;
    L.tlast = __builtin_amdgcn_s_memtime();
  }
  __syncthreads();
  lof_stamp(L, 7);                                // the candidates' copy from the host
  int ran = nadd;
  for (int i = 0; i < nadd; ++i) {
    const int n = s_n[i], p = s_p[i];
    for (int e = t; e < n; e += blockDim.x) { cs[e] = cand[i * stride + e]; cd[e] = cand_d[i * stride + e]; }
    lof_lds_sync();
    lof_stamp(L, 0);
    const bool fz = n <= 64;                         // targets' lists stay in LDS
    lof_insert_body(p, cs, cd, n, k, ignore_same, nb_slot, nb_dist, kdist, ok, lrd_ok, changed, nchanged, true,
                    L, kstamp, epoch0 + (uint32_t)i, fz ? lrd : nullptr, lstamp);
    lof_lds_sync();
    lof_score_body(cs, cd, n < k ? n : k, k, nb_slot, nb_dist, kdist, ok, lrd, lrd_ok, p,
                   res + (int64_t)i * out_stride, max_missing, nullptr, L, kstamp, lstamp, epoch0 + (uint32_t)i,
                   true, fz);
    __syncthreads();
    lof_stamp(L, 6);
    if (L.nmiss > 0) { ran = i + 1; break; }      // stopped: the later adds did not run
  }
  if (chain != nullptr && t == 0 && L.nmiss > 0) chain[0] = 1u;   // (the next batch on the stream sees it)
  // results to the host: every word but the statuses, acknowledged, then the
  // statuses (the last add's last: the host waits for it)
  const int nm = L.nmiss > 0 ? (L.nmiss < max_missing ? L.nmiss : max_missing) : 0;
  for (int i = t; i < ran; i += blockDim.x)
    for (int w = 1; w < 4; ++w) sys_store(out + (int64_t)i * out_stride + w, res[(int64_t)i * out_stride + w]);
  for (int w = t; w < nm; w += blockDim.x)
    sys_store(out + (int64_t)(ran - 1) * out_stride + 4 + w, res[(int64_t)(ran - 1) * out_stride + 4 + w]);
  sys_stores_block_done();
  for (int i = t; i < nadd - 1; i += blockDim.x)
    sys_store(out + (int64_t)i * out_stride, i < ran ? res[(int64_t)i * out_stride] : 3u);
  sys_stores_block_done();
  const int64_t last = (int64_t)(nadd - 1) * out_stride;
  if (t == 0) sys_store(out + last, nadd - 1 < ran ? res[last] : 3u);
  // phases (cycles): 0 candidates to LDS, 1 list loads, 2 edits, 3 write-back,
  // 4 (unused), 5 score loads, 6 score, 7 host copy; prof[8] adds
  if (prof != nullptr && t == 0) {
    for (int i = 0; i < 8; ++i) atomicAdd(prof + i, L.ph[i]);
    atomicAdd(prof + 8, (unsigned long long)ran);
  }
}

}  // namespace jb

static unsigned mark_blocks(int64_t nrows, int k) {
  const int64_t per_block = 256 * jb::kMarkPer;
  return (unsigned)((nrows * k + per_block - 1) / per_block);
}

extern "C" int jb_lof_mark(int64_t nrows, int k, const int32_t* nb_slot, const int32_t* changed,
                           const int32_t* nchanged, int clear_ok, uint8_t* ok, uint8_t* lrd_ok,
                           hipStream_t stream) {
  if (nrows <= 0) return 0;
  hipLaunchKernelGGL(jb::lof_mark_kernel, dim3(mark_blocks(nrows, k)), dim3(256), 0, stream, nrows, k,
                     nb_slot, changed, nchanged, clear_ok, ok, lrd_ok);
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
// scored from its k nearest (lof_score_kernel, lrd[p] stored). With stamps
// (kstamp / lstamp non-null, epoch = this add's, above every earlier one) and
// nc <= kLofArgMax the add is one launch instead (lof_add_score_kernel).
// Waits for the score; out_host = [status, score, lrd, nmissing, missing...].
extern "C" int jb_lof_add_st(int p, const int32_t* cs, const float* cd, int nc, int k,
                             int ignore_same, int64_t nrows, int32_t* nb_slot, float* nb_dist,
                             float* kdist, uint8_t* ok, float* lrd, uint8_t* lrd_ok,
                             int32_t* changed, int32_t* nchanged, uint32_t* kstamp, uint32_t* lstamp,
                             uint32_t epoch, uint32_t* out_host, int max_missing, hipStream_t stream) {
  if (k <= 0 || k > jb::kLofMaxK || nc < 0) return -2;
  jb::LofArgs a;
  out_host[0] = 0;
  if (kstamp != nullptr && lstamp != nullptr && nc <= jb::kLofArgMax) {
    int rc = fill_args(&a, cs, cd, nc);
    if (rc) return rc;
    hipLaunchKernelGGL(jb::lof_add_score_kernel, dim3(1), dim3(64), 0, stream, a, p, k, ignore_same, nb_slot,
                       nb_dist, kdist, ok, lrd, lrd_ok, changed, nchanged, kstamp, lstamp, epoch, out_host,
                       max_missing, (int32_t*)nullptr);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    return jb::wait_nonzero(out_host, stream);
  }
  // the candidates travel in the kernel arguments, kLofArgMax per launch: the
  // first launch sets p's own list (its k nearest are the head of the first
  // chunk) and the reverse inserts of that chunk, later ones (a
  // reverse_nearest_neighbor_num above the argument budget) only insert p
  // into their candidates' lists
  for (int c0 = 0; c0 == 0 || c0 < nc; c0 += jb::kLofArgMax) {
    const int cn = nc - c0 < jb::kLofArgMax ? nc - c0 : jb::kLofArgMax;
    int rc = fill_args(&a, cs + c0, cd + c0, cn < 0 ? 0 : cn);
    if (rc) return rc;
    hipLaunchKernelGGL(jb::lof_add_kernel, dim3(1), dim3(64), 0, stream, a, p, k, ignore_same,
                       nb_slot, nb_dist, kdist, ok, lrd_ok, changed, nchanged, c0 == 0 ? 1 : 0);
  }
  int rc = fill_args(&a, cs, cd, nc < jb::kLofArgMax ? nc : jb::kLofArgMax);
  if (rc) return rc;
  hipLaunchKernelGGL(jb::lof_mark_kernel, dim3(mark_blocks(nrows, k)), dim3(256), 0, stream, nrows, k,
                     nb_slot, changed, nchanged, 0, ok, lrd_ok);
  a.n = nc < k ? nc : k;               // score from the k nearest
  hipLaunchKernelGGL(jb::lof_score_kernel, dim3(1), dim3(64), 0, stream, a, k, nb_slot, nb_dist,
                     kdist, ok, lrd, lrd_ok, p, out_host, max_missing, (int32_t*)nullptr,
                     (const uint32_t*)kstamp, lstamp, epoch);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return jb::wait_nonzero(out_host, stream);
}

extern "C" int jb_lof_add(int p, const int32_t* cs, const float* cd, int nc, int k,
                          int ignore_same, int64_t nrows, int32_t* nb_slot, float* nb_dist,
                          float* kdist, uint8_t* ok, float* lrd, uint8_t* lrd_ok,
                          int32_t* changed, int32_t* nchanged, uint32_t* out_host,
                          int max_missing, hipStream_t stream) {
  return jb_lof_add_st(p, cs, cd, nc, k, ignore_same, nrows, nb_slot, nb_dist, kdist, ok, lrd, lrd_ok,
                       changed, nchanged, nullptr, nullptr, 0, out_host, max_missing, stream);
}

// A batch of adds in arrival order, one launch and one wait
// (lof_add_batch_kernel). ps / nc / cs / cd: pinned host memory the kernel
// reads ([nadd][stride] candidates, ascending, p excluded); cand: device
// scratch of 2 x nadd x stride words, res: of nadd x out_stride (the results
// before they go to the host); out_host[i * out_stride] = status 1
// done, 2 stopped on rows without a valid list (its insert is applied, its
// score is not), 3 not run. wait = 0: return once launched (the caller
// overlaps other work, then jb_lof_add_many_wait). chain (optional device
// word): a batch sets it when it stops, and a batch that finds it set does
// not run - batches queued back to back keep their order.
extern "C" int jb_lof_add_many(int nadd, const int32_t* ps, const int32_t* cs, const float* cd,
                               const int32_t* nc, int stride, int k, int ignore_same, int32_t* nb_slot,
                               float* nb_dist, float* kdist, uint8_t* ok, float* lrd, uint8_t* lrd_ok,
                               int32_t* changed, int32_t* nchanged, uint32_t* kstamp, uint32_t* lstamp,
                               uint32_t epoch0, int32_t* cand, uint32_t* res, uint32_t* out_host, int out_stride,
                               int max_missing, unsigned long long* prof, hipStream_t stream, int wait,
                               uint32_t* chain) {
  if (nadd <= 0) return 0;
  if (nadd > 64 || k <= 0 || k > jb::kLofMaxK || stride > jb::kLofArgMax || kstamp == nullptr ||
      lstamp == nullptr)
    return -2;
  for (int i = 0; i < nadd; ++i) {
    if (nc[i] < 0 || nc[i] > stride) return -2;
    out_host[(int64_t)i * out_stride] = 0;
  }
  hipLaunchKernelGGL(jb::lof_add_batch_kernel, dim3(1), dim3(64), 0, stream, nadd, ps, nc, cs, cd, stride, k,
                     ignore_same, nb_slot, nb_dist, kdist, ok, lrd, lrd_ok, changed, nchanged, kstamp, lstamp,
                     epoch0, cand, res, out_host, out_stride, max_missing, prof, chain);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return wait ? jb::wait_nonzero(out_host + (int64_t)(nadd - 1) * out_stride, stream) : 0;
}

// the wait of a jb_lof_add_many launched with wait = 0 (its last add's status)
extern "C" int jb_lof_add_many_wait(int nadd, uint32_t* out_host, int out_stride, hipStream_t stream) {
  if (nadd <= 0) return 0;
  return jb::wait_nonzero(out_host + (int64_t)(nadd - 1) * out_stride, stream);
}

// LOF of a point from its nt (<= 64) nearest (host arrays), lrd of the
// targets refreshed (stamped with epoch when kstamp / lstamp are given);
// waits; same out_host layout
extern "C" int jb_lof_score_st(const int32_t* ts, const float* td, int nt, int k,
                               const int32_t* nb_slot, const float* nb_dist, const float* kdist,
                               const uint8_t* ok, float* lrd, uint8_t* lrd_ok, int store_slot,
                               const uint32_t* kstamp, uint32_t* lstamp, uint32_t epoch,
                               uint32_t* out_host, int max_missing, hipStream_t stream) {
  if (nt > 64 || k > jb::kLofMaxK) return -2;
  jb::LofArgs a;
  int rc = fill_args(&a, ts, td, nt);
  if (rc) return rc;
  out_host[0] = 0;
  hipLaunchKernelGGL(jb::lof_score_kernel, dim3(1), dim3(64), 0, stream, a, k, nb_slot, nb_dist,
                     kdist, ok, lrd, lrd_ok, store_slot, out_host, max_missing, (int32_t*)nullptr,
                     kstamp, lstamp, epoch);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return jb::wait_nonzero(out_host, stream);
}

// Several independent scores (calc_score of a batch of queries), one launch
// (lof_score_many_kernel, a block per query): ts / td / nt in pinned host
// memory (query i's targets [i * stride, + nt[i])), its status and score go to
// out_host + i * out_stride. A query that finds rows without a valid list
// reports them (status 2) and the host finishes it alone.
extern "C" int jb_lof_score_many(int nq, const int32_t* ts, const float* td, const int32_t* nt, int stride,
                                 int k, const int32_t* nb_slot, const float* nb_dist, const float* kdist,
                                 const uint8_t* ok, float* lrd, uint8_t* lrd_ok, const uint32_t* kstamp,
                                 uint32_t* lstamp, uint32_t epoch, uint32_t* out_host, int out_stride,
                                 int max_missing, hipStream_t stream) {
  (void)epoch;
  if (nq <= 0) return 0;
  if (k > jb::kLofMaxK || stride > 64) return -2;
  for (int i = 0; i < nq; ++i) {
    if (nt[i] < 0 || nt[i] > stride) return -2;
    out_host[(int64_t)i * out_stride] = 0;
  }
  hipLaunchKernelGGL(jb::lof_score_many_kernel, dim3((unsigned)nq), dim3(64), 0, stream, ts, td, nt, stride, k,
                     nb_slot, nb_dist, kdist, ok, lrd, lrd_ok, kstamp, lstamp, out_host, out_stride, max_missing);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  for (int i = 0; i < nq; ++i) {          // the blocks finish in any order
    const int rc = jb::wait_nonzero(out_host + (int64_t)i * out_stride, stream);
    if (rc != 0) return rc;
  }
  return 0;
}

extern "C" int jb_lof_score(const int32_t* ts, const float* td, int nt, int k,
                            const int32_t* nb_slot, const float* nb_dist, const float* kdist,
                            const uint8_t* ok, float* lrd, uint8_t* lrd_ok, int store_slot,
                            uint32_t* out_host, int max_missing, hipStream_t stream) {
  return jb_lof_score_st(ts, td, nt, k, nb_slot, nb_dist, kdist, ok, lrd, lrd_ok, store_slot, nullptr,
                         nullptr, 0, out_host, max_missing, stream);
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
