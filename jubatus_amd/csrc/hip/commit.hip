// Delta committer: the serial-equivalent (update mode kSerial, the servers'
// default "exact") training of a batch of concurrent train requests for label
// capacities up to 64. The result is that of applying the batch's samples one
// after the other in request order - the reference's classifier applies every
// sample to the model the previous one left (classifier_serv.cpp:138-144).
//
// Design (MI355X-first; replaces serial.hip's bound committer for LC <= 64):
//
//   1. delta_s0_kernel (whole GPU, one wave per sample): every sample's LC
//      label scores against the model at the segment start M0 (the global
//      W / P tables, which nothing writes while the segment runs).
//   2. delta_commit_kernel (ONE 1024-thread workgroup, 16 waves = 64 groups
//      of 16 lanes; a group is a DPP row): walks the batch in order, 128
//      samples per round, each group owning 2 consecutive samples with
//      feature u / label u on lane u of the row. Everything the batch writes
//      lives in LDS until the segment ends:
//        dW[slot][LC], dP[slot][LC]  the summed increments since M0 of every
//                                    row the segment wrote (hash -> slot),
//      so the live model is M0 (global, never written, prefetchable) + the LDS
//      deltas. Each sample's scores are kept EXACT (not bounded): at round
//      start a lane adds x_u * dW[row_u][:] of the rows already written, and
//      after every update the stepping group publishes its per-row increments
//      (a small LDS step table) and every later sample of the round adds
//      x * dW_step to its scores of the two labels the update touched (one
//      probe per lane, two row sums). The first sample of the round whose
//      exact margin says it updates takes the exact step - its 16 lanes read
//      P0 + dP of (feature, y / best wrong), compute the method's
//      coefficients and add the increments into LDS - and the round
//      continues after it. A sample that does not update costs no table
//      access at all; an update costs two workgroup barriers and LDS work.
//   3. When the LDS row store is full the segment ends: the deltas are added
//      to W / P (one coalesced pass), and the next segment re-scores the rest
//      of the batch against the new tables. A sample wider than 64 features
//      ends the committer; the rest of the batch runs the single-stream exact
//      kernel (linear.hip kExact), as in serial.hip.
//
// Rounding: scores are S0 + incremental corrections, summed in another order
// than a fresh recomputation; a sample whose margin lies within a relative
// guard band of its update threshold re-scores itself from the live model
// (M0 + dW) before the decision, so decisions match a plain sequential fp32
// pass. Semantics per update (a repeated row counts every time, each
// occurrence against the pre-sample state) are those of linear.hip's direct
// path; the oracle is jubatus_amd/models/linear_oracle.py.
#include "jb_linear.hpp"

namespace jb {
namespace dc {

constexpr int kT = 512;               // committer threads (8 waves)
constexpr int kNG = kT / 16;          // groups (DPP rows) of 16 lanes
constexpr int kR = 4;                 // samples per group per round
constexpr int kNS = kNG * kR;         // samples per round
constexpr int kFC = 2;                // feature chunks of 16 held in registers
constexpr int kNFMax = 16 * kFC;      // widest sample the committer takes
constexpr int kSHS = 128;             // step-table hash slots (<= 32 rows per step)
constexpr float kGuard = 1e-4f;       // relative guard band of a decision
constexpr int kInf = 0x7fffffff;
// stop reasons (tail[kTailReason]); the values are serial.hip's
constexpr int64_t kStopDone = 0, kStopSaturated = 1, kStopDense = 2;
constexpr int kTailReason = 20;

constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }

template <int LC>
struct Geo {
  static constexpr int K = (LC + 15) / 16;                 // labels per lane
  static constexpr int NSLOT = 16384 / (LC > 16 ? LC : 16); // rows the LDS store holds
  static constexpr int HS = 2 * NSLOT;                      // row hash slots (load <= 1/2)
  static constexpr int HB = ilog2(HS);
};

__device__ __forceinline__ uint32_t hmix(int32_t r) { return (uint32_t)r * 0x9E3779B1u; }

template <int CTRL>
__device__ __forceinline__ float dppf(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

// best wrong label over a row of 16 lanes (lowest label on ties); the DPP
// pairings xor 1, xor 2, xor 7 (half mirror), xor 8 (rotate 8) span the row
__device__ __forceinline__ void row16_argmax(float& b, int& bl) {
#define JB_ARGSTEP(C)                                                              \
  {                                                                                \
    const float ob = dppf<C>(b);                                                   \
    const int ol = dppi<C>(bl);                                                    \
    if (ol >= 0 && (bl < 0 || ob > b || (ob == b && ol < bl))) { b = ob; bl = ol; } \
  }
  JB_ARGSTEP(kDppXor1)
  JB_ARGSTEP(kDppXor2)
  JB_ARGSTEP(kDppHalfMirror)
  JB_ARGSTEP(kDppRowRor8)
#undef JB_ARGSTEP
}

// value of lane (row base + u)
__device__ __forceinline__ float rowb_f(float v, int base, int u) { return __shfl(v, base + u, 64); }
__device__ __forceinline__ int rowb_i(int v, int base, int u) { return __shfl(v, base + u, 64); }

// margin of a sample held by a group: score(y) - best active wrong label
template <int LC>
__device__ __forceinline__ float group_margin(const float (&s)[Geo<LC>::K], int y,
                                              const bool (&act)[Geo<LC>::K], int sub, int base,
                                              int* lstar, float* sy_out, float* best_out) {
  constexpr int K = Geo<LC>::K;
  float sv = s[0];
#pragma unroll
  for (int k = 1; k < K; ++k)
    if (k == (y >> 4)) sv = s[k];
  const float sy = rowb_f(sv, base, y & 15);
  float b = -INFINITY;
  int bl = -1;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int lab = sub + 16 * k;
    if (lab < LC && act[k] && lab != y && s[k] > b) { b = s[k]; bl = lab; }
  }
  row16_argmax(b, bl);
  *lstar = bl;
  *sy_out = sy;
  *best_out = bl >= 0 ? b : 0.f;
  return sy - (bl >= 0 ? b : 0.f);
}

// may the sample update under its (exact up to rounding) margin? NaN: yes
// (the exact step decides). CW's threshold phi * var is bounded by
// phi * (1 or 2) * |x|^2: every precision is >= 1.
__device__ __forceinline__ bool may_update(int method, float m, float nrm, bool has_l, float C,
                                           float sy, float best) {
  const float g = kGuard * (1.f + fabsf(sy) + fabsf(best));
  switch (method) {
    case PERCEPTRON: return !(m > g);
    case PA: case PA1: case PA2: return nrm > 0.f && !(m >= 1.f + g);
    case CW: return nrm > 0.f && !(m >= C * (has_l ? 2.f : 1.f) * nrm + g);
    default: return !(m >= 1.f + g);
  }
}

// LDS row store: open-addressed row -> slot hash over HS entries
template <int LC>
__device__ __forceinline__ int cache_find(const int32_t* hkey, const int16_t* hslot, int32_t row) {
  using Gm = Geo<LC>;
  if (row < 0) return -1;
  uint32_t h = hmix(row) >> (32 - Gm::HB);
  for (int p = 0; p < Gm::HS; ++p) {
    const int32_t k = hkey[h];
    if (k == row) return hslot[h];
    if (k < 0) return -1;
    h = (h + 1) & (Gm::HS - 1);
  }
  return -1;
}

// insert (the stepping group only; the caller checked the capacity); returns
// the hash position - the slot is read from it once the group's inserts are
// done (a lane that found its row claimed by another lane of the same
// instruction reads the slot that lane stores)
template <int LC>
__device__ __forceinline__ uint32_t cache_insert(int32_t* hkey, int16_t* hslot, int32_t* ckey, int* cn,
                                                 int32_t row) {
  using Gm = Geo<LC>;
  uint32_t h = hmix(row) >> (32 - Gm::HB);
  for (int p = 0; p < Gm::HS; ++p) {
    const int32_t old = atomicCAS(&hkey[h], -1, row);
    if (old == -1) {
      const int s = atomicAdd(cn, 1);
      hslot[h] = (int16_t)s;
      ckey[s] = row;
      return h;
    }
    if (old == row) return h;
    h = (h + 1) & (Gm::HS - 1);
  }
  return 0;   // unreachable: the table is at most half full
}

__device__ __forceinline__ int step_find(const int32_t* skey, int32_t row) {
  if (row < 0) return -1;
  uint32_t h = hmix(row) >> (32 - ilog2(kSHS));
  for (int p = 0; p < kSHS; ++p) {
    const int32_t k = skey[h];
    if (k == row) return (int)h;
    if (k < 0) return -1;
    h = (h + 1) & (kSHS - 1);
  }
  return -1;
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
__device__ __forceinline__ void lds_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// ------------------------------------------------------------ S0 scores
template <int LC>
__global__ __launch_bounds__(256) void delta_s0_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int64_t* __restrict__ stream_ptr, int nstreams,
    const float* __restrict__ W, float* __restrict__ S0, const int64_t* __restrict__ reason) {
  using L = Lanes<LC>;
  static_assert(LC <= 64, "delta committer: LC <= 64");
  if (reason != nullptr && (*reason == kStopDense || *reason == kStopDone)) return;
  const int lane = threadIdx.x & 63;
  const int64_t beg = stream_ptr[0];
  const int64_t cnt = stream_ptr[nstreams] - beg;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int g = lane / L::LW;
  const int l0 = lane % L::LW;
  for (int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; wid < cnt; wid += nwaves) {
    const int64_t s = beg + wid;
    const int64_t fb = row_ptr[s];
    const int n = (int)(row_ptr[s + 1] - fb);
    float acc = 0.f;
    for (int j = g; j < n; j += L::G) {
      const int32_t idx = fidx[fb + j];
      if (idx >= 0) acc += fval[fb + j] * W[(int64_t)idx * LC + l0];
    }
#pragma unroll
    for (int off = L::LW; off < 64; off <<= 1) acc += __shfl_xor(acc, off, 64);
    if (lane < LC) S0[wid * LC + lane] = acc;
  }
}

// one sample's round data (group layout: lane u holds features u, u+16, ...)
struct Desc {
  int64_t fb;
  int nf;
  int y;
};

template <int LC>
struct Samp {
  int32_t fi[kFC];
  float fx[kFC];
  float s[Geo<LC>::K];
};

// ------------------------------------------------------------ committer
template <int LC>
__global__ __launch_bounds__(kT) void delta_commit_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, float* __restrict__ W,
    float* __restrict__ P, const int32_t* __restrict__ active, int method, float C,
    const float* __restrict__ S0, unsigned long long* __restrict__ stats,
    uint8_t* __restrict__ touched, int64_t* __restrict__ tail, int seg) {
  using Gm = Geo<LC>;
  constexpr int K = Gm::K;
  constexpr int NSLOT = Gm::NSLOT;
  constexpr int HS = Gm::HS;
  if (seg > 0 && (tail[kTailReason] == kStopDense || tail[kTailReason] == kStopDone)) return;
  __shared__ float s_dw[NSLOT * LC];
  __shared__ float s_dp[NSLOT * LC];
  __shared__ int32_t s_hkey[HS];
  __shared__ int16_t s_hslot[HS];
  __shared__ int32_t s_ckey[NSLOT];
  __shared__ int32_t s_skey[kSHS];
  __shared__ float s_sdy[kSHS];
  __shared__ float s_sdl[kSHS];
  __shared__ int32_t s_spos[kNFMax];
  __shared__ int s_sn, s_cn, s_stop, s_upd, s_yk, s_lk;
  __shared__ int s_first[2];
  __shared__ unsigned s_nupd, s_waste, s_refresh;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int sub = lane & 15;
  const int base = lane & 48;
  const int G = tid >> 4;
  const bool use_s = method >= CW;

  {
    float4* dw4 = reinterpret_cast<float4*>(s_dw);
    float4* dp4 = reinterpret_cast<float4*>(s_dp);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = tid; i < NSLOT * LC / 4; i += kT) { dw4[i] = z; dp4[i] = z; }
    for (int i = tid; i < HS; i += kT) s_hkey[i] = -1;
    for (int i = tid; i < kSHS; i += kT) { s_skey[i] = -1; s_sdy[i] = 0.f; s_sdl[i] = 0.f; }
    if (tid == 0) {
      s_sn = 0; s_cn = 0; s_stop = -1; s_upd = 0; s_yk = -1; s_lk = -1;
      s_first[0] = s_first[1] = kInf;
      s_nupd = 0; s_waste = 0; s_refresh = 0;
    }
  }
  bool act[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int lab = sub + 16 * k;
    act[k] = lab < LC && active[lab] != 0;
  }
  const int64_t beg = stream_ptr[0];
  const int64_t end = stream_ptr[nstreams];

  // two-deep prefetch: descriptors two rounds ahead, features / S0 one round ahead
  auto load_desc = [&](int64_t p, Desc (&d)[kR]) {
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int64_t j = p + G * kR + r;
      if (j < end) {
        d[r].y = labels[j];
        d[r].fb = row_ptr[j];
        d[r].nf = (int)(row_ptr[j + 1] - d[r].fb);
      } else {
        d[r].y = -1; d[r].fb = 0; d[r].nf = 0;
      }
    }
  };
  auto load_samp = [&](int64_t p, const Desc (&d)[kR], Samp<LC> (&sm)[kR]) {
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int64_t j = p + G * kR + r;
      const bool ok = j < end && d[r].y >= 0 && d[r].y < LC;
      const int32_t* fp = fidx + d[r].fb + sub;
      const float* vp = fval + d[r].fb + sub;
#pragma unroll
      for (int c = 0; c < kFC; ++c) {
        const bool v = ok && c * 16 + sub < d[r].nf;
        sm[r].fi[c] = v ? fp[c * 16] : -1;
        sm[r].fx[c] = v ? vp[c * 16] : 0.f;
      }
      const float* s0p = S0 + (j - beg) * LC + sub;
#pragma unroll
      for (int k = 0; k < K; ++k)
        sm[r].s[k] = (ok && sub + 16 * k < LC) ? s0p[16 * k] : 0.f;
    }
  };

  Desc dc[kR], dn[kR], dnn[kR];
  Samp<LC> sc[kR], sn[kR];
  load_desc(beg, dn);
  load_samp(beg, dn, sn);
  load_desc(beg + kNS, dnn);
  __syncthreads();

  int64_t stop = end;
  int64_t why = kStopDone;
  unsigned n_valid = 0;
  int iter = 0;
  int64_t n_steps = 0, n_rounds = 0;

  for (int64_t p = beg; p < end; p += kNS) {
#pragma unroll
    for (int r = 0; r < kR; ++r) { dc[r] = dn[r]; sc[r] = sn[r]; dn[r] = dnn[r]; }
    if (p + kNS < end) load_samp(p + kNS, dn, sn);
    if (p + 2 * kNS < end) load_desc(p + 2 * kNS, dnn);

    // ---- round start: deltas of the rows the segment wrote, margins
    bool alive[kR], unsafe[kR];
    float nrm[kR];
    int nch[kR];
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int64_t j = p + G * kR + r;
      const int y = dc[r].y;
      alive[r] = j < end && y >= 0 && y < LC;
      nch[r] = (dc[r].nf + 15) >> 4;
      unsafe[r] = false;
      nrm[r] = 0.f;
      if (!alive[r]) continue;
      if (dc[r].nf > kNFMax) { unsafe[r] = true; continue; }   // ends the committer when reached
      float q = 0.f;
#pragma unroll
      for (int c = 0; c < kFC; ++c) {
        if (c >= nch[r]) break;
        const int32_t row = sc[r].fi[c];
        const float x = sc[r].fx[c];
        if (row >= 0) q += x * x;
        const int slot = cache_find<LC>(s_hkey, s_hslot, row);
        // rows with a delta, over the whole wave: skip features no row of it has
        const uint64_t any = __builtin_amdgcn_ballot_w64(slot >= 0);
        if (any == 0) continue;
        for (int u = 0; u < 16; ++u) {
          // lanes u of the four rows
          if (((any >> u) | (any >> (16 + u)) | (any >> (32 + u)) | (any >> (48 + u))) & 1ull) {
            const int su = rowb_i(slot, base, u);
            const float xu = rowb_f(x, base, u);
            if (su >= 0) {
#pragma unroll
              for (int k = 0; k < K; ++k) {
                const int lab = sub + 16 * k;
                if (lab < LC) sc[r].s[k] += xu * s_dw[su * LC + lab];
              }
            }
          }
        }
      }
      nrm[r] = row16_sum(q);
      int ls;
      float sy, best;
      const float m = group_margin<LC>(sc[r].s, y, act, sub, base, &ls, &sy, &best);
      unsafe[r] = may_update(method, m, nrm[r], ls >= 0, C, sy, best);
    }

    int lim = -1;               // round positions <= lim are settled
    int rstop = kNS;            // first position this round did not settle
    for (;;) {
      int myfirst = kInf;
#pragma unroll
      for (int r = kR - 1; r >= 0; --r) {
        const int pos = G * kR + r;
        if (alive[r] && unsafe[r] && pos > lim) myfirst = pos;
      }
      myfirst = min(myfirst, partner16_i(myfirst, lane));
      myfirst = min(myfirst, partner32_i(myfirst, lane));
      if (lane == 0 && myfirst != kInf) atomicMin(&s_first[iter & 1], myfirst);
      lds_barrier();            // A: the first sample of the round that may update
      const int k = s_first[iter & 1];
      if (tid == 0) s_first[(iter + 1) & 1] = kInf;
      ++iter;
      if (k == kInf) break;
      if (G == k / kR) {
        // ---------------- the exact step of sample k (this group's 16 lanes)
        const int rk = k % kR;
        Samp<LC> t = sc[0];
        Desc dd = dc[0];
        float tn = nrm[0];
#pragma unroll
        for (int r = 1; r < kR; ++r)
          if (r == rk) { t = sc[r]; dd = dc[r]; tn = nrm[r]; }
        const int y = dd.y;
        // the previous step's table is no longer read (barrier A)
        for (int i = sub; i < s_sn; i += 16) {
          const int h = s_spos[i];
          s_skey[h] = -1; s_sdy[h] = 0.f; s_sdl[h] = 0.f;
        }
        int nvalid = 0;
#pragma unroll
        for (int c = 0; c < kFC; ++c) nvalid += t.fi[c] >= 0 ? 1 : 0;
        nvalid = (int)row16_sum((float)nvalid);
        lds_wait();
        if (sub == 0) s_sn = 0;
        if (dd.nf > kNFMax) {
          if (sub == 0) s_stop = (int)kStopDense;
        } else if (s_cn + nvalid > NSLOT) {
          if (sub == 0) s_stop = (int)kStopSaturated;
        } else {
          int slot[kFC];
          const int nc = (dd.nf + 15) >> 4;
#pragma unroll
          for (int c = 0; c < kFC; ++c) slot[c] = c < nc ? cache_find<LC>(s_hkey, s_hslot, t.fi[c]) : -1;
          float py[kFC], pl[kFC];
          int ls = -1;
          float m = 0.f, sy = 0.f, best = 0.f, var = 0.f;
          bool refreshed = false;
          for (;;) {
            m = group_margin<LC>(t.s, y, act, sub, base, &ls, &sy, &best);
            float v = 0.f;
#pragma unroll
            for (int c = 0; c < kFC; ++c) {
              py[c] = 1.f;
              pl[c] = 1.f;
              const int32_t row = t.fi[c];
              if (!use_s || row < 0) continue;
              const int64_t rb = (int64_t)row * LC;
              py[c] = P[rb + y] + (slot[c] >= 0 ? s_dp[slot[c] * LC + y] : 0.f);
              if (ls >= 0) pl[c] = P[rb + ls] + (slot[c] >= 0 ? s_dp[slot[c] * LC + ls] : 0.f);
              const float x2 = t.fx[c] * t.fx[c];
              v += x2 * (1.f / py[c] + (ls >= 0 ? 1.f / pl[c] : 0.f));
            }
            var = use_s ? row16_sum(v) : 0.f;
            if (refreshed) break;
            const float thr = method == PERCEPTRON ? 0.f : method == CW ? C * var : 1.f;
            const float g = kGuard * (1.f + fabsf(sy) + fabsf(best));
            if (!(fabsf(m - thr) < g)) break;
            // near the threshold: re-score from the live model (M0 + dW)
            refreshed = true;
            if (sub == 0) atomicAdd(&s_refresh, 1u);
            float ns[K];
#pragma unroll
            for (int kk = 0; kk < K; ++kk) ns[kk] = 0.f;
#pragma unroll
            for (int c = 0; c < kFC; ++c) {
              if (c >= nc) break;
              for (int u = 0; u < 16; ++u) {
                const int32_t ru = rowb_i(t.fi[c], base, u);
                const float xu = rowb_f(t.fx[c], base, u);
                const int su = rowb_i(slot[c], base, u);
                if (ru < 0) continue;
#pragma unroll
                for (int kk = 0; kk < K; ++kk) {
                  const int lab = sub + 16 * kk;
                  if (lab < LC)
                    ns[kk] += xu * (W[(int64_t)ru * LC + lab] + (su >= 0 ? s_dw[su * LC + lab] : 0.f));
                }
              }
            }
#pragma unroll
            for (int kk = 0; kk < K; ++kk) t.s[kk] = ns[kk];
          }
          float tau = 0.f, beta = 0.f;
          const bool up = step_coeffs(method, m, var, tn, ls >= 0, C, &tau, &beta);
          if (up) {
            uint32_t hp[kFC];
#pragma unroll
            for (int c = 0; c < kFC; ++c)
              hp[c] = (t.fi[c] >= 0 && slot[c] < 0)
                          ? cache_insert<LC>(s_hkey, s_hslot, s_ckey, &s_cn, t.fi[c]) : 0u;
            lds_wait();
#pragma unroll
            for (int c = 0; c < kFC; ++c)
              if (t.fi[c] >= 0 && slot[c] < 0) slot[c] = s_hslot[hp[c]];
#pragma unroll
            for (int c = 0; c < kFC; ++c) {
              const int32_t row = t.fi[c];
              if (row < 0) continue;
              const float x = t.fx[c];
              const float a = use_s ? 1.f / py[c] : 1.f;
              const float b = (use_s && ls >= 0) ? 1.f / pl[c] : 1.f;
              const float dwy = tau * a * x;
              const float dwl = ls >= 0 ? -tau * b * x : 0.f;
              float* dwr = s_dw + slot[c] * LC;
              atomicAdd(dwr + y, dwy);
              if (ls >= 0) atomicAdd(dwr + ls, dwl);
              if (use_s) {
                float* dpr = s_dp + slot[c] * LC;
                atomicAdd(dpr + y, dprec(method, beta, x, a));
                if (ls >= 0) atomicAdd(dpr + ls, dprec(method, beta, x, b));
              }
              // the step table: this update's increments per row
              uint32_t h = hmix(row) >> (32 - ilog2(kSHS));
              for (int q = 0; q < kSHS; ++q) {
                const int32_t old = atomicCAS(&s_skey[h], -1, row);
                if (old == -1) { s_spos[atomicAdd(&s_sn, 1)] = (int)h; break; }
                if (old == row) break;
                h = (h + 1) & (kSHS - 1);
              }
              atomicAdd(&s_sdy[h], dwy);
              atomicAdd(&s_sdl[h], dwl);
            }
          }
          if (sub == 0) {
            s_upd = up ? 1 : 0;
            s_yk = y;
            s_lk = ls;
            if (up) atomicAdd(&s_nupd, 1u); else atomicAdd(&s_waste, 1u);
          }
        }
      }
      lds_barrier();            // B: the step (or the stop) is visible
      ++n_steps;
      const int sc_stop = s_stop;
      if (sc_stop >= 0) {
        rstop = k;
        why = sc_stop;
        stop = p + k;
        break;
      }
      if (s_upd) {
        const int yk = s_yk, lk = s_lk;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          const int pos = G * kR + r;
          if (!alive[r] || pos <= k || dc[r].nf > kNFMax) continue;
          float cy = 0.f, cl = 0.f;
#pragma unroll
          for (int c = 0; c < kFC; ++c) {
            if (c >= nch[r]) break;
            const int h = step_find(s_skey, sc[r].fi[c]);
            if (h >= 0) {
              cy += sc[r].fx[c] * s_sdy[h];
              cl += sc[r].fx[c] * s_sdl[h];
            }
          }
          cy = row16_sum(cy);
          cl = row16_sum(cl);
#pragma unroll
          for (int kk = 0; kk < K; ++kk) {
            const int lab = sub + 16 * kk;
            if (lab == yk) sc[r].s[kk] += cy;
            if (lab == lk) sc[r].s[kk] += cl;
          }
          int ls;
          float sy, best;
          const float m = group_margin<LC>(sc[r].s, dc[r].y, act, sub, base, &ls, &sy, &best);
          unsafe[r] = may_update(method, m, nrm[r], ls >= 0, C, sy, best);
        }
      }
      lim = k;
    }
    ++n_rounds;
    if (sub == 0) {
#pragma unroll
      for (int r = 0; r < kR; ++r)
        if (alive[r] && G * kR + r < rstop) ++n_valid;
    }
    if (stop != end) break;
  }
  __syncthreads();
  // ---- segment end: the deltas into the tables (the committer is their only writer)
  {
    const int n = s_cn;
    for (int i = tid; i < n * LC; i += kT) {
      const int sl = i / LC;
      const int l = i % LC;
      const int64_t row = s_ckey[sl];
      W[row * LC + l] += s_dw[i];
      if (use_s) P[row * LC + l] += s_dp[i];
      if (l == 0 && touched != nullptr) touched[row] = 1;
    }
  }
  if (n_valid > 0 && stats != nullptr) atomicAdd(stats + 1, (unsigned long long)n_valid);
  if (tid == 0) {
    auto put = [&](int i, int64_t v) { tail[i] = seg == 0 ? v : tail[i] + v; };
    tail[0] = stop;
    tail[1] = end;
    tail[kTailReason] = why;
    put(2, n_steps);
    put(3, n_rounds);
    for (int i = 4; i < 20; ++i) put(i, 0);
    put(21, 1);
    put(22, (int64_t)s_waste);
    put(23, (int64_t)s_refresh);
    put(24, (int64_t)s_nupd);
    put(25, (int64_t)s_cn);
    if (stats != nullptr && s_nupd > 0) atomicAdd(stats, (unsigned long long)s_nupd);
  }
}

}  // namespace dc
}  // namespace jb

// Steps 1-2 of a kSerial batch for LC <= 64 (see the header); the caller
// runs the exact single-stream kernel over [tail[0], tail[1]) afterwards.
// scratch: [tail int64 x 32][S0: n_max x LC floats].
extern "C" int jb_delta_prepare(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                                int64_t n_max, float* W, float* S, const int32_t* active, int LC,
                                int method, float C, unsigned long long* stats, uint8_t* touched,
                                void* scratch, int nseg, hipStream_t stream) {
  if (LC > 64) return -1;
  int64_t* tail = (int64_t*)scratch;
  float* s0 = (float*)((uint8_t*)scratch + 256);
  const int64_t blocks = std::min<int64_t>((n_max * 64 + 255) / 256, 2048);
  for (int seg = 0; seg < nseg; ++seg) {
    const int64_t* sp = seg == 0 ? stream_ptr : tail;
    const int ns = seg == 0 ? nstreams : 1;
    const int64_t* why = seg == 0 ? nullptr : tail + jb::dc::kTailReason;
#define JB_DELTA(L)                                                                                \
  hipLaunchKernelGGL((jb::dc::delta_s0_kernel<L>), dim3((unsigned)blocks), dim3(256), 0, stream,  \
                     row_ptr, fidx, fval, sp, ns, W, s0, why);                                    \
  hipLaunchKernelGGL((jb::dc::delta_commit_kernel<L>), dim3(1), dim3(jb::dc::kT), 0, stream,       \
                     row_ptr, fidx, fval, labels, sp, ns, W, S, active, method, C, s0, stats,      \
                     touched, tail, seg);
    switch (LC) {
      case 8: JB_DELTA(8); break;
      case 16: JB_DELTA(16); break;
      case 32: JB_DELTA(32); break;
      case 64: JB_DELTA(64); break;
      default: return -1;
    }
#undef JB_DELTA
  }
  return (int)hipGetLastError();
}
