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

// Label capacities above 64: every sample on the direct path.
template <int LC, int MODE, typename WT>
__global__ __launch_bounds__(256) void linear_train_wide_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, WT* W, float* P,
    const int32_t* __restrict__ active, int method, float C,
    unsigned long long* __restrict__ stats, uint8_t* __restrict__ touched) {
  using L = Lanes<LC>;
  const int lane = threadIdx.x & 63;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (wid >= nstreams) return;
  bool act[L::K];
#pragma unroll
  for (int k = 0; k < L::K; ++k) act[k] = active[lane % L::LW + 64 * k] != 0;
  unsigned n_upd = 0, n_valid = 0;
  for (int64_t s = stream_ptr[wid]; s < stream_ptr[wid + 1]; ++s) {
    const int y = labels[s];
    if (y < 0 || y >= LC) continue;
    ++n_valid;
    const int64_t beg = row_ptr[s];
    if (general_sample<LC, MODE, WT>(fidx, fval, beg, (int)(row_ptr[s + 1] - beg), y, W, P, act, lane,
                                 method, C, touched))
      ++n_upd;
    if (MODE == kExact) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (stats != nullptr && lane == 0 && n_valid > 0) {
    atomicAdd(stats, (unsigned long long)n_upd);
    atomicAdd(stats + 1, (unsigned long long)n_valid);
  }
}

// ---------------------------------------------------------------------------
// Hot rows (concurrent modes). A feature row that most samples of a batch
// carry (the headline's always-present numeric keys, a bias feature) makes
// every stream issue memory-side atomics on the same few cache lines every
// sample; those serialise (~60 ns per line request): 9-11 ms per 131 072
// samples with 8 such rows (profiles/r01_train_kernel_contention.jsonl,
// profiles/r02_train_kernel_hot.jsonl). csrc/hip/hot.hip finds such rows per
// batch; the train kernel then keeps them out of the table:
//   * every block holds an LDS replica of the hot rows that its 4 streams
//     read and update (LDS atomics): the block's own updates are seen at once;
//   * blocks exchange their progress through kRep delta shards in global
//     memory (rep[r][t][e], block b adds to shard b % kRep): each sample, every
//     wave swaps the block's new increments of the entries it owns out of hA,
//     adds them to its shard with a returning atomic and reads the other
//     shards; a sample later (the round trip hides behind it) the other
//     blocks' progress is folded into hV. A shard line takes 1/kRep of the
//     atomics a table line took, and nothing writes the table rows;
//   * after the launch, hot_fold_kernel adds the summed shards to the table
//     and clears them.
// Every increment reaches the table exactly once; a stream sees other
// blocks' updates about two samples late (merge_every = 1). LDS per block:
//   hV  live value = table value at start + all shards seen + own since
//   hA  the block's increments not yet added to its shard
//   hB  the sum over shards at the block's last refresh
// Precision increments are additive (see header), so the same scheme serves
// W (t = 0) and P (t = 1).
#ifndef JB_KREP
#define JB_KREP 8
#endif
constexpr int kRep = JB_KREP;

template <int LC>
struct Hot {
  static constexpr int E = 512;                               // entries per table
  static constexpr int R = (E / LC) < 64 ? (E / LC) : 64;     // hot rows
  static constexpr int T = 128;                               // lookup slots
};

// hot slot of a row (-1: not hot); open addressing over hK/hS
__device__ __forceinline__ int hot_find(const int32_t* hK, const int32_t* hS, int32_t idx) {
  if (idx < 0) return -1;
  uint32_t h = ((uint32_t)idx * 0x9E3779B1u) >> 25;
  for (int p = 0; p < 128; ++p) {
    const int32_t k = hK[h];
    if (k == idx) return hS[h];
    if (k < 0) return -1;
    h = (h + 1) & 127;
  }
  return -1;
}

// Merge of the (chunk, table) pairs owned by wave `wv` (pair q = wv + NW k:
// chunk q / 2 of 64 entries, table q % 2), split in two: issue swaps the
// block delta out of hA, adds it to the block's shard (returning
// memory-side atomic) and loads the other shards; finish folds the other
// blocks' progress into hV and moves hB. The train loop issues a merge
// right after the sample's gather and descriptor loads and finishes it one
// sample later, before the next merge: the in-order vmcnt then never makes a
// gather wait for a merge (their ~us round trip stays off the sample chain),
// and the finish waits only for the merge itself.
template <int LC, int NW>
struct HotMerge {
  static constexpr int KQ = 2 * Hot<LC>::E / 64 / NW;  // pairs per wave
  float d[KQ];
  float own[KQ];
  float oth[KQ][kRep - 1];
  bool pending = false;

  template <int E>
  __device__ __forceinline__ void issue(const float* rep, int rr, bool use_s, int nent,
                                        float (*hA)[E], int wv, int lane) {
#pragma unroll
    for (int k = 0; k < KQ; ++k) {
      const int q = wv + NW * k;
      const int t = q & 1;
      const int e = (q >> 1) * 64 + lane;
      if (e < nent && (t == 0 || use_s)) {
        float* sh = const_cast<float*>(rep) + (int64_t)(rr * 2 + t) * E + e;
        d[k] = atomicExch(&hA[t][e], 0.f);
        own[k] = d[k] != 0.f ? atomicAdd(sh, d[k]) : ld_agent(sh);
#pragma unroll
        for (int j = 0; j < kRep - 1; ++j) {
          const int r = j < rr ? j : j + 1;
          oth[k][j] = ld_agent(rep + (int64_t)(r * 2 + t) * E + e);
        }
      }
    }
    pending = true;
  }

  template <int E>
  __device__ __forceinline__ void finish(bool use_s, int nent, float (*hV)[E], float (*hB)[E],
                                         float* hD, int wv, int lane) {
    if (!pending) return;
#pragma unroll
    for (int k = 0; k < KQ; ++k) {
      const int q = wv + NW * k;
      const int t = q & 1;
      const int e = (q >> 1) * 64 + lane;
      if (e < nent && (t == 0 || use_s)) {
        float S = own[k] + d[k];
#pragma unroll
        for (int j = 0; j < kRep - 1; ++j) S += oth[k][j];
        const float others = S - hB[t][e] - d[k];
        atomicAdd(&hV[t][e], others);
        if (t == 1) hD[e] = others;     // the other blocks' precision growth per merge
        hB[t][e] = S;
      }
    }
    pending = false;
  }
};

// After a hot launch: table += sum of the shards, shards := 0 (one thread
// per hot entry and table; stream-ordered after the train kernel, so plain
// read-modify-write).
template <int LC>
__global__ __launch_bounds__(256) void hot_fold_kernel(float* W, float* P, int use_s,
                                                       const int32_t* __restrict__ hot_rows,
                                                       const int32_t* __restrict__ hot_n,
                                                       float* __restrict__ rep,
                                                       uint8_t* __restrict__ touched) {
  constexpr int E = Hot<LC>::E;
  const int nh = min(*hot_n, Hot<LC>::R);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int e = i % E;
  const int t = i / E;
  if (e >= nh * LC || t > 1 || (t == 1 && !use_s)) return;
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < kRep; ++r) {
    float* p = rep + (int64_t)(r * 2 + t) * E + e;
    s += *p;
    *p = 0.f;
  }
  const int32_t row = hot_rows[e / LC];
  float* T = t == 0 ? W : P;
  if (s != 0.f) T[(int64_t)row * LC + (e % LC)] += s;
  if (touched != nullptr && t == 0 && e % LC == 0) touched[row] = 1;
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
// Features of hot rows (HOT) are staged as -2 - slot and read from the LDS
// replica at use time instead of being gathered.
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

__device__ __forceinline__ float readlane_f(float v, int i) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i));
}

// Issue the gather of one staged sample: lane (g, l0) loads W / P of
// features u*G + g, label l0. Every load is unconditional (invalid and hot
// slots read row 0) and nothing reads the results here, so the whole gather
// is U (or 2U) loads in flight; ``vmask`` bit u marks the valid slots for the
// commit.
template <int LC, typename WT>
__device__ __forceinline__ uint32_t gather_issue(const WT* W, const float* P, bool use_s,
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
      gw[u] = ldw(W + rows[u]);
      gp[u] = ld_agent(P + rows[u]);
    }
  } else {
#pragma unroll
    for (int u = 0; u < Q::U; ++u) {
      gw[u] = ldw(W + rows[u]);
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

// feature list of a sample into its LDS slot (lane j = feature j); hot rows
// are staged as -2 - slot
template <int LC>
__device__ __forceinline__ void put_features(int32_t* sI, float* sX, int32_t idx, int hs, float x,
                                             int n, int lane) {
  if (lane < Pipe<LC>::F) {
    const bool v = lane < n && idx >= 0;
    sI[lane] = v ? (hs >= 0 ? -2 - hs : idx) : -1;
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

template <int LC, int MODE, bool HOT, int NW, typename WT>
__global__ __launch_bounds__(64 * NW) void linear_train_pipe_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, WT* W, float* P,
    const int32_t* __restrict__ active, int method, float C, const int32_t* __restrict__ hot_rows,
    const int32_t* __restrict__ hot_n, float* __restrict__ hot_rep, int merge_every,
    unsigned long long* __restrict__ stats, uint8_t* __restrict__ touched) {
  using Q = Pipe<LC>;
  using HT = Hot<LC>;
  constexpr int F = Q::F;
  constexpr int HE = HOT ? HT::E : 1;
  constexpr int HK = HOT ? HT::T : 1;
  constexpr int HR = HOT ? HT::R : 1;
  __shared__ float sW[NW][2][F * LC];
  __shared__ float sP[NW][2][F * LC];
  __shared__ int32_t sI[NW][2][F];
  __shared__ float sX[NW][2][F];
  __shared__ float hV[2][HE];
  __shared__ float hA[2][HE];
  __shared__ float hB[2][HE];
  __shared__ float hD[HE];
  __shared__ int32_t hK[HK];
  __shared__ int32_t hS[HK];
  __shared__ int32_t hR[HR];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const bool use_s = method >= CW;
  int nent = 0;
  if (HOT) {
    const int nh = min(*hot_n, HT::R);
    nent = nh * LC;
    for (int i = threadIdx.x; i < HT::T; i += blockDim.x) hK[i] = -1;
    __syncthreads();
    if ((int)threadIdx.x < nh) {
      const int32_t r = hot_rows[threadIdx.x];
      hR[threadIdx.x] = r;
      uint32_t h = ((uint32_t)r * 0x9E3779B1u) >> 25;
      for (int p = 0; p < HT::T; ++p) {
        const int32_t old = atomicCAS(&hK[h], -1, r);
        if (old == -1) { hS[h] = threadIdx.x; break; }
        if (old == r) break;
        h = (h + 1) & 127;
      }
    }
    for (int e = threadIdx.x; e < nent; e += blockDim.x) {
      const int64_t a = (int64_t)hot_rows[e / LC] * LC + (e % LC);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (t == 1 && !use_s) break;
        float S = 0.f;                  // shards of blocks that ran before this one
#pragma unroll
        for (int r = 0; r < kRep; ++r) S += ld_agent(hot_rep + (int64_t)(r * 2 + t) * HE + e);
        hV[t][e] = (t == 0 ? ldw(W + a) : ld_agent(P + a)) + S;
        hB[t][e] = S;
        hA[t][e] = 0.f;
        if (t == 1) hD[e] = 0.f;
      }
    }
    __syncthreads();
  }
  const int rr = blockIdx.x % kRep;
  const int64_t s_beg = wid < nstreams ? stream_ptr[wid] : 0;
  const int64_t s_end = wid < nstreams ? stream_ptr[wid + 1] : 0;
  unsigned n_upd = 0, n_valid = 0;
  if (s_beg < s_end) {
  const int g = lane / LC;
  const int l0 = lane % LC;
  bool act[1] = {active[l0] != 0};
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
  int hs_s = (HOT && nent > 0) ? hot_find(hK, hS, idx_s) : -1;
  int hs1 = (HOT && nent > 0) ? hot_find(hK, hS, idx1) : -1;
  put_features<LC>(sI[wv][0], sX[wv][0], idx_s, hs_s, x_s, n_s, lane);
  put_features<LC>(sI[wv][1], sX[wv][1], idx1, hs1, x1, n1, lane);
  float gw[Q::U], gp[Q::U];
  uint32_t vmask = 0;
  bool staged = n_s <= F;
  if (staged) {
    vmask = gather_issue<LC, WT>(W, P, use_s, sI[wv][0], n_s, g, l0, gw, gp);
    gather_commit<LC>(sW[wv][0], sP[wv][0], use_s, n_s, g, l0, vmask, gw, gp);
  }
  int since_merge = 0;
  HotMerge<LC, NW> mrg;

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
    if (early) vmask = gather_issue<LC, WT>(W, P, use_s, sI[wv][c1], n1, g, l0, gw, gp);
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
    // 2b. hot rows: retire the previous merge, send the block's increments
    //     so far (see HotMerge for why here)
    if constexpr (HOT) {
      if (nent > 0 && ++since_merge >= merge_every) {
        since_merge = 0;
        mrg.template finish<HE>(use_s, nent, hV, hB, hD, wv, lane);
        mrg.template issue<HE>(hot_rep, rr, use_s, nent, hA, wv, lane);
      }
    }
    // 3. sample s (LDS + registers only while the loads above are in flight)
    bool upd = false;
    int lstar = -1;
    float dwy = 0.f, dwl = 0.f, dpy = 0.f, dpl = 0.f, py = 1.f, pl = 1.f, wy = 0.f, wl = 0.f;
    float tau_s = 0.f;
    bool ser = false, p_done = false;   // serialized confidence (atomic mode), P applied
    const bool mine = lane < n_s && idx_s >= 0;
    if (valid_s) ++n_valid;
    if (general_s) {
      const int i = (int)(s - wb);
      const int64_t b0 = readlane64(rp, i);
      upd = general_sample<LC, MODE, WT>(fidx, fval, b0, (int)(readlane64(rp, i + 1) - b0), y_s, W, P,
                                     act, lane, method, C, touched);
      if (upd) ++n_upd;
      upd = false;        // applied already
    } else if (valid_s) {
      const float* cw = sW[wv][c];
      const float* cp = sP[wv][c];
      const float* cx = sX[wv][c];
      const int32_t* ci = sI[wv][c];
      float acc = 0.f;
#pragma unroll
      for (int u = 0; u < Q::U; ++u) {
        const int j = u * Q::G + g;
        if (j < n_s) {
          float w = cw[j * LC + l0];
          if (HOT) {
            const int32_t si = ci[j];
            if (si <= -2) w = hV[0][(-2 - si) * LC + l0];
          }
          acc += cx[j] * w;
        }
      }
      acc = group_sum<LC>(acc, lane);
      const float sy = readlane_f(acc, y_s);
      float best = (act[0] && l0 != y_s) ? acc : -INFINITY;
      int bl = (act[0] && l0 != y_s) ? l0 : -1;
      group_argmax<LC>(best, bl, lane);
      lstar = __builtin_amdgcn_readfirstlane(bl);
      best = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(best)));
      const float margin = sy - (lstar >= 0 ? best : 0.f);
      float a = 1.f, b = 1.f, x2s = 0.f;
      if (mine) {
        x2s = x_s * x_s;
        if (HOT && hs_s >= 0) {
          const int hb = hs_s * LC;
          wy = hV[0][hb + y_s];
          wl = lstar >= 0 ? hV[0][hb + lstar] : 0.f;
          if (use_s) {
            py = hV[1][hb + y_s];
            pl = lstar >= 0 ? hV[1][hb + lstar] : 1.f;
          }
        } else {
          if (use_s) {
            py = cp[lane * LC + y_s];
            pl = lstar >= 0 ? cp[lane * LC + lstar] : 1.f;
          }
          wy = cw[lane * LC + y_s];
          wl = lstar >= 0 ? cw[lane * LC + lstar] : 0.f;
        }
        if (use_s) {
          a = 1.f / py;
          b = lstar >= 0 ? 1.f / pl : 0.f;
        }
      }
      const float var = use_s ? wave_sum_fast(x2s * (a + b), lane) : 0.f;
      const float nrm = wave_sum_fast(x2s, lane);
      float tau = 0.f, beta = 0.f;
      upd = step_coeffs(method, margin, var, nrm, lstar >= 0, C, &tau, &beta);
      if (upd) ++n_upd;
      if (upd && mine) {
        dwy = use_s ? tau * a * x_s : tau * x_s;
        dwl = use_s ? -tau * b * x_s : -tau * x_s;
        if (use_s) {
          dpy = dprec(method, beta, x_s, a);
          dpl = lstar >= 0 ? dprec(method, beta, x_s, b) : 0.f;
        }
      }
      // Serialized confidence (concurrent atomic streams, confidence methods):
      // the precision increment goes first with a returning atomic, and the W
      // step uses the variance 1/P at this update's place in the atomic order
      // of the row instead of the value gathered before the sample. Streams
      // that update a shared row at the same time then shrink each other's
      // steps as sequential updates would (without it, ~1000 streams sharing a
      // row all step with the same stale confidence and the weights grow
      // ~40x past the serial model's, profiles/r02_concurrent_vs_serial.jsonl).
      // One stream is unaffected: its returned P is the value it gathered.
      // Rows repeated inside the sample keep the gathered value (the
      // reference applies a sample's features against the pre-sample state).
      // Cost: one returning atomic per updated feature on the sample chain;
      // the worst case (every sample updates) runs ~10% slower end to end,
      // data with few updates is unchanged (profiles/r02_serialized_confidence.jsonl).
      if (MODE == kAtomic && use_s && upd) {
        bool dup = false;
        for (int j = 0; j < n_s; ++j) {
          const int32_t ij = __builtin_amdgcn_readlane(idx_s, j);
          dup |= mine && j != lane && ij == idx_s;
        }
        tau_s = tau;
        ser = mine && !dup;
        // (rows of the hot-row replica are serialized in LDS at apply time)
        if (ser && !(HOT && hs_s >= 0)) {
          const int64_t row = (int64_t)idx_s * LC;
          dwy = tau * x_s / atomicAdd(P + row + y_s, dpy);
          if (lstar >= 0) dwl = -tau * x_s / atomicAdd(P + row + lstar, dpl);
          p_done = true;
        }
      }
    }
    // 4. stage s+1 and forward s's own increments into it: lane k (feature k
    //    of s+1) scans s's features through readlane (registers only)
    if (early) {
      gather_commit<LC>(sW[wv][c1], sP[wv][c1], use_s, n1, g, l0, vmask, gw, gp);
      if (upd) {
        float fwy = 0.f, fwl = 0.f, fpy = 0.f, fpl = 0.f;
        const bool kv = lane < n1 && idx1 >= 0 && hs1 < 0;
        for (int j = 0; j < n_s; ++j) {
          const int32_t ij = __builtin_amdgcn_readlane(idx_s, j);
          const bool hit = kv && ij == idx1;
          if (__builtin_amdgcn_ballot_w64(hit)) {
            const float ay = readlane_f(dwy, j);
            const float al = readlane_f(dwl, j);
            const float by = readlane_f(dpy, j);
            const float bq = readlane_f(dpl, j);
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
    const int hs2 = (HOT && nent > 0) ? hot_find(hK, hS, idx2) : -1;
    // 5. apply s to the table. Plain-store modes first fold the increments
    //    of a repeated row (same index twice in one sample) into its first
    //    lane, so both count (as the atomic and LDS paths do).
    bool skip = false;
    if (MODE != kAtomic && upd) {
      float cy = 0.f, cl = 0.f, qy = 0.f, ql = 0.f;
      const bool plain = mine && hs_s < 0;
      for (int j = 0; j < n_s; ++j) {
        const int32_t ij = __builtin_amdgcn_readlane(idx_s, j);
        const bool same = plain && ij == idx_s && j != lane;
        if (__builtin_amdgcn_ballot_w64(same)) {
          const float ay = readlane_f(dwy, j);
          const float al = readlane_f(dwl, j);
          const float by = readlane_f(dpy, j);
          const float bq = readlane_f(dpl, j);
          if (same) {
            if (j < lane) skip = true;
            else { cy += ay; cl += al; qy += by; ql += bq; }
          }
        }
      }
      dwy += cy; dwl += cl; dpy += qy; dpl += ql;
    }
    if (upd && mine && !skip) {
      if (HOT && hs_s >= 0) {
        const int hb = hs_s * LC;
        if (use_s) {   // precision first: its returned value serializes the W step
          // inside the block; the other blocks' updates arrive a merge late,
          // so the growth they added since this replica's view (about one
          // merge's worth, estimated by the last merge's) is counted in full
          // (profiles/r02_serialized_confidence.jsonl: full 9.6x vs half
          // 10.9x weight distance to the serial order)
          const float p0 = atomicAdd(&hV[1][hb + y_s], dpy);
          atomicAdd(&hA[1][hb + y_s], dpy);
          if (MODE == kAtomic && ser) dwy = tau_s * x_s / (p0 + hD[hb + y_s]);
          if (lstar >= 0) {
            const float q0 = atomicAdd(&hV[1][hb + lstar], dpl);
            atomicAdd(&hA[1][hb + lstar], dpl);
            if (MODE == kAtomic && ser) dwl = -tau_s * x_s / (q0 + hD[hb + lstar]);
          }
        }
        atomicAdd(&hV[0][hb + y_s], dwy);
        atomicAdd(&hA[0][hb + y_s], dwy);
        if (lstar >= 0) {
          atomicAdd(&hV[0][hb + lstar], dwl);
          atomicAdd(&hA[0][hb + lstar], dwl);
        }
      } else {
        const int64_t row = (int64_t)idx_s * LC;
        const uint32_t ry = jb_mix32((uint32_t)(row + y_s), (uint32_t)s);
        const uint32_t rl = jb_mix32((uint32_t)(row + lstar), (uint32_t)s);
        if (MODE == kAtomic) {
          addw(W + row + y_s, dwy, ry);
          if (lstar >= 0) addw(W + row + lstar, dwl, rl);
          if (use_s && !p_done) {
            atomicAdd(P + row + y_s, dpy);
            if (lstar >= 0) atomicAdd(P + row + lstar, dpl);
          }
        } else {
          stw(W + row + y_s, wy + dwy, ry);
          if (lstar >= 0) stw(W + row + lstar, wl + dwl, rl);
          if (use_s) {
            P[row + y_s] = py + dpy;
            if (lstar >= 0) P[row + lstar] = pl + dpl;
          }
        }
        if (touched != nullptr) touched[idx_s] = 1;
      }
    }
    if (MODE == kExact && (upd || general_s)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // 6. s+1 not prefetched (s took the direct path): stage it now that s landed
    if (pipe1 && !early) {
      if (MODE != kExact) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      vmask = gather_issue<LC, WT>(W, P, use_s, sI[wv][c1], n1, g, l0, gw, gp);
      gather_commit<LC>(sW[wv][c1], sP[wv][c1], use_s, n1, g, l0, vmask, gw, gp);
    }
    // slot c is free again: it receives the features of s+2
    put_features<LC>(sI[wv][c], sX[wv][c], idx2, hs2, x2, n2, lane);
    __builtin_amdgcn_wave_barrier();
    staged = pipe1;
    idx_s = idx1; x_s = x1; n_s = n1; y_s = y1; hs_s = hs1;
    idx1 = idx2; x1 = x2; n1 = n2; y1 = y2; hs1 = hs2;
  }
  if constexpr (HOT) mrg.template finish<HE>(use_s, nent, hV, hB, hD, wv, lane);
  }  // s_beg < s_end
  if (stats != nullptr && lane == 0 && n_valid > 0) {
    atomicAdd(stats, (unsigned long long)n_upd);
    atomicAdd(stats + 1, (unsigned long long)n_valid);
  }
  if (HOT) {
    __syncthreads();      // every stream of the block has applied its last sample
    for (int e = threadIdx.x; e < nent; e += blockDim.x) {
      const float dw = hA[0][e];
      if (dw != 0.f) atomicAdd(hot_rep + (int64_t)(rr * 2) * HE + e, dw);
      if (use_s) {
        const float dp = hA[1][e];
        if (dp != 0.f) atomicAdd(hot_rep + (int64_t)(rr * 2 + 1) * HE + e, dp);
      }
    }
  }
}

template <int LC, typename WT>
__global__ __launch_bounds__(256) void linear_classify_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, int n_samples, const WT* W, float* __restrict__ out) {
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

// hot_rows / hot_n (device): rows to keep in the block LDS replica (nullptr:
// none; only the concurrent modes with LC <= 64 use them); hot_rep: the
// delta shards (jb_hot_rep_bytes(), zero-initialised once, left zero). stats (device,
// 2 x u64, nullable): += samples that updated, samples with a valid label.
// touched (device, H bytes, nullable): set to 1 for every row an update wrote.
// mode kSerial (several streams, serial-equivalent result, serial.hip) needs
// n_max >= the batch's sample count and scratch of jb_serial_scratch_bytes_lc(n_max, LC).
extern "C" int64_t jb_serial_scratch_bytes(int64_t n_max);
extern "C" int jb_serial_prepare(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                 const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                                 int64_t n_max, float* W, float* S, const int32_t* active, int LC,
                                 int method, float C, unsigned long long* stats, uint8_t* touched,
                                 void* scratch, int64_t scratch_bytes, int bail_after,
                                 hipStream_t stream);
// stepper.hip: one stream of samples applied in order from an LDS row cache
extern "C" int jb_stepper_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                const int32_t* labels, const int64_t* range, float* W, float* P,
                                const int32_t* active, int LC, int method, float C, unsigned long long* stats,
                                uint8_t* touched, int* err, hipStream_t stream);
extern "C" int jb_stepper_enabled();
// exact steps per 1024-sample committer round past which the rest of a
// kSerial batch goes to the sequential kernel (an exact step costs a few
// times a sequential sample; see serial.hip)
constexpr int kSerialBail = 128;

namespace jb {

// one stream spanning a whole batch: sp[0] .. sp[nstreams] (the streams are
// contiguous in request order, so this is the batch applied serially)
__global__ void stream_span_kernel(const int64_t* __restrict__ sp, int nstreams,
                                   int64_t* __restrict__ out) {
  if (threadIdx.x == 0) {
    out[0] = sp[0];
    out[1] = sp[nstreams];
  }
}

template <typename WT, int L, int M>
void launch_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                  const int32_t* labels, const int64_t* stream_ptr, int nstreams, WT* W, float* S,
                  const int32_t* active, int method, float C, bool hot, int hot_nw,
                  const int32_t* hot_rows, const int32_t* hot_n, float* hot_rep, int merge_every,
                  unsigned long long* stats, uint8_t* touched, hipStream_t stream) {
  const int threads = 256;
  const int blocks = (nstreams * 64 + threads - 1) / threads;
  const int hblocks = (nstreams + hot_nw - 1) / hot_nw;
#define JB_PIPE(H, NWV, B)                                                                      \
  hipLaunchKernelGGL((linear_train_pipe_kernel<L, M, H, NWV, WT>), dim3(B), dim3(64 * NWV), 0,  \
                     stream, row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S, active,   \
                     method, C, hot_rows, hot_n, hot_rep, merge_every, stats, touched);
  if constexpr (L <= 64) {
    // the hot-row replica (concurrent modes) keeps fp32 rows in LDS and folds
    // them into an fp32 table; bf16 tables train without it
    if constexpr (M != kExact && sizeof(WT) == 4) {
      if (hot) {
        if constexpr (L <= 16) {
          if (hot_nw == 16) { JB_PIPE(true, 16, hblocks) return; }
        }
        if (hot_nw == 4) { JB_PIPE(true, 4, hblocks) }
        else { JB_PIPE(true, 8, hblocks) }
        return;
      }
    }
    JB_PIPE(false, 4, blocks)
  } else {
    hipLaunchKernelGGL((linear_train_wide_kernel<L, M, WT>), dim3(blocks), dim3(threads), 0, stream,
                       row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S, active, method, C,
                       stats, touched);
  }
#undef JB_PIPE
}

template <typename WT, int L>
void launch_train_mode(int mode, const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                       const int32_t* labels, const int64_t* stream_ptr, int nstreams, WT* W,
                       float* S, const int32_t* active, int method, float C, bool hot, int hot_nw,
                       const int32_t* hot_rows, const int32_t* hot_n, float* hot_rep,
                       int merge_every, unsigned long long* stats, uint8_t* touched,
                       hipStream_t stream) {
#define JB_ARGS row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S, active, method, C, hot, \
                hot_nw, hot_rows, hot_n, hot_rep, merge_every, stats, touched, stream
  if (mode == kAtomic) launch_train<WT, L, kAtomic>(JB_ARGS);
  else if (mode == kHogwild) launch_train<WT, L, kHogwild>(JB_ARGS);
  else launch_train<WT, L, kExact>(JB_ARGS);
#undef JB_ARGS
}

}  // namespace jb

// kSerial over a bf16 table: the committer of serial.hip works on fp32
// tables, so the batch runs as one sequential stream (the same serial result)
template <typename WT>
static int linear_train_impl(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                             const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                             WT* W, float* S, const int32_t* active, int LC, int method, float C,
                             int mode, const int32_t* hot_rows, const int32_t* hot_n,
                             float* hot_rep, int merge_every, int hot_waves,
                             unsigned long long* stats, uint8_t* touched, int64_t n_max,
                             void* scratch, int64_t scratch_bytes, hipStream_t stream) {
  if (nstreams <= 0) return 0;
  if (mode == jb::kSerial && nstreams == 1) mode = jb::kExact;
  if (mode == jb::kExact && nstreams > 1) mode = jb::kSerial;   // exact means serial-equivalent
  if (mode == jb::kSerial) {
    if constexpr (sizeof(WT) == 4) {
      // score + ordered commit, then the sequential kernel over what is left
      const int rc = jb_serial_prepare(row_ptr, fidx, fval, labels, stream_ptr, nstreams, n_max,
                                       W, S, active, LC, method, C, stats, touched, scratch,
                                       scratch_bytes, kSerialBail, stream);
      if (rc != 0) return rc;
    } else {
      if (scratch == nullptr || scratch_bytes < 16) return -3;
      hipLaunchKernelGGL(jb::stream_span_kernel, dim3(1), dim3(64), 0, stream, stream_ptr,
                         nstreams, (int64_t*)scratch);
    }
    stream_ptr = (const int64_t*)scratch;
    nstreams = 1;
    mode = jb::kExact;
    hot_rows = nullptr;
  }
  // one exact stream (a single request, or a kSerial batch's rest after its
  // committer) over an fp32 table: the stepper
  if constexpr (sizeof(WT) == 4) {
    if (mode == jb::kExact && nstreams == 1 && LC <= 64 && jb_stepper_enabled())
      return jb_stepper_train(row_ptr, fidx, fval, labels, stream_ptr, W, S, active, LC, method, C,
                              stats, touched, nullptr, stream);
  }
  const bool hot = sizeof(WT) == 4 && hot_rows != nullptr && hot_n != nullptr &&
                   hot_rep != nullptr && mode != jb::kExact && LC <= 64;
  if (merge_every < 1) merge_every = 1;
  // hot launches: 8 streams per block (half the blocks exchanging hot-row
  // progress through the shards; see "Hot rows")
  const int hot_nw = (hot_waves == 16 && LC <= 16) ? 16 : (hot_waves == 4 ? 4 : 8);
#define JB_TRAIN(L)                                                                             \
  jb::launch_train_mode<WT, L>(mode, row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S,   \
                               active, method, C, hot, hot_nw, hot_rows, hot_n, hot_rep,        \
                               merge_every, stats, touched, stream);
  JB_LC_DISPATCH(LC, JB_TRAIN)
#undef JB_TRAIN
  if constexpr (sizeof(WT) == 4) {
    if (hot) {
#define JB_FOLD(L)                                                                            \
  hipLaunchKernelGGL((jb::hot_fold_kernel<(L <= 64 ? L : 64)>), dim3(2 * jb::Hot<64>::E / 256), \
                     dim3(256), 0, stream, W, S, method >= jb::CW ? 1 : 0, hot_rows, hot_n,     \
                     hot_rep, touched);
      JB_LC_DISPATCH(LC, JB_FOLD)
#undef JB_FOLD
    }
  }
  return (int)hipGetLastError();
}

extern "C" int jb_linear_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                               const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                               float* W, float* S, const int32_t* active, int LC, int method,
                               float C, int mode, const int32_t* hot_rows, const int32_t* hot_n,
                               float* hot_rep, int merge_every, int hot_waves,
                               unsigned long long* stats, uint8_t* touched, int64_t n_max,
                               void* scratch, int64_t scratch_bytes, hipStream_t stream) {
  return linear_train_impl<float>(row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S, active,
                                  LC, method, C, mode, hot_rows, hot_n, hot_rep, merge_every,
                                  hot_waves, stats, touched, n_max, scratch, scratch_bytes, stream);
}

// the same over a bf16 W table (fp32 S); hot-row arguments are ignored
extern "C" int jb_linear_train_bf16(const int64_t* row_ptr, const int32_t* fidx,
                                    const float* fval, const int32_t* labels,
                                    const int64_t* stream_ptr, int nstreams, jb::bf16_t* W,
                                    float* S, const int32_t* active, int LC, int method, float C,
                                    int mode, unsigned long long* stats, uint8_t* touched,
                                    void* scratch, int64_t scratch_bytes, hipStream_t stream) {
  return linear_train_impl<jb::bf16_t>(row_ptr, fidx, fval, labels, stream_ptr, nstreams, W, S,
                                       active, LC, method, C, mode, nullptr, nullptr, nullptr, 1,
                                       8, stats, touched, 0, scratch, scratch_bytes, stream);
}

// bytes of the hot-row delta shards (float [kRep][2][E]); zero on first use
extern "C" int64_t jb_hot_rep_bytes() { return (int64_t)jb::kRep * 2 * jb::Hot<8>::E * 4; }

template <typename WT>
static int linear_classify_impl(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                int n_samples, const WT* W, int LC, float* out,
                                hipStream_t stream) {
  if (n_samples <= 0) return 0;
  const int threads = 256;
  const int blocks = (n_samples * 64 + threads - 1) / threads;
#define JB_CLS(L)                                                                           \
  hipLaunchKernelGGL((jb::linear_classify_kernel<L, WT>), dim3(blocks), dim3(threads), 0, \
                     stream, row_ptr, fidx, fval, n_samples, W, out);
  JB_LC_DISPATCH(LC, JB_CLS)
#undef JB_CLS
  return (int)hipGetLastError();
}

extern "C" int jb_linear_classify(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                  int n_samples, const float* W, int LC, float* out,
                                  hipStream_t stream) {
  return linear_classify_impl<float>(row_ptr, fidx, fval, n_samples, W, LC, out, stream);
}

extern "C" int jb_linear_classify_bf16(const int64_t* row_ptr, const int32_t* fidx,
                                       const float* fval, int n_samples, const jb::bf16_t* W,
                                       int LC, float* out, hipStream_t stream) {
  return linear_classify_impl<jb::bf16_t>(row_ptr, fidx, fval, n_samples, W, LC, out, stream);
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
