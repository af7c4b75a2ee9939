// Exact top-k (smallest distances) for the similarity engines, fused with
// the signature scan.
//
// Reference: similar_row_* / neighbor_row_* / LOF kNN (recommender_serv.cpp:170-200,
// nearest_neighbor_serv.cpp:138-172, anomaly_serv.cpp:157-244; the search
// itself is jubatus_core, EXTERNAL). Replaces "write an nq x N distance
// matrix, then a radix-select top-k over it" with:
//
//   K1  grid (blocks, nq): every block scans tiles of 2048 rows (8 per
//       thread, coalesced), computes the distance in registers (fused
//       XOR+popcount over the signature table for lsh / minhash /
//       euclid_lsh, or a read of a precomputed score vector), drops rows
//       worse than the block's running k-th best, and merges the survivors
//       into the block's top-k. Per wave the selection is a "pop" loop over
//       per-lane sorted register lists: each round is one wave64 butterfly
//       arg-min (64-wide, 6 shuffle steps) and the winning lane shifts its
//       list; it stops as soon as the wave minimum is +inf, so after the
//       first tile the pops cost almost nothing (few rows beat the
//       threshold). Output: k candidates per block.
//   K2  one block per query merges the blocks' candidates (same code).
//
// Ties are broken by the lower row index (the CPU oracle's stable order).
// Distances: metric 0 lsh (hamming / hash_num), 2 minhash (mismatch
// fraction), 1 euclid_lsh (law of cosines on the norms). Invalid rows: +inf.
#include <limits.h>

#include <atomic>
#include <stdlib.h>

#include "jb_device.hpp"
#include "jb_host_wait.hpp"

namespace jb {

constexpr int kTopThreads = 256;
constexpr int kTopR = 8;                          // rows per thread per tile
constexpr int kTopTile = kTopThreads * kTopR;     // 2048
constexpr int kTopMaxK = 128;
constexpr int kTopMaxWords = 16;                  // hash_num <= 1024

__device__ __forceinline__ bool lt_pair(float a, int ia, float b, int ib) {
  return a < b || (a == b && ia < ib);
}

// ascending insertion network over N register values (compile-time indices)
template <int N>
__device__ __forceinline__ void sort_regs(float (&d)[N], int (&ix)[N]) {
#pragma unroll
  for (int i = 1; i < N; ++i) {
#pragma unroll
    for (int j = i; j > 0; --j) {
      const bool sw = lt_pair(d[j], ix[j], d[j - 1], ix[j - 1]);
      const float a = d[j - 1], b = d[j];
      const int ia = ix[j - 1], ib = ix[j];
      d[j - 1] = sw ? b : a; d[j] = sw ? a : b;
      ix[j - 1] = sw ? ib : ia; ix[j] = sw ? ia : ib;
    }
  }
}

// wave64 arg-min of (v, id) with every lane getting the result, in
// registers only: DPP quad / half-row / row mirrors, then permlane16/32
// swaps (gfx950). A ds_bpermute butterfly costs an LDS round trip per step.
template <int CTRL>
__device__ __forceinline__ void argmin_step_dpp(float& v, int& id) {
  const float ov = dpp_f<CTRL>(v);
  const int oid = dpp_i<CTRL>(id);
  if (lt_pair(ov, oid, v, id)) { v = ov; id = oid; }
}

__device__ __forceinline__ void wave_argmin(float& v, int& id, int lane) {
  argmin_step_dpp<kDppXor1>(v, id);
  argmin_step_dpp<kDppXor2>(v, id);
  argmin_step_dpp<kDppHalfMirror>(v, id);
  argmin_step_dpp<kDppMirror>(v, id);
  {
    const float ov = partner16_f(v, lane);
    const int oid = partner16_i(id, lane);
    if (lt_pair(ov, oid, v, id)) { v = ov; id = oid; }
  }
  {
    const float ov = partner32_f(v, lane);
    const int oid = partner32_i(id, lane);
    if (lt_pair(ov, oid, v, id)) { v = ov; id = oid; }
  }
}

// Pops the k smallest (d, ix) of the wave's per-lane sorted lists into
// od/oi[0..k); stops early at +inf and pads with (+inf, INT_MAX). Returns
// the k-th value (or +inf when fewer than k finite values exist).
template <int N>
__device__ __forceinline__ float wave_pop(float (&d)[N], int (&ix)[N], int k,
                                          float* od, int* oi, int lane, int* popped = nullptr) {
  int r = 0;
  float last = INFINITY;
  for (; r < k; ++r) {
    float v = d[0];
    int id = ix[0];
    wave_argmin(v, id, lane);
    if (!(v < INFINITY)) break;                 // uniform across the wave
    const bool win = (ix[0] == id) && (d[0] == v);
#pragma unroll
    for (int j = 0; j < N - 1; ++j) {
      d[j] = win ? d[j + 1] : d[j];
      ix[j] = win ? ix[j + 1] : ix[j];
    }
    if (win) { d[N - 1] = INFINITY; ix[N - 1] = INT_MAX; }
    if (lane == 0) { od[r] = v; oi[r] = id; }
    last = v;
  }
  for (int j = r + lane; j < k; j += 64) { od[j] = INFINITY; oi[j] = INT_MAX; }
  if (popped != nullptr) *popped = r;
  return r == k ? last : INFINITY;
}

struct TopkSrc {
  // MODE 0: fused signature scan
  const uint64_t* qbits;
  const float* qnorm;
  const uint64_t* tbits;
  const float* tnorm;
  const uint8_t* valid;
  int words, hash_num, metric;
  // MODE 1: score vector [nq][n] (flip: distance = 1 - score)
  // MODE 2: candidate pairs [nq][n]
  const float* src_d;
  const int32_t* src_i;
  int flip;
};

// The distance of row r (n: rows of the source, 0 = r is out of range).
// Branch-free: an out-of-range row loads row 0 and is masked afterwards, and
// the norm's address is selected rather than branched on, so the loads of a
// thread's R rows sit in one basic block and issue back to back (a branch per
// row made the compiler drain vmcnt after every load: R serial HBM round
// trips per tile).
template <int MODE>
__device__ __forceinline__ void load_item(const TopkSrc& s, int q, int64_t n, int64_t r,
                                          const uint64_t* qb, float qn, float& d, int& id) {
  const bool in = r < n;
  const int64_t rr = in ? r : 0;
  if (MODE == 0) {
    const int64_t w0 = rr * s.words;
    const uint8_t ok = s.valid[rr];
    // metric 1 reads the norm; the others read (and ignore) 4 bytes of the
    // row's own signature, which always exist
    const float* np = s.metric == 1 ? s.tnorm + rr : reinterpret_cast<const float*>(s.tbits + w0);
    const float braw = *np;
    int ham = __popcll(qb[0] ^ s.tbits[w0]);
    if (s.words > 1) {
#pragma unroll
      for (int w = 1; w < kTopMaxWords; ++w)
        if (w < s.words) ham += __popcll(qb[w] ^ s.tbits[w0 + w]);
    }
    const float b = s.metric == 1 ? braw : 0.f;
    const float frac = (float)ham / (float)s.hash_num;
    if (s.metric == 1)
      d = sqrtf(fmaxf(0.f, qn * qn + b * b - 2.f * qn * b * __cosf(3.14159265f * frac)));
    else
      d = frac;
    if (!ok) d = INFINITY;
  } else if (MODE == 1) {
    const float v = s.src_d[(int64_t)q * n + rr];
    d = s.flip ? 1.f - v : v;
    if (!(d < INFINITY) || d != d) d = INFINITY;   // -inf scores / NaN -> absent
  } else {
    d = s.src_d[(int64_t)q * n + rr];
    id = s.src_i[(int64_t)q * n + rr];
  }
  if (MODE != 2) id = (int)r;
  if (!in) { d = INFINITY; id = INT_MAX; }
}

// R rows at once (nn[u]: n for row u, 0 = out of range). MODE 0 in phases -
// every row's valid byte, norm and first signature word, then (tables wider
// than 64 bits only) the other words, then the distances - so the first
// phase's loads are one basic block and all R rows are in flight together
template <int MODE, int R>
__device__ __forceinline__ void load_rows(const TopkSrc& s, int q, const int64_t (&nn)[R],
                                          const int64_t (&r)[R], const uint64_t* qb, float qn,
                                          float (&d)[R], int (&id)[R], const float* ctab = nullptr) {
  if (MODE != 0) {
#pragma unroll
    for (int u = 0; u < R; ++u) load_item<MODE>(s, q, nn[u], r[u], qb, qn, d[u], id[u]);
    return;
  }
  int64_t w0[R];
  uint8_t ok[R];
  float braw[R];
  uint64_t b0[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const int64_t rr = r[u] < nn[u] ? r[u] : 0;
    w0[u] = rr * s.words;
    ok[u] = s.valid[rr];
    const float* np = s.metric == 1 ? s.tnorm + rr : reinterpret_cast<const float*>(s.tbits + w0[u]);
    braw[u] = *np;
    b0[u] = s.tbits[w0[u]];
  }
  int ham[R];
#pragma unroll
  for (int u = 0; u < R; ++u) ham[u] = __popcll(qb[0] ^ b0[u]);
  if (s.words > 1) {
#pragma unroll
    for (int u = 0; u < R; ++u)
      for (int w = 1; w < s.words; ++w) ham[u] += __popcll(qb[w] ^ s.tbits[w0[u] + w]);
  }
#pragma unroll
  for (int u = 0; u < R; ++u) {
    const float frac = (float)ham[u] / (float)s.hash_num;
    float v;
    if (s.metric == 1) {
      // ctab[h] = the same cos expression per hamming distance (bit-identical)
      const float c = ctab != nullptr ? ctab[ham[u]] : __cosf(3.14159265f * frac);
      v = sqrtf(fmaxf(0.f, qn * qn + braw[u] * braw[u] - 2.f * qn * braw[u] * c));
    } else {
      v = frac;
    }
    const bool in = r[u] < nn[u];
    d[u] = (in && ok[u]) ? v : INFINITY;
    id[u] = in ? (int)r[u] : INT_MAX;
  }
}

// number of entries of the sorted list (d, ix)[0, len) that precede (v, id)
__device__ __forceinline__ int rank_in(const float* d, const int* ix, int len, float v, int id) {
  int lo = 0, hi = len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (lt_pair(d[mid], ix[mid], v, id)) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Block-parallel merge of the carry (sorted, cc real entries) with NW sorted
// wave lists (wave w: cnt[w] real entries at wd/wi + w k) into the k
// smallest, written to nd/ni: every real entry's final position is its index
// in its own list plus its rank (binary search) in each other non-empty list
// - all (d, row) pairs are distinct, so the positions are a permutation.
// Replaces a serial k-round wave pop, which costs k dependent arg-min
// rounds per tile. Returns the merged count (<= k). Called by all threads;
// the caller synchronises before reading nd/ni.
template <int NW>
__device__ __forceinline__ int rank_merge(const float* cd, const int* ci, int cc, const float* wd,
                                          const int* wi, const int* cnt, int k, float* nd,
                                          int* ni, int t, int T) {
  int total = cc;
#pragma unroll
  for (int w = 0; w < NW; ++w) total += cnt[w];
  for (int e = t; e < total; e += T) {
    // locate element e: carry first, then the wave lists in order
    int list = -1, i = e;
    if (i >= cc) {
      i -= cc;
      list = 0;
      while (i >= cnt[list]) { i -= cnt[list]; ++list; }
    }
    const float v = list < 0 ? cd[i] : wd[list * k + i];
    const int id = list < 0 ? ci[i] : wi[list * k + i];
    int r = i;
    if (list >= 0) r += rank_in(cd, ci, cc, v, id);
    for (int w = 0; w < NW && r < k; ++w)
      if (w != list && cnt[w] > 0) r += rank_in(wd + w * k, wi + w * k, cnt[w], v, id);
    if (r < k) { nd[r] = v; ni[r] = id; }
  }
  return total < k ? total : k;
}

// NW waves per block (4 or 16); the carry merge is block-parallel (rank_merge).
template <int MODE, int NW = 4>
__global__ __launch_bounds__(NW * 64) void topk_kernel(const TopkSrc s, int64_t n,
                                                           int64_t per_block, int k,
                                                           float* __restrict__ out_d,
                                                           int32_t* __restrict__ out_i,
                                                           volatile uint32_t* done = nullptr,
                                                           uint32_t seq = 0) {
  constexpr int T = NW * 64;
  constexpr int TILE = T * kTopR;
  __shared__ float s_wd[NW * kTopMaxK];   // wave w's list at [w k, w k + k)
  __shared__ int s_wi[NW * kTopMaxK];
  __shared__ int s_cnt[NW];
  __shared__ float s_cbd[2][kTopMaxK];    // carry, double-buffered
  __shared__ int s_cbi[2][kTopMaxK];
  __shared__ float s_thr;
  __shared__ uint64_t s_q[kTopMaxWords];
  __shared__ float s_cos[MODE == 0 ? kTopMaxWords * 64 + 1 : 1];   // euclid_lsh: cos(pi h / hash_num)
  const int q = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int cur = 0, cc = 0;                     // carry buffer / real entries (block-uniform)
  float qn = 0.f;
  const float* ctab = nullptr;
  if (MODE == 0) {
    for (int w = t; w < s.words; w += T) s_q[w] = s.qbits[(int64_t)q * s.words + w];
    qn = s.qnorm[q];
    if (s.metric == 1 && s.hash_num <= kTopMaxWords * 64) {
      for (int h = t; h <= s.hash_num; h += T) s_cos[h] = __cosf(3.14159265f * ((float)h / (float)s.hash_num));
      ctab = s_cos;
    }
  }
  if (t == 0) s_thr = INFINITY;
  __syncthreads();
  uint64_t qb[kTopMaxWords];
#pragma unroll
  for (int w = 0; w < kTopMaxWords; ++w) qb[w] = (MODE == 0 && w < s.words) ? s_q[w] : 0ull;
  const int64_t b0 = (int64_t)blockIdx.x * per_block;
  const int64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  float* wd = &s_wd[wv * k];
  int* wi = &s_wi[wv * k];
  for (int64_t base = b0; base < b1; base += TILE) {
    const float thr = s_thr;
    float d[kTopR];
    int ix[kTopR];
    bool any = false;
    {
      int64_t rows[kTopR], nn[kTopR];
#pragma unroll
      for (int r = 0; r < kTopR; ++r) {
        rows[r] = base + (int64_t)r * T + t;
        nn[r] = rows[r] < b1 ? n : 0;
      }
      load_rows<MODE, kTopR>(s, q, nn, rows, qb, qn, d, ix, ctab);
    }
#pragma unroll
    for (int r = 0; r < kTopR; ++r) {
      // MODE 0/1 visit rows in increasing index order, so a row that ties
      // the carry's k-th distance loses the (distance, index) tie-break:
      // drop it too (quantized hamming distances tie a lot). MODE 2 lists
      // are distance-sorted per block, not index-ordered: keep ties.
      if (MODE != 2 ? d[r] >= thr : d[r] > thr) { d[r] = INFINITY; ix[r] = INT_MAX; }
      any |= d[r] < INFINITY;
    }
    // once the block's k-th best is known almost every row fails the
    // threshold: a wave with no survivor skips the sort and the selection
    int cnt = 0;
    if (__ballot(any)) {
      sort_regs<kTopR>(d, ix);
      wave_pop<kTopR>(d, ix, k, wd, wi, lane, &cnt);
    } else {
      for (int j = lane; j < k; j += 64) { wd[j] = INFINITY; wi[j] = INT_MAX; }
    }
    if (lane == 0) s_cnt[wv] = cnt;
    __syncthreads();
    int total = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) total += s_cnt[w];
    if (total > 0) {                       // block-uniform
      const int nn = rank_merge<NW>(s_cbd[cur], s_cbi[cur], cc, s_wd, s_wi, s_cnt, k,
                                    s_cbd[cur ^ 1], s_cbi[cur ^ 1], t, T);
      cur ^= 1;
      cc = nn;
      __syncthreads();
      if (t == 0) s_thr = cc == k ? s_cbd[cur][k - 1] : INFINITY;
    }
    __syncthreads();
  }
  const int64_t o = ((int64_t)q * gridDim.x + blockIdx.x) * k;
  if (done != nullptr) {   // latency path: results to pinned host memory, then the flag
    for (int j = t; j < k; j += T) {
      sys_store(out_d + o + j, j < cc ? s_cbd[cur][j] : INFINITY);
      sys_store(out_i + o + j, j < cc ? s_cbi[cur][j] : (int32_t)INT_MAX);
    }
    sys_stores_block_done();
    if (t == 0) sys_store(const_cast<uint32_t*>(done) + q, seq);
    return;
  }
  for (int j = t; j < k; j += T) {
    out_d[o + j] = j < cc ? s_cbd[cur][j] : INFINITY;
    out_i[o + j] = j < cc ? s_cbi[cur][j] : INT_MAX;
  }
}

// Several queries per table pass (MODE 0, W <= 2 signature words): waves
// per query. A block of 16 waves loads each tile of 4096 rows (signatures,
// and the norm with the valid flag folded in) into LDS once; the G = 16 / nq
// waves of a query (G a power of two) take every G-th 512-row chunk of the
// tile and run the threshold-pruned selection with a wave-private carry
// (merged by rank inside the wave): no block barrier per query, and the table
// crosses HBM once per batch of up to 8 queries instead of once per query
// (the (blocks, nq) grid re-reads it). A query's G carries merge at the end.
// euclid_lsh takes cos(pi h / hash_num) from a per-block table of the
// hash_num + 1 values (the same expression as load_item, so distances are
// bit-identical). Each wave visits its rows in increasing index order, so the
// tie rule of topk_kernel holds. Output layout as topk_kernel's.
constexpr int kWqWaves = 16;
constexpr int kWqT = kWqWaves * 64;
constexpr int kWqLoads = 4;                       // rows a thread stages per tile
constexpr int kWqTile = kWqT * kWqLoads;          // 4096 rows per tile
constexpr int kWqChunks = kWqTile / 512;          // 512-row chunks (8 rows a lane)
// static LDS of topk_wq_kernel<W> (tile bits + norms + carries): ~128 KB at
// W = 2, which fits gfx950's 160 KB per workgroup only (CDNA3 has 64 KB);
// this library is built for gfx950 alone (build_ext.py ARCH)
constexpr int wq_lds_bytes(int w) {
  return kWqTile * 8 * w + kWqTile * 4 + (64 * w + 1) * 4 + kWqWaves * 2 * kTopMaxK * 8 +
         kWqWaves * kTopMaxK * 8 + kWqWaves * 8;
}
static_assert(wq_lds_bytes(2) <= 160 * 1024, "topk_wq_kernel<2> exceeds gfx950 LDS (160 KB)");

// wave-level LDS ordering: the lanes of one wave read what others wrote
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// merge two sorted lists of distinct (d, ix) pairs into the k smallest (one wave)
__device__ __forceinline__ int wave_merge(const float* ad, const int* ai, int na, const float* bd,
                                          const int* bi, int nb, int k, float* od, int* oi,
                                          int lane) {
  for (int e = lane; e < na + nb; e += 64) {
    const bool inA = e < na;
    const int i = inA ? e : e - na;
    const float v = inA ? ad[i] : bd[i];
    const int id = inA ? ai[i] : bi[i];
    const int r = i + (inA ? rank_in(bd, bi, nb, v, id) : rank_in(ad, ai, na, v, id));
    if (r < k) { od[r] = v; oi[r] = id; }
  }
  return na + nb < k ? na + nb : k;
}

template <int W>
__global__ __launch_bounds__(kWqT) void topk_wq_kernel(const TopkSrc s, int nq, int64_t n,
                                                       int64_t per_block, int k,
                                                       float* __restrict__ out_d,
                                                       int32_t* __restrict__ out_i) {
  __shared__ uint64_t s_bits[kWqTile * W];
  __shared__ float s_nv[kWqTile];                 // norm, or -1 for an invalid row
  __shared__ float s_lut[64 * W + 1];
  __shared__ float s_cd[kWqWaves][2][kTopMaxK];   // per-wave carry, double-buffered
  __shared__ int s_ci[kWqWaves][2][kTopMaxK];
  __shared__ float s_wd[kWqWaves][kTopMaxK];      // per-wave winners of a chunk
  __shared__ int s_wi[kWqWaves][kTopMaxK];
  __shared__ int s_cc[kWqWaves], s_cur[kWqWaves];
  const int t = threadIdx.x, lane = t & 63;
  // wave-uniform in scalar registers: the query's bits and norm come from
  // scalar loads, so no vector-memory wait inside the scan waits for them
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  int G = kWqWaves;                               // waves per query
  while (G > 1 && G * nq > kWqWaves) G >>= 1;
  const int q = wv / G, part = wv % G;
  const bool active = q < nq;
  const int qq = active ? q : 0;
  const bool euclid = s.metric == 1;
  uint64_t qb[W];
#pragma unroll
  for (int w = 0; w < W; ++w) qb[w] = s.qbits[(int64_t)qq * s.words + w];
  const float qn = s.qnorm[qq];
  const float hn = (float)s.hash_num;
  // per hamming distance h: cos(pi h / hash_num) (euclid_lsh) or h / hash_num
  // (lsh / minhash), the expressions of load_item
  for (int h = t; h <= s.hash_num && h <= 64 * W; h += kWqT)
    s_lut[h] = euclid ? __cosf(3.14159265f * ((float)h / hn)) : (float)h / hn;
  int cur = 0, cc = 0;                             // wave-uniform
  float thr = INFINITY;
  const int64_t b0 = (int64_t)blockIdx.x * per_block;
  const int64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  // the next tile's rows are fetched into registers while the current one is
  // scanned from LDS (the HBM latency hides behind the selection)
  uint64_t pb[kWqLoads][W];
  float pn[kWqLoads];
  uint32_t pv[kWqLoads];
  auto fetch = [&](int64_t base) {      // plain loads only: no branch waits on them
#pragma unroll
    for (int r = 0; r < kWqLoads; ++r) {
      const int64_t row = base + r * kWqT + t;
      const int64_t rc = row < b1 ? row : b1 - 1;  // clamped, never out of range
#pragma unroll
      for (int w = 0; w < W; ++w) pb[r][w] = s.tbits[rc * W + w];
      pn[r] = euclid ? s.tnorm[rc] : 0.f;
      pv[r] = s.valid[rc];
    }
  };
  if (b0 < b1) fetch(b0);
  for (int64_t base = b0; base < b1; base += kWqTile) {
    __syncthreads();                               // the previous tile is consumed
#pragma unroll
    for (int r = 0; r < kWqLoads; ++r) {
      const int j = r * kWqT + t;
#pragma unroll
      for (int w = 0; w < W; ++w) s_bits[j * W + w] = pb[r][w];
      s_nv[j] = (base + j < b1 && pv[r] != 0) ? pn[r] : -1.f;
    }
    __syncthreads();
    if (base + kWqTile < b1) fetch(base + kWqTile);
    if (!active) continue;
    for (int c = part; c < kWqChunks; c += G) {
      float d[kTopR];
      int ix[kTopR];
      bool any = false;
      // euclid: rows whose squared distance is surely above thr^2 skip the sqrt
      const float thr2 = thr < INFINITY ? thr * thr * 1.0001f + 1e-30f : INFINITY;
#pragma unroll
      for (int i = 0; i < kTopR; ++i) {
        const int j = c * 512 + i * 64 + lane;
        int ham = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) ham += __popcll(qb[w] ^ s_bits[j * W + w]);
        const float b = s_nv[j];
        float v;
        if (euclid) {
          const float x = qn * qn + b * b - 2.f * qn * b * s_lut[ham];
          v = x > thr2 ? INFINITY : sqrtf(fmaxf(0.f, x));
        } else {
          v = s_lut[ham];
        }
        if (b < 0.f || v >= thr) v = INFINITY;
        d[i] = v;
        ix[i] = v < INFINITY ? (int)(base + j) : INT_MAX;
        any |= v < INFINITY;
      }
      if (!__ballot(any)) continue;                // wave-uniform
      // survivors per register slot: past the first chunks a handful per
      // wave, which are compacted and ranked directly (no register sort and
      // no k pop rounds); a chunk with more than 64 takes the pop path
      uint64_t masks[kTopR];
      int total = 0;
#pragma unroll
      for (int i = 0; i < kTopR; ++i) {
        masks[i] = __ballot(d[i] < INFINITY);
        total += __popcll(masks[i]);
      }
      int cnt = 0;
      float* wd = s_wd[wv];
      int* wi = s_wi[wv];
      if (total <= 64) {
        int at = 64;                               // raw survivors at [64, 64 + total)
#pragma unroll
        for (int i = 0; i < kTopR; ++i) {
          if (d[i] < INFINITY) {
            const int pos = at + (int)__builtin_amdgcn_mbcnt_hi(
                                     (uint32_t)(masks[i] >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)masks[i], 0u));
            wd[pos] = d[i];
            wi[pos] = ix[i];
          }
          at += __popcll(masks[i]);
        }
        wave_sync();
        if (lane < total) {                        // sorted into [0, total) by rank
          const float v = wd[64 + lane];
          const int id = wi[64 + lane];
          int r = 0;
          for (int e = 0; e < total; ++e) r += lt_pair(wd[64 + e], wi[64 + e], v, id) ? 1 : 0;
          wd[r] = v;
          wi[r] = id;
        }
        cnt = total < k ? total : k;
      } else {
        sort_regs<kTopR>(d, ix);
        wave_pop<kTopR>(d, ix, k, wd, wi, lane, &cnt);
      }
      wave_sync();
      cc = wave_merge(s_cd[wv][cur], s_ci[wv][cur], cc, s_wd[wv], s_wi[wv], cnt, k,
                      s_cd[wv][cur ^ 1], s_ci[wv][cur ^ 1], lane);
      cur ^= 1;
      wave_sync();
      thr = cc == k ? s_cd[wv][cur][k - 1] : INFINITY;
    }
  }
  if (lane == 0) {
    s_cc[wv] = cc;
    s_cur[wv] = cur;
  }
  __syncthreads();
  if (!active || part != 0) return;
  // the query's first wave folds in the carries of its other G - 1 waves
  for (int g = 1; g < G; ++g) {
    const int ow = wv + g;
    cc = wave_merge(s_cd[wv][cur], s_ci[wv][cur], cc, s_cd[ow][s_cur[ow]], s_ci[ow][s_cur[ow]],
                    s_cc[ow], k, s_wd[wv], s_wi[wv], lane);
    wave_sync();
    for (int j = lane; j < cc; j += 64) {
      s_cd[wv][cur][j] = s_wd[wv][j];
      s_ci[wv][cur][j] = s_wi[wv][j];
    }
    wave_sync();
  }
  const int64_t o = ((int64_t)q * gridDim.x + blockIdx.x) * k;
  for (int j = lane; j < k; j += 64) {
    out_d[o + j] = j < cc ? s_cd[wv][cur][j] : INFINITY;
    out_i[o + j] = j < cc ? s_ci[wv][cur][j] : INT_MAX;
  }
}

// Multi-query scan with the queries in scalar registers (MODE 0, W <= 2
// signature words, k <= kMqMaxK, up to kMqMaxQ queries a launch), two launches:
//   M1  topk_mq_sample_kernel, one block per query: the distances of a sample
//       of the table (32 contiguous segments of 1024 rows, spread over it) into
//       an LDS histogram - hamming distance (lsh / minhash) or the top 11 bits
//       of the float (euclid_lsh) - and the bin where the count reaches k. The
//       sample's rows are table rows, so k of them lie at or below that bin:
//       its upper edge bounds the k-th distance of the whole table (exact
//       pruning, no retry).
//   M2  topk_mq_kernel: every wave streams its own contiguous row range from
//       HBM once - a lane holds 8 consecutive rows of a 512-row chunk (vector
//       loads) while the next chunk is in flight - and tests every row against
//       every query: xor + popcount against the query's bits (SGPRs) and one
//       compare with the query's bound. Only rows under the bound leave that
//       loop; they go through the wave's exact selection (compaction + rank, or
//       the register pop) into its per-query carry.
// Every bound is a key limit "survive iff key < lim" (key: the hamming
// distance, or the bits of the non-negative float distance): the sample's bin
// edge, the wave's own k-th key (a wave visits its chunks in index order, so a
// tie with its k-th loses) and the block's best k-th key + 1 over its waves
// (an LDS atomicMin; another wave's rows may precede in index order, so a tie
// survives). euclid_lsh prefilters on the squared distance against the limit
// squared (with a relative margin) and computes the exact distance (load_item's
// expression) for the rows that pass. A first chunk with more than 64 rows
// under the limit is cut to those at or below the k-th smallest of the lanes'
// minima (a radix select over ballots): k rows of the chunk lie at or below it.
// Replaces topk_wq_kernel's LDS tile + waves per query for k <= kMqMaxK: that
// kernel re-read each staged row from LDS per query and spent 10.3 K VALU per
// wave, 481 GB/s on 10M rows x 8 queries (profiles/r4_pmc_roofline.md:9).
// Measured dead ends (profiles/r5_topk_mq_ab.md): a grid-wide bound in one
// global word per query (the waves' k-th, atomicMax) - every wave polls and
// updates the same few addresses, which serialize at the memory channel, and
// the minimum of the waves' k-ths stays far above the k-th of the rows seen.
constexpr int kMqWaves = 8;
constexpr int kMqT = kMqWaves * 64;
constexpr int kMqR = 8;                        // consecutive rows per lane per chunk
constexpr int kMqChunk = 64 * kMqR;            // 512
constexpr int kMqMaxK = 32;
constexpr int kMqMaxQ = 8;
constexpr int64_t kMqMinRows = (int64_t)2 << 20;
constexpr int kMqBlocksMax = 511;                 // the scan's blocks (<= kMergeLists - 1 lists)
constexpr int kMqSampT = 1024;                 // sample: threads = rows per segment
constexpr int kMqSampSegMax = 32;              // sample: segments (16 a round of loads in flight)
constexpr int kMqBins = 2048;                  // euclid: float bits >> 20

// counters of the scan (JB_TOPK_MQ_STATS; global atomics, slow): survivor passes, chunks, cuts, insertions
__device__ unsigned long long g_mq_stats[4];

__device__ __forceinline__ uint64_t uniform64(uint64_t x) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// the k-th smallest of the wave's 64 keys (k <= 64), MSB-first radix select
// over ballots; the top bits above NB are assumed equal
template <int NB>
__device__ __forceinline__ uint32_t wave_kth_key(uint32_t key, int k) {
  uint32_t res = 0;
#pragma unroll
  for (int b = NB - 1; b >= 0; --b) {
    const uint32_t trial = res | (1u << b);
    if (__popcll(__ballot(key < trial)) < k) res = trial;
  }
  return res;
}

// the distance key of a row for one query (hamming distance, or the bits of
// the exact euclid_lsh distance - load_item's expression)
template <int W, bool EUC>
__device__ __forceinline__ uint32_t mq_key(const uint64_t (&qw)[W], float qq, const uint64_t* bits, float b,
                                           const float* lut, float* dist, float hn) {
  int ham = 0;
#pragma unroll
  for (int w = 0; w < W; ++w) ham += __popcll(qw[w] ^ bits[w]);
  if (EUC) {
    const float v = sqrtf(fmaxf(0.f, qq * qq + b * b - 2.f * qq * b * lut[ham]));
    *dist = v;
    return __float_as_uint(v);
  }
  *dist = (float)ham / hn;
  return (uint32_t)ham;
}

template <int W, bool EUC>
__global__ __launch_bounds__(kMqSampT) void topk_mq_sample_kernel(const TopkSrc s, int q0, int64_t n, int k,
                                                                  int nseg, uint32_t* __restrict__ lim_out) {
  constexpr int NB = EUC ? kMqBins : 64 * W + 1;
  constexpr int U = 16;                            // sampled rows in flight per thread
  __shared__ int hist[NB];
  __shared__ float s_lut[EUC ? 64 * W + 1 : 1];
  __shared__ int s_part[kMqSampT / 64 + 1];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int q = q0 + blockIdx.x;
  const float hn = (float)s.hash_num;
  for (int b = t; b < NB; b += kMqSampT) hist[b] = 0;
  if (EUC)
    for (int h = t; h <= s.hash_num && h <= 64 * W; h += kMqSampT) s_lut[h] = __cosf(3.14159265f * ((float)h / hn));
  uint64_t qw[W];
#pragma unroll
  for (int w = 0; w < W; ++w) qw[w] = s.qbits[(int64_t)q * s.words + w];
  const float qq = EUC ? s.qnorm[q] : 0.f;
  __syncthreads();
  // every thread: the minimum key of its sampled rows (one per segment);
  // k distinct threads hold a row at or below their minimum, so the k-th
  // smallest minimum bounds the table's k-th distance
  const int64_t S = (int64_t)nseg * kMqSampT;
  uint32_t mn = 0xffffffffu;
  for (int j0 = 0; j0 < nseg; j0 += U) {
    uint64_t bits[U][W];
    float nrm[U];
    uint32_t ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {                  // loads first, all in flight
      const int64_t row = n <= S ? (int64_t)(j0 + u) * kMqSampT + t : (n / nseg) * (j0 + u) + t;
      const int64_t rc = row < n ? row : n - 1;
#pragma unroll
      for (int w = 0; w < W; ++w) bits[u][w] = s.tbits[rc * W + w];
      nrm[u] = EUC ? s.tnorm[rc] : 0.f;
      ok[u] = row < n ? (uint32_t)s.valid[rc] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d;
      const uint32_t key = mq_key<W, EUC>(qw, qq, bits[u], nrm[u], s_lut, &d, hn);
      mn = (ok[u] != 0 && key < mn) ? key : mn;
    }
  }
  if (mn != 0xffffffffu) atomicAdd(&hist[EUC ? (int)(mn >> 20) : (int)mn], 1);
  __syncthreads();
  // the first bin where the running count reaches k
  constexpr int PER = (NB + kMqSampT - 1) / kMqSampT;
  int c = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) c += t * PER + i < NB ? hist[t * PER + i] : 0;
  int incl = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int x = __shfl_up(incl, o, 64);
    if (lane >= o) incl += x;
  }
  if (lane == 63) s_part[wv] = incl;
  __syncthreads();
  if (t == 0) {
    int run = 0;
    for (int w = 0; w < kMqSampT / 64; ++w) {
      const int x = s_part[w];
      s_part[w] = run;
      run += x;
    }
    s_part[kMqSampT / 64] = run;
  }
  __syncthreads();
  incl += s_part[wv];
  if (t == 0 && s_part[kMqSampT / 64] < k) lim_out[q] = 0xffffffffu;   // fewer than k sampled: no bound
  int run = incl - c;
  if (run < k && incl >= k) {
    int b = t * PER;
    for (int i = 0; i < PER; ++i, ++b) {
      run += hist[b];
      if (run >= k) break;
    }
    lim_out[q] = EUC ? (uint32_t)(b + 1) << 20 : (uint32_t)(b + 1);
  }
}

// lane j (< k) of (cd, ci) holds the wave's j-th best of one query so far;
// inserts (v, id) when it beats the k-th (one readlane pair, a ballot for
// its rank and a one-lane shift of the lanes behind it)
__device__ __forceinline__ void carry_insert(float& cd, int& ci, float v, int id, int k, int lane) {
  const float kd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cd), k - 1));
  const int ki = __builtin_amdgcn_readlane(ci, k - 1);
  if (!lt_pair(v, id, kd, ki)) return;             // wave-uniform
  const int p = __popcll(__ballot(lane < k && lt_pair(cd, ci, v, id)));
  float ud;
  int ui;
  if (k <= 16) {                                   // the carry sits in DPP row 0: row_shr:1
    ud = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(cd), __float_as_int(cd), 0x111, 0xF, 0xF, false));
    ui = __builtin_amdgcn_update_dpp(ci, ci, 0x111, 0xF, 0xF, false);
  } else {
    ud = __shfl_up(cd, 1, 64);
    ui = __shfl_up(ci, 1, 64);
  }
  if (lane > p && lane < k) {
    cd = ud;
    ci = ui;
  }
  if (lane == p) {
    cd = v;
    ci = id;
  }
}

template <int W, int NQ, bool EUC>
__global__ __launch_bounds__(kMqT) void topk_mq_kernel(const TopkSrc s, int nq, int q0, int64_t n,
                                                       int64_t per_block, int k,
                                                       const uint32_t* __restrict__ lim_in, int stats,
                                                       float* __restrict__ out_d,
                                                       int32_t* __restrict__ out_i) {
  static_assert(NQ <= kMqWaves, "one wave per query merges the block's carries");
  __shared__ float s_cd[kMqWaves][NQ][kMqMaxK];      // the waves' carries, for the block merge
  __shared__ int s_ci[kMqWaves][NQ][kMqMaxK];
  __shared__ float s_md[kMqWaves][2][kMqMaxK];       // merge buffers
  __shared__ int s_mi[kMqWaves][2][kMqMaxK];
  __shared__ int s_cc[kMqWaves][NQ];
  __shared__ uint32_t s_blk[NQ];             // the sample's limit, then min over waves of k-th key + 1
  __shared__ float s_lut[EUC ? 64 * W + 1 : 1];
  __shared__ uint64_t s_qb[NQ][W];
  __shared__ float s_qn[NQ];
  const int t = threadIdx.x, lane = t & 63;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  const float hn = (float)s.hash_num;
  if (EUC)
    for (int h = t; h <= s.hash_num && h <= 64 * W; h += kMqT) s_lut[h] = __cosf(3.14159265f * ((float)h / hn));
  if (t < NQ) s_blk[t] = t < nq ? (lim_in != nullptr ? lim_in[q0 + t] : 0xffffffffu) : 0u;   // (null: no bound)
  if (t < NQ * W) {
    const int q = t / W, w = t % W;
    s_qb[q][w] = q < nq ? s.qbits[(int64_t)(q0 + q) * s.words + w] : 0ull;
  }
  if (t < NQ) s_qn[t] = (EUC && t < nq) ? s.qnorm[q0 + t] : 0.f;
  __syncthreads();
  uint64_t qb[NQ][W];
  float qn[NQ];
  float cd[NQ];                                      // the wave's carries (lane j < k: j-th best)
  int ci[NQ];
  uint32_t own[NQ];                                  // survive: key < own (a tie with the k-th loses)
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
#pragma unroll
    for (int w = 0; w < W; ++w) qb[q][w] = uniform64(s_qb[q][w]);
    qn[q] = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(s_qn[q])));
    cd[q] = INFINITY;
    ci[q] = INT_MAX;
    own[q] = 0xffffffffu;
  }
  const int64_t b0 = (int64_t)blockIdx.x * per_block;
  const int64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  const int64_t pw = ((per_block / kMqWaves) + kMqChunk - 1) / kMqChunk * kMqChunk;
  const int64_t w0 = b0 + (int64_t)wv * pw;
  const int64_t w1 = w0 + pw < b1 ? w0 + pw : b1;

  // the next chunk in flight: raw loads only - nothing reads them before the
  // next iteration (a value used inside this one would make the compiler wait
  // for every load in flight, vmcnt counting in order)
  uint64_t pb[kMqR][W];
  float pn[kMqR];
  uint32_t pv[kMqR];                 // valid bytes: packed (pv[0..1], whole chunks) or one per row
  bool packed = false;
  auto fetch = [&](int64_t base) {
    const int64_t r0 = base + (int64_t)lane * kMqR;
    packed = base + kMqChunk <= w1;
    if (packed) {                    // a whole chunk: vector loads of the lane's 8 rows
      const ulonglong2* bp = reinterpret_cast<const ulonglong2*>(s.tbits + r0 * W);
#pragma unroll
      for (int j = 0; j < kMqR * W / 2; ++j) {
        const ulonglong2 v = bp[j];
        pb[(2 * j) / W][(2 * j) % W] = v.x;
        pb[(2 * j + 1) / W][(2 * j + 1) % W] = v.y;
      }
      const uint2 vv = *reinterpret_cast<const uint2*>(s.valid + r0);
      pv[0] = vv.x;
      pv[1] = vv.y;
#pragma unroll
      for (int i = 2; i < kMqR; ++i) pv[i] = 0u;   // constants: no copy of an older load's register
      if (EUC) {
        const float4* np = reinterpret_cast<const float4*>(s.tnorm + r0);
        const float4 a = np[0], b = np[1];
        pn[0] = a.x; pn[1] = a.y; pn[2] = a.z; pn[3] = a.w;
        pn[4] = b.x; pn[5] = b.y; pn[6] = b.z; pn[7] = b.w;
      }
    } else {                         // the table's last chunk: clamped rows
#pragma unroll
      for (int i = 0; i < kMqR; ++i) {
        const int64_t row = r0 + i;
        const int64_t rc = row < w1 ? row : w1 - 1;
#pragma unroll
        for (int w = 0; w < W; ++w) pb[i][w] = s.tbits[rc * W + w];
        pv[i] = s.valid[rc];
        if (EUC) pn[i] = s.tnorm[rc];
      }
    }
    if (!EUC) {
#pragma unroll
      for (int i = 0; i < kMqR; ++i) pn[i] = 0.f;
    }
  };

  int st_surv = 0, st_chunks = 0, st_cut = 0, st_ins = 0;
  if (w0 < w1) fetch(w0);
  for (int64_t base = w0; base < w1; base += kMqChunk) {
    ++st_chunks;
    uint64_t bb[kMqR][W];
    float bn[kMqR];
    uint32_t okl = 0;                                // the lane's valid rows (bit i: row i)
#pragma unroll
    for (int i = 0; i < kMqR; ++i) {
#pragma unroll
      for (int w = 0; w < W; ++w) bb[i][w] = pb[i][w];
      bn[i] = pn[i];
      const uint32_t vb = packed ? (pv[i >> 2] >> (8 * (i & 3))) & 0xffu : pv[i];
      okl |= (base + (int64_t)lane * kMqR + i < w1 && vb != 0) ? (1u << i) : 0u;
    }
    if (base + kMqChunk < w1) fetch(base + kMqChunk);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      if (q >= nq) break;
      const uint32_t blk = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(&s_blk[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      const uint32_t lim = own[q] < blk ? own[q] : blk;
      // the prefilter: xor + popcount and one compare per row
      bool any = false;
      if (EUC) {
        const float f = __uint_as_float(lim);          // 0xffffffff: NaN -> no bound
        const float t2 = f < INFINITY ? f * f * 1.0001f + 1e-30f : INFINITY;
        const float q2 = qn[q] * qn[q], tqn = 2.f * qn[q];
#pragma unroll
        for (int i = 0; i < kMqR; ++i) {
          int ham = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) ham += __popcll(qb[q][w] ^ bb[i][w]);
          const float b = bn[i];
          const float x = q2 + b * b - tqn * b * s_lut[ham];
          any |= ((okl >> i) & 1u) && x <= t2;
        }
      } else {
#pragma unroll
        for (int i = 0; i < kMqR; ++i) {
          int ham = 0;
#pragma unroll
          for (int w = 0; w < W; ++w) ham += __popcll(qb[q][w] ^ bb[i][w]);
          any |= ((okl >> i) & 1u) && (uint32_t)ham < lim;
        }
      }
      if (__ballot(any) == 0) continue;              // the common case: nothing of the chunk passes
      // the exact keys of the chunk's rows under the limit, into the carry
      ++st_surv;
      uint32_t key[kMqR];
      float d[kMqR];
      uint32_t kmin = 0xffffffffu;
#pragma unroll
      for (int i = 0; i < kMqR; ++i) {
        key[i] = mq_key<W, EUC>(qb[q], qn[q], bb[i], bn[i], s_lut, &d[i], hn);
        if (!((okl >> i) & 1u) || !(key[i] < lim)) key[i] = 0xffffffffu;
        kmin = key[i] < kmin ? key[i] : kmin;
      }
      int total = 0;
#pragma unroll
      for (int i = 0; i < kMqR; ++i) total += __popcll(__ballot(key[i] != 0xffffffffu));
      if (total > 2 * k) {
        ++st_cut;
        // at least k rows of the chunk lie at or below the k-th smallest lane
        // minimum (k distinct lanes): the rest cannot enter the carry
        const uint32_t kb = EUC ? wave_kth_key<32>(kmin, k) : wave_kth_key<8>(kmin, k);
#pragma unroll
        for (int i = 0; i < kMqR; ++i)
          if (key[i] > kb) key[i] = 0xffffffffu;
      }
#pragma unroll
      for (int i = 0; i < kMqR; ++i) {
        uint64_t m = __ballot(key[i] != 0xffffffffu);
        while (m != 0) {                             // wave-uniform
          const int l = __ffsll((long long)m) - 1;
          m &= m - 1;
          const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d[i]), l));
          carry_insert(cd[q], ci[q], v, (int)(base + (int64_t)l * kMqR + i), k, lane);
          ++st_ins;
        }
      }
      const float kd = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cd[q]), k - 1));
      if (kd < INFINITY) {
        const uint32_t kk = EUC ? __float_as_uint(kd) : (uint32_t)(int)rintf(kd * hn);
        own[q] = kk;
        if (lane == 0 && kk + 1u < blk) atomicMin(&s_blk[q], kk + 1u);
      }
    }
  }
  if (stats && lane == 0) {
    atomicAdd(&g_mq_stats[0], (unsigned long long)st_surv);
    atomicAdd(&g_mq_stats[1], (unsigned long long)st_chunks);
    atomicAdd(&g_mq_stats[2], (unsigned long long)st_cut);
    atomicAdd(&g_mq_stats[3], (unsigned long long)st_ins);
  }
  // the carries to LDS, then query q's wave merges the block's lists
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (q >= nq) break;
    if (lane < k) {
      s_cd[wv][q][lane] = cd[q];
      s_ci[wv][q][lane] = ci[q];
    }
    const int cc = __popcll(__ballot(lane < k && ci[q] != INT_MAX));
    if (lane == 0) s_cc[wv][q] = cc;
  }
  __syncthreads();
  if (wv >= nq) return;
  const int q = wv;
  const float* ad = s_cd[wv][q];
  const int* ai = s_ci[wv][q];
  int cc = s_cc[wv][q], cur = 0;
  for (int ow = 0; ow < kMqWaves; ++ow) {
    if (ow == wv) continue;
    const int oc = s_cc[ow][q];
    if (oc == 0) continue;
    cc = wave_merge(ad, ai, cc, s_cd[ow][q], s_ci[ow][q], oc, k, s_md[wv][cur], s_mi[wv][cur], lane);
    wave_sync();
    ad = s_md[wv][cur];
    ai = s_mi[wv][cur];
    cur ^= 1;
  }
  const int64_t o = ((int64_t)(q0 + q) * gridDim.x + blockIdx.x) * k;
  for (int j = lane; j < k; j += 64) {
    out_d[o + j] = j < cc ? ad[j] : INFINITY;
    out_i[o + j] = j < cc ? ai[j] : INT_MAX;
  }
}

// Small k (<= KL): every thread keeps its own sorted top-KL of the items it
// reads (strided across the block's range) in registers and the block merges
// once at the end (per-wave pops, then wave 0). Used for the final merge of
// the blocks' candidates (a few items per thread); on a long scan with random
// distances the per-thread insertions cost more than the tile kernel's
// threshold-pruned selection (measured, tools/bench_topk.py).
template <int MODE, int KL, int NW = 4>
__global__ __launch_bounds__(NW * 64) void topk_lists_kernel(const TopkSrc s, int64_t n,
                                                             int64_t per_block, int k,
                                                             float* __restrict__ out_d,
                                                             int32_t* __restrict__ out_i,
                                                             volatile uint32_t* done = nullptr,
                                                             uint32_t seq = 0) {
  constexpr int T = NW * 64;
  __shared__ float s_wd[NW * KL];
  __shared__ int s_wi[NW * KL];
  __shared__ float s_cd[KL];
  __shared__ int s_ci[KL];
  __shared__ uint64_t s_q[kTopMaxWords];
  const int q = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float qn = 0.f;
  if (MODE == 0) {
    for (int w = t; w < s.words; w += T) s_q[w] = s.qbits[(int64_t)q * s.words + w];
    qn = s.qnorm[q];
  }
  __syncthreads();
  uint64_t qb[kTopMaxWords];
#pragma unroll
  for (int w = 0; w < kTopMaxWords; ++w) qb[w] = (MODE == 0 && w < s.words) ? s_q[w] : 0ull;
  float ld[KL];
  int li[KL];
#pragma unroll
  for (int j = 0; j < KL; ++j) { ld[j] = INFINITY; li[j] = INT_MAX; }
  const int64_t b0 = (int64_t)blockIdx.x * per_block;
  const int64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  for (int64_t base = b0; base < b1; base += (int64_t)T * 4) {
    float d[4];
    int ix[4];
    {   // 4 rows in flight per thread
      int64_t rows[4], nn[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        rows[r] = base + (int64_t)r * T + t;
        nn[r] = rows[r] < b1 ? n : 0;
      }
      load_rows<MODE, 4>(s, q, nn, rows, qb, qn, d, ix);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = d[r];
      const int id = ix[r];
      if (lt_pair(v, id, ld[KL - 1], li[KL - 1])) {
#pragma unroll
        for (int j = KL - 1; j > 0; --j) {
          const bool up = lt_pair(v, id, ld[j - 1], li[j - 1]);
          const bool here = !up && lt_pair(v, id, ld[j], li[j]);
          ld[j] = up ? ld[j - 1] : (here ? v : ld[j]);
          li[j] = up ? li[j - 1] : (here ? id : li[j]);
        }
        if (lt_pair(v, id, ld[0], li[0])) { ld[0] = v; li[0] = id; }
      }
    }
  }
  wave_pop<KL>(ld, li, k, &s_wd[wv * k], &s_wi[wv * k], lane);
  __syncthreads();
  if (wv == 0) {
    constexpr int M = (NW * KL + 63) / 64;
    float m[M];
    int mi[M];
#pragma unroll
    for (int j = 0; j < M; ++j) {
      const int c = lane + 64 * j;
      if (c < NW * k) { m[j] = s_wd[c]; mi[j] = s_wi[c]; }
      else { m[j] = INFINITY; mi[j] = INT_MAX; }
    }
    __builtin_amdgcn_wave_barrier();
    sort_regs<M>(m, mi);
    wave_pop<M>(m, mi, k, s_cd, s_ci, lane);
  }
  __syncthreads();
  const int64_t o = ((int64_t)q * gridDim.x + blockIdx.x) * k;
  if (done != nullptr) {   // pinned host memory, then the flag (sys_store)
    for (int j = t; j < k; j += T) { sys_store(out_d + o + j, s_cd[j]); sys_store(out_i + o + j, s_ci[j]); }
    sys_stores_block_done();
    if (t == 0) sys_store(const_cast<uint32_t*>(done) + q, seq);
    return;
  }
  for (int j = t; j < k; j += T) { out_d[o + j] = s_cd[j]; out_i[o + j] = s_ci[j]; }
}

// ---------------------------------------------------------------------------
// Sampled-threshold top-k (latency path, large tables): O(N) with a small
// constant for any k <= 128, instead of the tile kernel's O(N k / tile).
//   S1  one block per query reads S evenly spaced rows and takes the j-th
//       smallest distance as threshold T (j chosen by the host so that
//       ~3k rows of the full table are expected at or below T);
//   S2  full scan: rows with d <= T are appended to a candidate buffer
//       (wave-aggregated atomics: one atomic per wave per pass);
//   S3  exact top-k of the candidates (topk_lists / topk_kernel), written to
//       pinned host memory; done[q] = seq, or seq | kTopRetry when T was too
//       low (fewer than k candidates) or the buffer overflowed - the host
//       then reruns the exact tile path.
constexpr uint32_t kTopRetry = 0x80000000u;
constexpr int kSampleThreads = 1024;

template <int MODE>
__global__ __launch_bounds__(kSampleThreads) void topk_sample_kernel(const TopkSrc s, int64_t n,
                                                                     int64_t S, int j,
                                                                     float* __restrict__ thr,
                                                                     int* __restrict__ count) {
  constexpr int KL = 16;
  constexpr int NW = kSampleThreads / 64;
  __shared__ float s_wd[NW * KL];
  __shared__ int s_wi[NW * KL];
  __shared__ float s_out[KL];
  __shared__ int s_oi[KL];
  __shared__ uint64_t s_q[kTopMaxWords];
  const int q = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float qn = 0.f;
  if (MODE == 0) {
    for (int w = t; w < s.words; w += kSampleThreads) s_q[w] = s.qbits[(int64_t)q * s.words + w];
    qn = s.qnorm[q];
  }
  __syncthreads();
  uint64_t qb[kTopMaxWords];
#pragma unroll
  for (int w = 0; w < kTopMaxWords; ++w) qb[w] = (MODE == 0 && w < s.words) ? s_q[w] : 0ull;
  float ld[KL];
  int li[KL];
#pragma unroll
  for (int x = 0; x < KL; ++x) { ld[x] = INFINITY; li[x] = INT_MAX; }
  for (int64_t i = t; i < S; i += kSampleThreads) {
    const int64_t row = (i * n) / S;
    float v;
    int id;
    load_item<MODE>(s, q, n, row, qb, qn, v, id);
    if (lt_pair(v, id, ld[KL - 1], li[KL - 1])) {
#pragma unroll
      for (int x = KL - 1; x > 0; --x) {
        const bool up = lt_pair(v, id, ld[x - 1], li[x - 1]);
        const bool here = !up && lt_pair(v, id, ld[x], li[x]);
        ld[x] = up ? ld[x - 1] : (here ? v : ld[x]);
        li[x] = up ? li[x - 1] : (here ? id : li[x]);
      }
      if (lt_pair(v, id, ld[0], li[0])) { ld[0] = v; li[0] = id; }
    }
  }
  wave_pop<KL>(ld, li, j, &s_wd[wv * j], &s_wi[wv * j], lane);
  __syncthreads();
  if (wv == 0) {
    constexpr int M = (NW * KL + 63) / 64;
    float m[M];
    int mi[M];
#pragma unroll
    for (int x = 0; x < M; ++x) {
      const int c = lane + 64 * x;
      if (c < NW * j) { m[x] = s_wd[c]; mi[x] = s_wi[c]; }
      else { m[x] = INFINITY; mi[x] = INT_MAX; }
    }
    __builtin_amdgcn_wave_barrier();
    sort_regs<M>(m, mi);
    const float jth = wave_pop<M>(m, mi, j, s_out, s_oi, lane);
    if (lane == 0) thr[q] = jth;   // +inf when fewer than j finite samples: collect all
  }
  if (t == 0) count[q] = 0;        // the collect kernel (next in the stream) appends from 0
}

template <int MODE>
__global__ __launch_bounds__(256) void topk_collect_kernel(const TopkSrc s, int64_t n,
                                                           const float* __restrict__ thr,
                                                           int cap, float* __restrict__ cand_d,
                                                           int32_t* __restrict__ cand_i,
                                                           int* __restrict__ count) {
  __shared__ uint64_t s_q[kTopMaxWords];
  const int q = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63;
  float qn = 0.f;
  if (MODE == 0) {
    for (int w = t; w < s.words; w += 256) s_q[w] = s.qbits[(int64_t)q * s.words + w];
    qn = s.qnorm[q];
  }
  __syncthreads();
  uint64_t qb[kTopMaxWords];
#pragma unroll
  for (int w = 0; w < kTopMaxWords; ++w) qb[w] = (MODE == 0 && w < s.words) ? s_q[w] : 0ull;
  const float T = thr[q];
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += stride * 4) {
    float d[4];
    int ix[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t row = base + r * stride + t;
      load_item<MODE>(s, q, n, row, qb, qn, d[r], ix[r]);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const bool pass = d[r] <= T && d[r] < INFINITY;
      const uint64_t m = __ballot(pass);
      if (m == 0) continue;
      int basei = 0;
      if (lane == 0) basei = atomicAdd(&count[q], __popcll(m));
      basei = __shfl(basei, 0, 64);
      if (pass) {
        const int pos = basei + __popcll(m & ((1ull << lane) - 1ull));
        if (pos < cap) {
          cand_d[(int64_t)q * cap + pos] = d[r];
          cand_i[(int64_t)q * cap + pos] = ix[r];
        }
      }
    }
  }
}

// exact top-k of the candidates (count from the device), results to host
__global__ __launch_bounds__(1024) void topk_final_kernel(const float* __restrict__ cand_d,
                                                          const int32_t* __restrict__ cand_i,
                                                          const int* __restrict__ count, int cap,
                                                          int k, const float* __restrict__ thr,
                                                          float* __restrict__ out_d,
                                                          int32_t* __restrict__ out_i,
                                                          volatile uint32_t* done, uint32_t seq) {
  constexpr int NW = 16;
  constexpr int T = NW * 64;
  constexpr int KL = 8;   // candidates held per thread per pass
  __shared__ float s_cd[kTopMaxK];
  __shared__ int s_ci[kTopMaxK];
  __shared__ float s_wd[NW * kTopMaxK];
  __shared__ int s_wi[NW * kTopMaxK];
  __shared__ int s_cnt[NW];
  const int q = blockIdx.x;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int c_all = count[q];
  const int nc = c_all < cap ? c_all : cap;
  for (int x = t; x < k; x += T) { s_cd[x] = INFINITY; s_ci[x] = INT_MAX; }
  __syncthreads();
  const float* cd = cand_d + (int64_t)q * cap;
  const int32_t* ci = cand_i + (int64_t)q * cap;
  // passes of T * KL candidates, each merged with the carry (as topk_kernel)
  for (int base = 0; base < nc; base += T * KL) {
    float d[KL];
    int ix[KL];
#pragma unroll
    for (int r = 0; r < KL; ++r) {
      const int c = base + r * T + t;
      d[r] = c < nc ? cd[c] : INFINITY;
      ix[r] = c < nc ? ci[c] : INT_MAX;
    }
    sort_regs<KL>(d, ix);
    // k <= 128 may exceed the 10-per-lane merge of 16 lists: pop at most
    // min(k, 40) per wave here, the carry merge keeps exactness because each
    // wave's list is complete up to what it popped and the rest is retried
    int cnt = 0;
    const int kw = k;
    wave_pop<KL>(d, ix, kw, &s_wd[wv * kw], &s_wi[wv * kw], lane, &cnt);
    if (lane == 0) s_cnt[wv] = cnt;
    __syncthreads();
    if (wv == 0) {
      // merge carry + 16 wave lists: at most (1 + 16) k <= 17 * 128 values,
      // gathered in slices of 640 with the running carry
      for (int off = 0; off < NW * kw; off += 640 - kw) {
        constexpr int M = 10;
        float m[M];
        int mi[M];
#pragma unroll
        for (int x = 0; x < M; ++x) {
          const int c = lane + 64 * x;
          if (c < kw) { m[x] = s_cd[c]; mi[x] = s_ci[c]; }
          else if (c - kw + off < NW * kw && c - kw < 640 - kw) {
            m[x] = s_wd[c - kw + off];
            mi[x] = s_wi[c - kw + off];
          }
          else { m[x] = INFINITY; mi[x] = INT_MAX; }
        }
        __builtin_amdgcn_wave_barrier();
        sort_regs<M>(m, mi);
        wave_pop<M>(m, mi, kw, s_cd, s_ci, lane);
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
  }
  // pinned host memory by system-scope stores, the flag after every
  // thread's stores are acknowledged (no L2 write-back fence)
  for (int x = t; x < k; x += T) {
    sys_store(out_d + (int64_t)q * k + x, s_cd[x]);
    sys_store(out_i + (int64_t)q * k + x, (int32_t)s_ci[x]);
  }
  sys_stores_block_done();
  // too few candidates is only a failure when T cut rows off (T < +inf)
  const bool retry = c_all > cap || (c_all < k && thr[q] < INFINITY);
  if (t == 0) sys_store(const_cast<uint32_t*>(done) + q, retry ? (seq | kTopRetry) : seq);
}

constexpr int kListK = 16;   // k up to this uses topk_lists_kernel

// Waves per block of the scan stage (MODE 0/1). Every block scans a
// contiguous range with a block-wide carry and two barriers per tile, so a
// CU holding one 4-wave block spends most of a tile waiting on HBM latency;
// 16 waves per block (one block per CU, k <= 37 so the 17 k merge fits) keep
// 4x the rows in flight at the same candidate count (measured choices below,
// frozen: tools/bench_topk.py, profiles/r01_topk_kernels.md).
inline int scan_waves(int k, int nq, int64_t nrows) {
  if (k > 37) return 4;
  // measured (tools/bench_topk.py): 16 waves win for one query over a large
  // table (one block per CU, latency-bound: 10M rows k 10 74 vs 165 us) and
  // lose once several queries fill the chip with 4-wave blocks (1M rows x 8
  // queries: 182 vs 55 us); equal at 1M rows x 1 query
  return nq == 1 && nrows >= ((int64_t)2 << 20) ? 16 : 4;
}

// the final merge of the blocks' candidates for k <= kListK uses per-thread
// register lists (measured ~3 us faster than the tile kernel's rank merge,
// profiles/r02_lsh_merge_ab.jsonl)

// JB_TOPK_MQ=0 turns the register multi-query scan off (A/B runs)
// JB_TOPK_MQ_MIN_ROWS: the table size from which the multi-query scan runs
// (kMqMinRows; A/B runs)
inline int64_t mq_min_rows() {
  static const int64_t v = [] {
    const char* e = getenv("JB_TOPK_MQ_MIN_ROWS");
    const long long x = e != nullptr ? atoll(e) : 0;
    return x > 0 ? (int64_t)x : kMqMinRows;
  }();
  return v;
}

inline bool mq_enabled() {
  static const bool on = [] {
    const char* e = getenv("JB_TOPK_MQ");
    return !(e != nullptr && e[0] == '0');
  }();
  return on;
}

inline int mq_stats_on() {
  static const int on = [] {
    const char* e = getenv("JB_TOPK_MQ_STATS");
    return (e != nullptr && e[0] == '1') ? 1 : 0;
  }();
  return on;
}

// sample size: one round of loads for few queries (its latency is the
// whole cost), two for many (each survivor of the looser bound costs every
// query's wave a pass; measured profiles/r5_topk_mq_ab.md)
inline int mq_sample_segments(int nq) { return nq >= 4 ? kMqSampSegMax : kMqSampSegMax / 2; }

// The sample launch is skipped for one query: the scan starts without a
// bound (each wave's first chunk is cut at the k-th of its lanes' minima, a
// full 32-bit radix select for euclid_lsh's float keys). Measured, 10M
// rows, k 10: one lsh query 44.5 -> 42.8 us, one euclid_lsh query 62.6 ->
// 54.4 us without the sample; eight lsh queries 72.9 -> 129.8 us (every
// wave's eight first-chunk cuts), so several queries keep it.
// JB_TOPK_MQ_SAMPLE=1: always (A/B runs)
inline bool mq_sample_on(int nq) {
  static const bool forced = [] {
    const char* e = getenv("JB_TOPK_MQ_SAMPLE");
    return e != nullptr && e[0] == '1';
  }();
  return forced || nq >= 2;
}

template <int W, int NQ>
inline void launch_mq_nq(const TopkSrc& s, int blocks, int nq, int q0, int64_t nrows, int64_t per_block, int k,
                         uint32_t* lim, float* out_d, int32_t* out_i, hipStream_t stream) {
  const bool samp = mq_sample_on(nq);
  if (s.metric == 1) {
    if (samp)
      hipLaunchKernelGGL((topk_mq_sample_kernel<W, true>), dim3(nq), dim3(kMqSampT), 0, stream, s, q0, nrows, k,
                         mq_sample_segments(nq), lim);
    hipLaunchKernelGGL((topk_mq_kernel<W, NQ, true>), dim3(blocks), dim3(kMqT), 0, stream, s, nq, q0, nrows,
                       per_block, k, samp ? lim : nullptr, mq_stats_on(), out_d, out_i);
  } else {
    if (samp)
      hipLaunchKernelGGL((topk_mq_sample_kernel<W, false>), dim3(nq), dim3(kMqSampT), 0, stream, s, q0, nrows, k,
                         mq_sample_segments(nq), lim);
    hipLaunchKernelGGL((topk_mq_kernel<W, NQ, false>), dim3(blocks), dim3(kMqT), 0, stream, s, nq, q0, nrows,
                       per_block, k, samp ? lim : nullptr, mq_stats_on(), out_d, out_i);
  }
}

template <int W>
inline void launch_mq_w(const TopkSrc& s, int blocks, int nq, int q0, int64_t nrows, int64_t per_block, int k,
                        uint32_t* lim, float* out_d, int32_t* out_i, hipStream_t stream) {
  if (nq <= 1) launch_mq_nq<W, 1>(s, blocks, nq, q0, nrows, per_block, k, lim, out_d, out_i, stream);
  else if (nq <= 2) launch_mq_nq<W, 2>(s, blocks, nq, q0, nrows, per_block, k, lim, out_d, out_i, stream);
  else if (nq <= 4) launch_mq_nq<W, 4>(s, blocks, nq, q0, nrows, per_block, k, lim, out_d, out_i, stream);
  else launch_mq_nq<W, 8>(s, blocks, nq, q0, nrows, per_block, k, lim, out_d, out_i, stream);
}

// Launches the scan stage; returns the number of blocks (= candidate lists
// per query, each of k entries, at out + (q * blocks + b) * k), <= blocks.
// JB_TOPK_MQ_BLOCKS: fewer scan blocks than kMqBlocksMax (A/B runs)
inline int mq_blocks_cap() {
  static const int v = [] {
    const char* e = getenv("JB_TOPK_MQ_BLOCKS");
    const int x = e != nullptr ? atoi(e) : kMqBlocksMax;
    return x < 1 ? 1 : (x > kMqBlocksMax ? kMqBlocksMax : x);
  }();
  return v;
}

template <int MODE>
inline int launch_scan(const TopkSrc& s, int blocks, int nq, int64_t nrows, int64_t per_block,
                       int k, float* out_d, int32_t* out_i, hipStream_t stream, int mq_lists = 0) {
  // (measured against topk_wq / topk_kernel, profiles/r5_topk_mq_ab.md: ahead
  // up to 8 queries for lsh / minhash, up to 4 for euclid_lsh, whose
  // prefilter costs a table lookup and a few FMAs per row and query)
  // Tables under ~2M rows keep the tile kernels: the sample launch and the
  // block merge cost more there than the scan saves (measured through the
  // servers: 1M-row euclid_lsh similar_row 53 -> 63 us p50, 100 K-row LOF
  // calc_score 54 -> 74 us)
  if (MODE == 0 && mq_enabled() && blocks > 1 && nrows >= mq_min_rows() && k <= kMqMaxK &&
      (s.words == 1 || s.words == 2) && s.hash_num <= 64 * s.words && nq <= (s.metric == 1 ? 4 : kMqMaxQ)) {
    // the sampled bound, then the table streamed once per launch of up to
    // kMqMaxQ queries (topk_mq_kernel); at least 4 chunks a wave so its carry
    // prunes, fewer blocks than the caller sized the candidate scratch for
    // (the sample's limits live past the candidates, at out_i + nq mb k)
    constexpr int64_t kPer = (int64_t)kMqWaves * kMqChunk;
    // (mq_lists: the candidate lists the caller's scratch holds - the mb
    // lists plus the sample's limits must fit)
    const int64_t room = (mq_lists > 1 ? mq_lists : blocks) - 1;
    const int64_t cap = room < mq_blocks_cap() ? room : mq_blocks_cap();
    int64_t mb = (nrows + 4 * kPer - 1) / (4 * kPer);
    mb = mb < 1 ? 1 : (mb > cap ? cap : mb);
    int64_t pb = (nrows + mb - 1) / mb;
    pb = (pb + kPer - 1) / kPer * kPer;
    mb = (nrows + pb - 1) / pb;
    uint32_t* lim = reinterpret_cast<uint32_t*>(out_i + (int64_t)nq * mb * k);
    for (int q0 = 0; q0 < nq; q0 += kMqMaxQ) {
      const int nqi = nq - q0 < kMqMaxQ ? nq - q0 : kMqMaxQ;
      if (s.words == 1)
        launch_mq_w<1>(s, (int)mb, nqi, q0, nrows, pb, k, lim, out_d, out_i, stream);
      else
        launch_mq_w<2>(s, (int)mb, nqi, q0, nrows, pb, k, lim, out_d, out_i, stream);
    }
    return (int)mb;
  }
  if (MODE == 0 && nq > 1 && nq <= kWqWaves && s.words <= 2 && s.hash_num <= 64 * s.words) {
    // several queries per table pass, one wave per query (topk_wq_kernel)
    if (s.words == 1)
      hipLaunchKernelGGL((topk_wq_kernel<1>), dim3(blocks), dim3(kWqT), 0, stream, s, nq, nrows,
                         per_block, k, out_d, out_i);
    else
      hipLaunchKernelGGL((topk_wq_kernel<2>), dim3(blocks), dim3(kWqT), 0, stream, s, nq, nrows,
                         per_block, k, out_d, out_i);
    return blocks;
  }
  if (scan_waves(k, nq, nrows) == 16)
    hipLaunchKernelGGL((topk_kernel<MODE, 16>), dim3(blocks, nq), dim3(16 * 64), 0, stream, s,
                       nrows, per_block, k, out_d, out_i, nullptr, 0u);
  else
    hipLaunchKernelGGL((topk_kernel<MODE, 4>), dim3(blocks, nq), dim3(4 * 64), 0, stream, s,
                       nrows, per_block, k, out_d, out_i, nullptr, 0u);
  return blocks;
}

// Final merge of the scan's per-block lists (each sorted, k entries) for
// k <= kListK and <= kMergeLists blocks: ONE wave per query. The lists go to
// LDS; lane l owns lists l, l + 64, ... and keeps their heads in registers;
// each of k rounds takes the wave's arg-min head (DPP / permlane) and its
// owner advances that list. The per-thread insertion lists of
// topk_lists_kernel cost ~20 us here (16 waves of VALU pops on a handful of
// real candidates); this is k rounds of a dozen register steps.
constexpr int kMergeLists = 512;
constexpr int kMergeStageT = 256;   // threads staging the lists into LDS (wave 0 merges)
__global__ __launch_bounds__(kMergeStageT) void topk_merge_sorted_kernel(const float* __restrict__ cd,
                                                               const int32_t* __restrict__ ci, int nb, int k,
                                                               float* __restrict__ out_d,
                                                               int32_t* __restrict__ out_i,
                                                               volatile uint32_t* done, uint32_t seq) {
  constexpr int L = kMergeLists / 64;
  extern __shared__ float s_mg[];    // [nb k] distances, then [nb k] rows
  float* s_d = s_mg;
  int* s_i = reinterpret_cast<int*>(s_mg + nb * k);
  __shared__ float s_rd[kListK];
  __shared__ int s_ri[kListK];
  const int q = blockIdx.x, lane = threadIdx.x;
  const int n = nb * k;
  const float* src_d = cd + (int64_t)q * n;
  const int32_t* src_i = ci + (int64_t)q * n;
  // (eight loads a thread in flight: one load-then-store a trip waited a
  // memory round trip each, most of this kernel's time)
  for (int e0 = threadIdx.x; e0 < n; e0 += 8 * kMergeStageT) {
    float vd[8];
    int vi[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * kMergeStageT;
      vd[u] = e < n ? src_d[e] : 0.f;
      vi[u] = e < n ? src_i[e] : 0;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * kMergeStageT;
      if (e < n) { s_d[e] = vd[u]; s_i[e] = vi[u]; }
    }
  }
  __syncthreads();
  if (threadIdx.x >= 64) return;                  // the merge is one wave's
  int pos[L];
  float hd[L];
  int hi[L];
#pragma unroll
  for (int u = 0; u < L; ++u) {
    const int list = lane + 64 * u;
    pos[u] = 0;
    hd[u] = list < nb ? s_d[list * k] : INFINITY;
    hi[u] = list < nb ? s_i[list * k] : INT_MAX;
  }
  for (int r = 0; r < k; ++r) {
    float v = hd[0];
    int id = hi[0], bu = 0;
#pragma unroll
    for (int u = 1; u < L; ++u)
      if (lt_pair(hd[u], hi[u], v, id)) { v = hd[u]; id = hi[u]; bu = u; }
    float wv = v;
    int wid = id;
    wave_argmin(wv, wid, lane);
    if (lane == 0) { s_rd[r] = wv; s_ri[r] = wid; }
    if (v == wv && id == wid) {          // the owner (padding entries may match on several lanes: harmless)
#pragma unroll
      for (int u = 0; u < L; ++u) {
        if (u != bu) continue;
        const int list = lane + 64 * u;
        const int p = ++pos[u];
        hd[u] = p < k ? s_d[list * k + p] : INFINITY;
        hi[u] = p < k ? s_i[list * k + p] : INT_MAX;
      }
    }
  }
  wave_sync();                          // (waves 1..3 have left: wave-level ordering only)
  const int64_t o = (int64_t)q * k;
  if (done != nullptr) {
    for (int j = lane; j < k; j += 64) { sys_store(out_d + o + j, s_rd[j]); sys_store(out_i + o + j, s_ri[j]); }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the wave's stores acknowledged, then the flag
    if (lane == 0) sys_store(const_cast<uint32_t*>(done) + q, seq);
    return;
  }
  for (int j = lane; j < k; j += 64) { out_d[o + j] = s_rd[j]; out_i[o + j] = s_ri[j]; }
}

// the final merge: one block per query; 16 waves when the (17 k) candidates
// of the merge stage fit (k <= 37), else 4
inline void launch_merge(const TopkSrc& m, int nq, int64_t nc, int k, float* out_d,
                         int32_t* out_i, volatile uint32_t* done, uint32_t seq,
                         hipStream_t stream) {
  if (k <= kListK && nc % k == 0 && nc / k <= kMergeLists) {
    hipLaunchKernelGGL(topk_merge_sorted_kernel, dim3(nq), dim3(kMergeStageT), (size_t)nc * 8, stream, m.src_d, m.src_i,
                       (int)(nc / k), k, out_d, out_i, done, seq);
  } else if (k <= kListK) {
    hipLaunchKernelGGL((topk_lists_kernel<2, kListK, 16>), dim3(1, nq), dim3(16 * 64), 0, stream,
                       m, nc, nc, k, out_d, out_i, done, seq);
  } else if (k <= 37) {
    const int64_t tile = 16 * 64 * kTopR;
    hipLaunchKernelGGL((topk_kernel<2, 16>), dim3(1, nq), dim3(16 * 64), 0, stream, m, nc,
                       ((nc + tile - 1) / tile) * tile, k, out_d, out_i, done, seq);
  } else {
    hipLaunchKernelGGL((topk_kernel<2, 4>), dim3(1, nq), dim3(4 * 64), 0, stream, m, nc,
                       ((nc + kTopTile - 1) / kTopTile) * kTopTile, k, out_d, out_i, done, seq);
  }
}

}  // namespace jb

// Top-k smallest distances of nq queries.
//   mode 0: fused signature scan (qbits [nq][words], tbits [nrows][words],
//           norms, valid, metric 0 lsh / 1 euclid_lsh / 2 minhash)
//   mode 1: score vector src_d [nq][nrows] (flip: distance = 1 - score)
// out_d / out_i: [nq][k] (+inf / INT_MAX padding). scratch_d / scratch_i:
// >= nq * jb_topk_blocks(nrows, k) * k entries each. k <= 128.
static int topk_tile_blocks(int64_t nrows, int k) {
  if (k <= 0 || nrows <= 0) return 0;
  const int64_t tiles = (nrows + jb::kTopTile - 1) / jb::kTopTile;
  // bound the candidates K2 merges; one block per CU is enough to stream
  // the table (the scan is a few bytes per row)
  // (256: more blocks measured slower for batched queries,
  // profiles/r02_lsh_block_cap.jsonl; again with the one-wave merge: 512
  // blocks took one query at 1M rows 44 -> 42 us but four 48 -> 65 us and one
  // at 10M rows 102 -> 121 us, profiles/r4_topk_lsh_blocks512.jsonl)
  constexpr int64_t cap = 256;
  int64_t max_blocks = 8192 / k < cap ? 8192 / k : cap;
  if (max_blocks < 1) max_blocks = 1;
  const int64_t tiles_per_block = (tiles + max_blocks - 1) / max_blocks;
  return (int)((tiles + tiles_per_block - 1) / tiles_per_block);
}

// candidate lists the scratch must hold per query: the tile kernels' grid,
// or the multi-query scan's (up to jb::kMqBlocksMax blocks on tables of
// kMqMinRows and more: two blocks a CU keep more rows in flight than one)
extern "C" int jb_topk_blocks(int64_t nrows, int k) {
  const int tb = topk_tile_blocks(nrows, k);
  if (tb > 0 && nrows >= jb::mq_min_rows() && k <= jb::kMqMaxK)
    return tb > jb::kMqBlocksMax + 1 ? tb : jb::kMqBlocksMax + 1;
  return tb;
}

extern "C" int jb_topk(int mode, const uint64_t* qbits, const float* qnorm, int nq,
                       const uint64_t* tbits, const float* tnorm, const uint8_t* valid,
                       int64_t nrows, int words, int hash_num, int metric, const float* src_d,
                       int flip, int k, float* scratch_d, int32_t* scratch_i, float* out_d,
                       int32_t* out_i, hipStream_t stream) {
  if (nq <= 0 || nrows <= 0 || k <= 0) return 0;
  if (k > jb::kTopMaxK || words > jb::kTopMaxWords || (mode != 0 && mode != 1)) return -2;
  const int blocks = topk_tile_blocks(nrows, k);
  const int lists = jb_topk_blocks(nrows, k);
  const int64_t tiles = (nrows + jb::kTopTile - 1) / jb::kTopTile;
  const int64_t per_block = ((tiles + blocks - 1) / blocks) * jb::kTopTile;
  jb::TopkSrc s{qbits, qnorm, tbits, tnorm, valid, words, hash_num, metric, src_d, nullptr, flip};
  const int used = mode == 0 ? jb::launch_scan<0>(s, blocks, nq, nrows, per_block, k, scratch_d, scratch_i, stream,
                                                  lists)
                              : jb::launch_scan<1>(s, blocks, nq, nrows, per_block, k, scratch_d, scratch_i, stream,
                                                  lists);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int64_t nc = (int64_t)used * k;   // candidates per query
  jb::TopkSrc m{nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, scratch_d, scratch_i, 0};
  jb::launch_merge(m, nq, nc, k, out_d, out_i, nullptr, 0u, stream);
  return (int)hipGetLastError();
}

// Latency path (mode 0): as jb_topk, but the final merge writes straight into
// fine-grained pinned host memory and publishes done[q] = seq per query
// (tile path).
static int topk_to_host_tile(const uint64_t* qbits, const float* qnorm, int nq,
                             const uint64_t* tbits, const float* tnorm, const uint8_t* valid,
                             int64_t nrows, int words, int hash_num, int metric, int k,
                             float* scratch_d, int32_t* scratch_i, float* out_d_host,
                             int32_t* out_i_host, uint32_t* done_host, uint32_t seq,
                             hipStream_t stream) {
  const int blocks = topk_tile_blocks(nrows, k);
  const int64_t tiles = (nrows + jb::kTopTile - 1) / jb::kTopTile;
  const int64_t per_block = ((tiles + blocks - 1) / blocks) * jb::kTopTile;
  jb::TopkSrc s{qbits, qnorm, tbits, tnorm, valid, words, hash_num, metric, nullptr, nullptr, 0};
  const int used = jb::launch_scan<0>(s, blocks, nq, nrows, per_block, k, scratch_d, scratch_i, stream,
                                      jb_topk_blocks(nrows, k));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  const int64_t nc = (int64_t)used * k;
  jb::TopkSrc m{nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, scratch_d, scratch_i, 0};
  jb::launch_merge(m, nq, nc, k, out_d_host, out_i_host, (volatile uint32_t*)done_host, seq,
                   stream);
  return (int)hipGetLastError();
}

// scratch layout of the sampled path (in scratch_d / scratch_i, sized by
// jb_topk_direct_scratch): thr[8] | count[8] | candidates [nq][kCandCap]
constexpr int kCandCap = 65536;
constexpr int64_t kSampleMax = 16384;

// j for the sampled threshold, 0 when the tile path is the better choice
// (below ~2M rows the tile path is as fast, and it cannot overflow on rows
// that tie at the threshold - e.g. duplicated data)
static int sample_j(int64_t nrows, int k) {
  if (nrows < (int64_t)2 << 20) return 0;
  const int64_t S = nrows < kSampleMax ? nrows : kSampleMax;
  const double j = 4.0 * k * (double)S / (double)nrows;
  const int jj = (int)j + 3;
  return jj <= 16 ? jj : 0;
}

// + the radix-select histograms of the score path: 2 levels x nq x 4096
constexpr int kRadixBins = 4096;
// the one-launch score top-k keeps per-query histograms and counters that
// must be zero when it starts (it leaves them zero when it ends): a fixed
// region after the candidates of 8 queries, out of reach of the tile path's
// block candidates (<= 8 x 256 x 128 entries)
constexpr int64_t kFuseStateOff = 64 + 8 * (int64_t)kCandCap;
constexpr int64_t kFuseStateWords = 2 * 8 * (int64_t)kRadixBins + 8 * 4;
extern "C" int64_t jb_topk_direct_scratch(int nq) {
  (void)nq;
  return kFuseStateOff + kFuseStateWords;
}

// zero the score top-k's state region of a scratch allocation (once, after
// allocating it; scratch_i as passed to jb_topk_scores_direct)
extern "C" int jb_topk_scratch_init(int32_t* scratch_i, hipStream_t stream) {
  hipError_t e = hipMemsetAsync(scratch_i + kFuseStateOff, 0, sizeof(int32_t) * kFuseStateWords,
                                stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);   // done before any stream uses it
  return (int)e;
}

template <int MODE>
static int topk_fused_launch(const jb::TopkSrc& s, int nq, int64_t nrows, int k,
                             float* scratch_d, int32_t* scratch_i, float* out_d_host,
                             int32_t* out_i_host, uint32_t* done_host, uint32_t seq,
                             hipStream_t stream);

template <int MODE>
static int topk_onepass_launch(const jb::TopkSrc& s, int nq, int64_t nrows, int k, float* scratch_d,
                               int32_t* scratch_i, float* out_d_host, int32_t* out_i_host,
                               uint32_t* done_host, uint32_t seq, hipStream_t stream);

template <int MODE>
static int topk_select_launch(const jb::TopkSrc& s, int nq, int64_t nrows, int k, float* scratch_d,
                              int32_t* scratch_i, float* out_d_host, int32_t* out_i_host,
                              uint32_t* done_host, uint32_t seq, hipStream_t stream);

// the LDS-select launch by default (tools/bench_topk_lsh.py, 100 K and 1M
// rows): for k past kListK while rows x k stays moderate (1M rows: k 31 67 us
// vs 80, 4 queries k 40 81 vs 131; k 100 106 vs 91 one launch), and for
// several queries on small tables (100 K rows, 4 x k 10: 38 vs 44 us; at 1M
// the tile path's multi-query scan wins, 49 vs 92)
static bool select_default(int64_t nrows, int k, int nq) {
  if (nrows < 16384) return false;
  if (k > jb::kListK) return nrows * k <= ((int64_t)64 << 20);
  return nq > 1 && nrows <= 256 * 1024;
}

// path: -1 default, 0 tile, 2 one launch (grid barriers), 3 one pass, 4 LDS select. Default (measured at 1M rows,
// profiles/r03_topk_paths_ab.jsonl): the tile path up to k = kListK (k 10:
// 58 us vs 86 us one launch, whose two grid barriers cost more than the
// tile path's second launch), one launch past it (k 100: 94 us vs 224 us,
// the tile path's per-tile selection grows with k); the sampled path from 2M
// rows
static int topk_to_host_any(const uint64_t* qbits, const float* qnorm, int nq,
                            const uint64_t* tbits, const float* tnorm, const uint8_t* valid,
                            int64_t nrows, int words, int hash_num, int metric, int k,
                            float* scratch_d, int32_t* scratch_i, float* out_d_host,
                            int32_t* out_i_host, uint32_t* done_host, uint32_t seq,
                            hipStream_t stream, int path = -1) {
  const int j = sample_j(nrows, k);
  if (path == 3) {
    jb::TopkSrc s{qbits, qnorm, tbits, tnorm, valid, words, hash_num, metric, nullptr, nullptr, 0};
    return topk_onepass_launch<0>(s, nq, nrows, k, scratch_d, scratch_i, out_d_host, out_i_host,
                                  done_host, seq, stream);
  }
  if (path == 4 || (path < 0 && j == 0 && select_default(nrows, k, nq))) {
    jb::TopkSrc s{qbits, qnorm, tbits, tnorm, valid, words, hash_num, metric, nullptr, nullptr, 0};
    return topk_select_launch<0>(s, nq, nrows, k, scratch_d, scratch_i, out_d_host, out_i_host, done_host,
                                 seq, stream);
  }
  if (path == 2 || (path < 0 && j == 0 && nrows >= 16384 && k > jb::kListK)) {
    jb::TopkSrc s{qbits, qnorm, tbits, tnorm, valid, words, hash_num, metric, nullptr, nullptr, 0};
    return topk_fused_launch<0>(s, nq, nrows, k, scratch_d, scratch_i, out_d_host, out_i_host,
                                done_host, seq, stream);
  }
  if (j == 0 || path == 0)
    return topk_to_host_tile(qbits, qnorm, nq, tbits, tnorm, valid, nrows, words, hash_num,
                             metric, k, scratch_d, scratch_i, out_d_host, out_i_host, done_host,
                             seq, stream);
  jb::TopkSrc s{qbits, qnorm, tbits, tnorm, valid, words, hash_num, metric, nullptr, nullptr, 0};
  float* thr = scratch_d;                         // [8]
  int* count = scratch_i;                         // [8]
  float* cand_d = scratch_d + 64;
  int32_t* cand_i = scratch_i + 64;
  const int64_t S = nrows < kSampleMax ? nrows : kSampleMax;
  hipLaunchKernelGGL(jb::topk_sample_kernel<0>, dim3(nq), dim3(jb::kSampleThreads), 0, stream, s,
                     nrows, S, j, thr, count);
  int64_t cblocks = (nrows + 1023) / 1024;        // 4 rows per thread
  if (cblocks > 1024) cblocks = 1024;
  hipLaunchKernelGGL(jb::topk_collect_kernel<0>, dim3((unsigned)cblocks, nq), dim3(256), 0, stream,
                     s, nrows, thr, kCandCap, cand_d, cand_i, count);
  hipLaunchKernelGGL(jb::topk_final_kernel, dim3(nq), dim3(1024), 0, stream, cand_d, cand_i,
                     count, kCandCap, k, thr, out_d_host, out_i_host,
                     (volatile uint32_t*)done_host, seq);
  return (int)hipGetLastError();
}

// launch + wait; a sampled run whose threshold missed reruns the tile path
static int topk_direct_run(const uint64_t* qbits, const float* qnorm, int nq,
                           const uint64_t* tbits, const float* tnorm, const uint8_t* valid,
                           int64_t nrows, int words, int hash_num, int metric, int k,
                           float* scratch_d, int32_t* scratch_i, float* out_d_host,
                           int32_t* out_i_host, uint32_t* done_host, hipStream_t stream,
                           int path = -1) {
  uint32_t seq = jb::next_seq();
  int rc = topk_to_host_any(qbits, qnorm, nq, tbits, tnorm, valid, nrows, words, hash_num, metric,
                            k, scratch_d, scratch_i, out_d_host, out_i_host, done_host, seq,
                            stream, path);
  if (rc != 0) return rc;
  bool retry = false;
  rc = jb::wait_flags_status(done_host, nq, seq, jb::kTopRetry, stream, &retry);
  if (rc != 0 || !retry) return rc;
  seq = jb::next_seq();
  rc = topk_to_host_tile(qbits, qnorm, nq, tbits, tnorm, valid, nrows, words, hash_num, metric, k,
                         scratch_d, scratch_i, out_d_host, out_i_host, done_host, seq, stream);
  if (rc != 0) return rc;
  return jb::wait_flags(done_host, nq, seq, stream);
}

// query signatures on the device -> top-k in pinned host memory, waited for
extern "C" int jb_topk_direct_query(const uint64_t* qbits, const float* qnorm, int nq,
                                    const uint64_t* tbits, const float* tnorm,
                                    const uint8_t* valid, int64_t nrows, int words, int hash_num,
                                    int metric, int k, float* scratch_d, int32_t* scratch_i,
                                    float* out_d_host, int32_t* out_i_host, uint32_t* done_host,
                                    hipStream_t stream) {
  if (nq <= 0 || nrows <= 0 || k <= 0) return 0;
  if (k > jb::kTopMaxK || words > jb::kTopMaxWords || nq > 8) return -2;
  return topk_direct_run(qbits, qnorm, nq, tbits, tnorm, valid, nrows, words, hash_num, metric, k,
                         scratch_d, scratch_i, out_d_host, out_i_host, done_host, stream);
}

// as jb_topk_direct_query with the path forced (A/B in tools/bench_topk_lsh.py):
// -1 default, 0 tile, 2 one launch
extern "C" int jb_topk_direct_query_path(const uint64_t* qbits, const float* qnorm, int nq,
                                         const uint64_t* tbits, const float* tnorm,
                                         const uint8_t* valid, int64_t nrows, int words,
                                         int hash_num, int metric, int k, float* scratch_d,
                                         int32_t* scratch_i, float* out_d_host,
                                         int32_t* out_i_host, uint32_t* done_host, int path,
                                         hipStream_t stream) {
  if (nq <= 0 || nrows <= 0 || k <= 0) return 0;
  if (k > jb::kTopMaxK || words > jb::kTopMaxWords || nq > 8) return -2;
  return topk_direct_run(qbits, qnorm, nq, tbits, tnorm, valid, nrows, words, hash_num, metric, k,
                         scratch_d, scratch_i, out_d_host, out_i_host, done_host, stream, path);
}

// Score-vector latency path (mode 1: [nq][nrows] similarity / distance from
// the inverted index scan, csrc/hip/sparse_pool.hip), exact two-level radix
// select instead of the tile kernel's per-tile selection:
//   R1  histogram of the top 12 bits of the order-preserving key of every
//       distance (LDS per block, then global atomics);
//   R2  one block per query: the bucket holding the k-th smallest;
//   R3  histogram of the next 12 bits inside that bucket;
//   R4  the sub-bucket holding the k-th smallest -> threshold T (all rows
//       with key <= T: at most k + that sub-bucket's size);
//   R5  collect the rows <= T (topk_collect_kernel), R6 exact top-k of the
//       candidates into pinned host memory (topk_final_kernel).
// Cost: three 4-byte reads per row, no per-tile sorting, independent of k.
// Ties beyond the candidate buffer (e.g. thousands of identical distances)
// flag a retry and the exact tile path reruns.
namespace jb {

__device__ __forceinline__ uint32_t dist_key(float d) {
  const uint32_t u = __float_as_uint(d);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);      // monotone in d
}
__device__ __forceinline__ float key_dist(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Histogram of one radix level's 12-bit digit of every distance (LDS per
// block, merged with global atomics). Most rows of a cosine score vector
// share one digit (score 0 -> distance 1, 99% of the rows here), so each
// wave adds the digit of its first active lane with one LDS atomic and only
// the other lanes add their own (hist 1 under the tracer: 13.1 -> 11.4 us).
// A last-block select fused into this kernel measured slower (the
// agent-scope fence per block, then 512 blocks serialized on the
// finished-block counter; profiles/r02_topk_scores.jsonl).
template <int LEVEL>
__global__ __launch_bounds__(256) void radix_hist_kernel(const float* __restrict__ src, int flip,
                                                         int64_t n,
                                                         const uint32_t* __restrict__ sel,
                                                         uint32_t* __restrict__ hist) {
  constexpr int T = 256;
  __shared__ uint32_t h[kRadixBins];
  const int q = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63;
  for (int i = t; i < kRadixBins; i += T) h[i] = 0;
  __syncthreads();
  const uint32_t pre = LEVEL == 2 ? sel[2 * q] : 0u;
  const float* sq = src + (int64_t)q * n;
  const int64_t stride = (int64_t)gridDim.x * T * 4;
  for (int64_t b = (int64_t)blockIdx.x * T * 4 + t; b < n; b += stride) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = b + u * T;
      v[u] = sq[i < n ? i : n - 1];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float d = flip ? 1.f - v[u] : v[u];
      const uint32_t key = dist_key(d);
      const uint32_t bin = LEVEL == 1 ? key >> 20 : (key >> 8) & 0xfff;
      // invalid rows / NaN (!(d < inf)) and, on level 2, rows outside the bucket
      const bool act = b + u * T < n && d < INFINITY && (LEVEL == 1 || (key >> 20) == pre);
      const uint64_t am = __ballot(act);
      if (am == 0) continue;
      const int leader = __ffsll((unsigned long long)am) - 1;
      const uint32_t b0 = __shfl(bin, leader, 64);
      const uint64_t same = __ballot(act && bin == b0);
      if (lane == leader) atomicAdd(&h[b0], (uint32_t)__popcll(same));
      else if (act && bin != b0) atomicAdd(&h[bin], 1u);
    }
  }
  __syncthreads();
  uint32_t* gh = hist + (int64_t)q * kRadixBins;
  for (int i = t; i < kRadixBins; i += T)
    if (h[i]) atomicAdd(&gh[i], h[i]);
}

// sel[2q] = level-1 bucket, sel[2q + 1] = rows below it; level 2 writes the
// float threshold thr[q] and zeroes the candidate count
template <int LEVEL>
__global__ __launch_bounds__(1024) void radix_select_kernel(const uint32_t* __restrict__ hist,
                                                            int k, uint32_t* __restrict__ sel,
                                                            float* __restrict__ thr,
                                                            int* __restrict__ count) {
  __shared__ uint32_t part[1024];
  const int q = blockIdx.x;
  const uint32_t* h = hist + (int64_t)q * kRadixBins;
  const int t = threadIdx.x;
  uint32_t c[4];
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) { c[j] = h[4 * t + j]; sum += c[j]; }
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {          // inclusive scan of the per-thread sums
    const uint32_t x = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  const uint32_t before_me = part[t] - sum;
  const uint32_t total = part[1023];
  const uint32_t need = LEVEL == 1 ? (uint32_t)k : (uint32_t)k - sel[2 * q + 1];
  if (t == 0 && total < need) {                 // fewer finite rows than needed
    if (LEVEL == 1) { sel[2 * q] = 0xffffffffu; sel[2 * q + 1] = 0; }
    else { thr[q] = INFINITY; count[q] = 0; }
  }
  uint32_t run = before_me;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (run < need && run + c[j] >= need) {     // exactly one bin satisfies this
      const uint32_t bin = 4 * t + j;
      if (LEVEL == 1) {
        sel[2 * q] = bin;
        sel[2 * q + 1] = run;
      } else {
        const uint32_t T = (sel[2 * q] << 20) | (bin << 8) | 0xffu;
        thr[q] = key_dist(T);
        count[q] = 0;
      }
    }
    run += c[j];
  }
}

}  // namespace jb

namespace jb {

// exact top-k of a small candidate set by ranking: every candidate's final
// position is the number of candidates before it in (distance, row) order;
// for k <= kListK and more than 32 candidates (ties at the threshold) register
// lists instead (the rank loop is LDS-latency bound: 156 tied candidates
// 20 us, lists ~5 us); more than kRankMax candidates -> retry on the tile path.
constexpr int kRankMax = 4096;
__global__ __launch_bounds__(1024) void topk_rank_final_kernel(
    const float* __restrict__ cand_d, const int32_t* __restrict__ cand_i,
    const int* __restrict__ count, int cap, int k, const float* __restrict__ thr,
    float* __restrict__ out_d, int32_t* __restrict__ out_i, volatile uint32_t* done,
    uint32_t seq) {
  __shared__ float s_d[kRankMax];
  __shared__ int32_t s_i[kRankMax];
  const int q = blockIdx.x;
  const int t = threadIdx.x;
  const int c_all = count[q];
  const bool over = c_all > kRankMax || c_all > cap;
  const int nc = over ? 0 : c_all;
  for (int j = t; j < nc; j += blockDim.x) {
    s_d[j] = cand_d[(int64_t)q * cap + j];
    s_i[j] = cand_i[(int64_t)q * cap + j];
  }
  for (int j = nc + t; j < k; j += blockDim.x) {          // fewer candidates than k: padding
    out_d[(int64_t)q * k + j] = INFINITY;
    out_i[(int64_t)q * k + j] = INT_MAX;
  }
  __syncthreads();
  if (k <= kListK && nc > 32) {
    // many candidates (ties at the threshold): per-thread sorted top-16 of
    // its strided candidates, per-wave pops, then wave 0 merges the 16 waves'
    // lists - O(nc k / threads) instead of the rank's O(nc^2 / threads)
    constexpr int NW = 16;
    float ld[kListK];
    int li[kListK];
#pragma unroll
    for (int j = 0; j < kListK; ++j) { ld[j] = INFINITY; li[j] = INT_MAX; }
    for (int j = t; j < nc; j += blockDim.x) {
      const float v = s_d[j];
      const int id = s_i[j];
      if (lt_pair(v, id, ld[kListK - 1], li[kListK - 1])) {
#pragma unroll
        for (int x = kListK - 1; x > 0; --x) {
          const bool up = lt_pair(v, id, ld[x - 1], li[x - 1]);
          const bool here = !up && lt_pair(v, id, ld[x], li[x]);
          ld[x] = up ? ld[x - 1] : (here ? v : ld[x]);
          li[x] = up ? li[x - 1] : (here ? id : li[x]);
        }
        if (lt_pair(v, id, ld[0], li[0])) { ld[0] = v; li[0] = id; }
      }
    }
    __syncthreads();                               // s_d / s_i reused for the wave lists
    const int lane = t & 63, wv = t >> 6;
    wave_pop<kListK>(ld, li, k, &s_d[wv * k], &s_i[wv * k], lane);
    __syncthreads();
    if (wv == 0) {
      constexpr int M = (NW * kListK + 63) / 64;
      float m[M];
      int mi[M];
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const int c = lane + 64 * j;
        if (c < NW * k) { m[j] = s_d[c]; mi[j] = s_i[c]; }
        else { m[j] = INFINITY; mi[j] = INT_MAX; }
      }
      __builtin_amdgcn_wave_barrier();
      sort_regs<M>(m, mi);
      wave_pop<M>(m, mi, k, out_d + (int64_t)q * k, out_i + (int64_t)q * k, lane);
    }
  } else {
    for (int j = t; j < nc; j += blockDim.x) {
      const float d = s_d[j];
      const int32_t id = s_i[j];
      int rank = 0;
      for (int x = 0; x < nc; ++x) {
        const float e = s_d[x];
        rank += (e < d) || (e == d && s_i[x] < id);
        if ((x & 63) == 63 && rank >= k) break;    // already out of the top k
      }
      if (rank < k) {
        sys_store(out_d + (int64_t)q * k + rank, d);
        sys_store(out_i + (int64_t)q * k + rank, (int32_t)id);
      }
    }
  }
  sys_stores_block_done();
  const bool retry = over || (c_all < k && thr[q] < INFINITY);
  if (t == 0) sys_store(const_cast<uint32_t*>(done) + q, retry ? (seq | kTopRetry) : seq);
}

}  // namespace jb

namespace jb {

// ---------------------------------------------------------------------------
// Exact top-k as ONE launch, for a score vector (MODE 1: the inverted-index
// scan's output) or straight off the signature table (MODE 0: lsh /
// minhash / euclid_lsh distances computed in place). Replaces chains of
// dependent launches (score path: hist / select / hist / select / collect /
// final plus a histogram memset; signature path: per-block tile top-k, then
// a merge of blocks x k candidates) whose gaps and serial merges dominated a
// ~1M-row query. A grid of B blocks per query, at most as many blocks as are
// co-resident (kFuseThreads threads, 48 KB of LDS each), every block owning a
// contiguous range of rows:
//   A  distances of its rows (kept in LDS for the first kFuseCache rows),
//      level-1 histogram of the top 12 key bits -> global h1
//   -- grid barrier (per query: arrival counter, agent-scope atomics) --
//   B  every block reads h1 and finds the bucket of the k-th smallest
//      (redundantly: no extra barrier), level-2 histogram of its rows in that
//      bucket -> global h2
//   -- grid barrier --
//   C  threshold T from h2, rows with key <= T appended to the candidates;
//      the last block to finish (finished-block counter) ranks the
//      candidates, writes the k results into pinned host memory, publishes
//      the flag and zeroes the query's histograms and counters for the next
//      launch (so no memset precedes it)
// HBM is read once for up to B x kFuseCache rows; passes B and C read LDS.
// Ties are broken by the lower row index (lt_pair), like the tile path.
constexpr int kFuseThreads = 256;
constexpr int kFuseMaxBlocks = 256;
constexpr int kFuseSync = 4;            // per query: arrivals, candidates, finished, pad
constexpr int kFuseCache = 8192;        // distances kept in LDS per block

__device__ __forceinline__ uint32_t ld_agent_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every block of the query arrives; returns once `target` blocks did
__device__ __forceinline__ void fused_barrier(uint32_t* arrive, uint32_t target) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();                                   // release this block's atomics / stores
    atomicAdd(arrive, 1u);
    while (ld_agent_u32(arrive) < target) __builtin_amdgcn_s_sleep(1);
    __threadfence();                                   // acquire
  }
  __syncthreads();
}

// bucket of the need-th smallest in a 4096-bin global histogram: out[0] bin
// (0xffffffff: fewer than `need` entries), out[1] entries below it
__device__ __forceinline__ void fused_select(const uint32_t* g, uint32_t need, uint32_t* part,
                                             uint32_t* out) {
  const int t = threadIdx.x;
  constexpr int P = kRadixBins / kFuseThreads;       // 16 bins per thread
  uint32_t c[P];
  uint32_t sum = 0;
#pragma unroll
  for (int j = 0; j < P; ++j) { c[j] = ld_agent_u32(g + P * t + j); sum += c[j]; }
  part[t] = sum;
  if (t == 0) out[0] = 0xffffffffu;
  __syncthreads();
  for (int o = 1; o < kFuseThreads; o <<= 1) {
    const uint32_t x = t >= o ? part[t - o] : 0u;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  uint32_t run = part[t] - sum;
#pragma unroll
  for (int j = 0; j < P; ++j) {
    if (run < need && run + c[j] >= need) { out[0] = P * t + j; out[1] = run; }
    run += c[j];
  }
  __syncthreads();
}

// histogram of a wave's 64 keys into LDS: most rows of a score vector (and
// many of a hamming scan) share one bin, so the wave's first active lane
// adds the count of its bin and the others their own
__device__ __forceinline__ void fused_bin(uint32_t* h, bool act, uint32_t bin, int lane) {
  const uint64_t am = __ballot(act);
  if (am == 0) return;
  const int leader = __ffsll((unsigned long long)am) - 1;
  const uint32_t b0 = __shfl(bin, leader, 64);
  const uint64_t same = __ballot(act && bin == b0);
  if (lane == leader) atomicAdd(&h[b0], (uint32_t)__popcll(same));
  else if (act && bin != b0) atomicAdd(&h[bin], 1u);
}

// the distance of row r (MODE as load_item; r < n)
template <int MODE>
__device__ __forceinline__ float fused_dist(const TopkSrc& s, int q, int64_t n, int64_t r,
                                            const uint64_t* qb, float qn) {
  float d;
  int id;
  load_item<MODE>(s, q, n, r, qb, qn, d, id);
  return d;
}

template <int MODE>
__global__ __launch_bounds__(kFuseThreads) void topk_fused_kernel(
    const TopkSrc s, int64_t n, int k, uint32_t* __restrict__ h1, uint32_t* __restrict__ h2,
    uint32_t* __restrict__ sync, float* __restrict__ cand_d, int32_t* __restrict__ cand_i,
    int cap, float* __restrict__ out_d, int32_t* __restrict__ out_i, volatile uint32_t* done,
    uint32_t seq) {
  __shared__ uint32_t h[kRadixBins];
  __shared__ float s_cache[kFuseCache];                // pass A distances; later the final's lists
  __shared__ uint64_t s_q[kTopMaxWords];
  __shared__ uint32_t sel[4];
  __shared__ int s_last;
  float* s_d = s_cache;                                // final stage: kRankMax candidates
  int32_t* s_i = reinterpret_cast<int32_t*>(s_cache + kRankMax);
  const int q = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63;
  const uint32_t B = gridDim.x;
  float qn = 0.f;
  if (MODE == 0) {
    for (int w = t; w < s.words; w += kFuseThreads) s_q[w] = s.qbits[(int64_t)q * s.words + w];
    qn = s.qnorm[q];
  }
  __syncthreads();
  uint64_t qb[kTopMaxWords];
#pragma unroll
  for (int w = 0; w < kTopMaxWords; ++w) qb[w] = (MODE == 0 && w < s.words) ? s_q[w] : 0ull;
  uint32_t* g1 = h1 + (int64_t)q * kRadixBins;
  uint32_t* g2 = h2 + (int64_t)q * kRadixBins;
  uint32_t* qs = sync + (int64_t)q * kFuseSync;
  const int64_t per = ((n + B - 1) / B + 1023) & ~(int64_t)1023;
  const int64_t beg = min(n, (int64_t)blockIdx.x * per);
  const int64_t end = min(n, beg + per);
  const int64_t cend = min(end, beg + kFuseCache);    // rows [beg, cend) cached in LDS
  // A: distances (4 rows in flight per thread), level-1 histogram
  for (int i = t; i < kRadixBins; i += kFuseThreads) h[i] = 0;
  __syncthreads();
  for (int64_t b = beg + t; b < end; b += 4 * kFuseThreads) {
    float d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t r = b + u * kFuseThreads;
      d[u] = fused_dist<MODE>(s, q, n, r < end ? r : end - 1, qb, qn);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t r = b + u * kFuseThreads;
      if (r < cend) s_cache[r - beg] = d[u];
      fused_bin(h, r < end && d[u] < INFINITY, dist_key(d[u]) >> 20, lane);
    }
  }
  __syncthreads();
  for (int i = t; i < kRadixBins; i += kFuseThreads)
    if (h[i]) atomicAdd(&g1[i], h[i]);
  fused_barrier(qs, B);
  // the distance of row r in passes B and C: LDS for the cached rows
  auto dist_of = [&](int64_t r) -> float {
    return r < cend ? s_cache[r - beg] : fused_dist<MODE>(s, q, n, r, qb, qn);
  };
  // B
  fused_select(g1, (uint32_t)k, h, sel);               // h doubles as the scan buffer
  const uint32_t b1 = sel[0];
  const uint32_t below = sel[1];
  float T = INFINITY;                                 // fewer finite rows than k: take them all
  if (b1 != 0xffffffffu) {
    for (int i = t; i < kRadixBins; i += kFuseThreads) h[i] = 0;
    __syncthreads();
    for (int64_t r = beg + t; r < end; r += kFuseThreads) {
      const float d = dist_of(r);
      const uint32_t key = dist_key(d);
      fused_bin(h, d < INFINITY && (key >> 20) == b1, (key >> 8) & 0xfff, lane);
    }
    __syncthreads();
    for (int i = t; i < kRadixBins; i += kFuseThreads)
      if (h[i]) atomicAdd(&g2[i], h[i]);
    fused_barrier(qs, 2 * B);
    fused_select(g2, (uint32_t)k - below, h, sel);
    T = key_dist((b1 << 20) | (sel[0] << 8) | 0xffu);
  }
  // C: candidates <= T
  for (int64_t r0 = beg; r0 < end; r0 += kFuseThreads) {
    const int64_t r = r0 + t;
    const float d = r < end ? dist_of(r) : INFINITY;
    const bool pass = d <= T && d < INFINITY;
    const uint64_t m = __ballot(pass);
    if (m == 0) continue;
    int base = 0;
    if (lane == 0) base = atomicAdd((int*)&qs[1], __popcll(m));
    base = __shfl(base, 0, 64);
    if (pass) {
      const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
      if (pos < cap) {
        cand_d[(int64_t)q * cap + pos] = d;
        cand_i[(int64_t)q * cap + pos] = (int32_t)r;
      }
    }
  }
  __syncthreads();
  if (t == 0) {
    __threadfence();
    s_last = atomicAdd(&qs[2], 1u) == B - 1;
    __threadfence();
  }
  __syncthreads();
  if (!s_last) return;
  // the last block of the query: exact top-k of the candidates
  // k <= kListK reads the candidates from L2 (any count up to cap: heavy
  // ties at the threshold, e.g. quantized hamming distances); larger k
  // ranks them in LDS (at most kRankMax)
  const int c_all = (int)ld_agent_u32(&qs[1]);
  const bool over = c_all > cap || (k > kListK && c_all > kRankMax);
  const int nc = over ? 0 : c_all;
  float* od = out_d + (int64_t)q * k;
  int32_t* oi = out_i + (int64_t)q * k;
  const float* gcd = cand_d + (int64_t)q * cap;
  const int32_t* gci = cand_i + (int64_t)q * cap;
  if (k > kListK) {
    for (int j = t; j < nc; j += kFuseThreads) {
      s_d[j] = __hip_atomic_load(gcd + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_i[j] = __hip_atomic_load(gci + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  for (int j = nc + t; j < k; j += kFuseThreads) { od[j] = INFINITY; oi[j] = INT_MAX; }
  __syncthreads();
  if (k <= kListK) {
    // per-thread sorted lists of the strided candidates, per-wave pops into
    // LDS, wave 0 pops the 4 waves' lists
    constexpr int NW = kFuseThreads / 64;
    float ld[kListK];
    int li[kListK];
#pragma unroll
    for (int j = 0; j < kListK; ++j) { ld[j] = INFINITY; li[j] = INT_MAX; }
    for (int j = t; j < nc; j += kFuseThreads) {
      const float v = __hip_atomic_load(gcd + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int id = __hip_atomic_load(gci + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lt_pair(v, id, ld[kListK - 1], li[kListK - 1])) {
#pragma unroll
        for (int x = kListK - 1; x > 0; --x) {
          const bool up = lt_pair(v, id, ld[x - 1], li[x - 1]);
          const bool here = !up && lt_pair(v, id, ld[x], li[x]);
          ld[x] = up ? ld[x - 1] : (here ? v : ld[x]);
          li[x] = up ? li[x - 1] : (here ? id : li[x]);
        }
        if (lt_pair(v, id, ld[0], li[0])) { ld[0] = v; li[0] = id; }
      }
    }
    const int wv = t >> 6;
    wave_pop<kListK>(ld, li, k, &s_d[wv * k], &s_i[wv * k], lane);
    __syncthreads();
    if (wv == 0) {
      float m[1];
      int mi[1];
      m[0] = lane < NW * k ? s_d[lane] : INFINITY;
      mi[0] = lane < NW * k ? s_i[lane] : INT_MAX;
      __builtin_amdgcn_wave_barrier();
      wave_pop<1>(m, mi, k, od, oi, lane);
    }
  } else {
    for (int j = t; j < nc; j += kFuseThreads) {
      const float d = s_d[j];
      const int32_t id = s_i[j];
      int rank = 0;
      for (int x = 0; x < nc; ++x) {
        const float e = s_d[x];
        rank += (e < d) || (e == d && s_i[x] < id);
        if ((x & 63) == 63 && rank >= k) break;
      }
      if (rank < k) { od[rank] = d; oi[rank] = id; }
    }
  }
  // state for the next launch
  for (int i = t; i < kRadixBins; i += kFuseThreads) { g1[i] = 0u; g2[i] = 0u; }
  if (t < kFuseSync) qs[t] = 0u;
  __threadfence_system();
  __syncthreads();
  const bool retry = over || (c_all < k && T < INFINITY);
  if (t == 0) done[q] = retry ? (seq | kTopRetry) : seq;
}

// ---------------------------------------------------------------------------
// One pass, one launch, no grid barrier (k <= kListK): B blocks of 256
// threads each stream a contiguous range of rows, 8 rows per thread in flight
// (every load of a round issued before the first use). A thread keeps its
// sorted top-KL (distance, row) pairs in registers and inserts only below its
// current KL-th, so after the first rounds a row costs a compare. The block
// pops its k best (wave pops, then wave 0) into global candidates (write-
// through stores, no fence) and counts itself finished; the last block of
// the query merges the B x k
// candidates the same way, writes the k results into pinned host memory,
// resets the counter and publishes done[q]. Every block's range is read once
// from HBM; the only serialization is the one counter per block.
constexpr int kOnepassRows = 8;

template <int MODE>
__global__ __launch_bounds__(256) void topk_onepass_kernel(const TopkSrc s, int64_t n, int64_t per_block,
                                                           int k, float* __restrict__ cand_d,
                                                           int32_t* __restrict__ cand_i, int cap,
                                                           uint32_t* __restrict__ counter,
                                                           float* __restrict__ out_d,
                                                           int32_t* __restrict__ out_i,
                                                           volatile uint32_t* done, uint32_t seq,
                                                           long long* __restrict__ prof) {
  constexpr int NW = 4, T = NW * 64, KL = kListK, R = kOnepassRows;
  // diagnostics (prof != nullptr): realtime stamps (100 MHz) per block:
  // start, rows done, block pop done, published; the last block adds merge
  // loads done, final pop done, end
  auto stamp = [&](int i) {
    if (prof != nullptr && threadIdx.x == 0)
      prof[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + i] = (long long)__builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  __shared__ float s_wd[NW * KL];
  __shared__ int s_wi[NW * KL];
  __shared__ float s_cd[KL];
  __shared__ int s_ci[KL];
  __shared__ uint64_t s_q[kTopMaxWords];
  __shared__ int s_last;
  const int q = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float qn = 0.f;
  if (MODE == 0) {
    for (int w = t; w < s.words; w += T) s_q[w] = s.qbits[(int64_t)q * s.words + w];
    qn = s.qnorm[q];
  }
  __syncthreads();
  uint64_t qb[kTopMaxWords];
#pragma unroll
  for (int w = 0; w < kTopMaxWords; ++w) qb[w] = (MODE == 0 && w < s.words) ? s_q[w] : 0ull;
  float ld[KL];
  int li[KL];
#pragma unroll
  for (int j = 0; j < KL; ++j) { ld[j] = INFINITY; li[j] = INT_MAX; }
  auto insert = [&](float v, int id) {
    if (lt_pair(v, id, ld[KL - 1], li[KL - 1])) {
#pragma unroll
      for (int j = KL - 1; j > 0; --j) {
        const bool up = lt_pair(v, id, ld[j - 1], li[j - 1]);
        const bool here = !up && lt_pair(v, id, ld[j], li[j]);
        ld[j] = up ? ld[j - 1] : (here ? v : ld[j]);
        li[j] = up ? li[j - 1] : (here ? id : li[j]);
      }
      if (lt_pair(v, id, ld[0], li[0])) { ld[0] = v; li[0] = id; }
    }
  };
  const int64_t b0 = (int64_t)blockIdx.x * per_block;
  const int64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  for (int64_t base = b0; base < b1; base += (int64_t)T * R) {
    float d[R];
    int ix[R];
    {
      int64_t rows[R], nn[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        rows[r] = base + (int64_t)r * T + t;
        nn[r] = rows[r] < b1 ? n : 0;
      }
      load_rows<MODE, R>(s, q, nn, rows, qb, qn, d, ix);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) insert(d[r], ix[r]);
  }
  stamp(1);
  // the block's k best (wave pops, then wave 0) -> s_cd / s_ci
  auto block_pop = [&]() {
    wave_pop<KL>(ld, li, k, &s_wd[wv * k], &s_wi[wv * k], lane);
    __syncthreads();
    if (wv == 0) {
      constexpr int M = (NW * KL + 63) / 64;
      float m[M];
      int mi[M];
#pragma unroll
      for (int j = 0; j < M; ++j) {
        const int c = lane + 64 * j;
        m[j] = c < NW * k ? s_wd[c] : INFINITY;
        mi[j] = c < NW * k ? s_wi[c] : INT_MAX;
      }
      __builtin_amdgcn_wave_barrier();
      sort_regs<M>(m, mi);
      wave_pop<M>(m, mi, k, s_cd, s_ci, lane);
    }
    __syncthreads();
  };
  block_pop();
  stamp(2);
  // publish the candidates [q][block][k] cross-XCD without a fence
  // (MI355X_MICROARCH.md, visibility): write-through (sc1) stores, every
  // storing wave drains them, a barrier, then ONE agent-scope add whose
  // returned value tells the last block; that block reads them with sc1 loads
  float* cd = cand_d + (int64_t)q * cap;
  int32_t* ci = cand_i + (int64_t)q * cap;
  if (t < k) {
    __hip_atomic_store(cd + (int64_t)blockIdx.x * k + t, s_cd[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ci + (int64_t)blockIdx.x * k + t, s_ci[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* qc = counter + (int64_t)q * kFuseSync;     // the query's counter word
  if (t == 0)
    s_last = __hip_atomic_fetch_add(qc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  stamp(3);
  if (!s_last) return;
  // the last block: merge the B x k candidates, 8 pairs in flight per
  // thread (a load -> insert loop would wait one L2 round trip per pair)
#pragma unroll
  for (int j = 0; j < KL; ++j) { ld[j] = INFINITY; li[j] = INT_MAX; }
  const int nc = (int)gridDim.x * k;
  for (int j0 = t; j0 < nc; j0 += 8 * T) {
    float v[8];
    int vi[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = j0 + u * T < nc ? j0 + u * T : nc - 1;
      v[u] = __hip_atomic_load(cd + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      vi[u] = __hip_atomic_load(ci + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (j0 + u * T < nc) insert(v[u], vi[u]);
  }
  stamp(4);
  block_pop();
  stamp(5);
  float* od = out_d + (int64_t)q * k;
  int32_t* oi = out_i + (int64_t)q * k;
  if (t < k) { od[t] = s_cd[t]; oi[t] = s_ci[t]; }
  if (t == 0) __hip_atomic_store(qc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
  __threadfence_system();
  __syncthreads();
  if (t == 0) done[q] = seq;
  stamp(6);
}

// ---------------------------------------------------------------------------
// Tables up to ~1M rows, k up to kTopMaxK, one launch without a grid barrier
// (the one-launch kernel above waits twice for every block): B blocks per
// query stream contiguous ranges in chunks of kSelChunk rows. The rows of a
// chunk that beat the block's running k-th (all of them until it has k) are
// appended to LDS after the running top-k, in row order, and an exact select
// keeps the k smallest (distance key, row) pairs: a radix select over the
// key's 8-bit digits, stopping at the first digit whose bin holds exactly the
// pairs still needed; pairs tied on the whole key go by row (the LDS order),
// so the result stays in row order for the next chunk. The block publishes its
// k (write-through stores, one counter add); the last block of the query
// selects the k of the B x k the same way (candidates in block order are in
// row order), ranks them and writes the results to pinned host memory. A
// block short of k rows pads with keys above +inf.
constexpr int kSelThreads = 256;
constexpr int kSelChunk = 4096;                       // rows per chunk (16 per thread)
constexpr int kSelRounds = kSelChunk / kSelThreads;   // 16
constexpr int kSelCap = kSelChunk + kTopMaxK;         // LDS pairs; the last block: B x k <= kSelChunk
constexpr uint32_t kSelPadKey = 0xffffffffu;          // above dist_key(+inf)

struct SelLds {
  uint32_t key[kSelCap];
  uint32_t id[kSelCap];
  uint32_t tk[kTopMaxK], ti[kTopMaxK];                // the selected pairs
  uint32_t hist[256];
  uint32_t cnt[kSelRounds * 4];                       // survivors per (round, wave), then offsets
  uint32_t wsum[4];
  uint64_t wmax[4];
  uint32_t st[4];                                     // digit, count before it, count in it
};

__device__ __forceinline__ uint64_t sel_comp(uint32_t key, uint32_t id) { return ((uint64_t)key << 32) | id; }

__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t x = __shfl_up(v, o, 64);
    if (lane >= o) v += x;
  }
  return v;
}

// exclusive block scan of v over the 256 threads
__device__ __forceinline__ uint32_t block_excl_scan(SelLds& L, uint32_t v) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const uint32_t incl = wave_incl_scan_u32(v, lane);
  if (lane == 63) L.wsum[w] = incl;
  __syncthreads();
  uint32_t off = 0;
  for (int j = 0; j < w; ++j) off += L.wsum[j];
  __syncthreads();
  return off + incl - v;
}

// the k smallest (key, id) of L[0, n) (n > k, ids increasing with the index
// among equal keys) -> L[0, k) in index order; returns the largest of them
// (want_max; else 0)
__device__ uint64_t block_select(SelLds& L, int n, int k, bool want_max) {
  const int t = threadIdx.x, lane = t & 63;
  uint32_t prefix = 0;
  int need = k, shift = 24;
  for (;; shift -= 8) {
    L.hist[t] = 0;
    __syncthreads();
    const uint32_t hi = shift == 24 ? 0u : prefix >> (shift + 8);
    for (int i = t; i < n; i += kSelThreads) {
      const uint32_t c = L.key[i];
      if (shift == 24 || (c >> (shift + 8)) == hi) atomicAdd(&L.hist[(c >> shift) & 255], 1u);
    }
    __syncthreads();
    if (t < 64) {
      const uint32_t h0 = L.hist[4 * lane], h1 = L.hist[4 * lane + 1];
      const uint32_t h2 = L.hist[4 * lane + 2], h3 = L.hist[4 * lane + 3];
      const uint32_t sum = h0 + h1 + h2 + h3;
      uint32_t run = wave_incl_scan_u32(sum, lane) - sum;
      const uint32_t hv[4] = {h0, h1, h2, h3};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (run < (uint32_t)need && run + hv[j] >= (uint32_t)need) {
          L.st[0] = 4 * lane + j;
          L.st[1] = run;
          L.st[2] = hv[j];
        }
        run += hv[j];
      }
    }
    __syncthreads();
    const uint32_t digit = L.st[0], before = L.st[1], inbin = L.st[2];
    prefix |= digit << shift;
    need -= (int)before;
    if ((int)inbin == need || shift == 0) break;
    __syncthreads();                                  // st / hist reused by the next digit
  }
  // taken: key digits (down to `shift`) below the prefix, and the first
  // `need` of those equal to it in index order (all of them when the bin
  // held exactly `need`). Thread t owns a contiguous index range.
  const uint32_t lim = prefix >> shift;
  const int per = (n + kSelThreads - 1) / kSelThreads;
  const int i0 = t * per, i1 = min(n, i0 + per);
  uint32_t cs = 0, ct = 0;
  for (int i = i0; i < i1; ++i) {
    const uint32_t d = L.key[i] >> shift;
    cs += d < lim;
    ct += d == lim;
  }
  const uint32_t ex = block_excl_scan(L, cs | (ct << 16));
  uint32_t sb = ex & 0xffffu, tb = ex >> 16;
  uint64_t mx = 0;
  for (int i = i0; i < i1; ++i) {
    const uint32_t key = L.key[i], d = key >> shift;
    int pos = -1;
    if (d < lim) {
      pos = (int)(sb + min(tb, (uint32_t)need));
      ++sb;
    } else if (d == lim) {
      if (tb < (uint32_t)need) pos = (int)(sb + tb);
      ++tb;
    }
    if (pos >= 0) {
      L.tk[pos] = key;
      L.ti[pos] = L.id[i];
      mx = max(mx, sel_comp(key, L.id[i]));
    }
  }
  if (want_max) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t x = ((uint64_t)(uint32_t)__shfl_xor((int)(mx >> 32), o, 64) << 32) |
                         (uint32_t)__shfl_xor((int)(uint32_t)mx, o, 64);
      mx = max(mx, x);
    }
    if (lane == 0) L.wmax[t >> 6] = mx;
  }
  __syncthreads();
  for (int i = t; i < k; i += kSelThreads) { L.key[i] = L.tk[i]; L.id[i] = L.ti[i]; }
  const uint64_t m = want_max ? max(max(L.wmax[0], L.wmax[1]), max(L.wmax[2], L.wmax[3])) : 0ull;
  __syncthreads();
  return m;
}

template <int MODE>
__global__ __launch_bounds__(kSelThreads) void topk_select_kernel(
    const TopkSrc s, int64_t n, int64_t per_block, int k, float* __restrict__ cand_d,
    int32_t* __restrict__ cand_i, int cap, uint32_t* __restrict__ counter, float* __restrict__ out_d,
    int32_t* __restrict__ out_i, volatile uint32_t* done, uint32_t seq) {
  __shared__ SelLds L;
  __shared__ uint64_t s_q[kTopMaxWords];
  __shared__ int s_last;
  const int q = blockIdx.y;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  float qn = 0.f;
  if (MODE == 0) {
    for (int w = t; w < s.words; w += kSelThreads) s_q[w] = s.qbits[(int64_t)q * s.words + w];
    qn = s.qnorm[q];
  }
  __syncthreads();
  uint64_t qb[kTopMaxWords];
#pragma unroll
  for (int w = 0; w < kTopMaxWords; ++w) qb[w] = (MODE == 0 && w < s.words) ? s_q[w] : 0ull;
  const int64_t b0 = (int64_t)blockIdx.x * per_block;
  const int64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  int have = 0;                                       // the running top-k: L[0, have), row order
  uint64_t tau = ~0ull;                               // its largest pair once have == k
  for (int64_t base = b0; base < b1; base += kSelChunk) {
    const int rows = (int)(b1 - base < kSelChunk ? b1 - base : kSelChunk);
    int m;
    if (tau == ~0ull) {
      // every row goes in (the running set is not full yet): at its own index
#pragma unroll
      for (int h = 0; h < kSelRounds / 8; ++h) {
        constexpr int R = 8;
        int64_t rr[R], nn[R];
        float d[R];
        int ix[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const int j = (h * R + u) * kSelThreads + t;
          rr[u] = base + j;
          nn[u] = j < rows ? n : 0;
        }
        load_rows<MODE, R>(s, q, nn, rr, qb, qn, d, ix);
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const int j = (h * R + u) * kSelThreads + t;
          if (j < rows) { L.key[have + j] = dist_key(d[u]); L.id[have + j] = (uint32_t)(base + j); }
        }
      }
      m = have + rows;
      __syncthreads();
    } else {
      // only rows below the running k-th, appended in row order
      uint32_t key[kSelRounds];
      uint64_t bits = 0;                              // survivor flags per round
#pragma unroll
      for (int h = 0; h < kSelRounds / 8; ++h) {
        constexpr int R = 8;
        int64_t rr[R], nn[R];
        float d[R];
        int ix[R];
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const int j = (h * R + u) * kSelThreads + t;
          rr[u] = base + j;
          nn[u] = j < rows ? n : 0;
        }
        load_rows<MODE, R>(s, q, nn, rr, qb, qn, d, ix);
#pragma unroll
        for (int u = 0; u < R; ++u) {
          const int r = h * R + u;
          const int j = r * kSelThreads + t;
          key[r] = dist_key(d[u]);
          const bool sv = j < rows && sel_comp(key[r], (uint32_t)(base + j)) < tau;
          const uint64_t bm = __ballot(sv);
          if (lane == 0) L.cnt[r * 4 + wv] = (uint32_t)__popcll(bm);
          if (sv) bits |= 1ull << r;
        }
      }
      __syncthreads();
      if (t < 64) {                                   // offsets of (round, wave) in row order
        const uint32_t c = L.cnt[lane];
        const uint32_t inc = wave_incl_scan_u32(c, lane);
        L.cnt[lane] = inc - c;
        if (lane == 63) L.st[3] = inc;                // the chunk's survivors
      }
      __syncthreads();
      m = have + (int)L.st[3];
#pragma unroll
      for (int r = 0; r < kSelRounds; ++r) {
        const bool sv = (bits >> r) & 1ull;
        const uint64_t bm = __ballot(sv);
        if (sv) {
          const int pos = have + (int)L.cnt[r * 4 + wv] + __popcll(bm & ((1ull << lane) - 1ull));
          L.key[pos] = key[r];
          L.id[pos] = (uint32_t)(base + r * kSelThreads + t);
        }
      }
      __syncthreads();
    }
    if (m > k) {
      tau = block_select(L, m, k, base + kSelChunk < b1);
      have = k;
    } else {
      have = m;
    }
  }
  __syncthreads();
  // publish the block's k (pads above +inf with distinct ids when short)
  float* cd = cand_d + (int64_t)q * cap;
  int32_t* ci = cand_i + (int64_t)q * cap;
  for (int j = t; j < k; j += kSelThreads) {
    const uint32_t key = j < have ? L.key[j] : kSelPadKey;
    const uint32_t id = j < have ? L.id[j] : (0x80000000u | (uint32_t)(blockIdx.x * kTopMaxK + j));
    __hip_atomic_store(reinterpret_cast<uint32_t*>(cd) + (int64_t)blockIdx.x * k + j, key, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(reinterpret_cast<uint32_t*>(ci) + (int64_t)blockIdx.x * k + j, id, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t* qc = counter + (int64_t)q * kFuseSync;
  // The hand-off is the guide's fence-free valid form (MI355X_MICROARCH.md,
  // inter-workgroup visibility, Consumer bullet conditions 1-4): every byte
  // is stored sc1 (agent atomic store) and read back sc1 (agent atomic load),
  // every storing wave drains (vmcnt(0)) before the barrier, one lane adds
  // behind it. No agent release / acquire fence is needed for sc1 traffic; a
  // fence per block is an L2 write-back (~1.7-3.5 us, measured +25 us per call
  // on the round-3 merge), which this kernel exists to avoid.
  if (t == 0)
    s_last = __hip_atomic_fetch_add(qc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  // the last block: the k of the B x k candidates, ranked
  const int nc = (int)gridDim.x * k;
  for (int j = t; j < nc; j += kSelThreads) {
    L.key[j] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(cd) + j, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    L.id[j] = __hip_atomic_load(reinterpret_cast<const uint32_t*>(ci) + j, __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (nc > k) block_select(L, nc, k, false);
  float* od = out_d + (int64_t)q * k;
  int32_t* oi = out_i + (int64_t)q * k;
  for (int i = t; i < k; i += kSelThreads) {
    const uint64_t c = sel_comp(L.key[i], L.id[i]);
    int rank = 0;
    for (int j = 0; j < k; ++j) rank += sel_comp(L.key[j], L.id[j]) < c;
    const uint32_t key = L.key[i];
    const bool fin = key < dist_key(INFINITY);
    od[rank] = fin ? key_dist(key) : INFINITY;
    oi[rank] = fin ? (int32_t)L.id[i] : INT_MAX;
  }
  if (t == 0) __hip_atomic_store(qc, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
  __threadfence_system();
  __syncthreads();
  if (t == 0) done[q] = seq;
}

}  // namespace jb

// blocks of one fused launch that are resident at once (all queries): the
// grid barrier needs every block running; bounded by kFuseMaxBlocks
static int fused_resident_blocks() {
  static int cached = 0;
  if (cached == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, jb::topk_fused_kernel<1>,
                                                     jb::kFuseThreads, 0) != hipSuccess) {
      cus = 64;
      per_cu = 1;
    }
    int64_t r = (int64_t)cus * (per_cu > 0 ? per_cu : 1);
    cached = (int)(r < jb::kFuseMaxBlocks ? r : jb::kFuseMaxBlocks);
  }
  return cached;
}

template <int MODE>
static int topk_fused_launch(const jb::TopkSrc& s, int nq, int64_t nrows, int k,
                             float* scratch_d, int32_t* scratch_i, float* out_d_host,
                             int32_t* out_i_host, uint32_t* done_host, uint32_t seq,
                             hipStream_t stream) {
  uint32_t* st = (uint32_t*)(scratch_i + kFuseStateOff);
  static const int64_t rows_per_block = [] {
    const char* e = getenv("JB_FUSE_ROWS");                // diagnostics: rows per block
    const long v = e != nullptr ? atol(e) : 0;
    return (int64_t)(v >= 256 ? v : 1024);
  }();
  int64_t B = (nrows + rows_per_block - 1) / rows_per_block;
  const int64_t bmax = fused_resident_blocks() / nq;
  if (B > bmax) B = bmax;
  if (B < 1) B = 1;
  hipLaunchKernelGGL(jb::topk_fused_kernel<MODE>, dim3((unsigned)B, nq), dim3(jb::kFuseThreads), 0,
                     stream, s, nrows, k, st, st + 8 * kRadixBins, st + 16 * kRadixBins,
                     scratch_d + 64, scratch_i + 64, kCandCap, out_d_host, out_i_host,
                     (volatile uint32_t*)done_host, seq);
  return (int)hipGetLastError();
}

// diagnostics: phase stamps of the one-pass kernel (tools/bench_topk_phases.py)
static long long* g_topk_prof = nullptr;
extern "C" void jb_topk_set_prof(long long* prof) { g_topk_prof = prof; }

// one-pass launch (k <= kListK): blocks of 2048 rows (one round of 8 rows a
// thread) up to 512 blocks; the counter is word 3 of the query's sync words
// in the zeroed state region (the fused kernel leaves it zero too)
template <int MODE>
static int topk_onepass_launch(const jb::TopkSrc& s, int nq, int64_t nrows, int k, float* scratch_d,
                               int32_t* scratch_i, float* out_d_host, int32_t* out_i_host,
                               uint32_t* done_host, uint32_t seq, hipStream_t stream) {
  if (k > jb::kListK) return -2;
  uint32_t* counter = (uint32_t*)(scratch_i + kFuseStateOff) + 16 * kRadixBins + 3;
  constexpr int64_t rows_per_round = 256 * jb::kOnepassRows;
  int64_t B = (nrows + rows_per_round - 1) / rows_per_round;
  if (B > 512) B = 512;
  const int64_t rounds = (nrows + B * rows_per_round - 1) / (B * rows_per_round);
  const int64_t per_block = rounds * rows_per_round;
  B = (nrows + per_block - 1) / per_block;
  hipLaunchKernelGGL(jb::topk_onepass_kernel<MODE>, dim3((unsigned)B, nq), dim3(256), 0, stream, s, nrows,
                     per_block, k, scratch_d + 64, scratch_i + 64, kCandCap, counter, out_d_host,
                     out_i_host, (volatile uint32_t*)done_host, seq, g_topk_prof);
  return (int)hipGetLastError();
}

// one-launch select path (k <= kTopMaxK): ~2048 rows a block, B x k
// candidates at most kSelChunk (the last block's LDS); counter as the one-pass
// launch's (each leaves it zero)
template <int MODE>
static int topk_select_launch(const jb::TopkSrc& s, int nq, int64_t nrows, int k, float* scratch_d,
                              int32_t* scratch_i, float* out_d_host, int32_t* out_i_host,
                              uint32_t* done_host, uint32_t seq, hipStream_t stream) {
  if (k > jb::kTopMaxK || nq > 8) return -2;
  uint32_t* counter = (uint32_t*)(scratch_i + kFuseStateOff) + 16 * kRadixBins + 3;
  int64_t B = (nrows + 2047) / 2048;
  const int64_t bmax = jb::kSelChunk / k;
  if (B > bmax) B = bmax;
  if (B > 256) B = 256;
  if (B < 1) B = 1;
  const int64_t per_block = (nrows + B - 1) / B;
  B = (nrows + per_block - 1) / per_block;
  hipLaunchKernelGGL(jb::topk_select_kernel<MODE>, dim3((unsigned)B, nq), dim3(jb::kSelThreads), 0, stream, s,
                     nrows, per_block, k, scratch_d + 64, scratch_i + 64, kCandCap, counter, out_d_host,
                     out_i_host, (volatile uint32_t*)done_host, seq);
  return (int)hipGetLastError();
}

// path: 0 tile scan + merge, 1 radix chain (6 launches + memset), 2 one launch
// (grid barriers), 3 one pass (k <= kListK), 4 one launch, LDS select
static int topk_scores_launch(const jb::TopkSrc& s, int nq, int64_t nrows, int k, int path,
                              float* scratch_d, int32_t* scratch_i, float* out_d_host,
                              int32_t* out_i_host, uint32_t* done_host, uint32_t seq,
                              hipStream_t stream) {
  if (path == 2)
    return topk_fused_launch<1>(s, nq, nrows, k, scratch_d, scratch_i, out_d_host, out_i_host,
                                done_host, seq, stream);
  if (path == 3)
    return topk_onepass_launch<1>(s, nq, nrows, k, scratch_d, scratch_i, out_d_host, out_i_host,
                                  done_host, seq, stream);
  if (path == 4)
    return topk_select_launch<1>(s, nq, nrows, k, scratch_d, scratch_i, out_d_host, out_i_host,
                                 done_host, seq, stream);
  if (path == 0) {
    const int blocks = topk_tile_blocks(nrows, k);
    const int64_t tiles = (nrows + jb::kTopTile - 1) / jb::kTopTile;
    const int64_t per_block = ((tiles + blocks - 1) / blocks) * jb::kTopTile;
    const int used = jb::launch_scan<1>(s, blocks, nq, nrows, per_block, k, scratch_d, scratch_i, stream,
                                        jb_topk_blocks(nrows, k));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
    const int64_t nc = (int64_t)used * k;
    jb::TopkSrc m{nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, scratch_d, scratch_i, 0};
    jb::launch_merge(m, nq, nc, k, out_d_host, out_i_host, (volatile uint32_t*)done_host, seq,
                     stream);
    return (int)hipGetLastError();
  }
  float* thr = scratch_d;                          // [8]
  int* count = scratch_i;                          // [8]
  uint32_t* sel = (uint32_t*)scratch_i + 16;       // [2 x 8]
  float* cand_d = scratch_d + 64;
  int32_t* cand_i = scratch_i + 64;
  uint32_t* h1 = (uint32_t*)(scratch_i + 64 + (int64_t)nq * kCandCap);
  uint32_t* h2 = h1 + (int64_t)nq * kRadixBins;
  hipError_t e = hipMemsetAsync(h1, 0, sizeof(uint32_t) * 2 * (size_t)nq * kRadixBins, stream);
  if (e != hipSuccess) return (int)e;
  // blocks of the histogram passes: every block adds its bins to the global
  // histogram with atomics, and on a score vector most rows share a bin, so
  // the block count bounds the atomics serialized on that address
  constexpr int64_t hb_max = 512;
  int64_t hb = (nrows + 1023) / 1024;
  if (hb > hb_max) hb = hb_max;
  const float* src = s.src_d;
  hipLaunchKernelGGL(jb::radix_hist_kernel<1>, dim3((unsigned)hb, nq), dim3(256), 0, stream, src,
                     s.flip, nrows, sel, h1);
  hipLaunchKernelGGL(jb::radix_select_kernel<1>, dim3(nq), dim3(1024), 0, stream, h1, k, sel, thr,
                     count);
  hipLaunchKernelGGL(jb::radix_hist_kernel<2>, dim3((unsigned)hb, nq), dim3(256), 0, stream, src,
                     s.flip, nrows, sel, h2);
  hipLaunchKernelGGL(jb::radix_select_kernel<2>, dim3(nq), dim3(1024), 0, stream, h2, k, sel, thr,
                     count);
  int64_t cblocks = (nrows + 1023) / 1024;
  if (cblocks > 1024) cblocks = 1024;
  hipLaunchKernelGGL(jb::topk_collect_kernel<1>, dim3((unsigned)cblocks, nq), dim3(256), 0, stream,
                     s, nrows, thr, kCandCap, cand_d, cand_i, count);
  hipLaunchKernelGGL(jb::topk_rank_final_kernel, dim3(nq), dim3(1024), 0, stream, cand_d, cand_i,
                     count, kCandCap, k, thr, out_d_host, out_i_host,
                     (volatile uint32_t*)done_host, seq);
  return (int)hipGetLastError();
}

// path_sel: -1 default (the radix chain from 16384 rows), 0 tile, 1 radix
// chain, 2 one launch (A/B in tools/bench_topk_scores.py: at 1M rows the
// chain measured 48-61 us, the one launch 80-86 us, and 6x slower on heavy
// ties at k = 100; profiles/r03_topk_paths_ab.jsonl)
extern "C" int jb_topk_scores_direct_path(const float* src_d, int flip, int nq, int64_t nrows,
                                          int k, float* scratch_d, int32_t* scratch_i,
                                          float* out_d_host, int32_t* out_i_host,
                                          uint32_t* done_host, int path_sel, hipStream_t stream) {
  if (nq <= 0 || nrows <= 0 || k <= 0) return 0;
  if (k > jb::kTopMaxK || nq > 8) return -2;
  jb::TopkSrc s{nullptr, nullptr, nullptr, nullptr, nullptr, 0, 0, 0, src_d, nullptr, flip};
  // default: one query on the LDS select (tools/bench_topk_scores.py, 1M rows:
  // k 10 44-56 us vs 47-101 on the radix chain, which degrades on quantized
  // scores - k 100 with 64 score levels: 105 vs 631 us); several queries on
  // the chain (4 x k 10: 55-66 vs 71-78 us without ties)
  const int path = nrows >= 16384 ? (path_sel < 0 ? (nq == 1 ? 4 : 1) : path_sel) : 0;
  uint32_t seq = jb::next_seq();
  int rc = topk_scores_launch(s, nq, nrows, k, path, scratch_d, scratch_i, out_d_host,
                              out_i_host, done_host, seq, stream);
  if (rc != 0) return rc;
  bool retry = false;
  rc = jb::wait_flags_status(done_host, nq, seq, jb::kTopRetry, stream, &retry);
  if (rc != 0 || !retry) return rc;
  seq = jb::next_seq();
  rc = topk_scores_launch(s, nq, nrows, k, 0, scratch_d, scratch_i, out_d_host, out_i_host,
                          done_host, seq, stream);
  if (rc != 0) return rc;
  return jb::wait_flags(done_host, nq, seq, stream);
}

extern "C" int jb_topk_scores_direct(const float* src_d, int flip, int nq, int64_t nrows, int k,
                                     float* scratch_d, int32_t* scratch_i, float* out_d_host,
                                     int32_t* out_i_host, uint32_t* done_host,
                                     hipStream_t stream) {
  return jb_topk_scores_direct_path(src_d, flip, nq, nrows, k, scratch_d, scratch_i, out_d_host,
                                    out_i_host, done_host, -1, stream);
}

// the scan counters since the last call (JB_TOPK_MQ_STATS=1; synchronizes the device)
extern "C" int jb_topk_mq_stats(unsigned long long* out4) {
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpyFromSymbol(out4, HIP_SYMBOL(jb::g_mq_stats), 4 * sizeof(unsigned long long));
  unsigned long long z[4] = {0, 0, 0, 0};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(jb::g_mq_stats), z, sizeof(z));
  return (int)e;
}
