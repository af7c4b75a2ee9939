// Squared euclidean distances points x centers on the matrix cores.
//
// Reference: the clustering engine's push / get_nearest_* paths
// (jubatus/server/server/clustering_serv.cpp:108-137) over jubatus_core's
// k-means / GMM on compressive coresets (EXTERNAL).
//
// D[i][j] = |x_i|^2 + |c_j|^2 - 2 x_i . c_j, with the Gram term X C^T on
// v_mfma_f32_16x16x4_f32 (fp32 in / fp32 accumulate: exact f32 products, the
// same numerics as an f32 fmaf chain). One wave computes a 16 x 16 tile
// (16 points x 16 centres) stepping K by 4; a 256-thread workgroup covers 64
// points. Fragment maps (gfx950, 16x16x4 f32):
//   A: lane l holds A[l & 15][k = l >> 4]     (X rows)
//   B: lane l holds B[k = l >> 4][l & 15]     (C^T, i.e. C[l & 15][k])
//   D: lane l, reg r -> row (l >> 4) * 4 + r, col l & 15
#include <stdlib.h>

#include "jb_device.hpp"

namespace jb {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void sqdist_mfma_kernel(
    const float* __restrict__ X, int64_t n, const float* __restrict__ C, int k, int d,
    const float* __restrict__ xn2, const float* __restrict__ cn2, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t row0 = ((int64_t)blockIdx.x * 4 + wv) * 16;
  const int col0 = blockIdx.y * 16;
  if (row0 >= n) return;
  const int ar = lane & 15;   // A row / B col inside the tile
  const int kq = lane >> 4;   // k offset 0..3
  const int64_t xi = row0 + ar;
  const int cj = col0 + ar;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int kk = 0; kk < d; kk += 4) {
    const int kc = kk + kq;
    const float a = (xi < n && kc < d) ? X[xi * d + kc] : 0.f;
    const float b = (cj < k && kc < d) ? C[(int64_t)cj * d + kc] : 0.f;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  const int col = col0 + (lane & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t row = row0 + (lane >> 4) * 4 + r;
    if (row < n && col < k) out[row * k + col] = fmaxf(0.f, xn2[row] + cn2[col] - 2.f * acc[r]);
  }
}

// ---------------------------------------------------------------------------
// Coreset construction and Lloyd on one workgroup (bucket-sized problems:
// bucket_size 1000 x a few hundred dims). A bucket is far too small to fill
// the chip, and the host path's cost is not the arithmetic but the round
// trip per k-means++ draw / per Lloyd iteration; here every draw and every
// iteration stays on the device, one launch each, no host sync in between.

constexpr int kClBlock = 1024;

// squared distance of row i to row c of X (d dims)
__device__ __forceinline__ float cl_dist2(const float* __restrict__ X, int64_t i, int64_t c, int d) {
  const float* a = X + i * d;
  const float* b = X + c * d;
  float s = 0.f;
  for (int j = 0; j < d; ++j) {
    const float t = a[j] - b[j];
    s = fmaf(t, t, s);
  }
  return s;
}

// block-wide weighted draw with Python's random.choices semantics
// (bisect_right over the running sum of the weights at u * total): each
// thread owns a contiguous chunk of rows; chunk sums are scanned in double.
// Returns the index, or -1 when the weights sum to zero.
__device__ int cl_draw(const float* __restrict__ wt, int n, double u, double* part, int* pick) {
  const int t = threadIdx.x;
  const int per = (n + kClBlock - 1) / kClBlock;
  const int i0 = t * per, i1 = min(n, i0 + per);
  double s = 0.0;
  for (int i = i0; i < i1; ++i) s += (double)wt[i];
  // inclusive scan of the chunk sums: within each wave by shuffles, then the
  // wave totals (a Hillis-Steele pass over all 1024 took ~20 barriers a draw)
  const int lane = t & 63, wv = t >> 6;
  constexpr int NWV = kClBlock / 64;
  double incl = s;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double x = __shfl_up(incl, o, 64);
    if (lane >= o) incl += x;
  }
  if (lane == 63) part[kClBlock + wv] = incl;    // wave totals
  __syncthreads();
  if (t == 0) {
    double run = 0.0;
    for (int w = 0; w < NWV; ++w) {
      const double x = part[kClBlock + w];
      part[kClBlock + w] = run;                  // exclusive prefix of the wave
      run += x;
    }
    part[kClBlock + NWV] = run;
  }
  __syncthreads();
  incl += part[kClBlock + wv];
  part[t] = incl;
  const double total = part[kClBlock + NWV];
  if (t == 0) *pick = -1;
  __syncthreads();
  if (total > 0.0) {
    const double target = u * total;
    double run = part[t] - s;                      // before my chunk
    if (run <= target && target < part[t]) {
      int r = i1 - 1;
      for (int i = i0; i < i1; ++i) {
        run += (double)wt[i];
        if (run > target) { r = i; break; }
      }
      *pick = r;
    }
  }
  __syncthreads();
  int r = *pick;
  if (r < 0 && total > 0.0) r = n - 1;             // u * total rounded onto the end
  return r;
}

// k-means++ seeding: m draws (u: host-drawn uniforms, one per draw, as the
// host path consumes its RNG). out[j] = chosen row, or status = 1 when every
// remaining weight is zero (the host continues with its uniform fallback).
__global__ __launch_bounds__(kClBlock) void kmeanspp_kernel(const float* __restrict__ Xg, int n,
                                                            int d, const float* __restrict__ wg,
                                                            const double* __restrict__ u, int m,
                                                            float* __restrict__ d2g,
                                                            float* __restrict__ probg,
                                                            int32_t* __restrict__ out,
                                                            int32_t* __restrict__ status, int lds_mode) {
  __shared__ double part[kClBlock + kClBlock / 64 + 1];   // chunk prefixes, wave prefixes, total
  __shared__ int pick;
  const int t = threadIdx.x;
  // lds_mode 1: weights, d2 and draw weights in LDS (every draw reads and
  // writes them; through global memory each was an L2 round trip); 2: the
  // points too
  extern __shared__ float s_pp[];
  const float* w = wg;
  float* d2 = d2g;
  float* prob = probg;
  const float* X = Xg;
  if (lds_mode > 0) {
    float* sw = s_pp;
    d2 = sw + n;
    prob = d2 + n;
    for (int i = t; i < n; i += kClBlock) sw[i] = wg[i];
    w = sw;
    if (lds_mode > 1) {
      float* sx = prob + n;
      for (int i = t; i < n * d; i += kClBlock) sx[i] = Xg[i];
      X = sx;
    }
    __syncthreads();
  }
  int c = cl_draw(w, n, u[0], part, &pick);
  if (t == 0) { out[0] = c; *status = c < 0 ? 1 : 0; }
  if (c < 0) return;
  for (int i = t; i < n; i += kClBlock) d2[i] = cl_dist2(X, i, c, d);
  __syncthreads();
  for (int j = 1; j < m; ++j) {
    for (int i = t; i < n; i += kClBlock) prob[i] = d2[i] * w[i];
    __syncthreads();
    c = cl_draw(prob, n, u[j], part, &pick);
    if (c < 0) {
      if (t == 0) { out[j] = -1; *status = 1 + j; }
      return;
    }
    if (t == 0) out[j] = c;
    for (int i = t; i < n; i += kClBlock) d2[i] = fminf(d2[i], cl_dist2(X, i, c, d));
    __syncthreads();
  }
}

// inclusive prefix sum of a double over the wave, in registers: DPP row
// shifts within each row of 16 lanes, then the row broadcasts of lanes 15 /
// 31 into the later rows (gfx9 DPP; a __shfl_up per step is an LDS round trip)
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, ROWS, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, ROWS, 0xF, true);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_incl_scan_d(double x) {
  x += dpp_d<0x111, 0xF>(x);   // row_shr:1
  x += dpp_d<0x112, 0xF>(x);   // row_shr:2
  x += dpp_d<0x114, 0xF>(x);   // row_shr:4
  x += dpp_d<0x118, 0xF>(x);   // row_shr:8
  x += dpp_d<0x142, 0xA>(x);   // row_bcast:15 into rows 1, 3
  x += dpp_d<0x143, 0xC>(x);   // row_bcast:31 into rows 2, 3
  return x;
}

// X [n][d] (row-major, global) into LDS column-major [d][np]: coalesced
// reads, eight in flight per thread (a load-then-store loop waited a memory
// round trip per element - ~160 of them a lane for 1000 x 10 points on one
// wave, the bulk of a k-means++ launch)
__device__ __forceinline__ void stage_cols(float* __restrict__ s_x, const float* __restrict__ Xg, int n, int d, int np,
                                           int tid, int nth) {
  const int tot = n * d;
  for (int e0 = tid; e0 < tot; e0 += 8 * nth) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * nth;
      v[u] = e < tot ? Xg[e] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int e = e0 + u * nth;
      if (e < tot) {
        const int i = e / d, j = e - i * d;
        s_x[j * np + i] = v[u];
      }
    }
  }
}

// acc[p] += sum_j (x[i0 + p][j] - x[c][j])^2 over the d columns of a
// column-major LDS table [d][NP], in column order (the host's order), four
// columns' loads issued before their arithmetic: one LDS round trip per four
// columns instead of one per column - the relax step of a k-means++ draw
template <int P, int NP>
__device__ __forceinline__ void relax_cols(const float* __restrict__ s_x, int d, int c, int i0, float (&acc)[P]) {
  int j = 0;
  for (; j + 4 <= d; j += 4) {
    float xc[4], v[4][P];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float* col = s_x + (int64_t)(j + q) * NP;
      xc[q] = col[c];
#pragma unroll
      for (int r = 0; r < P / 4; ++r) {
        const float4 f = reinterpret_cast<const float4*>(col + i0)[r];
        v[q][4 * r] = f.x; v[q][4 * r + 1] = f.y; v[q][4 * r + 2] = f.z; v[q][4 * r + 3] = f.w;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int p = 0; p < P; ++p) {
        const float tt = v[q][p] - xc[q];
        acc[p] = fmaf(tt, tt, acc[p]);
      }
  }
  for (; j < d; ++j) {
    const float* col = s_x + (int64_t)j * NP;
    const float xc = col[c];
#pragma unroll
    for (int r = 0; r < P / 4; ++r) {
      const float4 f = reinterpret_cast<const float4*>(col + i0)[r];
      const float vv[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float tt = vv[e] - xc;
        acc[4 * r + e] = fmaf(tt, tt, acc[4 * r + e]);
      }
    }
  }
}

constexpr int kKppMaxM = 1024;   // draws whose uniforms the wave kernel stages in LDS

// k-means++ seeding on ONE wave (n <= 64 P points): lane l owns rows
// [l P, l P + P) - a contiguous chunk, as cl_draw's threads - with their
// weights and distances in registers and the points in LDS, column-major
// (dimension j of the lane's P rows is P / 4 b128 reads). A draw is a wave
// prefix sum of the lanes' chunk sums in double (DPP, no barrier), a ballot
// for the lane holding u * total and that lane's walk over its chunk: the same
// bisect_right pick as cl_draw without its 4 block barriers per draw.
template <int P>
__global__ __launch_bounds__(64) void kmeanspp_wave_kernel(const float* __restrict__ Xg, int n, int d,
                                                           const float* __restrict__ wg,
                                                           const double* __restrict__ u, int m,
                                                           int32_t* __restrict__ out,
                                                           int32_t* __restrict__ status) {
  static_assert(P % 4 == 0, "b128 column reads");
  extern __shared__ float s_x[];                   // [d][64 P]
  __shared__ double s_u[kKppMaxM];                 // the draws' uniforms (a global read per draw
                                                   // was a memory round trip on the chain)
  constexpr int NP = 64 * P;
  const int lane = threadIdx.x;
  stage_cols(s_x, Xg, n, d, NP, lane, 64);   // (rows past n stay unread: their d2 stays INFINITY)
  // the draws' uniforms in LDS, kKppMaxM at a time (an LDS read per draw; a
  // pointer select between LDS and global memory compiled to a flat load
  // that waited on the vector memory path every draw)
  auto stage_u = [&](int j0) {
    __builtin_amdgcn_wave_barrier();
    for (int j = j0 + lane; j < m && j < j0 + kKppMaxM; j += 64) s_u[j - j0] = u[j];
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  };
  stage_u(0);
  const int i0 = lane * P;
  float w[P], d2[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    w[p] = i0 + p < n ? wg[i0 + p] : 0.f;
    d2[p] = INFINITY;
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // the row of draw j over weights wt (-1: total 0)
  auto draw = [&](const float (&wt)[P], double uj) -> int {
    double sum = 0.0;
#pragma unroll
    for (int p = 0; p < P; ++p) sum += (double)wt[p];
    const double incl = wave_incl_scan_d(sum);
    const double total = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(incl), 63),
                                          __builtin_amdgcn_readlane(__double2loint(incl), 63));
    if (!(total > 0.0)) return -1;
    const double target = uj * total;
    double run = incl - sum;                       // before my chunk
    const bool mine = run <= target && target < incl;
    int r = i0 + P - 1;
    if (mine) {
#pragma unroll
      for (int p = 0; p < P; ++p) {
        run += (double)wt[p];
        if (run > target) { r = i0 + p; break; }
      }
    }
    const uint64_t b = __ballot(mine);
    if (b == 0) return n - 1;                      // u * total rounded onto the end
    return __builtin_amdgcn_readlane(r, __ffsll((long long)b) - 1);
  };
  auto relax = [&](int c) {
    float acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = 0.f;
    relax_cols<P, NP>(s_x, d, c, i0, acc);
#pragma unroll
    for (int p = 0; p < P; ++p)
      if (i0 + p < n) d2[p] = fminf(d2[p], acc[p]);
  };
  auto uj = [&](int j) -> double {
    if (j % kKppMaxM == 0 && j > 0) stage_u(j);
    return s_u[j % kKppMaxM];
  };
  int c = draw(w, uj(0));
  if (lane == 0) { out[0] = c; *status = c < 0 ? 1 : 0; }
  if (c < 0) return;
  relax(c);
  for (int j = 1; j < m; ++j) {
    float pr[P];
#pragma unroll
    for (int p = 0; p < P; ++p) pr[p] = d2[p] < INFINITY ? d2[p] * w[p] : 0.f;
    c = draw(pr, uj(j));
    if (c < 0) {
      if (lane == 0) { out[j] = -1; *status = 1 + j; }
      return;
    }
    if (lane == 0) out[j] = c;
    relax(c);
  }
}

// k-means++ seeding on NW waves (256 < n <= 64 NW P points): the wave
// kernel's draw with a quarter of its rows a lane. Each draw: the lanes'
// chunk sums scanned in double per wave (DPP), the wave totals through LDS
// (one barrier), every thread's interval [lo, hi) of the running sum from the
// same sequential sums (lane i's hi is lane i + 1's lo bit for bit, so at
// most one lane holds u * total), that lane's walk over its chunk, the pick
// through LDS (a second barrier), then every thread relaxes its rows. The
// wave kernel's relax (P rows x d dims a lane) was ~70 % of a draw at P 16.
template <int P, int NW>
__global__ __launch_bounds__(NW * 64) void kmeanspp_blk_kernel(const float* __restrict__ Xg, int n, int d,
                                                               const float* __restrict__ wg,
                                                               const double* __restrict__ u, int m,
                                                               int32_t* __restrict__ out,
                                                               int32_t* __restrict__ status) {
  static_assert(P % 4 == 0, "b128 column reads");
  extern __shared__ float s_x[];                   // [d][NT P]
  __shared__ double s_u[kKppMaxM];
  __shared__ double s_tot[2][NW];
  __shared__ int s_pick[2];
  constexpr int NT = NW * 64, NP = NT * P;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  stage_cols(s_x, Xg, n, d, NP, t, NT);
  for (int j = t; j < m && j < kKppMaxM; j += NT) s_u[j] = u[j];   // (past kKppMaxM: restaged below)
  if (t == 0) { s_pick[0] = n - 1; s_pick[1] = n - 1; }
  const int i0 = t * P;
  float w[P], d2[P];
#pragma unroll
  for (int p = 0; p < P; ++p) {
    w[p] = i0 + p < n ? wg[i0 + p] : 0.f;
    d2[p] = INFINITY;
  }
  __syncthreads();
  auto draw = [&](const float (&wt)[P], double uj, int j) -> int {
    const int b = j & 1;
    double sum = 0.0;
#pragma unroll
    for (int p = 0; p < P; ++p) sum += (double)wt[p];
    const double incl = wave_incl_scan_d(sum);
    const int phi = __shfl_up(__double2hiint(incl), 1, 64), plo = __shfl_up(__double2loint(incl), 1, 64);
    const double excl = lane == 0 ? 0.0 : __hiloint2double(phi, plo);
    if (lane == 63) s_tot[b][wv] = incl;
    __syncthreads();
    // the next draw's default (every thread has read the previous draw's pick)
    if (t == 0) s_pick[b ^ 1] = n - 1;
    double off = 0.0, total = 0.0;
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      if (q == wv) off = total;
      total += s_tot[b][q];
    }
    if (!(total > 0.0)) return -1;                 // (block-uniform)
    const double target = uj * total;
    const double lo = off + excl, hi = off + incl;
    if (lo <= target && target < hi) {
      double run = lo;
      int r = i0 + P - 1;
#pragma unroll
      for (int p = 0; p < P; ++p) {
        run += (double)wt[p];
        if (run > target) { r = i0 + p; break; }
      }
      s_pick[b] = r;
    }
    __syncthreads();
    return s_pick[b];
  };
  auto relax = [&](int c) {
    float acc[P];
#pragma unroll
    for (int p = 0; p < P; ++p) acc[p] = 0.f;
    relax_cols<P, NP>(s_x, d, c, i0, acc);
#pragma unroll
    for (int p = 0; p < P; ++p)
      if (i0 + p < n) d2[p] = fminf(d2[p], acc[p]);
  };
  auto uj = [&](int j) -> double {
    if (j % kKppMaxM == 0 && j > 0) {   // (block-uniform)
      __syncthreads();
      for (int i = j + t; i < m && i < j + kKppMaxM; i += NT) s_u[i - j] = u[i];
      __syncthreads();
    }
    return s_u[j % kKppMaxM];
  };
  int c = draw(w, uj(0), 0);
  if (t == 0) { out[0] = c; *status = c < 0 ? 1 : 0; }
  if (c < 0) return;
  relax(c);
  for (int j = 1; j < m; ++j) {
    float pr[P];
#pragma unroll
    for (int p = 0; p < P; ++p) pr[p] = d2[p] < INFINITY ? d2[p] * w[p] : 0.f;
    c = draw(pr, uj(j), j);
    if (c < 0) {
      if (t == 0) { out[j] = -1; *status = 1 + j; }
      return;
    }
    if (t == 0) out[j] = c;
    relax(c);
  }
}

// Weighted Lloyd iterations to convergence (|C' - C| <= atol + rtol |C|, as
// torch.allclose) or `iters`, then the final assignment. C [k, d] in/out.
__global__ __launch_bounds__(kClBlock) void lloyd_kernel(const float* __restrict__ X, int n, int d,
                                                         const float* __restrict__ w,
                                                         float* __restrict__ C, int k, int iters,
                                                         float atol, float rtol,
                                                         int32_t* __restrict__ assign,
                                                         float* __restrict__ S,
                                                         int32_t* __restrict__ done_iters) {
  extern __shared__ float s_c[];                   // C [k][d] | S [k][d] | W [k]
  float* s_s = s_c + (int64_t)k * d;
  float* s_w = s_s + (int64_t)k * d;
  __shared__ int changed;
  const int t = threadIdx.x;
  for (int i = t; i < k * d; i += kClBlock) s_c[i] = C[i];
  __syncthreads();
  int it = 0;
  for (; it <= iters; ++it) {
    // assignment (the last pass only assigns)
    for (int i = t; i < n; i += kClBlock) {
      const float* x = X + (int64_t)i * d;
      int best = 0;
      float bd = INFINITY;
      for (int j = 0; j < k; ++j) {
        float s = 0.f;
        for (int q = 0; q < d; ++q) {
          const float tt = x[q] - s_c[j * d + q];
          s = fmaf(tt, tt, s);
        }
        if (s < bd) { bd = s; best = j; }
      }
      assign[i] = best;
    }
    if (it == iters) break;
    for (int i = t; i < k * d; i += kClBlock) s_s[i] = 0.f;
    for (int i = t; i < k; i += kClBlock) s_w[i] = 0.f;
    if (t == 0) changed = 0;
    __syncthreads();
    for (int i = t; i < n; i += kClBlock) {
      const int a = assign[i];
      const float wi = w[i];
      atomicAdd(&s_w[a], wi);
      const float* x = X + (int64_t)i * d;
      for (int q = 0; q < d; ++q) atomicAdd(&s_s[a * d + q], wi * x[q]);
    }
    __syncthreads();
    for (int i = t; i < k * d; i += kClBlock) {
      const int j = i / d;
      const float nc = s_w[j] > 0.f ? s_s[i] / fmaxf(s_w[j], 1e-12f) : s_c[i];
      if (fabsf(nc - s_c[i]) > atol + rtol * fabsf(s_c[i])) changed = 1;
      s_c[i] = nc;
    }
    __syncthreads();
    if (!changed) {                                // converged: final assignment next
      it = iters - 1;
    }
    __syncthreads();
  }
  for (int i = t; i < k * d; i += kClBlock) C[i] = s_c[i];
  if (t == 0) *done_iters = it;
}

// Diagonal-covariance GMM EM, every iteration in one single-workgroup launch
// (the Python path ran ~10 torch launches per iteration). Same formulas as
// models/clustering.py _em: responsibilities r_ij = w_i softmax_j(log N(x_i |
// C_j, var_j) + log pi_j); nk = max(sum_i r_ij, 1e-9); C = S1 / nk;
// var = max(S2 / nk - C^2, 1e-6); pi = nk / sum nk. LDS: C, var, S1, S2
// [k][d], nk / logdet / log pi [k].
// XL: the points and weights are staged in LDS (a compile-time choice: a
// runtime select between LDS and global pointers compiles to flat loads,
// which wait on the vector memory path)
template <int T, bool XL>
__global__ __launch_bounds__(T) void gmm_em_kernel(const float* __restrict__ Xg, int n, int d,
                                                          const float* __restrict__ wg, float* __restrict__ C,
                                                          float* __restrict__ var, float* __restrict__ pi,
                                                          int k, int iters, int32_t* __restrict__ assign,
                                                          bool staged) {
  constexpr bool xlds = XL;
  extern __shared__ float s_em[];
  float* sC = s_em;
  float* sV = sC + k * d;
  float* s1 = sV + k * d;
  float* s2 = s1 + k * d;
  float* nk = s2 + k * d;          // [k]
  float* lc = nk + k;              // [k] log pi_j - 0.5 sum_q log(2 pi var_jq)
  float* spi = lc + k;             // [k] pi (staged loop)
  float* sR = spi + k;             // [n][k] responsibilities (staged)
  float* sIV = sR + (staged ? (size_t)n * k : 0);   // [k][d] 1 / var (staged)
  float* sX = sIV + (staged ? (size_t)k * d : 0);   // [n][d] the points (xlds)
  float* sW = sX + (xlds ? (size_t)n * d : 0);       // [n] the weights (xlds): read every iteration
  __shared__ float s_tot;
  const int t = threadIdx.x;
  // the points in LDS when they fit: every E- and M-step pass reads them
  if (xlds)
    for (int i = t; i < n * d; i += T) sX[i] = Xg[i];
  const float* __restrict__ X = xlds ? sX : Xg;
  if (xlds)
    for (int i = t; i < n; i += T) sW[i] = wg[i];
  const float* __restrict__ w = xlds ? sW : wg;
  const float kLog2Pi = 1.8378770664093453f;
  for (int i = t; i < k * d; i += T) { sC[i] = C[i]; sV[i] = var[i]; }
  for (int j = t; j < k; j += T) { nk[j] = pi[j]; spi[j] = pi[j]; }   // (nk: pi until the first M-step)
  __syncthreads();
  // staged: four barriers an iteration - (lc, 1 / var) | E-step | normalize |
  // M-step sums (nk floored where it is summed) | C, var, pi - the reads of
  // each phase follow the writes of the one before it
  // an iteration that leaves C, var and pi bit for bit as they were is a
  // fixed point: every later one would too (the staged loop is deterministic:
  // no atomics), so the loop stops there with the result of all `iters`
  __shared__ int s_moved;
  if (t == 0) s_moved = 0;
  for (int it = 0; staged && it < iters; ++it) {
    for (int j = t; j < k; j += T) {
      float ld = 0.f;
      for (int q = 0; q < d; ++q) ld += logf(6.283185307179586f * sV[j * d + q]);
      lc[j] = logf(fmaxf(spi[j], 1e-12f)) - 0.5f * ld;
    }
    for (int i = t; i < k * d; i += T) sIV[i] = 1.f / sV[i];
    __syncthreads();
    if (t == 0) s_moved = 0;   // (every thread read the last iteration's flag before the barrier above)
    for (int e = t; e < n * k; e += T) {
      const int i = e / k, j = e - i * k;
      const float* x = X + (int64_t)i * d;
      const float* c = sC + j * d;
      const float* iv = sIV + j * d;
      float q2 = 0.f;
      for (int q = 0; q < d; ++q) {
        const float df = x[q] - c[q];
        q2 += df * df * iv[q];
      }
      sR[e] = lc[j] - 0.5f * q2;
    }
    __syncthreads();
    for (int i = t; i < n; i += T) {
      float* r = sR + (size_t)i * k;
      float mx = -INFINITY;
      for (int j = 0; j < k; ++j) mx = fmaxf(mx, r[j]);
      float den = 0.f;
      for (int j = 0; j < k; ++j) den += expf(r[j] - mx);
      const float wi = w[i] / den;
      for (int j = 0; j < k; ++j) r[j] = wi * expf(r[j] - mx);
    }
    __syncthreads();
    {
      const int lane = t & 63, wave = t >> 6, cols = 2 * d + 1;
      for (int pr = wave; pr < k * cols; pr += T / 64) {
        const int j = pr / cols, col = pr - j * cols;
        float acc = 0.f;
        for (int i = lane; i < n; i += 64) {
          const float r = sR[(size_t)i * k + j];
          if (col == 2 * d) {
            acc += r;
          } else {
            const float xv = X[(int64_t)i * d + (col < d ? col : col - d)];
            acc += col < d ? r * xv : r * xv * xv;
          }
        }
        acc = wave_sum_fast(acc, lane);              // DPP / permlane: no LDS round trips
        if (lane == 0) {
          if (col == 2 * d) nk[j] = fmaxf(acc, 1e-9f);
          else if (col < d) s1[j * d + col] = acc;
          else s2[j * d + col - d] = acc;
        }
      }
    }
    __syncthreads();
    bool moved = false;
    for (int i = t; i < k * d; i += T) {
      const float m = nk[i / d];
      const float c = s1[i] / m;
      const float v = fmaxf(s2[i] / m - c * c, 1e-6f);
      moved |= __float_as_uint(c) != __float_as_uint(sC[i]) || __float_as_uint(v) != __float_as_uint(sV[i]);
      sC[i] = c;
      sV[i] = v;
    }
    if (t < k) {
      float tot = 0.f;
      for (int j = 0; j < k; ++j) tot += nk[j];
      const float pn = nk[t] / tot;               // pi of the next E-step
      moved |= __float_as_uint(pn) != __float_as_uint(spi[t]);
      spi[t] = pn;
    }
    if (moved) s_moved = 1;
    __syncthreads();
    if (s_moved == 0) break;                      // (block-uniform)
  }
  if (staged)
    for (int j = t; j < k; j += T) nk[j] = spi[j];
  for (int it = 0; !staged && it < iters; ++it) {
    for (int j = t; j < k; j += T) {
      float ld = 0.f;
      for (int q = 0; q < d; ++q) ld += logf(6.283185307179586f * sV[j * d + q]);
      lc[j] = logf(fmaxf(nk[j], 1e-12f)) - 0.5f * ld;
    }
    for (int i = t; i < k * d; i += T) { s1[i] = 0.f; s2[i] = 0.f; }
    __syncthreads();
    for (int j = t; j < k; j += T) nk[j] = 0.f;
    __syncthreads();
    (void)kLog2Pi;
    if (staged) {
      // E-step: one thread per (point, component) - the d-long distance
      // multiplies by 1 / var (one divide per (j, q) an iteration, not one
      // per point) - then one thread per point normalizes its k entries
      for (int i = t; i < k * d; i += T) sIV[i] = 1.f / sV[i];
      __syncthreads();
      for (int e = t; e < n * k; e += T) {
        const int i = e / k, j = e - i * k;
        const float* x = X + (int64_t)i * d;
        const float* c = sC + j * d;
        const float* iv = sIV + j * d;
        float q2 = 0.f;
        for (int q = 0; q < d; ++q) {
          const float df = x[q] - c[q];
          q2 += df * df * iv[q];
        }
        sR[e] = lc[j] - 0.5f * q2;
      }
      __syncthreads();
      for (int i = t; i < n; i += T) {
        float* r = sR + (size_t)i * k;
        float mx = -INFINITY;
        for (int j = 0; j < k; ++j) mx = fmaxf(mx, r[j]);
        float den = 0.f;
        for (int j = 0; j < k; ++j) den += expf(r[j] - mx);
        const float wi = w[i] / den;
        for (int j = 0; j < k; ++j) r[j] = wi * expf(r[j] - mx);
      }
      __syncthreads();
      // M-step sums: one wave per (cluster, column) pair, lanes over the
      // points, a shuffle reduction and one plain store (no LDS atomics)
      const int lane = t & 63, wave = t >> 6, cols = 2 * d + 1;
      for (int pr = wave; pr < k * cols; pr += T / 64) {
        const int j = pr / cols, col = pr - j * cols;
        float acc = 0.f;
        for (int i = lane; i < n; i += 64) {
          const float r = sR[(size_t)i * k + j];
          if (col == 2 * d) {
            acc += r;
          } else {
            const float xv = X[(int64_t)i * d + (col < d ? col : col - d)];
            acc += col < d ? r * xv : r * xv * xv;
          }
        }
        for (int off = 32; off; off >>= 1) acc += __shfl_xor(acc, off, 64);
        if (lane == 0) {
          if (col == 2 * d) nk[j] = acc;
          else if (col < d) s1[j * d + col] = acc;
          else s2[j * d + col - d] = acc;
        }
      }
    }
    for (int i = staged ? n : t; i < n; i += T) {
      const float* x = X + (int64_t)i * d;
      // log-sum-exp over the clusters (k is small: two passes over d)
      float mx = -INFINITY;
      for (int j = 0; j < k; ++j) {
        float q2 = 0.f;
        for (int q = 0; q < d; ++q) {
          const float df = x[q] - sC[j * d + q];
          q2 += df * df / sV[j * d + q];
        }
        mx = fmaxf(mx, lc[j] - 0.5f * q2);
      }
      float den = 0.f;
      for (int j = 0; j < k; ++j) {
        float q2 = 0.f;
        for (int q = 0; q < d; ++q) {
          const float df = x[q] - sC[j * d + q];
          q2 += df * df / sV[j * d + q];
        }
        den += expf(lc[j] - 0.5f * q2 - mx);
      }
      const float wi = w[i];
      for (int j = 0; j < k; ++j) {
        float q2 = 0.f;
        for (int q = 0; q < d; ++q) {
          const float df = x[q] - sC[j * d + q];
          q2 += df * df / sV[j * d + q];
        }
        const float r = wi * expf(lc[j] - 0.5f * q2 - mx) / den;
        if (r == 0.f) continue;
        atomicAdd(&nk[j], r);
        for (int q = 0; q < d; ++q) {
          atomicAdd(&s1[j * d + q], r * x[q]);
          atomicAdd(&s2[j * d + q], r * x[q] * x[q]);
        }
      }
    }
    __syncthreads();
    for (int j = t; j < k; j += T) nk[j] = fmaxf(nk[j], 1e-9f);
    __syncthreads();
    for (int i = t; i < k * d; i += T) {
      const float m = nk[i / d];
      const float c = s1[i] / m;
      sC[i] = c;
      sV[i] = fmaxf(s2[i] / m - c * c, 1e-6f);
    }
    if (t == 0) {
      float tot = 0.f;
      for (int j = 0; j < k; ++j) tot += nk[j];
      s_tot = tot;
    }
    __syncthreads();
    for (int j = t; j < k; j += T) nk[j] = nk[j] / s_tot;   // pi of the next E-step
    __syncthreads();
  }
  for (int i = t; i < k * d; i += T) { C[i] = sC[i]; var[i] = sV[i]; }
  for (int j = t; j < k; j += T) pi[j] = nk[j];
  if (assign == nullptr) return;
  // the most likely component of every point under the final parameters
  // (models/clustering.py _assign: argmax of the log responsibilities)
  for (int j = t; j < k; j += T) {
    float ld = 0.f;
    for (int q = 0; q < d; ++q) ld += logf(6.283185307179586f * sV[j * d + q]);
    lc[j] = logf(fmaxf(nk[j], 1e-12f)) - 0.5f * ld;
  }
  __syncthreads();
  for (int i = t; i < n; i += T) {
    const float* x = X + (int64_t)i * d;
    int best = 0;
    float bv = -INFINITY;
    for (int j = 0; j < k; ++j) {
      float q2 = 0.f;
      for (int q = 0; q < d; ++q) {
        const float df = x[q] - sC[j * d + q];
        q2 += df * df / sV[j * d + q];
      }
      const float v = lc[j] - 0.5f * q2;
      if (v > bv) { bv = v; best = j; }
    }
    assign[i] = best;
  }
}

}  // namespace jb

extern "C" int jb_gmm_em(const float* X, int n, int d, const float* w, float* C, float* var, float* pi, int k,
                         int iters, int32_t* assign, hipStream_t stream) {
  if (n <= 0 || k <= 0 || d <= 0) return 0;
  size_t lds = sizeof(float) * (4 * (size_t)k * d + 3 * (size_t)k);
  if (lds > 64 * 1024) return -2;
  // responsibilities staged in LDS when they fit: the M-step then reduces
  // per (cluster, column) instead of contending on LDS float atomics
  const size_t staged = lds + sizeof(float) * ((size_t)n * k + (size_t)k * d);   // + 1 / var
  const bool stage = staged <= 64 * 1024;
  if (stage) lds = staged;
  const size_t withx = lds + sizeof(float) * (size_t)n * (d + 1);   // the points and their weights
  const bool xlds = stage && withx <= 64 * 1024;
  if (xlds) lds = withx;
  // (measured: 256 threads ran the bench's 300-point coresets in 784 us for
  // 50 iterations, 1024 threads in 341 us - the per-thread work, not the
  // barriers, sets the iteration's time)
  if (xlds)
    hipLaunchKernelGGL((jb::gmm_em_kernel<jb::kClBlock, true>), dim3(1), dim3(jb::kClBlock), lds, stream, X, n, d, w,
                       C, var, pi, k, iters, assign, stage);
  else
    hipLaunchKernelGGL((jb::gmm_em_kernel<jb::kClBlock, false>), dim3(1), dim3(jb::kClBlock), lds, stream, X, n, d,
                       w, C, var, pi, k, iters, assign, stage);
  return (int)hipGetLastError();
}

namespace jb {
// the first nearest column of every row of D [n][k] (strict <, as the
// host's argmin loop and torch.argmin): the compress step's assignment
// without copying the n x k distances to the host
__global__ __launch_bounds__(256) void argmin_rows_kernel(const float* __restrict__ D, int64_t n, int k,
                                                          int32_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float* r = D + i * k;
  int a = 0;
  float best = r[0];
  for (int j = 1; j < k; ++j) {
    const float v = r[j];
    if (v < best) { best = v; a = j; }
  }
  out[i] = a;
}
// the same for rows of 32+ columns: one wave a row, coalesced reads, lane
// minima (first index on ties) merged by shuffles - the first minimum of
// the row, as the loop above (a thread a row read its k columns strided by k)
__global__ __launch_bounds__(256) void argmin_rows_wave_kernel(const float* __restrict__ D, int64_t n, int k,
                                                               int32_t* __restrict__ out) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  const float* r = D + i * k;
  float best = INFINITY;
  int a = INT_MAX;
  for (int j = lane; j < k; j += 64) {
    const float v = r[j];
    if (v < best || (a == INT_MAX && !(v > best))) { best = v; a = j; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oa = __shfl_xor(a, o, 64);
    if (ob < best || (ob == best && oa < a) || (a == INT_MAX && oa != INT_MAX && !(ob > best))) {
      best = ob;
      a = oa;
    }
  }
  if (lane == 0) out[i] = a == INT_MAX ? 0 : a;
}
}  // namespace jb

extern "C" int jb_argmin_rows(const float* D, int64_t n, int k, int32_t* out, hipStream_t stream) {
  if (n <= 0 || k <= 0) return 0;
  if (k >= 32) {
    hipLaunchKernelGGL(jb::argmin_rows_wave_kernel, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, stream, D,
                       n, k, out);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(jb::argmin_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, D, n, k,
                     out);
  return (int)hipGetLastError();
}

extern "C" int jb_sqdist_mfma(const float* X, int64_t n, const float* C, int k, int d,
                              const float* xn2, const float* cn2, float* out, hipStream_t stream) {
  if (n <= 0 || k <= 0) return 0;
  dim3 grid((unsigned)((n + 63) / 64), (unsigned)((k + 15) / 16));
  hipLaunchKernelGGL(jb::sqdist_mfma_kernel, grid, dim3(256), 0, stream, X, n, C, k, d, xn2, cn2, out);
  return (int)hipGetLastError();
}

extern "C" int jb_kmeanspp(const float* X, int n, int d, const float* w, const double* u, int m,
                           float* d2, float* prob, int32_t* out, int32_t* status,
                           hipStream_t stream) {
  if (n <= 0 || m <= 0) return 0;
  // one wave when the points fit its registers / LDS (JB_KMEANSPP_BLOCK=1: the block kernel)
  static const bool block_only = [] {
    const char* e = getenv("JB_KMEANSPP_BLOCK");
    return e != nullptr && e[0] == '1';
  }();
  // past 256 points: four waves, 4 or 8 rows a lane (JB_KMEANSPP_WAVE=1:
  // the one-wave kernel there too, for A/B runs)
  static const bool wave_only = [] {
    const char* e = getenv("JB_KMEANSPP_WAVE");
    return e != nullptr && e[0] == '1';
  }();
  if (!block_only && !wave_only && n > 64 * 4 && n <= 256 * 8) {
    const int P4 = n <= 256 * 4 ? 4 : 8;
    const size_t xb4 = sizeof(float) * (size_t)(256 * P4) * d;
    if (xb4 <= 64 * 1024) {
      if (P4 == 4)
        hipLaunchKernelGGL((jb::kmeanspp_blk_kernel<4, 4>), dim3(1), dim3(256), xb4, stream, X, n, d, w, u, m, out,
                           status);
      else
        hipLaunchKernelGGL((jb::kmeanspp_blk_kernel<8, 4>), dim3(1), dim3(256), xb4, stream, X, n, d, w, u, m, out,
                           status);
      return (int)hipGetLastError();
    }
  }
  const int P = n <= 64 * 4 ? 4 : n <= 64 * 8 ? 8 : n <= 64 * 16 ? 16 : 32;
  const size_t xb = sizeof(float) * (size_t)(64 * P) * d;   // column-major, padded to 64 P rows
  if (!block_only && n <= 64 * 32 && xb <= 64 * 1024) {
#define JB_KPP(P)                                                                                             \
  hipLaunchKernelGGL((jb::kmeanspp_wave_kernel<P>), dim3(1), dim3(64), xb, stream, X, n, d, w, u, m, out, status); \
  return (int)hipGetLastError();
    if (n <= 64 * 4) { JB_KPP(4) }
    if (n <= 64 * 8) { JB_KPP(8) }
    if (n <= 64 * 16) { JB_KPP(16) }
    JB_KPP(32)
#undef JB_KPP
  }
  const size_t base = sizeof(float) * 3 * (size_t)n;
  const size_t withx = base + sizeof(float) * (size_t)n * d;
  const int mode = withx <= 64 * 1024 ? 2 : (base <= 64 * 1024 ? 1 : 0);
  hipLaunchKernelGGL(jb::kmeanspp_kernel, dim3(1), dim3(jb::kClBlock), mode == 2 ? withx : (mode == 1 ? base : 0),
                     stream, X, n, d, w, u, m, d2, prob, out, status, mode);
  return (int)hipGetLastError();
}

extern "C" int jb_lloyd(const float* X, int n, int d, const float* w, float* C, int k, int iters,
                        float atol, float rtol, int32_t* assign, float* S, int32_t* done_iters,
                        hipStream_t stream) {
  if (n <= 0 || k <= 0) return 0;
  const size_t lds = sizeof(float) * (2 * (size_t)k * d + k);
  if (lds > 64 * 1024) return -2;
  (void)S;
  hipLaunchKernelGGL(jb::lloyd_kernel, dim3(1), dim3(jb::kClBlock), lds, stream, X, n, d, w, C, k,
                     iters, atol, rtol, assign, S, done_iters);
  return (int)hipGetLastError();
}
