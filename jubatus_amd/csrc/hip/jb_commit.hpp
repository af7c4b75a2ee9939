// Pieces shared by the serial-equivalent committers of label capacities up to
// 64 (commit.hip: the delta committer; vcommit.hip: the verified committer):
// the LDS row store (2-choice 4-way buckets of row keys), the exact margin of a
// sample held by a 16-lane group, its slack to the method's update threshold,
// and the round-start score correction over the store's delta rows.
#pragma once
#include <stdlib.h>

#include "jb_linear.hpp"

namespace jb {
namespace dc {

constexpr int kT = 512;               // committer threads (8 waves)
constexpr int kNG = kT / 16;          // groups (DPP rows) of 16 lanes
constexpr int kR = 2;                 // samples per group per round
constexpr int kNS = kNG * kR;         // samples per round
constexpr int kFC = 2;                // feature chunks of 16 held in registers
constexpr int kNFMax = 16 * kFC;      // widest sample the committer takes
constexpr float kGuard = 1e-4f;       // relative guard band of a decision
constexpr int kInf = 0x7fffffff;
// stop reasons (tail[kTailReason]); the values are serial.hip's
constexpr int64_t kStopDone = 0, kStopSaturated = 1, kStopDense = 2, kStopWindow = 3;
constexpr int kTailReason = 20;
// A segment scores and commits a window of the batch, not its whole rest:
// twice the samples the previous segment took, at least kWinMin (the S0
// pass of a segment that saturates early would otherwise re-score the whole
// rest of the batch every time). tail[kTailWin]: samples the last segment took.
constexpr int kTailWin = 29;
constexpr int64_t kWinMin = 8192;
__device__ __forceinline__ int64_t window_end(int64_t beg, int64_t end, const int64_t* tail) {
  int64_t w = tail[kTailWin];   // the previous batch's last segment for a batch's first one
  w = (w <= 0 || w > ((int64_t)1 << 30)) ? kWinMin : (2 * w > kWinMin ? 2 * w : kWinMin);
  return beg + w < end ? beg + w : end;
}
// phase timing (tail[4..19]): shader cycles of wave 0 per phase, the wall
// clock of the kernel and every wave's own round-start work
// (a kernel argument: JB_COMMIT_PROF=1 turns them on; they cost ~6 % of a
// steady batch, so the default run leaves them off)

constexpr int ilog2(int v) { return v <= 1 ? 0 : 1 + ilog2(v / 2); }

template <int LC>
struct Geo {
  static constexpr int K = (LC + 15) / 16;                 // labels per lane
  static constexpr int NSLOT = 16384 / (LC > 16 ? LC : 16); // rows the LDS store holds
  static constexpr int NB = NSLOT / 4;                      // 4-way buckets of row keys
  static constexpr int BB = ilog2(NB);
  static constexpr int PAD = LC + 16;   // a zero row (slot NSLOT) + read overrun of LC = 8
};

// best wrong label over a row of 16 lanes (lowest label on ties): the row's
// maximum (4 DPP max steps over the pairings xor 1, xor 2, xor 7 - half
// mirror - and xor 8 - rotate 8 - which span the row), then the lowest label
// holding it (4 DPP min steps). b: the lane's best candidate (-inf: none),
// bl its label; every lane gets the row's (b, bl), bl = -1 when no lane has one.
__device__ __forceinline__ void row16_argmax(float& b, int& bl) {
  float m = b;
  m = fmaxf(m, dpp_f<kDppXor1>(m));
  m = fmaxf(m, dpp_f<kDppXor2>(m));
  m = fmaxf(m, dpp_f<kDppHalfMirror>(m));
  m = fmaxf(m, dpp_f<kDppRowRor8>(m));
  int c = (bl >= 0 && b == m) ? bl : 0x7fff;
  c = min(c, dpp_i<kDppXor1>(c));
  c = min(c, dpp_i<kDppXor2>(c));
  c = min(c, dpp_i<kDppHalfMirror>(c));
  c = min(c, dpp_i<kDppRowRor8>(c));
  bl = c == 0x7fff ? -1 : c;
  b = m;
}

// exact margin of a sample held by a group: score(y) - best active wrong
// label (every lane of the row gets the same values)
template <int LC>
__device__ __forceinline__ float group_margin(const float (&s)[Geo<LC>::K], int y,
                                              const int (&act)[Geo<LC>::K], int sub,
                                              int* lstar, float* sy_out, float* best_out) {
  constexpr int K = Geo<LC>::K;
  float v = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k == (y >> 4) && sub == (y & 15)) v = s[k];
  const float sy = row16_sum(v);   // one non-zero term: exact
  float b = -INFINITY;
  int bl = -1;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int lab = sub + 16 * k;
    if (lab < LC && act[k] != 0 && lab != y && s[k] > b) { b = s[k]; bl = lab; }
  }
  row16_argmax(b, bl);
  *lstar = bl;
  *sy_out = sy;
  *best_out = bl >= 0 ? b : 0.f;
  return sy - (bl >= 0 ? b : 0.f);
}

// distance of a margin to the update threshold of the method, less the guard
// band: a sample updates only if this is not positive (NaN: it may). CW's
// threshold phi * var is bounded by phi * (1 or 2) * |x|^2 (precisions >= 1).
__device__ __forceinline__ float slack_of(int method, float m, float nrm, bool has_l, float C,
                                          float sy, float best) {
  const float g = kGuard * (1.f + fabsf(sy) + fabsf(best));
  switch (method) {
    case PERCEPTRON: return m - g;
    case PA: case PA1: case PA2: return nrm > 0.f ? m - 1.f - g : INFINITY;
    case CW: return nrm > 0.f ? m - C * (has_l ? 2.f : 1.f) * nrm - g : INFINITY;
    default: return m - 1.f - g;
  }
}

// LDS row store: row keys in 2-choice 4-way buckets; a row's slot is its
// position in the key array (its dW / dP rows live at that index), so a
// lookup is two 16-byte LDS reads and eight compares, no probe loop
template <int LC>
__device__ __forceinline__ void buckets_of(int32_t row, int* b1, int* b2) {
  using Gm = Geo<LC>;
  const int x = (int)(((uint32_t)row * 0x9E3779B1u) >> (32 - Gm::BB));
  const int y = (int)((((uint32_t)row ^ 0x5BD1E995u) * 0x85EBCA77u) >> (32 - Gm::BB));
  *b1 = x;
  *b2 = y == x ? (y ^ 1) : y;
}

template <int LC>
__device__ __forceinline__ int cache_find(const int32_t* key, int32_t row) {
  int b1, b2;
  buckets_of<LC>(row, &b1, &b2);
  const int4 k1 = reinterpret_cast<const int4*>(key)[b1];
  const int4 k2 = reinterpret_cast<const int4*>(key)[b2];
  const int32_t r = row < 0 ? -2 : row;     // no key is -2 (free entries are -1)
  int s = -1;
  s = k1.x == r ? 4 * b1 : s;
  s = k1.y == r ? 4 * b1 + 1 : s;
  s = k1.z == r ? 4 * b1 + 2 : s;
  s = k1.w == r ? 4 * b1 + 3 : s;
  s = k2.x == r ? 4 * b2 : s;
  s = k2.y == r ? 4 * b2 + 1 : s;
  s = k2.z == r ? 4 * b2 + 2 : s;
  s = k2.w == r ? 4 * b2 + 3 : s;
  return s;
}

// the stepping group's lanes add their new rows (the emptier bucket first;
// keys are only added during a segment, so a bucket fills in order); a lane
// whose row another lane of the same instruction added takes that slot.
// -1: both buckets are full (the segment ends)
template <int LC>
__device__ __forceinline__ int cache_insert(int32_t* key, int32_t row) {
  int b1, b2;
  buckets_of<LC>(row, &b1, &b2);
  const int4 k1 = reinterpret_cast<const int4*>(key)[b1];
  const int4 k2 = reinterpret_cast<const int4*>(key)[b2];
  // added meanwhile (an earlier feature chunk of the same sample)
  if (k1.x == row) return 4 * b1;
  if (k1.y == row) return 4 * b1 + 1;
  if (k1.z == row) return 4 * b1 + 2;
  if (k1.w == row) return 4 * b1 + 3;
  if (k2.x == row) return 4 * b2;
  if (k2.y == row) return 4 * b2 + 1;
  if (k2.z == row) return 4 * b2 + 2;
  if (k2.w == row) return 4 * b2 + 3;
  const int n1 = (k1.x >= 0) + (k1.y >= 0) + (k1.z >= 0) + (k1.w >= 0);
  const int n2 = (k2.x >= 0) + (k2.y >= 0) + (k2.z >= 0) + (k2.w >= 0);
  const int first = n2 < n1 ? b2 : b1;
  const int second = first == b1 ? b2 : b1;
  for (int t = first == b1 ? n1 : n2; t < 8; ++t) {
    const int pos = t < 4 ? 4 * first + t : 4 * second + (t - 4);
    const int old = atomicCAS(&key[pos], -1, row);
    if (old == -1 || old == row) return pos;
  }
  return -1;
}

// round-start correction: s[k] (label sub + 16k) += sum over the row's lanes
// of x_c * dW[slot_c][label]. Lane i reads the quads of its row in the order
// q ^ (i >> 2); the mirror (lane 15 - i) and half-mirror (lane i ^ 7) DPP
// adds then leave lane i the quad of labels 4 (i >> 2) .. + 3 summed over 4
// lanes, and two quad-permute steps hand each lane its own label.
// Branch-free: a lane without a row reads the zero row (slot NSLOT); with
// LC = 8 the quads past the labels read padding / the next row, which only
// ever sums into labels >= LC (lanes 8..15), never read.
template <int LC, int FC>
__device__ __forceinline__ void row_correct(const float* dw, const int (&slot)[FC],
                                            const float (&x)[FC], int sub, bool two,
                                            float (&s)[Geo<LC>::K]) {
  constexpr int K = Geo<LC>::K;
  const int qs = sub >> 2;
#pragma unroll
  for (int b = 0; b < K; ++b) {
    float4 v[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int c = 0; c < FC; ++c) {
      if (c > 0 && !two) break;              // wave-uniform
      const float xc = x[c];
      const float* rowp = dw + (slot[c] >= 0 ? slot[c] : Geo<LC>::NSLOT) * LC + 16 * b;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 w = *reinterpret_cast<const float4*>(rowp + 4 * (q ^ qs));
        v[q].x += xc * w.x; v[q].y += xc * w.y; v[q].z += xc * w.z; v[q].w += xc * w.w;
      }
    }
#define JB_DADD(D, S, C) \
  D.x += dpp_f<C>(S.x); D.y += dpp_f<C>(S.y); D.z += dpp_f<C>(S.z); D.w += dpp_f<C>(S.w);
    JB_DADD(v[0], v[3], kDppMirror)
    JB_DADD(v[1], v[2], kDppMirror)
    JB_DADD(v[0], v[1], kDppHalfMirror)
#undef JB_DADD
    const bool h2 = (sub & 2) != 0;
    float k0 = h2 ? v[0].z : v[0].x;
    float k1 = h2 ? v[0].w : v[0].y;
    const float s0 = h2 ? v[0].x : v[0].z;
    const float s1 = h2 ? v[0].y : v[0].w;
    k0 += dpp_f<kDppXor2>(s0);
    k1 += dpp_f<kDppXor2>(s1);
    const bool h1 = (sub & 1) != 0;
    float kk = h1 ? k1 : k0;
    kk += dpp_f<kDppXor1>(h1 ? k0 : k1);
    s[b] += kk;
  }
}

// a wave-uniform value moved into a VGPR: the committer holds more loop
// invariants than the SGPR file (a spilled SGPR costs a v_readlane at every
// use); the prefetch's base pointers and bounds live in VGPRs instead
__device__ __forceinline__ uint64_t in_vgpr(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32), vl, vh;
  asm("v_mov_b32 %0, %1" : "=v"(vl) : "s"(lo));
  asm("v_mov_b32 %0, %1" : "=v"(vh) : "s"(hi));
  return (uint64_t)vl | ((uint64_t)vh << 32);
}
template <class T>
__device__ __forceinline__ T* in_vgpr(T* p) { return (T*)in_vgpr((uint64_t)p); }

// a load through the global address space: a pointer that went through
// in_vgpr is generic to the compiler, and a flat load counts on lgkmcnt too,
// so every LDS wait would also wait for the prefetches in flight
template <class T>
__device__ __forceinline__ T gld(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}
// HIP's vector structs copy through generic references: load native vectors
typedef float jb_f2v __attribute__((ext_vector_type(2)));
typedef int jb_i4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float2 gld(const float2* p) {
  const jb_f2v v = *(const __attribute__((address_space(1))) jb_f2v*)p;
  return make_float2(v.x, v.y);
}
__device__ __forceinline__ int4 gld(const int4* p) {
  const jb_i4v v = *(const __attribute__((address_space(1))) jb_i4v*)p;
  return make_int4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ int aux_pack(int y, int ls, int n) {
  return (y & 0xff) | ((ls & 0xff) << 8) | ((n < 0xffff ? n : 0xffff) << 16);
}
__device__ __forceinline__ int aux_y(int v) { return (int)(int8_t)(v & 0xff); }
__device__ __forceinline__ int aux_ls(int v) { return (int)(int8_t)((v >> 8) & 0xff); }
__device__ __forceinline__ int aux_nf(int v) { return (int)((unsigned)v >> 16); }

}  // namespace dc
}  // namespace jb
