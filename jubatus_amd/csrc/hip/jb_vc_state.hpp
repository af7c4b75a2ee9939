// The verified committer's device state words (vcommit.hip), shared with the
// sequential stepper (stepper.hip): after an update-dense committed window
// (status kDense) the stepper applies the next chunk of the batch in order
// from the window's end, then hands the batch back to the committer
// (status kNew at the chunk's end, kDone at the batch end).
#pragma once
#include <stdint.h>

namespace jb {
namespace vc {

enum : int { kNew = 0, kRetry = 1, kDone = 2, kDense = 3 };
// state words (int64 each, 512 B)
enum : int {
  S_MAGIC = 0, S_BEG, S_BEND, S_STATUS, S_LW, S_T, S_NCAND, S_PEND, S_WHY, S_NUPD, S_NSLOTS, S_VIOL,
  S_DONEB, S_NVALID, S_RETRYW, S_WEND,
  // batch counters
  S_WINDOWS, S_RETRIES, S_STEPS, S_ROUNDS, S_WASTED, S_REFRESH, S_EXACT, S_CAND, S_UPD, S_SAT, S_TICKS,
  S_NONC, S_PH0, S_PH1, S_PH2, S_PH3, S_PH4, S_PHW, S_WIDE, S_DENSE_PM,
  S_DCHUNK,    // samples of the next stepper chunk (doubles while windows stay dense)
  S_STEPPED,   // samples the stepper chunks applied in this batch
  S_NCHUNK,    // stepper chunks in this batch
  S_BBEG,      // the batch's first sample
  S_CSMODE,    // 1: this window's candidates are walked by the stepper (kernel B decides)
  S_CSN,       // windows the stepper walked in this batch
  S_NWORDS = 64
};
// committer stop reasons (S_WHY)
enum : int { kWhyEnd = 0, kWhySat = 1, kWhyDense = 2 };
// first stepper chunk after a dense window; chunks double up to kDenseChunkMax
constexpr int64_t kDenseChunk0 = 8192, kDenseChunkMax = 1 << 20;
// tail words (the batch's int64 x 32 diagnostics, jb_commit.hpp) the stepper
// chunks report through
constexpr int kTailStepped = 16, kTailChunks = 17, kTailSegEst = 18, kTailCsWindows = 19;
// tail[kTailReasonW]: the batch's stop reason (jb_commit.hpp dc::kTailReason / kStop*)
constexpr int kTailReasonW = 20;
constexpr int64_t kReasonDone = 0, kReasonSaturated = 1;

// Candidates on the stepper (JB_VC_CS / JB_VC_CS_PM, see vcommit.hip): an
// update-heavy window's candidates are walked by the sequential stepper instead of the
// one-wave committer C - in candidate order, from the model at the window's
// start, without writing W / P: its updated rows stay pinned in its LDS
// cache and are staged like C's store (keys, rmax, dW, dP) in the stepper's
// own slot layout, which kernel D then verifies against and commits.
constexpr int kSpSlotBytes = 98304;   // the stepper's W / P row cache
// the stepper's cache slots at label capacity lc (2-choice, 4-way buckets)
__host__ __device__ constexpr int sp_nslot(int lc) {
  return kSpSlotBytes / (8 * lc) > 1024 ? 1024 : kSpSlotBytes / (8 * lc);
}
// the stepper's two buckets of a row (nb buckets)
__device__ __forceinline__ void sp_buckets(int row, int nb, int* b1, int* b2) {
  const uint32_t h1 = (uint32_t)row * 0x9E3779B1u;
  uint32_t h2 = ((uint32_t)row ^ 0x5bd1e995u) * 0x85EBCA77u;
  h2 ^= h2 >> 13;
  h2 *= 0xC2B2AE35u;
  *b1 = (int)__umulhi(h1, (uint32_t)nb);
  int c = (int)__umulhi(h2, (uint32_t)nb);
  if (c == *b1) c = c + 1 == nb ? 0 : c + 1;
  *b2 = c;
}
// a row's slot in a stepper-layout key table (-1: absent)
__device__ __forceinline__ int sp_find(const int32_t* key, int nb, int32_t row) {
  if (row < 0) return -1;
  int b1, b2;
  sp_buckets(row, nb, &b1, &b2);
  const int4 k1 = reinterpret_cast<const int4*>(key)[b1];
  const int4 k2 = reinterpret_cast<const int4*>(key)[b2];
  int s = -1;
  s = k1.x == row ? 4 * b1 : s;
  s = k1.y == row ? 4 * b1 + 1 : s;
  s = k1.z == row ? 4 * b1 + 2 : s;
  s = k1.w == row ? 4 * b1 + 3 : s;
  s = k2.x == row ? 4 * b2 : s;
  s = k2.y == row ? 4 * b2 + 1 : s;
  s = k2.z == row ? 4 * b2 + 2 : s;
  s = k2.w == row ? 4 * b2 + 3 : s;
  return s;
}

// segments the batch would have used without stepper chunks (its windows and
// retries, plus the chunks' samples at the batch's mean committed window) -
// the next batch's segment budget (serial.hip): a batch that is sparse again
// after a dense one must not run out of segments
__device__ inline int64_t seg_estimate(const int64_t* st) {
  const int64_t wins = st[S_WINDOWS], stepped = st[S_STEPPED];
  const int64_t committed = st[S_BEG] - st[S_BBEG] - stepped;
  // (a dense batch's windows commit few samples each: at least 1024 a window,
  // or a worst-case batch would queue ~1500 empty segments for the next one)
  int64_t per = committed > 0 && wins > 0 ? committed / wins : 2048;
  per = per < 1024 ? 1024 : per;
  return wins + st[S_RETRIES] + (stepped + per - 1) / per;
}

}  // namespace vc
}  // namespace jb
