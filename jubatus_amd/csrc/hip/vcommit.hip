// Verified committer: the serial-equivalent training (update mode kSerial, the
// servers' default "exact") of a batch for label capacities up to 64. The
// result is that of applying the batch's samples one after the other in
// request order, as the reference's classifier does
// (jubatus/server/server/classifier_serv.cpp:138-144).
//
// Why a new committer (round 5). The delta committer (commit.hip) walks every
// sample of a batch through one 512-thread workgroup, 64 samples per round and
// a workgroup barrier per round and per step, although ~98 % of the samples
// never come near their update threshold. The host study of the bench stream
// (tools/exact_study.py over jb_cpu_serial.cpp) shows that a sample's slack at
// the segment start almost always exceeds the bound on what the segment's
// updates can move its margin: with T = 0.5, ~6 % of a window are candidates
// and the final bound clears every other sample. So:
//
//   A vc_score_kernel   (whole GPU, one wave per sample) scores the window
//                       [beg, beg + lw) against the model M0 (W / P, which
//                       nothing writes until the window is verified): the
//                       slack of every sample to its update threshold, and a
//                       candidate bit for every slack <= T.
//   B vc_gather_kernel  (whole GPU, one wave per candidate) writes the
//                       candidates' records in candidate order (rank = prefix
//                       count of the bits): S0 scores, labels, |x|^2, slack,
//                       window position, features and their P0 precisions.
//   C vc_commit_kernel  (ONE wave, no barriers) walks only the candidates in
//                       order, 16 per round (4 DPP rows x 4 samples), and keeps
//                       everything the window writes in an LDS row store
//                       (dc:: 2-choice buckets): exact scores are S0 + x . dW,
//                       a step's increments go to the store, and every later
//                       candidate of the round gets the step's correction from
//                       the stamped rows. Candidate scores stay lazy under the
//                       bounded slack (2 sum_f |x_f| rmax_f), as in commit.hip.
//                       The store, the per-row bound rmax and the stop
//                       position are staged to global memory.
//   D vc_verify_kernel  (whole GPU, one thread per sample) proves that no
//                       non-candidate of [beg, stop) could have updated: its
//                       slack at M0 must exceed 2 sum_f |x_f| rmax_f with the
//                       FINAL rmax of the window (an upper bound on the bound
//                       at its own position). The last block then either
//                       commits the window (W / P += staged deltas, the next
//                       window starts at the stop) or, if some sample is not
//                       cleared, marks it a candidate and the window runs
//                       again (C and D; A is skipped, M0 did not change) with a
//                       higher T for the windows after.
//
// The window ends where the committer stops: at its end, when the LDS store is
// full (the next window re-scores from there), or at a candidate wider than 32
// features. Such a window, and one whose updates were dense (JB_VC_DENSE_PM),
// hands the next chunk of the batch to the sequential stepper (stepper.hip,
// launched after every segment, empty unless the status says kDense); the
// next segment continues after the chunk. Chunks double while the windows
// between them stay dense. Windows adapt their length to where the store
// fills. Decisions follow commit.hip's guard band (a margin within 1e-4 of its
// threshold is re-scored from the live model M0 + dW before the decision).
//
// Device state (int64 words, 512 B) lives in the kSerial scratch; every kernel
// reads the status first, so a batch's segments are queued without a host round
// trip and the finished ones cost an empty launch each.
#include <string.h>

#include <type_traits>

#include "jb_commit.hpp"
#include "jb_vc_state.hpp"

namespace jb {
namespace vc {

using dc::Geo;
constexpr int kFCMax = 2;               // feature chunks of 16 per lane (a sample of <= 32 features)
constexpr int kRec = 16 * kFCMax;       // feature slots of a candidate record
constexpr int64_t kLwMin = 2048, kLwMax = 65536, kLwInit = 8192;
constexpr int kBitWords = (int)(kLwMax / 64);
// candidate rule (kernel A): slack0 <= T, T adapting (x1.5 on a
// verification failure, x0.97 per committed window, >= kTMin). Measured on
// the bench stream (tools/exact_study.py rules_w8192): at 0.125 the final
// bound clears every other sample of a window; a rule predicting each
// sample's bound from the previous window's row steps cuts candidates by
// ~40 % but fails verification ~once a window, and a failed window runs its
// committer again (costlier than the rounds saved).
constexpr float kTInit = 0.5f, kTMin = 0.125f, kTMax = 64.f;
constexpr int64_t kMagic = 0x56434f4d4d495433LL;
constexpr int kRetryForce = 3;          // retries of one window before all its samples are candidates
// (status, state words and stop reasons: jb_vc_state.hpp, shared with the stepper)
static_assert(kTailReasonW == dc::kTailReason && kReasonDone == dc::kStopDone &&
                  kReasonSaturated == dc::kStopSaturated,
              "jb_vc_state.hpp mirrors jb_commit.hpp's tail words");

__device__ __forceinline__ float st_T(const int64_t* st) { return __int_as_float((int)st[S_T]); }
__device__ __forceinline__ int64_t ld_st(const int64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool live(int status) { return status == kNew || status == kRetry; }

// The committer's arithmetic with hardware reciprocals (v_rcp_f32, 1 ulp)
// instead of IEEE divisions (a ten-instruction sequence each): a one-wave
// step is instruction-bound (4 cycles per wave64 VALU op). Same formulas as
// jb_linear.hpp step_coeffs / dprec; the guard band (1e-4 relative) absorbs
// the ulp, and the oracle comparisons hold at rtol 2e-3.
__device__ __forceinline__ float frcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ bool step_coeffs_fast(int method, float margin, float var, float nrm, bool has_l, float C,
                                                 float* tau, float* beta) {
  switch (method) {
    case PERCEPTRON:
      if (margin <= 0.f) { *tau = 1.f; *beta = 0.f; return true; }
      return false;
    case PA: case PA1: case PA2: {
      const float loss = 1.f - margin;
      if (!(loss > 0.f && nrm > 0.f)) return false;
      const float sq = (has_l ? 2.f : 1.f) * nrm;
      if (method == PA) *tau = loss * frcp(sq);
      else if (method == PA1) *tau = fminf(C, loss * frcp(sq));
      else *tau = loss * frcp(sq + 0.5f * frcp(C));
      *beta = 0.f;
      return true;
    }
    case CW: {
      if (!(var > 0.f)) return false;
      const float phi = C;
      const float b = 1.f + 2.f * phi * margin;
      const float disc = b * b - 8.f * phi * (margin - phi * var);
      const float gamma = (-b + sqrtf(fmaxf(disc, 0.f))) * frcp(4.f * phi * var);
      if (!(gamma > 0.f)) return false;
      *tau = gamma; *beta = 2.f * gamma * phi;
      return true;
    }
    case AROW:
      if (!(margin < 1.f)) return false;
      *beta = frcp(var + frcp(C));
      *tau = (1.f - margin) * *beta;
      return true;
    case NHERD: {
      if (!(margin < 1.f)) return false;
      *tau = (1.f - margin) * frcp(var + frcp(C));
      const float cv = 1.f + C * var;
      *beta = (C * C * var + 2.f * C) * frcp(cv * cv);
      return true;
    }
    default: return false;
  }
}
__device__ __forceinline__ float dprec_fast(int method, float beta, float x, float s) {
  const float bx2 = beta * x * x;
  return method == CW ? bx2 : bx2 * frcp(1.f - bx2 * s);
}

// ------------------------------------------------------------ init
// per batch: the range, the status, zero candidate bits; the window length and
// T persist across batches on the same scratch (a model's stream)
__global__ __launch_bounds__(256) void vc_init_kernel(int64_t* __restrict__ st, const int64_t* __restrict__ sp,
                                                      int nstreams, unsigned long long* __restrict__ bits,
                                                      int64_t* __restrict__ tail, float t_force,
                                                      int32_t* __restrict__ g_key, float* __restrict__ g_rmax,
                                                      int dense_pm) {
  for (int i = threadIdx.x; i < kBitWords; i += blockDim.x) bits[i] = 0ull;
  const bool fresh = st[S_MAGIC] != kMagic;
  if (fresh)      // no previous window: the candidate rule's row bounds are empty
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) { g_key[i] = -1; g_rmax[i] = 0.f; }
  __syncthreads();
  if (threadIdx.x != 0) return;
  if (fresh) {
    for (int i = 0; i < S_NWORDS; ++i) st[i] = 0;
    st[S_MAGIC] = kMagic;
    st[S_LW] = kLwInit;
    st[S_T] = __float_as_int(kTInit);
  }
  if (t_force > 0.f) st[S_T] = __float_as_int(t_force);
  const int64_t beg = sp[0], bend = sp[nstreams];
  st[S_BEG] = beg;
  st[S_BEND] = bend;
  st[S_WEND] = beg;
  st[S_STATUS] = beg < bend ? kNew : kDone;
  for (int i = S_NCAND; i <= S_RETRYW; ++i) st[i] = 0;
  for (int i = S_WINDOWS; i < S_NWORDS; ++i) st[i] = 0;
  st[S_DENSE_PM] = dense_pm;
  st[S_DCHUNK] = kDenseChunk0;
  st[S_BBEG] = beg;
  for (int i = 0; i < 32; ++i) tail[i] = 0;
  tail[0] = beg < bend ? beg : bend;
  tail[1] = bend;
  tail[31] = 1;    // marker: the verified committer ran this batch
}

// ------------------------------------------------------------ A: score + candidate bits
// one wave per sample (lanes as Lanes<LC>, as delta_s0_kernel)
template <int LC>
__device__ __forceinline__ void wave_score(const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
                                           const float* __restrict__ fval, const float* __restrict__ W,
                                           int64_t s, int lane, bool la, int* n_out, float* acc_out,
                                           float* q_out) {
  using L = Lanes<LC>;
  const int g = lane / L::LW;
  const int l0 = lane % L::LW;
  const int64_t fb = row_ptr[s];
  const int n = (int)(row_ptr[s + 1] - fb);
  float acc = 0.f;
  for (int j = g; j < n; j += L::G) {
    const int32_t idx = fidx[fb + j];
    if (idx >= 0) acc += fval[fb + j] * W[(int64_t)idx * LC + l0];
  }
#pragma unroll
  for (int off = L::LW; off < 64; off <<= 1) acc += __shfl_xor(acc, off, 64);
  float q = 0.f;
  for (int j = lane; j < n; j += 64) {
    const float x = fval[fb + j];
    q += x * x;
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) q += __shfl_xor(q, off, 64);
  (void)la;
  *n_out = n;
  *acc_out = acc;
  *q_out = q;
}

// best active wrong label over the lanes of one label group, the margin at M0
// and its slack (dc::slack_of); y must be a valid label
template <int LC>
__device__ __forceinline__ float wave_slack(float acc, int y, bool la, int lane, int method, float C,
                                            float q, int* bl_out) {
  using L = Lanes<LC>;
  const int l0 = lane % L::LW;
  float b = (la && l0 != y) ? acc : -INFINITY;
  int bl = (la && l0 != y) ? l0 : -1;
#pragma unroll
  for (int off = 1; off < L::LW; off <<= 1) {
    const float ob = __shfl_xor(b, off, 64);
    const int ol = __shfl_xor(bl, off, 64);
    if (ol >= 0 && (bl < 0 || ob > b || (ob == b && ol < bl))) { b = ob; bl = ol; }
  }
  const float sy = __shfl(acc, y, 64);
  const float best = bl >= 0 ? b : 0.f;
  *bl_out = bl;
  return dc::slack_of(method, sy - best, q, bl >= 0, C, sy, best);
}

template <int LC>
__global__ __launch_bounds__(256) void vc_score_kernel(
    const int64_t* __restrict__ st, const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels, const float* __restrict__ W,
    const int32_t* __restrict__ active, int method, float C, float* __restrict__ SL,
    unsigned long long* __restrict__ bits, const int32_t* __restrict__ g_key, const float* __restrict__ g_rmax) {
  using L = Lanes<LC>;
  static_assert(LC <= 64, "verified committer: LC <= 64");
  if (st[S_STATUS] != kNew) return;
  (void)g_key;
  (void)g_rmax;
  const int lane = threadIdx.x & 63;
  const int64_t beg = st[S_BEG], bend = st[S_BEND];
  const int64_t lw = st[S_LW];
  const float T = st_T(st);
  const int64_t cnt = (beg + lw < bend ? beg + lw : bend) - beg;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int l0 = lane % L::LW;
  const bool la = l0 < LC && active[l0] != 0;
  for (int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; wid < cnt; wid += nwaves) {
    const int64_t s = beg + wid;
    int n;
    float acc, q;
    wave_score<LC>(row_ptr, fidx, fval, W, s, lane, la, &n, &acc, &q);
    const int y = labels[s];
    if (y < 0 || y >= LC) {
      if (lane == 0) SL[wid] = INFINITY;
      continue;
    }
    int bl;
    const float sl0 = wave_slack<LC>(acc, y, la, lane, method, C, q, &bl);
    if (lane == 0) {
      SL[wid] = sl0;
      if (!(sl0 > T)) atomicOr(bits + (wid >> 6), 1ull << (wid & 63));
    }
  }
}

// ------------------------------------------------------------ B: candidate records
// record k (the k-th candidate of the window): S0[k * LC + l], AUX[k] = (labels
// and feature count, |x|^2, slack at M0, position in the window), FI / FX[k * 32
// + f], PP0[k * 32 + f] = (P0(row_f, y), P0(row_f, best wrong label at M0))
template <int LC>
__global__ __launch_bounds__(256) void vc_gather_kernel(
    int64_t* __restrict__ st, const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels, const float* __restrict__ W,
    const float* __restrict__ P, const int32_t* __restrict__ active, int method, float C,
    const unsigned long long* __restrict__ bits, float* __restrict__ S0, int4* __restrict__ AUX,
    float2* __restrict__ PP0, int32_t* __restrict__ FI, float* __restrict__ FX, int cs_min, int cs_pm) {
  using L = Lanes<LC>;
  if (!live((int)st[S_STATUS])) return;
  __shared__ int s_pref[kBitWords + 1];
  __shared__ int s_wsum[4];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int64_t beg = st[S_BEG], bend = st[S_BEND], lw = st[S_LW];
  const int64_t we = beg + lw < bend ? beg + lw : bend;
  const int nw = (int)((we - beg + 63) >> 6);
  // exclusive prefix of the words' popcounts (each thread 4 consecutive words)
  int c[4], tot = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int w = 4 * tid + j;
    c[j] = w < nw ? __popcll(bits[w]) : 0;
    tot += c[j];
  }
  int incl = tot;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int o = __shfl_up(incl, off, 64);
    if (lane >= off) incl += o;
  }
  if (lane == 63) s_wsum[tid >> 6] = incl;
  __syncthreads();
  int base = 0;
  for (int w = 0; w < (tid >> 6); ++w) base += s_wsum[w];
  int run = base + incl - tot;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s_pref[4 * tid + j] = run;
    run += c[j];
  }
  if (tid == 255) s_pref[kBitWords] = run;
  __syncthreads();
  const int ncand = s_pref[kBitWords];
  if (blockIdx.x == 0 && tid == 0) {
    // the stepper walks the candidates (stepper.hip, candidate mode) when
    // there are enough and the last window updated on more than cs_pm per
    // mille of its candidates: kernel C pays ~2.3 us an update and little for
    // the rest, the stepper ~0.8 us a candidate either way
    const int64_t pn = st[S_NCAND], pu = st[S_NUPD];
    st[S_CSMODE] = (cs_min > 0 && ncand >= cs_min && pu * 1000 >= (int64_t)cs_pm * (pn > 0 ? pn : 1)) ? 1 : 0;
    st[S_NCAND] = ncand;
    st[S_WEND] = we;
  }
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int g = lane / L::LW;
  const int l0 = lane % L::LW;
  const bool la = l0 < LC && active[l0] != 0;
  for (int64_t k = ((int64_t)blockIdx.x * blockDim.x + tid) >> 6; k < ncand; k += nwaves) {
    // the word holding candidate k (largest w with s_pref[w] <= k), then its bit
    int lo = 0, hi = nw - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_pref[mid] <= k) lo = mid; else hi = mid - 1;
    }
    unsigned long long word = bits[lo];
    for (int j = (int)k - s_pref[lo]; j > 0; --j) word &= word - 1;
    const int pos = 64 * lo + (__ffsll((long long)word) - 1);
    const int64_t s = beg + pos;
    int n;
    float acc, q;
    wave_score<LC>(row_ptr, fidx, fval, W, s, lane, la, &n, &acc, &q);
    const int64_t fb = row_ptr[s];
    if (lane < kRec) {
      const bool in = lane < n;
      FI[k * kRec + lane] = in ? fidx[fb + lane] : -1;
      FX[k * kRec + lane] = in ? fval[fb + lane] : 0.f;
    }
    if (lane == 0 && n > 16) atomicOr((unsigned long long*)&st[S_WIDE], 1ull);
    if (lane < LC) S0[k * LC + lane] = acc;
    (void)g;
    const int y = labels[s];
    if (y < 0 || y >= LC) {      // (a window forced whole after repeated retries)
      if (lane == 0) AUX[k] = make_int4(dc::aux_pack(-1, -1, n), __float_as_int(q), __float_as_int(1.f), pos);
      continue;
    }
    int bl;
    const float sl0 = wave_slack<LC>(acc, y, la, lane, method, C, q, &bl);
    if (lane == 0) AUX[k] = make_int4(dc::aux_pack(y, bl, n), __float_as_int(q), __float_as_int(sl0), pos);
    if (P == nullptr) continue;
    if (lane < kRec) {
      float2 pp = make_float2(1.f, 1.f);
      if (lane < n) {
        const int32_t idx = fidx[fb + lane];
        if (idx >= 0) {
          pp.x = P[(int64_t)idx * LC + y];
          if (bl >= 0) pp.y = P[(int64_t)idx * LC + bl];
        }
      }
      PP0[k * kRec + lane] = pp;
    }
  }
}

// ------------------------------------------------------------ C: the committer
template <int LC, int FC>
struct Raw {
  int32_t fi[FC];
  float fx[FC];
  float2 pp[FC];
  float s[Geo<LC>::K];
  int aux;
  float nrm;
  float slack0;
  int pos;
};

template <int LC, int FC>
struct Samp {
  int32_t fi[FC];
  float fx[FC];
  float py[FC];    // P0(row, y), P0(row, best wrong label at M0)
  float pl[FC];
  float s[Geo<LC>::K];
  int y;           // -1: no candidate / label out of range
  int ls0;
  int nf;
  float nrm;
  float slack0;
  int pos;
};

// stamp of a store row (one b128 read): id of the last step that wrote it (int
// bits), that step's increments of its labels y / l*, and rmax - a bound on
// max_l |dW[row][l]| (the summed step magnitudes)
struct __attribute__((aligned(16))) Stamp { float sid, dy, dl, rmax; };

template <int LC, int MT, int R_, int PD_, int FC_>
__global__ __launch_bounds__(64) void vc_commit_kernel(
    int64_t* __restrict__ st, const float* __restrict__ W, const float* __restrict__ P,
    const int32_t* __restrict__ active, float C, const float* __restrict__ S0_k,
    const int4* __restrict__ AUX_k, const float2* __restrict__ PP0_k, const int32_t* __restrict__ FI_k,
    const float* __restrict__ FX_k, int32_t* __restrict__ g_key, float* __restrict__ g_rmax,
    float* __restrict__ g_dw, float* __restrict__ g_dp, int prof) {
  using Gm = Geo<LC>;
  using Rw = Raw<LC, FC_>;
  using S = Samp<LC, FC_>;
  // FC_ feature chunks of 16 per lane: 1 when no candidate of the window has
  // more than 16 features (kernel B's wide flag), else 2
  constexpr int kFC = FC_;
  constexpr int kNFM = 16 * FC_;
  // R_ samples per group and round, PD_ rounds of records in flight: the code
  // of a round is instantiated R_ x PD_ times (the instruction cache decides)
  constexpr int kR = R_;
  constexpr int kNS = 4 * R_;
  constexpr int kPD = PD_;
  constexpr int K = Gm::K;
  constexpr int NSLOT = Gm::NSLOT;
  constexpr int method = MT;
  constexpr bool use_s = MT >= CW;
  constexpr bool use_nrm = MT == PA || MT == PA1 || MT == PA2 || MT == CW;
  constexpr float kG = dc::kGuard;
  if (!live((int)st[S_STATUS])) return;
  if (st[S_CSMODE] == 1) return;   // (the stepper walks this window's candidates)
  if ((st[S_WIDE] != 0) != (FC_ == 2)) return;
  __shared__ __attribute__((aligned(16))) float s_dw[NSLOT * LC + Gm::PAD];
  __shared__ __attribute__((aligned(16))) float s_dp[use_s ? NSLOT * LC + Gm::PAD : 4];
  __shared__ __attribute__((aligned(16))) int32_t s_key[NSLOT];
  __shared__ __attribute__((aligned(16))) Stamp s_sg[NSLOT + 1];

  const int lane = threadIdx.x;
  const int sub = lane & 15;
  const int G = lane >> 4;
  const uint64_t t_k0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t t_c0 = __builtin_amdgcn_s_memtime();
  {
    float4* dw4 = reinterpret_cast<float4*>(s_dw);
    float4* dp4 = reinterpret_cast<float4*>(s_dp);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = lane; i < (NSLOT * LC + Gm::PAD) / 4; i += 64) {
      dw4[i] = z;
      if (use_s) dp4[i] = z;
    }
    for (int i = lane; i < NSLOT; i += 64) s_key[i] = -1;
    for (int i = lane; i <= NSLOT; i += 64) s_sg[i] = Stamp{__int_as_float(-1), 0.f, 0.f, 0.f};
  }
  int act[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int lab = sub + 16 * k;
    act[k] = (lab < LC && active[lab] != 0) ? 1 : 0;
  }
  const int64_t ncand = (int64_t)dc::in_vgpr((uint64_t)st[S_NCAND]);
  const int64_t wb = (int64_t)dc::in_vgpr((uint64_t)st[S_BEG]);
  const int64_t we = (int64_t)dc::in_vgpr((uint64_t)st[S_WEND]);
  const float* __restrict__ S0 = dc::in_vgpr(S0_k);
  const int4* __restrict__ AUX = dc::in_vgpr(AUX_k);
  const float2* __restrict__ PP0 = dc::in_vgpr(PP0_k);
  const int32_t* __restrict__ FI = dc::in_vgpr(FI_k);
  const float* __restrict__ FX = dc::in_vgpr(FX_k);

  // records kPD rounds ahead, at addresses of the candidate index alone; past
  // the last candidate a lane re-reads the last record (the round masks it)
  auto load_raw = [&](int64_t k0, Rw (&rw)[kR]) {
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      int64_t j = k0 + G * kR + r;
      j = j < ncand ? j : ncand - 1;
      j = j < 0 ? 0 : j;
#pragma unroll
      for (int c = 0; c < kFC; ++c) {
        const int64_t o = j * kRec + c * 16 + sub;
        rw[r].fi[c] = dc::gld(FI + o);
        rw[r].fx[c] = dc::gld(FX + o);
        if (use_s) rw[r].pp[c] = dc::gld(PP0 + o);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int lab = sub + 16 * k;
        rw[r].s[k] = dc::gld(S0 + j * LC + (lab < LC ? lab : LC - 1));
      }
      const int* a = reinterpret_cast<const int*>(AUX + j);
      rw[r].aux = dc::gld(a);
      rw[r].slack0 = __int_as_float(dc::gld(a + 2));
      rw[r].pos = dc::gld(a + 3);
      if (use_nrm) rw[r].nrm = __int_as_float(dc::gld(a + 1));
    }
  };
  auto unpack = [&](int64_t k0, const Rw (&rw)[kR], S (&sm)[kR]) {
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const bool ok = k0 + G * kR + r < ncand;
#pragma unroll
      for (int c = 0; c < kFC; ++c) {
        sm[r].fi[c] = ok ? rw[r].fi[c] : -1;
        sm[r].fx[c] = ok ? rw[r].fx[c] : 0.f;
        sm[r].py[c] = (use_s && ok) ? rw[r].pp[c].x : 1.f;
        sm[r].pl[c] = (use_s && ok) ? rw[r].pp[c].y : 1.f;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) sm[r].s[k] = (ok && sub + 16 * k < LC) ? rw[r].s[k] : 0.f;
      const int aux = rw[r].aux;
      sm[r].y = ok ? dc::aux_y(aux) : -1;
      sm[r].ls0 = (use_s && ok) ? dc::aux_ls(aux) : -1;
      sm[r].nf = ok ? dc::aux_nf(aux) : 0;
      sm[r].nrm = (use_nrm && ok) ? rw[r].nrm : 0.f;
      sm[r].slack0 = ok ? rw[r].slack0 : 1.f;
      sm[r].pos = rw[r].pos;
    }
  };

  S sc[kR];
  Rw pf[kPD][kR];
#pragma unroll
  for (int i = 0; i < kPD; ++i) load_raw((int64_t)i * kNS, pf[i]);

  int stopped = 0;            // wave-uniform
  int64_t pend = we;
  int why = kWhyEnd;
  // the step id stays in a register; the other counters live in LDS (lane 0
  // adds), which keeps them out of the SGPR file (a spilled SGPR costs a
  // v_writelane / v_readlane pair at every use)
  int n_steps = 0, n_exact = 0;
  __shared__ int s_cnt[4];                 // updates, wasted steps, refreshes, rounds
  __shared__ unsigned long long s_ph[5];   // phase cycles (prof)
  if (lane < 4) s_cnt[lane] = 0;
  if (lane < 5) s_ph[lane] = 0;
  auto bump = [&](int i) __attribute__((always_inline)) {
    if (lane == 0) s_cnt[i] += 1;
  };
  const uint64_t kLead = 0x0001000100010001ull;   // lane 0 of each DPP row

  // phase stamps (prof, JB_COMMIT_PROF=1: shader cycles summed per phase -
  // round start, step selection, decision, apply, corrections; each stamp
  // waits for the LDS operations in flight, so they cost a little)
  const bool kProf = prof != 0;

  uint64_t tp = kProf ? __builtin_amdgcn_s_memtime() : 0;
  auto stamp = [&](int i) __attribute__((always_inline)) {
    if (!kProf) return;
    const uint64_t t = __builtin_amdgcn_s_memtime();
    if (lane == 0) s_ph[i] += t - tp;
    tp = t;
  };
  auto round = [&](int64_t k0) __attribute__((always_inline)) {
    int alive[kR], unsafe[kR], exact[kR];
    float slack[kR];
    int slot[kR][kFC];
    bool widew = false;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      alive[r] = (sc[r].y >= 0 && sc[r].y < LC) ? 1 : 0;
      widew |= alive[r] && sc[r].nf > 16;
    }
    const bool two = kFC == 2 && __builtin_amdgcn_ballot_w64(widew) != 0;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const bool ok = alive[r] && sc[r].nf <= kNFM;
      slot[r][0] = ok ? dc::cache_find<LC>(s_key, sc[r].fi[0]) : -1;
      if (kFC == 2) slot[r][kFC - 1] = (two && ok) ? dc::cache_find<LC>(s_key, sc[r].fi[kFC - 1]) : -1;
    }
    // samples of the round whose slack ran out (positions > after): exact
    // scores S0 + x . dW against the live store, exact margin and slack
    auto make_exact = [&](int after) {
      bool need[kR];
      bool anyneed = false;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        need[r] = alive[r] && !exact[r] && sc[r].nf <= kNFM && G * kR + r > after && !(slack[r] > 0.f);
        anyneed |= need[r];
      }
      if (__builtin_amdgcn_ballot_w64(anyneed) == 0) return;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        if (__builtin_amdgcn_ballot_w64(need[r]) == 0) continue;
        float t[K];
#pragma unroll
        for (int k = 0; k < K; ++k) t[k] = sc[r].s[k];
        dc::row_correct<LC, kFC>(s_dw, slot[r], sc[r].fx, sub, two, t);
        int ls;
        float sy, best;
        const float m = dc::group_margin<LC>(t, sc[r].y, act, sub, &ls, &sy, &best);
        const float sl = dc::slack_of(method, m, sc[r].nrm, ls >= 0, C, sy, best);
        if (need[r]) {
#pragma unroll
          for (int k = 0; k < K; ++k) sc[r].s[k] = t[k];
          slack[r] = sl;
          exact[r] = 1;
          if (sub == 0) ++n_exact;
        }
      }
    };
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      float bsum = 0.f;
#pragma unroll
      for (int c = 0; c < kFC; ++c)
        bsum += slot[r][c] >= 0 ? fabsf(sc[r].fx[c]) * s_sg[slot[r][c]].rmax : 0.f;
      slack[r] = sc[r].slack0 - 2.f * (1.f + 4.f * kG) * row16_sum(bsum);
      exact[r] = 0;
    }
    make_exact(-1);
    stamp(0);
#pragma unroll
    for (int r = 0; r < kR; ++r) unsafe[r] = (alive[r] && (sc[r].nf > kNFM || !(slack[r] > 0.f))) ? 1 : 0;

    int lim = -1;
    for (;;) {
      // the first position > lim that may update (wave-uniform)
      int k = dc::kInf;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        const uint64_t b = __builtin_amdgcn_ballot_w64(unsafe[r] && G * kR + r > lim) & kLead;
        if (b != 0) {
          const int gk = (__ffsll((long long)b) - 1) >> 4;
          k = min(k, gk * kR + r);
        }
      }
      stamp(1);
      if (k == dc::kInf) break;
      const int Gk = k / kR, rk = k % kR;
      (void)rk;
      const bool mine = G == Gk;
      // the step of sample k, with its round slot a compile-time index (a
      // runtime one puts the samples in scratch memory: a load that drains
      // every prefetch in flight)
      auto step_of = [&](auto RKc) __attribute__((always_inline)) -> int {
        constexpr int rk = decltype(RKc)::value;
        S t = sc[rk];
        int sl[kFC];
#pragma unroll
        for (int c = 0; c < kFC; ++c) sl[c] = slot[rk][c];
        const int kpos = __builtin_amdgcn_readlane(t.pos, Gk * 16);
        const int knf = __builtin_amdgcn_readlane(t.nf, Gk * 16);
        if (knf > kNFM) {
          stopped = 1;
          why = kWhyDense;
          pend = wb + kpos;
          return 1;
        }
        const int y = t.y;
        int ls = -1;
        float m = 0.f, sy = 0.f, best = 0.f, var = 0.f;
        float py[kFC], pl[kFC];
        bool refreshed = false;
        for (;;) {
          m = dc::group_margin<LC>(t.s, y, act, sub, &ls, &sy, &best);
          // P0 of the best wrong label: prefetched for the one at M0; another
          // one is read from the table behind a wave-uniform branch (a
          // conditional load the compiler joins waits for every load in flight)
          float p0l[kFC];
#pragma unroll
          for (int c = 0; c < kFC; ++c) p0l[c] = t.pl[c];
          if (use_s && __builtin_amdgcn_ballot_w64(mine && ls >= 0 && ls != t.ls0) != 0) {
            // scalar loads at the group's (uniform) rows: they count on
            // lgkmcnt, so waiting for them does not wait for the prefetches
            const int lsu = __builtin_amdgcn_readlane(ls, Gk * 16);
#pragma unroll
            for (int c = 0; c < kFC; ++c) {
              if (c > 0 && !two) break;
              for (int u = 0; u < 16; ++u) {
                const int ru = __builtin_amdgcn_readlane(t.fi[c], Gk * 16 + u);
                if (ru < 0) continue;
                const float pv = P[(int64_t)ru * LC + lsu];
                p0l[c] = sub == u ? pv : p0l[c];
              }
            }
          }
          float v = 0.f;
#pragma unroll
          for (int c = 0; c < kFC; ++c) {
            py[c] = 1.f;
            pl[c] = 1.f;
            const int32_t row = t.fi[c];
            if (!use_s || row < 0) continue;
            const float* dpr = s_dp + (sl[c] >= 0 ? sl[c] : NSLOT) * LC;
            py[c] = t.py[c] + dpr[y];
            if (ls >= 0) pl[c] = p0l[c] + dpr[ls];
            const float x2 = t.fx[c] * t.fx[c];
            v += x2 * (frcp(py[c]) + (ls >= 0 ? frcp(pl[c]) : 0.f));
          }
          var = use_s ? row16_sum(v) : 0.f;
          if (refreshed) break;
          const float thr = method == PERCEPTRON ? 0.f : method == CW ? C * var : 1.f;
          const float g = kG * (1.f + fabsf(sy) + fabsf(best));
          if (__builtin_amdgcn_ballot_w64(mine && fabsf(m - thr) < g) == 0) break;
          // near the threshold: re-score from the live model (M0 + dW)
          refreshed = true;
          bump(2);
          float ns[K];
#pragma unroll
          for (int kk = 0; kk < K; ++kk) ns[kk] = 0.f;
#pragma unroll
          for (int c = 0; c < kFC; ++c) {
#pragma unroll 1
            for (int u = 0; u < 16; ++u) {
              const int32_t ru = __shfl(t.fi[c], (lane & 48) + u, 64);
              const float xu = __shfl(t.fx[c], (lane & 48) + u, 64);
              const int su0 = __shfl(sl[c], (lane & 48) + u, 64);
              const int su = su0 >= 0 ? su0 : NSLOT;
              if (ru < 0) continue;
#pragma unroll
              for (int kk = 0; kk < K; ++kk) {
                const int lab = sub + 16 * kk;
                if (lab < LC) ns[kk] += xu * (W[(int64_t)ru * LC + lab] + s_dw[su * LC + lab]);
              }
            }
          }
#pragma unroll
          for (int kk = 0; kk < K; ++kk) t.s[kk] = ns[kk];
        }
        float tau = 0.f, beta = 0.f;
        const bool up_l = step_coeffs_fast(method, m, var, t.nrm, ls >= 0, C, &tau, &beta);
        const bool up = __builtin_amdgcn_ballot_w64(mine && up_l) != 0;
        stamp(2);
        const int sid = n_steps++;
        if (!up) {
          bump(1);
        } else {
          // the sample's rows not in the store yet; a full bucket pair ends the
          // window before this candidate (nothing of its step is applied)
          bool full = false;
          bool any_new = false;
#pragma unroll
          for (int c = 0; c < kFC; ++c) {
            const bool need = mine && t.fi[c] >= 0 && sl[c] < 0;
            any_new |= need;
            if (need) {
              sl[c] = dc::cache_insert<LC>(s_key, t.fi[c]);
              full |= sl[c] < 0;
            }
          }
          if (__builtin_amdgcn_ballot_w64(full) != 0) {
            stopped = 1;
            why = kWhySat;
            pend = wb + kpos;
            return 1;
          }
          const bool nins = __builtin_amdgcn_ballot_w64(any_new) != 0;
          bump(0);
          if (mine) {
#pragma unroll
            for (int c = 0; c < kFC; ++c)
              if (t.fi[c] >= 0) {
                float* sg = reinterpret_cast<float*>(&s_sg[sl[c]]);
                sg[0] = __int_as_float(sid);
                sg[1] = 0.f;
                sg[2] = 0.f;
              }
#pragma unroll
            for (int c = 0; c < kFC; ++c) {
              if (t.fi[c] < 0) continue;
              const float x = t.fx[c];
              const float a = use_s ? frcp(py[c]) : 1.f;
              const float b = (use_s && ls >= 0) ? frcp(pl[c]) : 1.f;
              const float dwy = tau * a * x;
              const float dwl = ls >= 0 ? -tau * b * x : 0.f;
              float* dwr = s_dw + sl[c] * LC;
              atomicAdd(dwr + y, dwy);
              if (ls >= 0) atomicAdd(dwr + ls, dwl);
              if (use_s) {
                float* dpr = s_dp + sl[c] * LC;
                atomicAdd(dpr + y, dprec_fast(method, beta, x, a));
                if (ls >= 0) atomicAdd(dpr + ls, dprec_fast(method, beta, x, b));
              }
              float* sg = reinterpret_cast<float*>(&s_sg[sl[c]]);
              atomicAdd(sg + 1, dwy);
              atomicAdd(sg + 2, dwl);
              atomicAdd(sg + 3, fmaxf(fabsf(dwy), fabsf(dwl)));
            }
          }
          // the later samples of the round: slots of the rows the step added,
          // then the step's increments of their stamped rows
          stamp(3);
          const int yk = __builtin_amdgcn_readlane(y, Gk * 16);
          const int lk = __builtin_amdgcn_readlane(ls, Gk * 16);
          if (nins) {
#pragma unroll
            for (int r = 0; r < kR; ++r) {
              if (G * kR + r <= k || !alive[r]) continue;
#pragma unroll
              for (int c = 0; c < kFC; ++c)
                if ((c == 0 || two) && slot[r][c] < 0 && sc[r].fi[c] >= 0)
                  slot[r][c] = dc::cache_find<LC>(s_key, sc[r].fi[c]);
            }
          }
#pragma unroll
          for (int r = 0; r < kR; ++r) {
            const int pos = G * kR + r;
            if (!alive[r] || pos <= k || sc[r].nf > kNFM) continue;
            float cy = 0.f, cl = 0.f;
#pragma unroll
            for (int c = 0; c < kFC; ++c) {
              const int s = slot[r][c];
              if (s >= 0) {
                const Stamp sg = s_sg[s];
                if (__float_as_int(sg.sid) == sid) {
                  cy += sc[r].fx[c] * sg.dy;
                  cl += sc[r].fx[c] * sg.dl;
                }
              }
            }
            cy = row16_sum(cy);
            cl = row16_sum(cl);
            if (exact[r]) {
#pragma unroll
              for (int kk = 0; kk < K; ++kk) {
                const int lab = sub + 16 * kk;
                if (lab == yk) sc[r].s[kk] += cy;
                if (lab == lk) sc[r].s[kk] += cl;
              }
            }
            slack[r] -= (fabsf(cy) + fabsf(cl)) * (1.f + 4.f * kG);
            if (exact[r] && !(slack[r] > 0.f)) {
              int ls2;
              float sy2, best2;
              const float m2 = dc::group_margin<LC>(sc[r].s, sc[r].y, act, sub, &ls2, &sy2, &best2);
              slack[r] = dc::slack_of(method, m2, sc[r].nrm, ls2 >= 0, C, sy2, best2);
            }
          }
          make_exact(k);
#pragma unroll
          for (int r = 0; r < kR; ++r)
            if (G * kR + r > k) unsafe[r] = (alive[r] && (sc[r].nf > kNFM || !(slack[r] > 0.f))) ? 1 : 0;
        }
        return 0;
      };
      int stop_code = 0;
      switch (rk) {
        case 0: stop_code = step_of(std::integral_constant<int, 0>{}); break;
        case 1: if constexpr (kR > 1) stop_code = step_of(std::integral_constant<int, (kR > 1 ? 1 : 0)>{}); break;
        case 2: if constexpr (kR > 2) stop_code = step_of(std::integral_constant<int, (kR > 2 ? 2 : 0)>{}); break;
        default: if constexpr (kR > 3) stop_code = step_of(std::integral_constant<int, (kR > 3 ? 3 : 0)>{}); break;
      }
      stamp(4);
      if (stop_code) break;
      lim = k;
    }
    bump(3);
  };
  // the round loop unrolled kPD times (each round reads its own prefetch slot
  // and refills it kPD rounds ahead: no register copies of loads in flight)
  for (int64_t p0 = 0; p0 < ncand && !stopped; p0 += kPD * kNS) {
#pragma unroll
    for (int u = 0; u < kPD; ++u) {
      const int64_t p = p0 + u * kNS;
      unpack(p, pf[u], sc);
      load_raw(p + kPD * kNS, pf[u]);
      if (p < ncand && !stopped) round(p);
    }
  }
  // stage the store: keys and rmax of every slot, the delta rows of the used ones
  int nslots = 0;
  for (int i = lane; i < NSLOT; i += 64) {
    const int32_t key = s_key[i];
    g_key[i] = key;
    g_rmax[i] = s_sg[i].rmax;
    nslots += key >= 0;
  }
  {
    constexpr int Q = LC / 4;
    for (int i = lane; i < NSLOT * Q; i += 64) {
      if (s_key[i / Q] < 0) continue;
      reinterpret_cast<float4*>(g_dw)[i] = reinterpret_cast<const float4*>(s_dw)[i];
      if (use_s) reinterpret_cast<float4*>(g_dp)[i] = reinterpret_cast<const float4*>(s_dp)[i];
    }
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) nslots += __shfl_xor(nslots, off, 64);
  if (lane == 0) {
    st[S_PEND] = pend;
    st[S_WHY] = why;
    st[S_NUPD] = s_cnt[0];
    st[S_NSLOTS] = nslots;
    st[S_STEPS] += n_steps;
    st[S_ROUNDS] += s_cnt[3];
    st[S_WASTED] += s_cnt[1];
    st[S_REFRESH] += s_cnt[2];
    st[S_EXACT] += n_exact;
    st[S_CAND] += ncand;
    st[S_TICKS] += (int64_t)(__builtin_amdgcn_s_memrealtime() - t_k0);
    if (kProf) {
      for (int i = 0; i < 5; ++i) st[S_PH0 + i] += (int64_t)s_ph[i];
      st[S_PHW] += (int64_t)(__builtin_amdgcn_s_memtime() - t_c0);
    }
  }
}

// ------------------------------------------------------------ D: verify + commit
template <int LC>
__global__ __launch_bounds__(256) void vc_verify_kernel(
    int64_t* __restrict__ st, const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels, const float* __restrict__ SL,
    unsigned long long* __restrict__ bits, const int32_t* __restrict__ g_key,
    const float* __restrict__ g_rmax, const float* __restrict__ g_dw, const float* __restrict__ g_dp,
    float* __restrict__ W, float* __restrict__ P, uint8_t* __restrict__ touched,
    unsigned long long* __restrict__ stats, int64_t* __restrict__ tail) {
  using Gm = Geo<LC>;
  constexpr int NSLOT = Gm::NSLOT;
  constexpr float kG = dc::kGuard;
  const int status = (int)st[S_STATUS];
  if (!live(status)) return;
  __shared__ __attribute__((aligned(16))) int32_t s_key[NSLOT];
  __shared__ float s_rmax[NSLOT];
  __shared__ unsigned s_valid, s_viol;
  __shared__ int s_last, s_force;
  const int tid = threadIdx.x;
  for (int i = tid; i < NSLOT; i += blockDim.x) {
    s_key[i] = g_key[i];
    s_rmax[i] = g_rmax[i];
  }
  if (tid == 0) { s_valid = 0; s_viol = 0; }
  __syncthreads();
  const int64_t wb = st[S_BEG], pe = st[S_PEND];
  const bool cs_mode = st[S_CSMODE] == 1;
  unsigned nvalid = 0, nviol = 0, nnonc = 0;
  for (int64_t i = wb + (int64_t)blockIdx.x * blockDim.x + tid; i < pe; i += (int64_t)gridDim.x * blockDim.x) {
    const int y = labels[i];
    if (y < 0 || y >= LC) continue;
    ++nvalid;
    const int64_t rel = i - wb;
    const unsigned long long bit = 1ull << (rel & 63);
    if (bits[rel >> 6] & bit) continue;
    ++nnonc;
    float bound = 0.f;
    for (int64_t j = row_ptr[i]; j < row_ptr[i + 1]; ++j) {
      const int32_t row = fidx[j];
      if (row < 0) continue;
      // (the store's layout: kernel C's, or the stepper cache's in candidate mode)
      const int s = cs_mode ? sp_find(s_key, sp_nslot(LC) / 4, row) : dc::cache_find<LC>(s_key, row);
      if (s >= 0) bound += fabsf(fval[j]) * s_rmax[s];
    }
    bound *= 2.f * (1.f + 4.f * kG);
    if (!(SL[rel] > bound)) {
      atomicOr(bits + (rel >> 6), bit);
      ++nviol;
    }
  }
  if (nvalid) atomicAdd(&s_valid, nvalid);
  if (nviol) atomicAdd(&s_viol, nviol);
  if (nnonc) atomicAdd((unsigned long long*)&st[S_NONC], (unsigned long long)nnonc);
  __syncthreads();
  if (tid == 0) {
    if (s_valid) atomicAdd((unsigned long long*)&st[S_NVALID], (unsigned long long)s_valid);
    if (s_viol) atomicAdd((unsigned long long*)&st[S_VIOL], (unsigned long long)s_viol);
    __threadfence();
    s_last = atomicAdd((unsigned long long*)&st[S_DONEB], 1ull) == (unsigned long long)(gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  const int64_t viol = ld_st(&st[S_VIOL]);
  const int64_t wend = st[S_WEND];
  if (viol == 0) {
    // commit the window: the staged deltas into W / P (this block is their
    // only writer). The used slots first (a window writes a few hundred of
    // NSLOT), then kU read-modify-writes per thread in flight at once: one
    // item per loop trip waited a whole HBM round trip per item
    __shared__ int s_used[NSLOT];
    __shared__ int s_nused;
    if (tid == 0) s_nused = 0;
    __syncthreads();
    for (int i = tid; i < NSLOT; i += blockDim.x)
      if (s_key[i] >= 0) s_used[atomicAdd(&s_nused, 1)] = i;
    __syncthreads();
    constexpr int Q = LC / 4;
    constexpr int kU = 4;
    const int items = s_nused * Q;
    for (int b0 = 0; b0 < items; b0 += kU * (int)blockDim.x) {
      float4 w[kU], d[kU], pv[kU], dp[kU];
      int64_t off[kU];
      bool on[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int it = b0 + u * (int)blockDim.x + tid;
        on[u] = it < items;
        const int sl = s_used[on[u] ? it / Q : 0];
        const int q = it % Q;
        off[u] = (int64_t)s_key[sl] * Q + q;
        const int gi = sl * Q + q;
        if (on[u]) {
          w[u] = reinterpret_cast<const float4*>(W)[off[u]];
          d[u] = reinterpret_cast<const float4*>(g_dw)[gi];
          if (P != nullptr) {
            pv[u] = reinterpret_cast<const float4*>(P)[off[u]];
            dp[u] = reinterpret_cast<const float4*>(g_dp)[gi];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        if (!on[u]) continue;
        w[u].x += d[u].x; w[u].y += d[u].y; w[u].z += d[u].z; w[u].w += d[u].w;
        reinterpret_cast<float4*>(W)[off[u]] = w[u];
        if (P != nullptr) {
          pv[u].x += dp[u].x; pv[u].y += dp[u].y; pv[u].z += dp[u].z; pv[u].w += dp[u].w;
          reinterpret_cast<float4*>(P)[off[u]] = pv[u];
        }
        if (off[u] % Q == 0 && touched != nullptr) touched[off[u] / Q] = 1;
      }
    }
    for (int i = tid; i < kBitWords; i += blockDim.x) bits[i] = 0ull;
    if (tid == 0) {
      const int64_t nupd = st[S_NUPD];
      const int64_t nv = ld_st(&st[S_NVALID]);
      if (stats != nullptr) {
        if (nupd > 0) atomicAdd(stats, (unsigned long long)nupd);
        if (nv > 0) atomicAdd(stats + 1, (unsigned long long)nv);
      }
      const int why = (int)st[S_WHY];
      const int64_t bend = st[S_BEND];
      st[S_BEG] = pe;
      st[S_WINDOWS] += 1;
      st[S_UPD] += nupd;
      if (why == kWhySat) st[S_SAT] += 1;
      // an update-dense window (more than dense_pm per mille of its samples
      // updated): the next chunk of the batch goes to the sequential stepper
      // (stepper.hip, ~0.8 us a sample whatever updates), which beats this
      // committer's ~2.2 us a step once updates are that frequent; the
      // segment after it continues from the chunk's end
      const int64_t dpm = st[S_DENSE_PM];
      const bool dense = dpm > 0 && pe < bend && nupd * 1000 > dpm * (pe - wb);
      st[S_STATUS] = (why == kWhyDense || dense) ? kDense : (pe >= bend ? kDone : kNew);
      if (!(why == kWhyDense || dense)) st[S_DCHUNK] = kDenseChunk0;   // sparse again: chunks start small
      // the window length follows where the store fills; T relaxes slowly
      int64_t lw = st[S_LW];
      if (why == kWhySat) {
        const int64_t took = pe - wb;
        lw = took + took / 4;
      } else if (pe - wb >= lw) {
        lw = 2 * lw;
      }
      lw = lw < kLwMin ? kLwMin : (lw > kLwMax ? kLwMax : lw);
      st[S_LW] = lw;
      const float T = fmaxf(kTMin, st_T(st) * 0.97f);
      st[S_T] = __float_as_int(T);
      st[S_RETRYW] = 0;
    }
  } else {
    if (tid == 0) {
      st[S_RETRIES] += 1;
      st[S_RETRYW] += 1;
      const float T = fminf(kTMax, st_T(st) * 1.5f);
      st[S_T] = __float_as_int(T);
      st[S_STATUS] = kRetry;
      s_force = st[S_RETRYW] >= kRetryForce;
    }
    __syncthreads();
    if (s_force) {
      // every sample of the window a candidate: nothing left to verify
      const int64_t n = wend - wb;
      for (int64_t w = tid; w < (n + 63) / 64; w += blockDim.x) {
        const int64_t rem = n - 64 * w;
        bits[w] = rem >= 64 ? ~0ull : ((1ull << rem) - 1);
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    st[S_DONEB] = 0;
    st[S_NVALID] = 0;
    st[S_VIOL] = 0;
    const int s2 = (int)st[S_STATUS];
    if (s2 != kRetry) st[S_WIDE] = 0;   // a retry keeps the window's candidates (and width)
    tail[0] = s2 == kDone ? st[S_BEND] : st[S_BEG];
    tail[1] = st[S_BEND];
    tail[2] = st[S_STEPS];
    tail[3] = st[S_ROUNDS];
    // stop reason: done / saturated (segments ran out) / dense
    tail[dc::kTailReason] = s2 == kDone ? dc::kStopDone : s2 == kDense ? dc::kStopDense : dc::kStopSaturated;
    tail[21] = st[S_WINDOWS] + st[S_RETRIES];   // segments used
    tail[kTailStepped] = st[S_STEPPED];
    tail[kTailChunks] = st[S_NCHUNK];
    tail[kTailSegEst] = seg_estimate(st);
    tail[kTailCsWindows] = st[S_CSN];
    tail[22] = st[S_WASTED];
    tail[23] = st[S_REFRESH];
    tail[24] = st[S_UPD];
    tail[25] = st[S_NSLOTS];
    tail[26] = st[S_EXACT];
    tail[27] = st[S_CAND];
    tail[28] = st[S_RETRIES];
    tail[29] = st[S_SAT];
    tail[30] = st[S_TICKS];
    for (int i = 0; i < 5; ++i) tail[10 + i] = st[S_PH0 + i];
    tail[15] = st[S_PHW];
    tail[8] = st[S_LW];
    tail[9] = st[S_T];
    tail[7] = st[S_NONC];
  }
}

}  // namespace vc
}  // namespace jb

// bytes of the verified committer's fixed region (after the per-sample arrays):
// state (512 B), candidate bits, the staged store (keys, rmax, dW, dP)
static constexpr int64_t kVcFixed = 512 + 8 * jb::vc::kBitWords + 4 * 1024 + 4 * 1024 + 2 * 4 * 16384;
extern "C" int64_t jb_vcommit_fixed_bytes() { return kVcFixed; }

// stepper.hip
extern "C" int jb_stepper_enabled();
extern "C" int jb_stepper_chunk(const int64_t* row_ptr, const int32_t* fidx, const float* fval, const int32_t* labels,
                                float* W, float* P, const int32_t* active, int LC, int method, float C,
                                unsigned long long* stats, uint8_t* touched, int64_t* vst, int64_t* vtail,
                                hipStream_t stream);
extern "C" int jb_stepper_cand(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                               const int32_t* labels, float* W, float* P, const int32_t* active, int LC, int method,
                               float C, int64_t* vst, const int4* aux, int32_t* g_key, float* g_rmax, float* g_dw,
                               float* g_dp, hipStream_t stream);

template <int L>
static int launch_vc(int method, const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                     const int32_t* labels, float* W, float* S, const int32_t* active, float C, int64_t* st,
                     float* sl, unsigned long long* bits, float* s0, int4* aux, float2* pp0, int32_t* fi,
                     float* fx, int32_t* gk, float* gr, float* gdw, float* gdp, uint8_t* touched,
                     unsigned long long* stats, int64_t* tail, int nseg, bool chunks, int cs_min, int cs_pm,
                     hipStream_t stream) {
  using namespace jb::vc;
  static const int prof = [] {
    const char* e = getenv("JB_COMMIT_PROF");
    return (e != nullptr && e[0] == '1') ? 1 : 0;
  }();
  // committer shape (samples per group x rounds in flight), for A/B runs:
  // JB_VC_SHAPE = r1pd1; default r1pd2 (measured: r1pd2 7.19, r1pd1 7.27,
  // r1pd3 7.25, r2pd1 8.47, r2pd2 8.45 ms per steady 131 K batch)
  static const int shape = [] {
    const char* e = getenv("JB_VC_SHAPE");
    if (e == nullptr) return 0;
    if (strcmp(e, "r2pd2") == 0) return 1;
    if (strcmp(e, "r2pd1") == 0) return 2;
    if (strcmp(e, "r1pd1") == 0) return 3;
    if (strcmp(e, "r1pd3") == 0) return 4;
    return 0;
  }();
  float* Pp = method >= jb::CW ? S : nullptr;
  for (int seg = 0; seg < nseg; ++seg) {
    hipLaunchKernelGGL((vc_score_kernel<L>), dim3(1024), dim3(256), 0, stream, st, row_ptr, fidx, fval, labels,
                       W, active, method, C, sl, bits, gk, gr);
    hipLaunchKernelGGL((vc_gather_kernel<L>), dim3(512), dim3(256), 0, stream, st, row_ptr, fidx, fval, labels,
                       W, Pp, active, method, C, bits, s0, aux, pp0, fi, fx, cs_min, cs_pm);
#define JB_VC_S(M, R, PD)                                                                                       \
  hipLaunchKernelGGL((vc_commit_kernel<L, M, R, PD, 1>), dim3(1), dim3(64), 0, stream, st, W, Pp, active, C, s0, \
                     aux, pp0, fi, fx, gk, gr, gdw, gdp, prof);                                                  \
  hipLaunchKernelGGL((vc_commit_kernel<L, M, R, PD, 2>), dim3(1), dim3(64), 0, stream, st, W, Pp, active, C, s0, \
                     aux, pp0, fi, fx, gk, gr, gdw, gdp, prof);
#define JB_VC_M(M)                               \
  if (shape == 3) { JB_VC_S(M, 1, 1) }           \
  else { JB_VC_S(M, 1, 2) }                      \
  break;
    switch (method) {
      case jb::PERCEPTRON: JB_VC_M(jb::PERCEPTRON)
      case jb::PA: JB_VC_M(jb::PA)
      case jb::PA1: JB_VC_M(jb::PA1)
      case jb::PA2: JB_VC_M(jb::PA2)
      case jb::CW: JB_VC_M(jb::CW)
      case jb::AROW: JB_VC_M(jb::AROW)
      case jb::NHERD: JB_VC_M(jb::NHERD)
      default: return -1;
    }
#undef JB_VC_M
#undef JB_VC_S
    // candidate mode (kernel B's choice): the stepper walks the candidates
    if (cs_min > 0) {
      const int rc = jb_stepper_cand(row_ptr, fidx, fval, labels, W, Pp, active, L, method, C, st, aux, gk, gr, gdw,
                                     gdp, stream);
      if (rc != 0) return rc;
    }
    hipLaunchKernelGGL((vc_verify_kernel<L>), dim3(256), dim3(256), 0, stream, st, row_ptr, fidx, fval, labels,
                       sl, bits, gk, gr, gdw, gdp, W, Pp, touched, stats, tail);
    // after an update-dense window: the stepper's chunk (an empty launch
    // otherwise), then the next segment continues from its end
    if (chunks) {
      const int rc = jb_stepper_chunk(row_ptr, fidx, fval, labels, W, Pp, active, L, method, C, stats, touched, st,
                                      tail, stream);
      if (rc != 0) return rc;
    }
  }
  return 0;
}

// Steps 1-2 of a kSerial batch for LC <= 64 with the verified committer; the
// caller runs the exact single-stream kernel over [tail[0], tail[1]) afterwards
// (empty when every window committed). scratch: [tail int64 x 32][S0: n_max x
// 64 floats][PP0: n_max x 32 float2][FI: n_max x 32][FX: n_max x 32][AUX: n_max
// int4][SL: n_max floats][fixed region, 256-aligned: state, bits, staged store]
extern "C" int jb_vcommit_prepare(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                  const int32_t* labels, const int64_t* stream_ptr, int nstreams, int64_t n_max,
                                  float* W, float* S, const int32_t* active, int LC, int method, float C,
                                  unsigned long long* stats, uint8_t* touched, void* scratch, int nseg,
                                  hipStream_t stream) {
  if (LC > 64) return -1;
  int64_t* tail = (int64_t*)scratch;
  uint8_t* base = (uint8_t*)scratch + 256;
  float* s0 = (float*)base;
  float2* pp0 = (float2*)(base + 256 * n_max);
  int32_t* fi = (int32_t*)(base + 512 * n_max);
  float* fx = (float*)(base + 640 * n_max);
  int4* aux = (int4*)(base + 768 * n_max);
  float* sl = (float*)(base + 784 * n_max);
  uint8_t* fixed = base + ((788 * n_max + 255) & ~(int64_t)255);
  int64_t* st = (int64_t*)fixed;
  unsigned long long* bits = (unsigned long long*)(fixed + 512);
  int32_t* gk = (int32_t*)(fixed + 512 + 8 * jb::vc::kBitWords);
  float* gr = (float*)((uint8_t*)gk + 4 * 1024);
  float* gdw = (float*)((uint8_t*)gr + 4 * 1024);
  float* gdp = gdw + 16384;
  // JB_VERIFIED_T: the candidate threshold at every batch start (tests force
  // verification failures with a tiny one); unset: T adapts across batches
  const char* te = getenv("JB_VERIFIED_T");
  const float t_force = te != nullptr ? (float)atof(te) : 0.f;
  // JB_VC_DENSE_PM: updates per mille of a committed window past which the
  // next chunk of the batch goes to the stepper (0: never; default 300 - the
  // committer costs ~2.2 us an update, the stepper ~0.8 us a sample)
  const char* de = getenv("JB_VC_DENSE_PM");
  const int dense_pm = de != nullptr ? atoi(de) : 300;
  hipLaunchKernelGGL(jb::vc::vc_init_kernel, dim3(1), dim3(256), 0, stream, st, stream_ptr, nstreams, bits, tail,
                     t_force, gk, gr, dense_pm);
  // fp32 tables with the stepper on: dense windows hand the next chunk to it
  // inside the segment sequence (else the batch's rest goes to the caller's
  // single-stream kernel at the end)
  const bool chunks = dense_pm > 0 && jb_stepper_enabled();
  // JB_VC_CS=n (0 / unset: off): windows of at least n candidates go to the
  // stepper when the last window updated on more than JB_VC_CS_PM per mille
  // of its candidates (default 350). Off by default: measured on the bench
  // stream (tools/bench_serial.py, batches 20-30: ~22 % of candidates update)
  // with every window on the stepper 11.3 ms a batch against kernel C's 6.8
  // (the stepper costs ~0.8 us a candidate, C ~2.3 us an update and little
  // else, and the stepper's windows end at fewer pinned rows), and on the
  // served learning stream (18 % updates) 1.61 M samples/s against 1.65 M
  const char* cs_e = getenv("JB_VC_CS");
  const char* cs_p = getenv("JB_VC_CS_PM");
  const int cs_min = (jb_stepper_enabled() && cs_e != nullptr) ? atoi(cs_e) : 0;
  const int cs_pm = cs_p != nullptr ? atoi(cs_p) : 350;
  int rc = 0;
#define JB_VC_L(L)                                                                                            \
  rc = launch_vc<L>(method, row_ptr, fidx, fval, labels, W, S, active, C, st, sl, bits, s0, aux, pp0, fi, fx, \
                    gk, gr, gdw, gdp, touched, stats, tail, nseg, chunks, cs_min, cs_pm, stream);              \
  break;
  switch (LC) {
    case 8: JB_VC_L(8)
    case 16: JB_VC_L(16)
    case 32: JB_VC_L(32)
    case 64: JB_VC_L(64)
    default: return -1;
  }
#undef JB_VC_L
  if (rc) return rc;
  return (int)hipGetLastError();
}
