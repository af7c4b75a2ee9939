// Sequential stepper: the servers' default "exact" training of an
// update-dense run of samples, every sample applied to the model in request
// order exactly as the reference's classifier does
// (jubatus/server/server/classifier_serv.cpp:138-144; update rules in
// jb_linear.hpp, oracle jubatus_amd/models/linear_oracle.py).
//
// Why. The verified committer (vcommit.hip) is fast when few samples update
// (it walks only the candidates), but on a stream where most samples update
// its one-wave chain costs ~2.2 us a step (a hashed LDS store probe per
// feature, lazy bounds, corrections of the later candidates) and a window
// ends every ~130 samples when that store fills. The old sequential kernel
// (linear.hip, one wave reading W / P from HBM) pays two HBM round trips a
// sample. Here one wave steps and never touches global memory: the model rows
// the samples need are staged in an LDS row cache ahead of it.
//
// One workgroup of four waves on one CU, handing work on through LDS rings:
//   wave 2  (meta)    reads the samples' labels, row offsets and features
//                     from HBM, 64 samples at a time, into a sample header
//                     ring and a feature ring;
//   wave 1  (lookup)  maps every feature row of the next sample to a slot of
//                     a 2-choice 4-way set-associative LDS cache of W / P
//                     rows: hits stay; a miss takes an empty way or the least
//                     recently used one whose last sample the stepper has
//                     passed (CAS on the way's key) and becomes a fetch job;
//   wave 3  (fetch)   takes the jobs in order: writes the way's previous row
//                     back to HBM when the stepper had written it, fetches the
//                     new row with LDS-DMA loads (global_load_lds_dwordx4) into
//                     a staging area - kK stages in flight, counted vmcnt
//                     waits - copies a landed stage into its slots and then
//                     publishes the samples it completes;
//   wave 0  (stepper) takes the published samples in order: scores of every
//                     label (lanes = label x feature group), best wrong label
//                     by DPP max + ballot, the variance, the method's step
//                     (jb_linear.hpp step_coeffs, IEEE divisions; per-feature
//                     inverse precisions by rcp + one Newton step) and the
//                     updated values stored into the cached rows (LDS float
//                     adds when the meta wave saw a row twice in the sample). The next sample's
//                     header and entries are read while a sample computes, so
//                     a step is one LDS round trip (its rows) plus VALU work,
//                     no HBM.
// A sample the cache cannot hold (more than kFMax features, or more rows in
// one bucket pair than its ways) is applied on HBM directly by the stepper
// after the loader has written back and dropped its cached rows.
//
// Waves hand data over through LDS only (in-order per CU); every wait has a
// time limit (an error code instead of a hung GPU).
#include <string.h>

#include "jb_linear.hpp"
#include "jb_vc_state.hpp"

namespace jb {
namespace sp {

constexpr int kT = 256;
constexpr int kSR = 256;            // sample header ring (power of two)
constexpr int kFR = 1024;           // feature ring entries (power of two)
constexpr int kFMax = 256;          // features of a cached sample (<= kFR / 2)
constexpr int kNMask = 0x3fff;      // header word z: (y + 1) << 16 | dup bit | (n + 1)
constexpr int kDupBit = 0x8000;
constexpr int kK = 8;               // fetch stages in flight
constexpr int kC = 5;               // VMEM instructions per stage (see issue_stage)
constexpr int kSlotBytes = vc::kSpSlotBytes;   // the W / P row cache
constexpr int kJR = 512;            // fetch job ring (power of two, >= kFMax + 64)
constexpr int64_t kTimeout = 200000000;   // 2 s of s_memrealtime (100 MHz)

template <int LC>
struct Geo {
  static_assert(LC >= 8 && LC <= 64, "stepper: 8 <= LC <= 64");
  static constexpr int G = 64 / LC;                                    // feature groups of a step
  static constexpr int NSLOT = vc::sp_nslot(LC);
  static constexpr int NB = NSLOT / 4;                                 // 4-way buckets
  static constexpr int RPS = 256 / LC;                                 // rows per fetch stage
  static constexpr int LPR = 64 / RPS;                                 // lanes per row (16 B of W, 16 B of P)
  static constexpr int QC = 16 / G;                                   // features per lane of a 16-feature sample
  // LDS carve (bytes, every offset a multiple of 16)
  static constexpr int oW = 0;
  // W / P rows of NSLOT cache slots + one dummy slot (index NSLOT) that
  // absent features of a sample point at (zero x, adds of zero)
  static constexpr int oP = oW + (NSLOT + 1) * LC * 4;
  static constexpr int oKey = oP + (NSLOT + 1) * LC * 4;
  static constexpr int oUse = oKey + (NSLOT + 4) * 4;
  static constexpr int oDirty = oUse + (NSLOT + 4) * 4;
  static constexpr int oHdr = oDirty + (NSLOT + 4) * 4;  // int4 [kSR]: meta/ready seq, y|n, off
  static constexpr int oFend = oHdr + kSR * 16;                        // int [kSR]
  static constexpr int oFR = oFend + kSR * 4;                          // int2 [kFR]: row (then slot), x
  static constexpr int oStage = oFR + kFR * 8;                         // [kK][W 1 KB | P 1 KB]
  static constexpr int oStSlot = oStage + kK * 2048;                   // int [kK][64]
  static constexpr int oStPub = oStSlot + kK * 64 * 4;                 // int [kK] (padded to 64 B)
  static constexpr int oLk = oStPub + 64;                              // int4 [kSR]: lk_seq, job pos, misses
  static constexpr int oJobs = oLk + kSR * 16;                         // int4 [kJR]: row, slot, previous row
  static constexpr int oDps = oJobs + kJR * 16;                        // float [kFMax][2]: a wide sample's dP
  static constexpr int oDps2 = oDps + 2 * kFMax * 4;                   // float [kFMax][2]: its P / sigma values
  static constexpr int oRmx = oDps2 + 2 * kFMax * 4;                   // float [NSLOT + 4]: rows' step bounds (CS)
  static constexpr int oCtl = oRmx + (NSLOT + 4) * 4;                  // control words
  static constexpr int kBytes = oCtl + 64;
  static_assert(kBytes <= 160 * 1024, "stepper LDS");
};

// control words (int [16] at oCtl)
// C_STOP: the first sample not taken (candidate mode: the cache cannot pin
// another updated row - the window ends there)
enum : int { C_PROGRESS = 0, C_ABORT = 1, C_WHY = 2, C_JDONE = 3, C_STOP = 4, C_NUPD = 5 };
// launch modes: a range (single stream), a chunk after a dense window, the
// candidates of a verified-committer window (vcommit.hip, kernel C's place)
enum : int { kModeRange = 0, kModeChunk = 1, kModeCand = 2 };
// abort reasons (stats[2] when non-zero)
enum : int { kErrTimeoutStep = 1, kErrTimeoutLoad = 2, kErrTimeoutMeta = 3, kErrTimeoutFetch = 4 };

__device__ float g_dummy[1024] __attribute__((aligned(256)));   // target of padding stores / loads
__device__ int g_err;                                            // first abort reason of any launch
// JB_STEPPER_PROF=1: per-wave shader cycles of the launches since the last
// jb_stepper_prof() (accumulated by lane 0 of each wave)
enum : int {
  P_STEP_TOTAL = 0, P_STEP_WAIT, P_LOAD_IDLE, P_LOAD_RETIRE, P_LOAD_STUCK, P_META_ROOM, P_SAMPLES, P_STAGES,
  P_MISSES, P_DIRECT, P_LOAD_LOOKUP, P_LOAD_ISSUE, P_LOAD_TOTAL, P_META_TOTAL, P_FETCH_TOTAL, P_LK_ITERS,
  P_LK_KEYS, P_LK_CAS, P_ST_READ, P_ST_REDUCE, P_ST_COEF, P_ST_APPLY, P_NWORDS = 24
};
__device__ unsigned long long g_prof[P_NWORDS];

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
// 16 B per lane from HBM into LDS at lds_dst + 16 * lane (lds_dst wave-uniform);
// sc1: past the CU's L1 (a row written back by this CU earlier is read from L2)
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds_dst) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off sc1\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(gsrc), "s"(lds_dst)
               : "memory");
}
// wait until at most kC * n of the loader's VMEM instructions are in flight
__device__ __forceinline__ void wait_stages(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(25)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(30)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(35)" ::: "memory"); break;
  }
}
static_assert(kC * (kK - 1) <= 35, "wait_stages covers kK - 1 stages");

// LDS reads / writes the compiler may neither cache nor move across the
// other waves' hand-offs (vector types through a plain access between
// compiler barriers: HIP vector types have no volatile accessors)
template <class T>
__device__ __forceinline__ T lds_ld(const T* p) {
  asm volatile("" ::: "memory");
  const T v = *p;
  asm volatile("" ::: "memory");
  return v;
}
template <class T>
__device__ __forceinline__ void lds_st(T* p, T v) {
  asm volatile("" ::: "memory");
  *p = v;
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ void buckets(int row, int NB, int* b1, int* b2) { vc::sp_buckets(row, NB, b1, b2); }
__device__ __forceinline__ int find_in(const int* key, int b1, int b2, int row) {
  const int4 k1 = lds_ld(reinterpret_cast<const int4*>(key + 4 * b1));
  const int4 k2 = lds_ld(reinterpret_cast<const int4*>(key + 4 * b2));
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

__device__ __forceinline__ bool timed_out(uint64_t t0) {
  return (int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > kTimeout;
}

// floats as ints of the same order (non-NaN): negative values flip their
// magnitude bits
__device__ __forceinline__ int ord_i(float f) {
  const int b = __float_as_int(f);
  return b ^ ((b >> 31) & 0x7fffffff);
}
// max over the LC labels of a group (lanes [k LC, (k + 1) LC))
template <int LC>
__device__ __forceinline__ int group_max_i(int v, int lane) {
  v = max(v, dpp_i<kDppXor1>(v));
  v = max(v, dpp_i<kDppXor2>(v));
  v = max(v, dpp_i<kDppHalfMirror>(v));
  if constexpr (LC >= 16) v = max(v, dpp_i<kDppMirror>(v));
  if constexpr (LC >= 32) v = max(v, partner16_i(v, lane));
  if constexpr (LC >= 64) v = max(v, partner32_i(v, lane));
  return v;
}
__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// s and a second per-lane sum q reduced over the G feature groups together:
// one permlane swap exchanges s's odd rows with q's even rows, so one add
// sums both (s's totals land in lanes [0, LC), q's at kQOff + [0, LC);
// LC 64 has one group - nothing to reduce, q stays in its own register)
template <int LC>
struct PairLanes {
  static constexpr int kQOff = LC <= 16 ? 16 : 32;
};
template <int LC>
__device__ __forceinline__ float pair_sum(float s, float q) {
  if constexpr (LC == 64) {
    return s;
  } else if constexpr (LC == 32) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(q), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);   // [s_lo + s_hi | q_lo + q_hi]
  } else {
    if constexpr (LC == 8) {
      s += dpp_f<kDppRowRor8>(s);
      q += dpp_f<kDppRowRor8>(q);
    }
    // rows [s0 s1 s2 s3] [q0 q1 q2 q3] -> [s0 q0 s2 q2] + [s1 q1 s3 q3]
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(q), false, false);
    const float t = __uint_as_float(r[0]) + __uint_as_float(r[1]);
    // -> [S Q S Q]
    const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(t), __float_as_uint(t), false, false);
    return __uint_as_float(h[0]) + __uint_as_float(h[1]);
  }
}

// 1 / p to within ~1 ulp: the hardware reciprocal and one Newton step (three
// instructions instead of the ten of an IEEE division). Used for the
// per-feature inverse precisions only; the step coefficients (one per
// sample) keep IEEE divisions (jb_linear.hpp step_coeffs)
__device__ __forceinline__ float rcp_nr(float p) {
  const float r = __builtin_amdgcn_rcpf(p);
  return fmaf(r, fmaf(-p, r, 1.f), r);
}
__device__ __forceinline__ float4 rcp4(float4 v) {
  return make_float4(rcp_nr(v.x), rcp_nr(v.y), rcp_nr(v.z), rcp_nr(v.w));
}
// jb_linear.hpp dprec with rcp_nr for the division
__device__ __forceinline__ float dprec_nr(int method, float beta, float x, float s) {
  const float bx2 = beta * x * x;
  return method == CW ? bx2 : bx2 * rcp_nr(1.f - bx2 * s);
}

template <int LC, int MT, bool PROF>
__global__ __launch_bounds__(kT) void stepper_kernel(const int64_t* __restrict__ row_ptr,
                                                     const int32_t* __restrict__ fidx,
                                                     const float* __restrict__ fval,
                                                     const int32_t* __restrict__ labels,
                                                     const int64_t* __restrict__ range, float* W, float* P,
                                                     const int32_t* __restrict__ active, float C,
                                                     unsigned long long* __restrict__ stats,
                                                     uint8_t* __restrict__ touched, int* __restrict__ err,
                                                     unsigned long long* __restrict__ prof, int64_t* vst,
                                                     int64_t* vtail, int mode, const int4* __restrict__ aux,
                                                     int32_t* __restrict__ g_key, float* __restrict__ g_rmax,
                                                     float* __restrict__ g_dw, float* __restrict__ g_dp) {
  using Gm = Geo<LC>;
  constexpr bool use_s = MT >= CW;
  // AROW / NHERD: the cache holds sigma = 1 / P (converted when a row lands
  // and when it goes back): P += b x^2 / (1 - b x^2 sigma) is then
  // sigma -= b x^2 sigma^2 - no reciprocal in a step (CW's P += b x^2 keeps P)
  constexpr bool kSig = MT == AROW || MT == NHERD;
  auto to_hbm = [](float4 v) __attribute__((always_inline)) { return kSig ? rcp4(v) : v; };
  constexpr bool use_nrm = MT == PA || MT == PA1 || MT == PA2;
  constexpr int NSLOT = Gm::NSLOT, NB = Gm::NB, G = Gm::G, RPS = Gm::RPS, LPR = Gm::LPR;
  constexpr int QC = Gm::QC;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* Wc = reinterpret_cast<float*>(smem + Gm::oW);
  float* Pc = reinterpret_cast<float*>(smem + Gm::oP);
  int* key = reinterpret_cast<int*>(smem + Gm::oKey);
  int* use = reinterpret_cast<int*>(smem + Gm::oUse);
  int* dirty = reinterpret_cast<int*>(smem + Gm::oDirty);
  int4* hdr = reinterpret_cast<int4*>(smem + Gm::oHdr);
  int* fend = reinterpret_cast<int*>(smem + Gm::oFend);
  int2* fring = reinterpret_cast<int2*>(smem + Gm::oFR);
  char* stage = smem + Gm::oStage;
  int* st_slot = reinterpret_cast<int*>(smem + Gm::oStSlot);
  int* st_pub = reinterpret_cast<int*>(smem + Gm::oStPub);
  int4* lk = reinterpret_cast<int4*>(smem + Gm::oLk);
  int4* jobs = reinterpret_cast<int4*>(smem + Gm::oJobs);
  float* dps = reinterpret_cast<float*>(smem + Gm::oDps);
  float* dps2 = reinterpret_cast<float*>(smem + Gm::oDps2);
  float* rmx = reinterpret_cast<float*>(smem + Gm::oRmx);
  int* ctl = reinterpret_cast<int*>(smem + Gm::oCtl);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  // vst (a verified committer's state, vcommit.hip): a chunk after an
  // update-dense window - nothing to do unless the committer stopped dense
  // kModeCand: the window's candidates (kernel B's records, in order) from
  // the model at the window's start; nothing is written to W / P
  const bool cs = mode == kModeCand;
  int64_t beg, end;
  if (cs) {
    const int stv = (int)vst[vc::S_STATUS];
    if (!(stv == vc::kNew || stv == vc::kRetry) || vst[vc::S_CSMODE] != 1) return;
    beg = vst[vc::S_BEG];
    end = beg + vst[vc::S_NCAND];    // (N candidates; sample t is beg + aux[t].w)
  } else if (vst != nullptr) {
    if (vst[vc::S_STATUS] != vc::kDense) return;
    beg = vst[vc::S_BEG];
    end = min(vst[vc::S_BEND], beg + vst[vc::S_DCHUNK]);
  } else {
    beg = range[0];
    end = range[1];
  }
  if (end <= beg && vst == nullptr) return;
  const int N = (int)(end > beg ? end - beg : 0);
  auto sidx = [&](int t) __attribute__((always_inline)) -> int64_t { return cs ? beg + aux[t].w : beg + t; };

  // ---- init (all waves)
  for (int i = tid; i < NSLOT + 4; i += kT) {
    key[i] = -1;
    use[i] = -1;
    dirty[i] = 0;
    rmx[i] = 0.f;
  }
  for (int i = tid; i < (NSLOT + 1) * LC; i += kT) {   // empty slots hold the initial model
    Wc[i] = 0.f;
    Pc[i] = 1.f;
  }
  for (int i = tid; i < kSR; i += kT) {
    hdr[i] = make_int4(-1, -1, 0, 0);
    lk[i] = make_int4(-1, 0, 0, 0);
  }
  if (tid < 16) ctl[tid] = tid == C_STOP ? N : 0;
  __syncthreads();
  // phase cycles of this wave (prof != nullptr only)
  unsigned long long pc[P_NWORDS];
#pragma unroll
  for (int i = 0; i < P_NWORDS; ++i) pc[i] = 0;
  auto clk = [&]() __attribute__((always_inline)) -> uint64_t {
    if constexpr (PROF) return __builtin_amdgcn_s_memtime();
    return 0;
  };
  const uint64_t c_start = clk();
  auto abort_with = [&](int why) __attribute__((always_inline)) {
    if (lane == 0) {
      lds_st(&ctl[C_ABORT], 1);
      if (lds_ld(&ctl[C_WHY]) == 0) lds_st(&ctl[C_WHY], why);
    }
  };
  // wait until ctl[C_PROGRESS] >= want (every wait bounded)
  auto wait_progress = [&](int want, int why) __attribute__((always_inline)) -> bool {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (lds_ld(&ctl[C_PROGRESS]) < want) {
      if (lds_ld(&ctl[C_ABORT]) != 0 || timed_out(t0)) { abort_with(why); return false; }
      __builtin_amdgcn_s_sleep(1);
    }
    return true;
  };

  if (wave == 0) {
    // ================================================================ stepper
    const int l = lane % LC;
    const int g = lane / LC;
    const bool act = active[l] != 0;
    unsigned n_upd = 0, n_valid = 0;
    // the next sample's header and first-chunk entries, read while the
    // current one computes (neither depends on its adds); valid when the
    // header's ready word names the sample
    int4 hd = lds_ld(&hdr[0]);
    int2 e[QC];
    auto entries = [&](int off) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < QC; ++u) e[u] = fring[(off + u * G + g) & (kFR - 1)];
    };
    entries(hd.w);
    for (int t = 0; t < N; ++t) {
      if (hd.y != t) {
        const uint64_t w0 = clk();
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        bool dead = false;
        for (;;) {
          __builtin_amdgcn_s_sleep(1);
          hd = lds_ld(&hdr[t & (kSR - 1)]);
          if (hd.y == t) break;
          if (cs && lds_ld(&ctl[C_STOP]) <= t) { dead = true; break; }   // the window ends before t
          if (lds_ld(&ctl[C_ABORT]) != 0 || timed_out(t0)) { abort_with(kErrTimeoutStep); dead = true; break; }
        }
        pc[P_STEP_WAIT] += clk() - w0;
        if (dead) break;
        entries(hd.w);
      }
      const int y = __builtin_amdgcn_readfirstlane((hd.z >> 16) - 1);
      const int n = __builtin_amdgcn_readfirstlane((hd.z & kNMask) - 1);
      const bool dup = __builtin_amdgcn_readfirstlane(hd.z & kDupBit) != 0;
      const int off = __builtin_amdgcn_readfirstlane(hd.w);
      int sl[QC];
      float xv[QC], inv[QC];
#pragma unroll
      for (int u = 0; u < QC; ++u) {
        const bool ok = u * G + g < n && e[u].x >= 0;
        sl[u] = ok ? e[u].x : NSLOT;
        xv[u] = ok ? __int_as_float(e[u].y) : 0.f;
      }
      // the next sample's header and entries (stale if it is not published yet)
      const int tn = t + 1;
      hd = lds_ld(&hdr[tn & (kSR - 1)]);
      entries(hd.w);
      uint64_t s3 = 0;
      if (y >= 0) {
        ++n_valid;
        if (n < 0) {
          // a sample the cache does not hold: on HBM (the loader wrote back
          // and dropped its rows), drained before the progress word moves
          const int64_t s = sidx(t);
          const int64_t rb = row_ptr[s];
          const bool ak[1] = {act};
          if (general_sample<LC, kAtomic, float>(fidx, fval, rb, (int)(row_ptr[s + 1] - rb), y, W, P, ak, lane, MT,
                                                 C, touched))
            ++n_upd;
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
          // scores, |x|^2 and x^2 / P of this lane's label over its features
          // (lanes: label l x feature group g); all reads before any add
          // (absent features: the dummy slot, x 0 - no selects, no branches)
          float s = 0.f, vq = 0.f, nq = 0.f;
          const bool one = n <= QC * G;
          const uint64_t s0 = clk();
          float w[QC], p[QC];
          auto chunk = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < QC; ++u) {
              w[u] = Wc[sl[u] * LC + l];
              p[u] = use_s ? Pc[sl[u] * LC + l] : 1.f;
            }
#pragma unroll
            for (int u = 0; u < QC; ++u) {
              s = fmaf(xv[u], w[u], s);
              if (use_nrm) nq = fmaf(xv[u], xv[u], nq);
              if (use_s) {
                inv[u] = kSig ? p[u] : rcp_nr(p[u]);
                vq = fmaf(xv[u] * xv[u], inv[u], vq);
              } else {
                inv[u] = 1.f;
              }
            }
          };
          chunk();
          for (int q0 = QC; q0 * G < n; q0 += QC) {   // wide: the further chunks
#pragma unroll
            for (int u = 0; u < QC; ++u) {
              const int j = (q0 + u) * G + g;
              const int2 ej = fring[(off + j) & (kFR - 1)];
              const bool ok = j < n && ej.x >= 0;
              sl[u] = ok ? ej.x : NSLOT;
              xv[u] = ok ? __int_as_float(ej.y) : 0.f;
            }
            chunk();
          }
          const uint64_t s1 = clk();
          pc[P_ST_READ] += s1 - s0;
          // s and the method's second sum (x^2 / P or |x|^2) reduced together
          const float q = use_s ? vq : nq;
          const float r = pair_sum<LC>(s, q);
          // best wrong label: max over the labels as order-preserving ints
          // (one fused DPP max per step, no float canonicalisation)
          const int v = (act && l != y) ? ord_i(r) : ord_i(-INFINITY);
          const int m = group_max_i<LC>(v, lane);
          const uint64_t bal = __ballot(lane < LC && act && l != y && v == m && v > ord_i(-INFINITY));
          const int bl = bal != 0ull ? (int)__ffsll((long long)bal) - 1 : -1;
          const int blr = bl >= 0 ? bl : y;   // a lane to read without a branch (discarded if bl < 0)
          auto rq = [&](int i) __attribute__((always_inline)) {
            return LC == 64 ? readlane_f(q, i) : readlane_f(r, PairLanes<LC>::kQOff + i);
          };
          const float sy = readlane_f(r, y);
          const float sb = readlane_f(r, blr);
          const float best = bl >= 0 ? sb : 0.f;
          const float qb = rq(blr);
          const float var = use_s ? rq(y) + (bl >= 0 ? qb : 0.f) : 0.f;
          const float nrm = use_nrm ? rq(0) : 0.f;
          float tau = 0.f, beta = 0.f;
          const uint64_t s2 = clk();
          pc[P_ST_REDUCE] += s2 - s1;
          const bool upd = step_coeffs(MT, sy - best, var, nrm, bl >= 0, C, &tau, &beta);
          s3 = clk();
          pc[P_ST_COEF] += s3 - s2;
          if (upd) {
            ++n_upd;
            if (cs && one && !(kSig && dup)) {   // (kSig repeats: the wide loops below)
              // candidate mode: the step's bound on every row it writes (for
              // kernel D) - the larger |dW| of its two labels, the best wrong
              // label's from its lane by a permute - added to the row's rmax;
              // the row stays pinned in the cache until the window is staged
              const float sgl = l == y ? tau : -tau;
              const int src = g * LC + (bl >= 0 ? bl : y);
#pragma unroll
              for (int u = 0; u < QC; ++u) {
                const float a = fabsf(sgl * inv[u] * xv[u]);
                const float b = __shfl(a, src, 64);
                if (l == y) {
                  atomicAdd(&rmx[sl[u]], bl >= 0 ? fmaxf(a, b) : a);
                  dirty[sl[u]] = 1;
                }
              }
            }
            const bool isy = l == y, isl = l == bl;
            if (isy || isl) {
              const float sg = isy ? tau : -tau;
              if (one && !dup) {
                // distinct slots: the values read above plus the deltas
                // (absent features store the dummy slot's value back)
#pragma unroll
                for (int u = 0; u < QC; ++u) {
                  Wc[sl[u] * LC + l] = fmaf(sg * inv[u], xv[u], w[u]);
                  if (kSig) {
                    const float bx = beta * xv[u] * xv[u] * p[u];
                    Pc[sl[u] * LC + l] = fmaf(-bx, p[u], p[u]);   // sigma - b x^2 sigma^2
                  } else if (use_s) {
                    Pc[sl[u] * LC + l] = p[u] + dprec_nr(MT, beta, xv[u], inv[u]);
                  }
                }
              } else if (one && !kSig) {
#pragma unroll
                for (int u = 0; u < QC; ++u) {   // (absent features add 0 to the dummy slot)
                  atomicAdd(&Wc[sl[u] * LC + l], sg * inv[u] * xv[u]);
                  if (use_s) atomicAdd(&Pc[sl[u] * LC + l], dprec_nr(MT, beta, xv[u], inv[u]));
                }
              } else {
                // wide sample: the entries again, chunk by chunk. Every
                // precision is read before this sample's first P add (the
                // oracle's semantics for a row repeated across chunks): W adds
                // go at once, the P increments wait in dps until all are read
                for (int q0 = 0; q0 * G < n; q0 += QC) {
#pragma unroll
                  for (int u = 0; u < QC; ++u) {
                    const int j = (q0 + u) * G + g;
                    const int2 ej = fring[(off + j) & (kFR - 1)];
                    const int sj = j < n ? ej.x : -1;
                    if (sj < 0) continue;
                    const float x = __int_as_float(ej.y);
                    const float pv = use_s ? Pc[sj * LC + l] : 1.f;
                    const float iv = kSig ? pv : (use_s ? rcp_nr(pv) : 1.f);
                    atomicAdd(&Wc[sj * LC + l], sg * iv * x);
                    if (use_s) dps[2 * j + (isy ? 0 : 1)] = dprec_nr(MT, beta, x, iv);
                    if (kSig) dps2[2 * j + (isy ? 0 : 1)] = pv;
                    if (cs) {   // (wide: both labels' |dW| summed - an upper bound of their max)
                      atomicAdd(&rmx[sj], fabsf(sg * iv * x));
                      if (isy) dirty[sj] = 1;
                    }
                  }
                }
                // sigma cache, a row repeated in the sample (or wide): the
                // precisions back as P, the increments added, sigma again -
                // each pass reads everything before it writes
                auto each = [&](auto&& fn) __attribute__((always_inline)) {
                  for (int q0 = 0; q0 * G < n; q0 += QC) {
#pragma unroll
                    for (int u = 0; u < QC; ++u) {
                      const int j = (q0 + u) * G + g;
                      const int sj = j < n ? fring[(off + j) & (kFR - 1)].x : -1;
                      if (sj >= 0) fn(sj, 2 * j + (isy ? 0 : 1));
                    }
                  }
                };
                if (kSig) {
                  each([&](int sj, int d) { Pc[sj * LC + l] = rcp_nr(dps2[d]); });
                  each([&](int sj, int d) { atomicAdd(&Pc[sj * LC + l], dps[d]); });
                  each([&](int sj, int d) { dps2[d] = Pc[sj * LC + l]; });
                  each([&](int sj, int d) { Pc[sj * LC + l] = rcp_nr(dps2[d]); });
                } else if (use_s) {
                  for (int q0 = 0; q0 * G < n; q0 += QC) {
#pragma unroll
                    for (int u = 0; u < QC; ++u) {
                      const int j = (q0 + u) * G + g;
                      const int sj = j < n ? fring[(off + j) & (kFR - 1)].x : -1;
                      if (sj >= 0) atomicAdd(&Pc[sj * LC + l], dps[2 * j + (isy ? 0 : 1)]);
                    }
                  }
                }
              }
            }
          }
        }
      }
      if (lane == 0) lds_st(&ctl[C_PROGRESS], t + 1);
      if (s3 != 0) pc[P_ST_APPLY] += clk() - s3;
    }
    if (cs) {
      if (lane == 0) lds_st(&ctl[C_NUPD], (int)n_upd);   // (kernel D counts a committed window's updates)
    } else if (lane == 0 && stats != nullptr) {
      if (n_upd) atomicAdd(stats, (unsigned long long)n_upd);
      if (n_valid) atomicAdd(stats + 1, (unsigned long long)n_valid);
    }
    pc[P_STEP_TOTAL] = clk() - c_start;
    pc[P_SAMPLES] = (unsigned long long)N;
  } else if (wave == 2) {
    // ================================================================ meta
    int t0 = 0;
    int head = 0;   // feature ring write position (monotonic)
    while (t0 < N) {
      const int t = t0 + lane;
      const bool in = t < N;
      int64_t rp0 = 0, rp1 = 0;
      int y = -1;
      if (in) {
        const int64_t si = sidx(t);
        rp0 = row_ptr[si];
        rp1 = row_ptr[si + 1];
        y = labels[si];
      }
      const int n = (int)(rp1 - rp0);
      const bool vy = in && y >= 0 && y < LC;
      const int ns = (vy && n <= kFMax) ? n : 0;
      const int hn = !vy ? 0 : (n <= kFMax ? n : -1);
      int inc = ns;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const int v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
      }
      // a chunk whose features fit half the ring (a prefix of the lanes)
      const bool take = in && inc <= kFR / 2;
      const int cnt = __popcll(__ballot(take));
      const int total = __shfl(inc, cnt - 1, 64);
      const int ex = inc - ns;
      // room: the headers of [t0, t0 + cnt) and the chunk's features; strict
      // so the chunk never reuses the header (and fend) of sample prog - 1
      const uint64_t tw = __builtin_amdgcn_s_memrealtime();
      const uint64_t w0 = clk();
      bool dead = false;
      for (;;) {
        const int prog = lds_ld(&ctl[C_PROGRESS]);
        const int cons = prog > 0 ? lds_ld(&fend[(prog - 1) & (kSR - 1)]) : 0;
        if (t0 + cnt < prog + kSR && head + total - cons <= kFR) break;
        if (cs && lds_ld(&ctl[C_STOP]) < N) { dead = true; break; }   // the window ended: no more headers
        if (lds_ld(&ctl[C_ABORT]) != 0 || timed_out(tw)) { abort_with(kErrTimeoutMeta); dead = true; break; }
        __builtin_amdgcn_s_sleep(2);
      }
      pc[P_META_ROOM] += clk() - w0;
      if (dead) break;
      int mx = take ? ns : 0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = max(mx, __shfl_xor(mx, o, 64));
      const int base = head + ex;
      // dup: two features of the sample share a row (so a slot) - the stepper
      // then applies with LDS atomics; else with plain stores. Decided for
      // samples of <= 16 features (the stepper's one-pass case)
      int dup = 0;
      if (mx <= 16) {
        int id[16];
        float xv[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const bool on = take && i < ns;
          id[i] = on ? fidx[rp0 + i] : -1 - i;
          xv[i] = on ? fval[rp0 + i] : 0.f;
        }
#pragma unroll
        for (int i = 1; i < 16; ++i)
#pragma unroll
          for (int k = 0; k < i; ++k) dup |= id[i] == id[k] ? 1 : 0;
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (take && i < ns) fring[(base + i) & (kFR - 1)] = make_int2(id[i], __float_as_int(xv[i]));
      } else {
        for (int f0 = 0; f0 < mx; f0 += 8) {
          int id[8];
          float xv[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const bool on = take && f0 + i < ns;
            id[i] = on ? fidx[rp0 + f0 + i] : -1;
            xv[i] = on ? fval[rp0 + f0 + i] : 0.f;
          }
#pragma unroll
          for (int i = 0; i < 8; ++i)
            if (take && f0 + i < ns) fring[(base + f0 + i) & (kFR - 1)] = make_int2(id[i], __float_as_int(xv[i]));
        }
        dup = 1;
      }
      if (take) {
        const int hh = t & (kSR - 1);
        int* hp = reinterpret_cast<int*>(&hdr[hh]);
        lds_st(&hp[2], ((vy ? y : -1) + 1) << 16 | (dup ? kDupBit : 0) | ((hn + 1) & kNMask));
        lds_st(&hp[3], base);
        lds_st(&fend[hh], base + ns);
        lds_st(&hp[0], t);   // meta_seq last
      }
      head += total;
      t0 += cnt;
    }
    pc[P_META_TOTAL] = clk() - c_start;
  } else if (wave == 1) {
    // ================================================================ lookup
    // every feature row of the next sample -> a cache slot: hits keep their
    // way; a miss takes an empty way or the least recently used one the
    // stepper has passed (CAS on its key), and becomes a fetch job (row,
    // slot, the way's previous row) for the fetch wave
    int jhead = 0;   // job ring write position (monotonic)
    bool dead = false;
    // a sample the cache does not hold (wider than kFMax, or overflow): every
    // earlier sample stepped, its cached rows (and the previous rows of the
    // ways its partial lookup took) written back and dropped, then it is
    // handed on as direct; the lookup waits until the stepper is past it
    // (y < 0: a sample without a label whose group overflowed - only the
    // partial lookup is undone, the sample is handed on as it was)
    auto go_direct = [&](int t, int y, int jpos0) __attribute__((always_inline)) {
      if (!wait_progress(t, kErrTimeoutLoad)) { dead = true; return; }
      auto drop = [&](int sl, int wrow) {
        if (wrow >= 0 && dirty[sl] != 0) {
          for (int c = 0; c < LC; c += 4) {
            *reinterpret_cast<float4*>(W + (int64_t)wrow * LC + c) = *reinterpret_cast<const float4*>(Wc + sl * LC + c);
            if (use_s)
              *reinterpret_cast<float4*>(P + (int64_t)wrow * LC + c) =
                  to_hbm(*reinterpret_cast<const float4*>(Pc + sl * LC + c));
          }
          if (touched != nullptr) touched[wrow] = 1;
        }
        key[sl] = -1;
        use[sl] = -1;
        dirty[sl] = 0;
        for (int c = 0; c < LC; ++c) {
          Wc[sl * LC + c] = 0.f;
          Pc[sl * LC + c] = 1.f;
        }
      };
      // the ways this sample's partial lookup took: their previous rows go back
      for (int i = jpos0 + lane; i < jhead; i += 64) {
        const int4 jb = jobs[i & (kJR - 1)];
        drop(jb.y, jb.z);
      }
      jhead = jpos0;
      const int64_t s = sidx(t);
      const int64_t rb = row_ptr[s];
      const int n = y >= 0 ? (int)(row_ptr[s + 1] - rb) : 0;
      for (int j0 = 0; j0 < n; j0 += 64) {
        const int j = j0 + lane;
        const int row = j < n ? fidx[rb + j] : -1;
        int sl = -1;
        if (row >= 0) {
          int b1, b2;
          buckets(row, NB, &b1, &b2);
          sl = find_in(key, b1, b2, row);
        }
        // one lane per slot (a row repeated in the sample)
        for (;;) {
          const uint64_t want = __ballot(sl >= 0);
          if (want == 0ull) break;
          const int lead = (int)__ffsll((long long)want) - 1;
          const int s0 = __builtin_amdgcn_readlane(sl, lead);
          if (lane == lead) drop(s0, row);
          if (sl == s0) sl = -1;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        if (y >= 0) lds_st(reinterpret_cast<int*>(&hdr[t & (kSR - 1)]) + 2, (y + 1) << 16);   // n = -1: direct
        int* lp = reinterpret_cast<int*>(&lk[t & (kSR - 1)]);
        lds_st(&lp[1], jhead);
        lds_st(&lp[2], -1);
        lds_st(&lp[0], t);
      }
      if (!wait_progress(t + 1, kErrTimeoutLoad)) dead = true;
    };
    auto lk_done = [&](int t, int jpos, int m) __attribute__((always_inline)) {
      if (lane == 0) {
        int* lp = reinterpret_cast<int*>(&lk[t & (kSR - 1)]);
        lds_st(&lp[1], jpos);
        lds_st(&lp[2], m);
        lds_st(&lp[0], t);   // lk_seq last
      }
    };

    // Samples of at most 16 features are looked up four at a time (lanes
    // 16 k + j: feature j of sample t + k), wider ones alone in 64-lane
    // chunks. A group's fetch jobs all count for its first sample, which is
    // then published last of them landing - the later ones of the group
    // carry no jobs, and the fetch wave publishes in order.
    int jdone_c = 0;   // the fetch wave's consumed-job count, as last read
    for (int t = 0; t < N && !dead;) {
      int4 h0 = lds_ld(&hdr[t & (kSR - 1)]);
      if (h0.x != t) {
        const uint64_t w0 = clk();
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while ((h0 = lds_ld(&hdr[t & (kSR - 1)])).x != t) {
          if (lds_ld(&ctl[C_ABORT]) != 0 || timed_out(t0)) { abort_with(kErrTimeoutLoad); dead = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        pc[P_LOAD_IDLE] += clk() - w0;
        if (dead) break;
      }
      const int y0 = (h0.z >> 16) - 1;
      const int n0 = (h0.z & kNMask) - 1;
      if (y0 >= 0 && n0 < 0) {
        if (cs) {   // (candidate mode writes no HBM rows: the window ends before t)
          if (lane == 0) lds_st(&ctl[C_STOP], t);
          break;
        }
        pc[P_DIRECT] += 1;
        go_direct(t, y0, jhead);
        ++t;
        continue;
      }
      // the group: sample t and the next ready ones of <= 16 features
      const int gk = lane >> 4, gj = lane & 15;
      const int4 hk = gk == 0 ? h0 : lds_ld(&hdr[(t + gk) & (kSR - 1)]);
      const int yk = (hk.z >> 16) - 1, nk = (hk.z & kNMask) - 1;
      const bool small_k = hk.x == t + gk && t + gk < N && (yk < 0 || (nk >= 0 && nk <= 16));
      const uint64_t okm = __ballot(gj == 0 && small_k) & 0x0001000100010001ull;
      // consecutive ready groups from k = 0 (the bit of group k is lane 16 k)
      int K = 0;
      while (K < 4 && ((okm >> (16 * K)) & 1ull)) ++K;
      const bool single = K == 0;   // sample t is wider than 16 features
      if (single) K = 1;
      const int n_lanes = single ? n0 : 16;
      const uint64_t l0 = clk();
      const int jpos0 = jhead;
      int prog = lds_ld(&ctl[C_PROGRESS]);
      bool overflow = false;
      for (int c0 = 0; c0 < n_lanes && !overflow && !dead; c0 += 64) {
        // room in the job ring for this pass's misses
        if (jhead + 64 - jdone_c > kJR) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          while (jhead + 64 - (jdone_c = lds_ld(&ctl[C_JDONE])) > kJR) {
            if (lds_ld(&ctl[C_ABORT]) != 0 || timed_out(t0)) { abort_with(kErrTimeoutLoad); dead = true; break; }
            __builtin_amdgcn_s_sleep(1);
          }
          if (dead) break;
        }
        const int kk = single ? 0 : gk;
        const int j = single ? c0 + lane : gj;
        const int tk = t + kk;
        const int4 hh = single ? h0 : hk;
        const int yh = (hh.z >> 16) - 1, nh = (hh.z & kNMask) - 1;
        const bool in = kk < K && yh >= 0 && j < nh;
        int2* fe = &fring[(hh.w + j) & (kFR - 1)];
        const int row = in ? lds_ld(&fe->x) : -1;
        int b1 = 0, b2 = 0;
        if (row >= 0) buckets(row, NB, &b1, &b2);
        int4 k1 = make_int4(-1, -1, -1, -1), k2 = k1;
        if (row >= 0) {
          k1 = lds_ld(reinterpret_cast<const int4*>(key + 4 * b1));
          k2 = lds_ld(reinterpret_cast<const int4*>(key + 4 * b2));
        }
        auto match = [&]() -> int {
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
        };
        int sl = row >= 0 ? match() : -1;
        const uint64_t lk1 = clk();
        pc[P_LK_KEYS] += lk1 - l0;
        // hits are marked (the latest sample of the group that holds the
        // row) before any lane reads the ways' last uses - LDS keeps this
        // wave's order - so no lane evicts a row the group holds
        if (sl >= 0) atomicMax(&use[sl], tk);
        bool need = row >= 0 && sl < 0;
        bool first = true;
        uint64_t ts = 0;
        while (__ballot(need) != 0ull) {
          bool mine = false, stuck = false;
          int vk = -1;
          if (need) {
            if (!first) {   // another lane may have taken this row's way meanwhile
              k1 = lds_ld(reinterpret_cast<const int4*>(key + 4 * b1));
              k2 = lds_ld(reinterpret_cast<const int4*>(key + 4 * b2));
              sl = match();
              if (sl >= 0) { atomicMax(&use[sl], tk); need = false; }
            }
            if (need) {
              const int4 u1 = lds_ld(reinterpret_cast<const int4*>(use + 4 * b1));
              const int4 u2 = lds_ld(reinterpret_cast<const int4*>(use + 4 * b2));
              // (candidate mode: a way holding an updated row stays pinned)
              int4 d1 = make_int4(0, 0, 0, 0), d2 = d1;
              if (cs) {
                d1 = lds_ld(reinterpret_cast<const int4*>(dirty + 4 * b1));
                d2 = lds_ld(reinterpret_cast<const int4*>(dirty + 4 * b2));
              }
              int v = -1, vu = 0x7fffffff;
              auto cand = [&](int s, int k, int u, int dv) {
                const int score = k < 0 ? -2 : u;   // an empty way first, else the least recently used
                if ((k < 0 || (u < prog && dv == 0)) && score < vu) { v = s; vu = score; vk = k; }
              };
              cand(4 * b1, k1.x, u1.x, d1.x);
              cand(4 * b1 + 1, k1.y, u1.y, d1.y);
              cand(4 * b1 + 2, k1.z, u1.z, d1.z);
              cand(4 * b1 + 3, k1.w, u1.w, d1.w);
              cand(4 * b2, k2.x, u2.x, d2.x);
              cand(4 * b2 + 1, k2.y, u2.y, d2.y);
              cand(4 * b2 + 2, k2.z, u2.z, d2.z);
              cand(4 * b2 + 3, k2.w, u2.w, d2.w);
              if (v >= 0) {
                if (atomicCAS(&key[v], vk, row) == vk) {
                  atomicMax(&use[v], tk);
                  sl = v;
                  need = false;
                  mine = true;
                }
              } else {
                stuck = true;
              }
            }
          }
          first = false;
          pc[P_LK_ITERS] += 1;
          const uint64_t mb = __ballot(mine);
          if (mine) {
            const int pos = jhead + __popcll(mb & ((1ull << lane) - 1ull));
            jobs[pos & (kJR - 1)] = make_int4(row, sl, vk, 0);
          }
          jhead += __popcll(mb);
          const uint64_t nb = __ballot(need);
          if (nb != 0ull && nb == __ballot(stuck)) {
            // every open lane lacks a free way: wait for the stepper; once it
            // has passed every earlier sample, the group itself holds the ways
            // (overflow: sample t goes direct, the rest of the group again)
            const uint64_t w0 = clk();
            if (prog >= t) {
              overflow = true;
            } else {
              if (ts == 0) ts = __builtin_amdgcn_s_memrealtime();
              if (lds_ld(&ctl[C_ABORT]) != 0 || timed_out(ts)) { abort_with(kErrTimeoutLoad); dead = true; break; }
              __builtin_amdgcn_s_sleep(1);
              prog = lds_ld(&ctl[C_PROGRESS]);
            }
            pc[P_LOAD_STUCK] += clk() - w0;
            if (overflow) break;
          }
        }
        pc[P_LK_CAS] += clk() - lk1;
        if (!overflow && in) lds_st(&fe->x, sl);
      }
      pc[P_LOAD_LOOKUP] += clk() - l0;
      if (dead) break;
      if (overflow) {
        if (cs) {   // the cache cannot pin another updated row: the window ends before t
          if (lane == 0) lds_st(&ctl[C_STOP], t);
          break;
        }
        pc[P_DIRECT] += 1;
        go_direct(t, y0, jpos0);
        ++t;
        continue;
      }
      pc[P_MISSES] += (unsigned long long)(jhead - jpos0);
      // the group's lookup records (its jobs on the first sample), in order
      if (gj == 0 && gk < K) {
        int* lp = reinterpret_cast<int*>(&lk[(t + gk) & (kSR - 1)]);
        lds_st(&lp[1], gk == 0 ? jpos0 : jhead);
        lds_st(&lp[2], gk == 0 ? jhead - jpos0 : 0);
        lds_st(&lp[0], t + gk);
      }
      t += K;
    }
    if (dead) abort_with(kErrTimeoutLoad);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pc[P_LOAD_TOTAL] = clk() - c_start;
  } else {
    // ================================================================ fetch
    // the jobs of each looked-up sample, in order: the way's previous row
    // written back when the stepper had written it, the new row fetched with
    // LDS-DMA loads into a staging buffer (kK stages in flight, counted
    // vmcnt waits), copied into its slot when it lands; then the samples a
    // landed stage completes are published to the stepper
    const int part = lane % LPR;   // this lane's 16 B of a row in a fetch stage
    const int rin = lane / LPR;    // its row within the stage
    float* dummy = g_dummy + 4 * lane;
    int pend = 0;                  // stages in flight
    int shead = 0;                 // next stage buffer
    int pub_done = 0;              // samples published: [0, pub_done)
    bool dead = false;
    auto publish_to = [&](int upto) __attribute__((always_inline)) {
      for (int b = pub_done; b <= upto; b += 64) {
        const int s = b + lane;
        if (s <= upto) lds_st(reinterpret_cast<int*>(&hdr[s & (kSR - 1)]) + 1, s);
      }
      pub_done = upto + 1;
    };
    auto retire = [&]() __attribute__((always_inline)) {
      const uint64_t w0 = clk();
      wait_stages(pend - 1);
      pc[P_LOAD_RETIRE] += clk() - w0;
      const int b = (shead - pend + kK) & (kK - 1);
      const int sl = lds_ld(&st_slot[b * 64 + lane]);
      const int pub = lds_ld(&st_pub[b]);
      const float4 w = lds_ld(reinterpret_cast<const float4*>(stage + b * 2048 + 16 * lane));
      float4 p = w;
      if (use_s) p = lds_ld(reinterpret_cast<const float4*>(stage + b * 2048 + 1024 + 16 * lane));
      if (sl >= 0) {
        *reinterpret_cast<float4*>(Wc + sl * LC + 4 * part) = w;
        if (use_s) *reinterpret_cast<float4*>(Pc + sl * LC + 4 * part) = kSig ? rcp4(p) : p;
      }
      if (pub >= 0) publish_to(pub);
      --pend;
    };
    // one fetch stage: jobs [jp, jp + m) (m <= RPS); kC VMEM instructions
    // every time (padding to g_dummy), so the waits can count
    auto issue_stage = [&](int jp, int m, int pub) __attribute__((always_inline)) {
      if (pend == kK) retire();
      pc[P_STAGES] += 1;
      const int b = shead;
      const bool on = rin < m;
      const int4 jb = jobs[(jp + (on ? rin : 0)) & (kJR - 1)];
      const int row = on ? jb.x : -1;
      const int sl = on ? jb.y : 0;
      const int old = on ? jb.z : -1;
      // the way's previous contents, read whether or not they go back
      const int dv = dirty[sl];
      const float4 ow = lds_ld(reinterpret_cast<const float4*>(Wc + sl * LC + 4 * part));
      float4 op = ow;
      if (use_s) op = to_hbm(lds_ld(reinterpret_cast<const float4*>(Pc + sl * LC + 4 * part)));
      const bool dirt = on && old >= 0 && dv != 0;
      float* dw = dirt ? W + (int64_t)old * LC + 4 * part : dummy;
      float* dp = (dirt && use_s) ? P + (int64_t)old * LC + 4 * part : dummy;
      uint8_t* dt = (dirt && part == 0 && touched != nullptr) ? touched + old : reinterpret_cast<uint8_t*>(dummy);
      *reinterpret_cast<float4*>(dw) = ow;
      *reinterpret_cast<float4*>(dp) = op;
      *dt = 1;
      // every cached row goes back when evicted; candidate mode: only rows the
      // stepper updated count (and those are never evicted), with their bound
      if (on && part == 0) {
        dirty[sl] = cs ? 0 : 1;
        if (cs) rmx[sl] = 0.f;
      }
      const float* sw = on ? W + (int64_t)row * LC + 4 * part : dummy;
      const float* sp = (on && use_s) ? P + (int64_t)row * LC + 4 * part : dummy;
      const uint32_t lb = __builtin_amdgcn_readfirstlane(lds_addr(stage + b * 2048));
      glds16(sw, lb);
      glds16(sp, lb + 1024);
      st_slot[b * 64 + lane] = on ? sl : -1;
      if (lane == 0) st_pub[b] = pub;
      shead = (shead + 1) & (kK - 1);
      ++pend;
    };

    int t = 0;
    uint64_t tw = __builtin_amdgcn_s_memrealtime();
    while (!dead) {
      const int Ne = cs ? min(N, lds_ld(&ctl[C_STOP])) : N;   // (candidate mode: up to the window's end)
      if (!(t < Ne || pend > 0)) break;
      int4 lkv = make_int4(-1, 0, 0, 0);
      if (t < Ne) lkv = lds_ld(&lk[t & (kSR - 1)]);
      if (t >= Ne || lkv.x != t) {
        if (pend > 0) {
          retire();
        } else {
          if (lds_ld(&ctl[C_ABORT]) != 0 || timed_out(tw)) { abort_with(kErrTimeoutFetch); dead = true; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        continue;
      }
      tw = __builtin_amdgcn_s_memrealtime();
      const uint64_t i0c = clk();
      const int jpos = lkv.y, m = lkv.z;
      if (m <= 0) {   // nothing to fetch (m -1: direct, everything before it is published)
        if (pend == 0) publish_to(t);
        else if (lane == 0) st_pub[(shead - 1) & (kK - 1)] = t;
      } else {
        for (int i0 = 0; i0 < m; i0 += RPS) issue_stage(jpos + i0, min(RPS, m - i0), i0 + RPS >= m ? t : -1);
        if (lane == 0) lds_st(&ctl[C_JDONE], jpos + m);
      }
      pc[P_LOAD_ISSUE] += clk() - i0c;
      ++t;
    }
    if (dead) abort_with(kErrTimeoutFetch);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    pc[P_FETCH_TOTAL] = clk() - c_start;
  }
  // ---- write the cache back (all waves)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  constexpr int Q = LC / 4;
  if (cs) {
    // candidate mode: the window's updated rows staged as kernel C stages its
    // store - keys and rmax in this cache's slot layout (kernel D looks rows
    // up with vc::sp_find), the deltas to the model at the window's start
    constexpr int NSD = 16384 / (LC > 16 ? LC : 16);   // kernel D's table (jb_commit.hpp dc::Geo NSLOT)
    static_assert(NSLOT <= NSD, "the staged table holds the cache");
    for (int i = tid; i < NSD; i += kT) {
      const bool on = i < NSLOT && key[i] >= 0 && dirty[i] != 0;
      g_key[i] = on ? key[i] : -1;
      g_rmax[i] = on ? rmx[i] : 0.f;
    }
    for (int i = tid; i < NSLOT * Q; i += kT) {
      const int sl = i / Q;
      const int k = key[sl];
      if (k < 0 || dirty[sl] == 0) continue;
      const int c = (i % Q) * 4;
      const float4 w0 = *reinterpret_cast<const float4*>(W + (int64_t)k * LC + c);
      const float4 wn = *reinterpret_cast<const float4*>(Wc + sl * LC + c);
      *reinterpret_cast<float4*>(g_dw + sl * LC + c) =
          make_float4(wn.x - w0.x, wn.y - w0.y, wn.z - w0.z, wn.w - w0.w);
      if (use_s) {
        const float4 p0 = *reinterpret_cast<const float4*>(P + (int64_t)k * LC + c);
        const float4 pn = to_hbm(*reinterpret_cast<const float4*>(Pc + sl * LC + c));
        *reinterpret_cast<float4*>(g_dp + sl * LC + c) =
            make_float4(pn.x - p0.x, pn.y - p0.y, pn.z - p0.z, pn.w - p0.w);
      }
    }
    if (tid == 0) {
      const int stop = ctl[C_STOP];
      const bool stopped = stop < N;
      int nsl = 0;
      for (int i = 0; i < NSLOT; ++i) nsl += (key[i] >= 0 && dirty[i] != 0) ? 1 : 0;
      vst[vc::S_PEND] = stopped ? beg + aux[stop].w : vst[vc::S_WEND];
      vst[vc::S_WHY] = stopped ? vc::kWhySat : vc::kWhyEnd;
      vst[vc::S_NUPD] = ctl[C_NUPD];
      vst[vc::S_NSLOTS] = nsl;
      vst[vc::S_STEPS] += stopped ? stop : N;
      vst[vc::S_CAND] += N;
      vst[vc::S_CSN] += 1;
    }
  } else {
    for (int i = tid; i < NSLOT * Q; i += kT) {
      const int sl = i / Q;
      const int k = key[sl];
      if (k < 0 || dirty[sl] == 0) continue;
      const int c = (i % Q) * 4;
      *reinterpret_cast<float4*>(W + (int64_t)k * LC + c) = *reinterpret_cast<const float4*>(Wc + sl * LC + c);
      if (use_s)
        *reinterpret_cast<float4*>(P + (int64_t)k * LC + c) =
            to_hbm(*reinterpret_cast<const float4*>(Pc + sl * LC + c));
      if (c == 0 && touched != nullptr) touched[k] = 1;
    }
  }
  if (tid == 0 && ctl[C_ABORT] != 0 && err != nullptr) atomicMax(err, ctl[C_WHY] != 0 ? ctl[C_WHY] : 9);
  if (tid == 0 && mode == kModeChunk) {
    // the batch back to the committer from the chunk's end
    const int64_t bend = vst[vc::S_BEND];
    const bool done = end >= bend;
    vst[vc::S_BEG] = end;
    vst[vc::S_STATUS] = done ? vc::kDone : vc::kNew;
    vst[vc::S_STEPPED] += end - beg;
    vst[vc::S_NCHUNK] += 1;
    vst[vc::S_DCHUNK] = min(2 * vst[vc::S_DCHUNK], vc::kDenseChunkMax);
    vtail[0] = done ? bend : end;
    vtail[1] = bend;
    vtail[vc::kTailReasonW] = done ? vc::kReasonDone : vc::kReasonSaturated;
    vtail[vc::kTailStepped] = vst[vc::S_STEPPED];
    vtail[vc::kTailChunks] = vst[vc::S_NCHUNK];
    vtail[vc::kTailSegEst] = vc::seg_estimate(vst);
  }
  if (PROF && prof != nullptr && lane == 0) {
#pragma unroll
    for (int i = 0; i < P_NWORDS; ++i)
      if (pc[i] != 0) atomicAdd(prof + i, pc[i]);
  }
}

}  // namespace sp
}  // namespace jb

// The stepper over samples [range[0], range[1]) (device int64 pair) of a
// batch, applied one after another to W / P (fp32, LC <= 64). err (device
// int, nullable): set > 0 if a wait timed out (the kernel then ends early;
// never expected). Returns -1 for a label capacity it does not cover.
// stepper abort reason since the last call (0: none); resets it
extern "C" int jb_stepper_error() {
  int v = 0;
  if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(jb::sp::g_err), sizeof(int), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  if (v != 0) {
    const int z = 0;
    (void)hipMemcpyToSymbol(HIP_SYMBOL(jb::sp::g_err), &z, sizeof(int), 0, hipMemcpyHostToDevice);
  }
  return v;
}

// JB_STEPPER_PROF=1: the launches accumulate per-wave phase cycles into
// g_prof (label capacities 8 and 16; the others run unprofiled);
// jb_stepper_prof copies them out (uint64 [P_NWORDS]) and resets them
static bool stepper_prof_on() {
  static const bool on = [] {
    const char* e = getenv("JB_STEPPER_PROF");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}
extern "C" int jb_stepper_prof(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(jb::sp::g_prof), sizeof(unsigned long long) * jb::sp::P_NWORDS, 0,
                          hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  unsigned long long z[jb::sp::P_NWORDS] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(jb::sp::g_prof), z, sizeof z, 0, hipMemcpyHostToDevice);
  return 0;
}

// JB_STEPPER=0: the single-stream exact samples go to the old one-wave
// kernel (linear.hip) instead (A/B runs)
extern "C" int jb_stepper_enabled() {
  static const int on = [] {
    const char* e = getenv("JB_STEPPER");
    return (e != nullptr && e[0] == '0') ? 0 : 1;
  }();
  return on;
}

static int stepper_launch(const int64_t* row_ptr, const int32_t* fidx, const float* fval, const int32_t* labels,
                          const int64_t* range, float* W, float* P, const int32_t* active, int LC, int method,
                          float C, unsigned long long* stats, uint8_t* touched, int* err, int64_t* vst,
                          int64_t* vtail, hipStream_t stream, int mode = jb::sp::kModeRange,
                          const int4* aux = nullptr, int32_t* g_key = nullptr, float* g_rmax = nullptr,
                          float* g_dw = nullptr, float* g_dp = nullptr) {
  if (LC < 8 || LC > 64) return -1;
  if (method >= jb::CW && P == nullptr) return -4;
  if (err == nullptr) {
    static int* g = [] {
      void* a = nullptr;
      return hipGetSymbolAddress(&a, HIP_SYMBOL(jb::sp::g_err)) == hipSuccess ? (int*)a : nullptr;
    }();
    err = g;
  }
  unsigned long long* prof = nullptr;
  if (stepper_prof_on()) {
    static unsigned long long* gp = [] {
      void* a = nullptr;
      return hipGetSymbolAddress(&a, HIP_SYMBOL(jb::sp::g_prof)) == hipSuccess ? (unsigned long long*)a : nullptr;
    }();
    prof = gp;
  }
#define JB_SP_LAUNCH_P(L, M, PR)                                                                              \
  {                                                                                                           \
    static bool attr = [] {                                                                                   \
      return hipFuncSetAttribute((const void*)jb::sp::stepper_kernel<L, M, PR>,                              \
                                 hipFuncAttributeMaxDynamicSharedMemorySize, jb::sp::Geo<L>::kBytes) ==      \
             hipSuccess;                                                                                      \
    }();                                                                                                      \
    (void)attr;                                                                                               \
    hipLaunchKernelGGL((jb::sp::stepper_kernel<L, M, PR>), dim3(1), dim3(jb::sp::kT), jb::sp::Geo<L>::kBytes, \
                       stream, row_ptr, fidx, fval, labels, range, W, P, active, C, stats, touched, err, prof,     \
                       vst, vtail, mode, aux, g_key, g_rmax, g_dw, g_dp);                                    \
  }
  // the phase counters are compiled into the label-capacity 8 and 16 kernels only
#define JB_SP_LAUNCH(L, M)                                   \
  if constexpr (L <= 16) {                                   \
    if (prof != nullptr) JB_SP_LAUNCH_P(L, M, true)          \
    else JB_SP_LAUNCH_P(L, M, false)                         \
  } else {                                                   \
    JB_SP_LAUNCH_P(L, M, false)                              \
  }
#define JB_SP_M(L)                                          \
  switch (method) {                                         \
    case jb::PERCEPTRON: JB_SP_LAUNCH(L, jb::PERCEPTRON) break; \
    case jb::PA: JB_SP_LAUNCH(L, jb::PA) break;             \
    case jb::PA1: JB_SP_LAUNCH(L, jb::PA1) break;           \
    case jb::PA2: JB_SP_LAUNCH(L, jb::PA2) break;           \
    case jb::CW: JB_SP_LAUNCH(L, jb::CW) break;             \
    case jb::AROW: JB_SP_LAUNCH(L, jb::AROW) break;         \
    case jb::NHERD: JB_SP_LAUNCH(L, jb::NHERD) break;       \
    default: return -1;                                     \
  }
  switch (LC) {
    case 8: JB_SP_M(8) break;
    case 16: JB_SP_M(16) break;
    case 32: JB_SP_M(32) break;
    case 64: JB_SP_M(64) break;
    default: return -1;
  }
#undef JB_SP_M
#undef JB_SP_LAUNCH
#undef JB_SP_LAUNCH_P
  return (int)hipGetLastError();
}

extern "C" int jb_stepper_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                const int32_t* labels, const int64_t* range, float* W, float* P,
                                const int32_t* active, int LC, int method, float C, unsigned long long* stats,
                                uint8_t* touched, int* err, hipStream_t stream) {
  return stepper_launch(row_ptr, fidx, fval, labels, range, W, P, active, LC, method, C, stats, touched, err, nullptr,
                        nullptr, stream);
}

// One chunk of a verified-committer batch after an update-dense window
// (vcommit.hip launches it after every segment): [S_BEG, S_BEG + S_DCHUNK)
// of the batch when vst's status is kDense, then the status is kNew (kDone at
// the batch end) and the next segment continues from the chunk's end; an
// empty launch otherwise.
extern "C" int jb_stepper_chunk(const int64_t* row_ptr, const int32_t* fidx, const float* fval, const int32_t* labels,
                                float* W, float* P, const int32_t* active, int LC, int method, float C,
                                unsigned long long* stats, uint8_t* touched, int64_t* vst, int64_t* vtail,
                                hipStream_t stream) {
  if (vst == nullptr || vtail == nullptr) return -2;
  return stepper_launch(row_ptr, fidx, fval, labels, nullptr, W, P, active, LC, method, C, stats, touched, nullptr,
                        vst, vtail, stream, jb::sp::kModeChunk);
}

// The candidates of a verified-committer window (vcommit.hip, in kernel C's
// place when kernel B set S_CSMODE): [0, S_NCAND) in order, sample
// S_BEG + aux[k].w, from the model at the window's start; the updated rows
// staged into (g_key, g_rmax, g_dw, g_dp) as kernel C stages its store, the
// stop position / updates into the state words; W / P untouched. An empty
// launch unless the window is live and in candidate mode.
extern "C" int jb_stepper_cand(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                               const int32_t* labels, float* W, float* P, const int32_t* active, int LC, int method,
                               float C, int64_t* vst, const int4* aux, int32_t* g_key, float* g_rmax, float* g_dw,
                               float* g_dp, hipStream_t stream) {
  if (vst == nullptr || aux == nullptr || g_key == nullptr) return -2;
  return stepper_launch(row_ptr, fidx, fval, labels, nullptr, W, P, active, LC, method, C, nullptr, nullptr, nullptr,
                        vst, nullptr, stream, jb::sp::kModeCand, aux, g_key, g_rmax, g_dw, g_dp);
}
