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
//      W / P tables, which nothing writes while the segment runs), its best
//      wrong label at M0 and, per feature, the precisions P0(row, y) and
//      P0(row, that label) - the step of a sample reads them from its
//      registers instead of a dependent global load.
//   2. delta_commit_kernel (ONE 512-thread workgroup, 8 waves = 32 groups of
//      16 lanes; a group is a DPP row): walks the batch in order, 64 samples
//      per round, each group owning 2 consecutive samples with feature u /
//      label u on lane u of the row. Everything the segment writes lives in
//      LDS until it ends:
//        dW[slot][LC], dP[slot][LC]  the summed increments since M0 of every
//                                    row the segment wrote (row -> slot hash),
//      so the live model is M0 + the LDS deltas. Scores are kept EXACT:
//        - round start: lane u reads the dW row of its feature (4 x b128) and
//          a 16 x 16 transpose-reduce over the row (mirror / half-mirror /
//          quad DPP adds, no LDS round trip) gives lane l the correction of
//          label l; the exact margin gives the sample's slack to its update
//          threshold;
//        - the first sample whose slack is not positive takes the exact step
//          (its group reads P0 + dP, computes the method's coefficients and
//          adds the increments into LDS), stamping the rows it wrote with the
//          step id and their increments of the two labels it moved;
//        - every later sample of the round adds x * increment of its stamped
//          rows to those two label scores (one LDS probe per feature, two row
//          sums) and lowers its slack by the correction's size; only a sample
//          whose slack runs out recomputes its exact margin.
//      A sample that does not update costs no table access beyond these.
//   3. When the LDS row store is full the segment ends: the deltas are added
//      to W / P (one coalesced pass over the row hash), and the next segment
//      re-scores the rest of the batch against the new tables. A sample wider
//      than 32 features ends the committer; the rest of the batch runs the
//      single-stream exact kernel (linear.hip kExact), as in serial.hip.
//
// Rounding: scores are S0 + incremental corrections, summed in another order
// than a fresh recomputation; a sample whose margin lies within a relative
// guard band of its update threshold re-scores itself from the live model
// (M0 + dW) before the decision, so decisions match a plain sequential fp32
// pass. Semantics per update (a repeated row counts every time, each
// occurrence against the pre-sample state) are those of linear.hip's direct
// path; the oracle is jubatus_amd/models/linear_oracle.py.
#include "jb_commit.hpp"

namespace jb {
namespace dc {

// ------------------------------------------------------------ S0 scores
// Per sample i of the segment (sample beg + i), everything the committer
// reads of it, at addresses that depend on i alone (no descriptor load
// before the feature loads, so the committer prefetches two rounds ahead):
//   S0[i * LC + l]   score of label l at the segment start
//   AUX[i]           (label y | best active wrong label there << 8 | feature
//                    count << 16 - labels as int8, -1: none / invalid y;
//                    |x|^2, the slack to the method's update threshold
//                    there - both as float bits; 0)
//   FI / FX[i * 32 + f]  row and value of feature f < 32 (-1 / 0 past the end)
//   PP0[i * 32 + f]  (P0(row_f, y), P0(row_f, that label)) (P != nullptr)
// *wide: set when a sample has more than 16 features (the committer with
// two feature chunks per lane takes the segment)
template <int LC>
__global__ __launch_bounds__(256) void delta_s0_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, const int32_t* __restrict__ labels,
    const int64_t* __restrict__ stream_ptr, int nstreams, const float* __restrict__ W,
    const float* __restrict__ P, const int32_t* __restrict__ active, int method, float C,
    float* __restrict__ S0, int4* __restrict__ AUX, float2* __restrict__ PP0, int32_t* __restrict__ FI,
    float* __restrict__ FX, unsigned long long* __restrict__ wide, const int64_t* __restrict__ tail,
    const int64_t* __restrict__ reason) {
  using L = Lanes<LC>;
  static_assert(LC <= 64, "delta committer: LC <= 64");
  if (reason != nullptr && (*reason == kStopDense || *reason == kStopDone)) return;
  const int lane = threadIdx.x & 63;
  const int64_t beg = stream_ptr[0];
  const int64_t cnt = window_end(beg, stream_ptr[nstreams], tail) - beg;
  const int64_t nwaves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const int g = lane / L::LW;
  const int l0 = lane % L::LW;
  const bool la = l0 < LC && active[l0] != 0;
  for (int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; wid < cnt; wid += nwaves) {
    const int64_t s = beg + wid;
    const int64_t fb = row_ptr[s];
    const int n = (int)(row_ptr[s + 1] - fb);
    if (lane < kNFMax) {
      const bool in = lane < n;
      FI[wid * kNFMax + lane] = in ? fidx[fb + lane] : -1;
      FX[wid * kNFMax + lane] = in ? fval[fb + lane] : 0.f;
    }
    if (lane == 0 && n > 16) atomicOr(wide, 1ull);
    float acc = 0.f;
    for (int j = g; j < n; j += L::G) {
      const int32_t idx = fidx[fb + j];
      if (idx >= 0) acc += fval[fb + j] * W[(int64_t)idx * LC + l0];
    }
#pragma unroll
    for (int off = L::LW; off < 64; off <<= 1) acc += __shfl_xor(acc, off, 64);
    if (lane < LC) S0[wid * LC + lane] = acc;
    // |x|^2 over the sample's features (hashed-out slots count too, as in
    // the sequential kernel's norm)
    float q = 0.f;
    for (int j = lane; j < n; j += 64) {
      const float x = fval[fb + j];
      q += x * x;
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) q += __shfl_xor(q, off, 64);
    const int y = labels[s];
    if (y < 0 || y >= LC) {
      if (lane == 0) AUX[wid] = make_int4(aux_pack(-1, -1, n), __float_as_int(q), 0, 0);
      continue;
    }
    float b = (la && l0 != y) ? acc : -INFINITY;
    int bl = (la && l0 != y) ? l0 : -1;
#pragma unroll
    for (int off = 1; off < L::LW; off <<= 1) {
      const float ob = __shfl_xor(b, off, 64);
      const int ol = __shfl_xor(bl, off, 64);
      if (ol >= 0 && (bl < 0 || ob > b || (ob == b && ol < bl))) { b = ob; bl = ol; }
    }
    // the margin at M0 and its slack (group_margin / slack_of of the committer)
    const float sy = __shfl(acc, y, 64);
    const float best = bl >= 0 ? b : 0.f;
    const float sl0 = slack_of(method, sy - best, q, bl >= 0, C, sy, best);
    if (lane == 0) AUX[wid] = make_int4(aux_pack(y, bl, n), __float_as_int(q), __float_as_int(sl0), 0);
    if (P == nullptr) continue;
    if (lane < kNFMax) {
      float2 pp = make_float2(1.f, 1.f);
      if (lane < n) {
        const int32_t idx = fidx[fb + lane];
        if (idx >= 0) {
          pp.x = P[(int64_t)idx * LC + y];
          if (bl >= 0) pp.y = P[(int64_t)idx * LC + bl];
        }
      }
      PP0[wid * kNFMax + lane] = pp;
    }
  }
}

// one sample's record as loaded (group layout: lane u holds features u,
// u + 16); nothing reads it until the round it belongs to, so its loads stay
// in flight for PD rounds
template <int LC, int FC>
struct Raw {
  int32_t fi[FC];
  float fx[FC];
  float2 pp[FC];
  float s[Geo<LC>::K];
  int aux;       // AUX .x (labels, feature count)
  float nrm;     // AUX .y (read only by the methods that use |x|^2)
  float slack0;  // AUX .z
};

// one sample's round data
template <int LC, int FC>
struct Samp {
  int32_t fi[FC];
  float fx[FC];
  float py[FC];    // P0(row, y), P0(row, ls0)
  float pl[FC];
  float s[Geo<LC>::K];
  int y;           // -1: no sample / label out of range
  int ls0;
  int nf;
  float nrm;       // |x|^2
  float slack0;    // slack at M0 (the segment start)
};

// ------------------------------------------------------------ committer
// MT: the method, a template argument - the step's coefficient code, the
// precision path (CW / AROW / NHERD) and the slack thresholds fold away for
// the other methods. FC: feature chunks of 16 a lane holds (1: samples of at
// most 16 features, the registers it frees buy a deeper prefetch; 2: up to
// 32). Both are launched per segment; *wide (the S0 pass) picks one.
template <int LC, int MT, int FC>
__global__ __launch_bounds__(kT) void delta_commit_kernel(
    const int64_t* __restrict__ stream_ptr, int nstreams, float* __restrict__ W,
    float* __restrict__ P, const int32_t* __restrict__ active, float C,
    const float* __restrict__ S0_k, const int4* __restrict__ AUX_k, const float2* __restrict__ PP0_k,
    const int32_t* __restrict__ FI_k, const float* __restrict__ FX_k,
    unsigned long long* __restrict__ wide, unsigned long long* __restrict__ stats,
    uint8_t* __restrict__ touched, int64_t* __restrict__ tail, int seg, int prof) {
  const bool kProf = prof != 0;      // uniform: scalar branches
  auto cyc = [&]() -> uint64_t { return kProf ? __builtin_amdgcn_s_memtime() : 0; };
  using Gm = Geo<LC>;
  using S = Samp<LC, FC>;
  constexpr int K = Gm::K;
  constexpr int NSLOT = Gm::NSLOT;
  constexpr int NFM = 16 * FC;        // widest sample this variant takes
  if (seg > 0 && (tail[kTailReason] == kStopDense || tail[kTailReason] == kStopDone)) return;
  if ((*wide != 0) != (FC == 2)) return;
  __shared__ __attribute__((aligned(16))) float s_dw[NSLOT * LC + Gm::PAD];
  __shared__ __attribute__((aligned(16))) float s_dp[NSLOT * LC + Gm::PAD];
  __shared__ __attribute__((aligned(16))) int32_t s_key[NSLOT];   // row of each slot (-1: free)
  __shared__ int32_t s_sst[NSLOT];    // id of the last step that wrote the slot
  __shared__ float s_sdy[NSLOT];      // that step's increment of labels y / l
  __shared__ float s_sdl[NSLOT];
  __shared__ float s_rmax[NSLOT];     // a bound on max_l |dW[slot][l]| (sum of the |increments|)
  __shared__ unsigned s_nexact, s_nalive;
  __shared__ int s_cn, s_stop, s_upd, s_yk, s_lk, s_nins;
  __shared__ int s_first[2];
  __shared__ unsigned s_nupd, s_waste, s_refresh;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int sub = lane & 15;
  const int G = tid >> 4;
  const int wv = tid >> 6;
  constexpr int method = MT;
  constexpr bool use_s = MT >= CW;
  constexpr bool use_nrm = MT == PA || MT == PA1 || MT == PA2 || MT == CW;   // |x|^2 (slack_of, step_coeffs)
  const uint64_t t_k0 = cyc();
  const uint64_t w_k0 = kProf ? __builtin_amdgcn_s_memrealtime() : 0;
  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};   // start, barrier A, step, corrections, flush, init
  uint64_t wwork = 0;

  {
    float4* dw4 = reinterpret_cast<float4*>(s_dw);
    float4* dp4 = reinterpret_cast<float4*>(s_dp);
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int i = tid; i < (NSLOT * LC + Gm::PAD) / 4; i += kT) { dw4[i] = z; if (use_s) dp4[i] = z; }
    for (int i = tid; i < NSLOT; i += kT) s_key[i] = -1;
    for (int i = tid; i < NSLOT; i += kT) s_sst[i] = -1;
    for (int i = tid; i < NSLOT; i += kT) s_rmax[i] = 0.f;
    if (tid == 0) {
      s_cn = 0; s_stop = -1; s_upd = 0; s_yk = -1; s_lk = -1; s_nins = 0;
      s_first[0] = s_first[1] = kInf;
      s_nupd = 0; s_waste = 0; s_refresh = 0; s_nexact = 0; s_nalive = 0;
    }
  }
  int act[K];   // ints, not lane masks: every bool array held across the loop is an SGPR pair
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int lab = sub + 16 * k;
    act[k] = (lab < LC && active[lab] != 0) ? 1 : 0;
  }
  const float* __restrict__ S0 = in_vgpr(S0_k);
  const int4* __restrict__ AUX = in_vgpr(AUX_k);
  const float2* __restrict__ PP0 = in_vgpr(PP0_k);
  const int32_t* __restrict__ FI = in_vgpr(FI_k);
  const float* __restrict__ FX = in_vgpr(FX_k);
  // [beg, end): this segment's window; bend: the batch end
  const int64_t bend = stream_ptr[nstreams];
  const int64_t beg = (int64_t)in_vgpr((uint64_t)stream_ptr[0]);
  const int64_t end = (int64_t)in_vgpr((uint64_t)window_end(stream_ptr[0], bend, tail));

  // sample loads PD rounds ahead, at addresses of the sample index alone;
  // no branches: a position past the batch reads the last sample's record
  // (the round that uses it selects the neutral values)
  using R = Raw<LC, FC>;
  auto load_raw = [&](int64_t p, R (&rw)[kR]) {
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int64_t j = p + G * kR + r;
      int64_t jc = (j < end ? j : end - 1) - beg;
      jc = jc < 0 ? 0 : jc;             // an empty range reads record 0 (the scratch holds >= 1)
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        const int64_t o = jc * kNFMax + c * 16 + sub;
        rw[r].fi[c] = gld(FI + o);
        rw[r].fx[c] = gld(FX + o);
        if (use_s) rw[r].pp[c] = gld(PP0 + o);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const int lab = sub + 16 * k;
        rw[r].s[k] = gld(S0 + jc * LC + (lab < LC ? lab : LC - 1));
      }
      // only the words the method reads: a loaded register nothing reads
      // is reused at once, and that write waits for the load (vmcnt(0))
      const int* a = reinterpret_cast<const int*>(AUX + jc);
      rw[r].aux = gld(a);
      rw[r].slack0 = __int_as_float(gld(a + 2));
      if (use_nrm) rw[r].nrm = __int_as_float(gld(a + 1));
    }
  };
  auto unpack = [&](int64_t p, const R (&rw)[kR], S (&sm)[kR]) {
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const bool ok = p + G * kR + r < end;
#pragma unroll
      for (int c = 0; c < FC; ++c) {
        sm[r].fi[c] = ok ? rw[r].fi[c] : -1;
        sm[r].fx[c] = ok ? rw[r].fx[c] : 0.f;
        sm[r].py[c] = (use_s && ok) ? rw[r].pp[c].x : 1.f;
        sm[r].pl[c] = (use_s && ok) ? rw[r].pp[c].y : 1.f;
      }
#pragma unroll
      for (int k = 0; k < K; ++k) sm[r].s[k] = (ok && sub + 16 * k < LC) ? rw[r].s[k] : 0.f;
      const int aux = rw[r].aux;
      sm[r].y = ok ? aux_y(aux) : -1;
      sm[r].ls0 = (use_s && ok) ? aux_ls(aux) : -1;
      sm[r].nf = ok ? aux_nf(aux) : 0;
      sm[r].nrm = (use_nrm && ok) ? rw[r].nrm : 0.f;
      sm[r].slack0 = ok ? rw[r].slack0 : 1.f;
    }
  };

  // pf[i]: the records of round p + i kNS (prefetch depth PD)
  constexpr int PD = FC == 1 ? 3 : 2;
  S sc[kR];
  R pf[PD][kR];
#pragma unroll
  for (int i = 0; i < PD; ++i) load_raw(beg + i * kNS, pf[i]);
  __syncthreads();
  ph[5] = cyc() - t_k0;

  int64_t stop = end;
  int64_t why = kStopDone;
  unsigned n_valid = 0;
  int iter = 0;
  int n_steps = 0;
  int64_t n_rounds = 0;

  // one round at p (the samples p .. p + kNS - 1, already in sc)
  auto round = [&](int64_t p, uint64_t tt) __attribute__((always_inline)) {

    // ---- round start: slots, deltas of the rows the segment wrote, slacks
    int alive[kR], unsafe[kR], exact[kR];
    float slack[kR];
    int slot[kR][FC];
    bool widew = false;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      alive[r] = (sc[r].y >= 0 && sc[r].y < LC) ? 1 : 0;
      widew |= alive[r] && sc[r].nf > 16;
    }
    // the second feature chunk only when a sample of the wave has one
    const bool two = FC == 2 && __builtin_amdgcn_ballot_w64(widew) != 0;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const bool ok = alive[r] && sc[r].nf <= NFM;
      slot[r][0] = ok ? cache_find<LC>(s_key, sc[r].fi[0]) : -1;
      if (FC == 2) {
        slot[r][FC - 1] = -1;
        if (two) slot[r][FC - 1] = ok ? cache_find<LC>(s_key, sc[r].fi[FC - 1]) : -1;
      }
    }
    // samples of this wave whose slack ran out (positions > after) and are
    // still on S0 scores: exact scores S0 + x . dW (the live deltas), exact
    // margin and slack. Wave-uniform call; most waves have none.
    auto make_exact = [&](int after) {
      bool need[kR];
      bool anyneed = false;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        need[r] = alive[r] && !exact[r] && sc[r].nf <= NFM && G * kR + r > after && !(slack[r] > 0.f);
        anyneed |= need[r];
      }
      if (__builtin_amdgcn_ballot_w64(anyneed) == 0) return;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        float t[K];
#pragma unroll
        for (int k = 0; k < K; ++k) t[k] = sc[r].s[k];
        row_correct<LC, FC>(s_dw, slot[r], sc[r].fx, sub, two, t);
        int ls;
        float sy, best;
        const float m = group_margin<LC>(t, sc[r].y, act, sub, &ls, &sy, &best);
        const float sl = slack_of(method, m, sc[r].nrm, ls >= 0, C, sy, best);
        if (need[r]) {
#pragma unroll
          for (int k = 0; k < K; ++k) sc[r].s[k] = t[k];
          slack[r] = sl;
          exact[r] = 1;
          if (kProf && sub == 0) atomicAdd(&s_nexact, 1u);
        }
      }
    };
    // slack at round start: the slack at M0 less a bound on what the
    // segment's deltas moved the margin (2 sum_f |x_f| max_l |dW_f[l]|; the
    // guard band moves by 1e-4 of it). Scores stay S0 until a sample's slack
    // runs out; then (make_exact) it is scored exactly against M0 + dW.
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      float bsum = 0.f;
#pragma unroll
      for (int c = 0; c < FC; ++c)
        bsum += slot[r][c] >= 0 ? fabsf(sc[r].fx[c]) * s_rmax[slot[r][c]] : 0.f;
      slack[r] = sc[r].slack0 - 2.f * (1.f + 4.f * kGuard) * row16_sum(bsum);
      exact[r] = 0;
    }
    make_exact(-1);
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      unsafe[r] = (alive[r] && (sc[r].nf > NFM || !(slack[r] > 0.f))) ? 1 : 0;
      if (kProf && sub == 0 && alive[r] && sc[r].nf <= NFM) atomicAdd(&s_nalive, 1u);
    }
    {
      const uint64_t t2 = cyc();
      ph[0] += t2 - tt;
      wwork += t2 - tt;
      tt = t2;
    }

    int lim = -1;               // round positions <= lim are settled
    int rstop = kNS;            // first position this round did not settle
    for (;;) {
      int myfirst = kInf;
#pragma unroll
      for (int r = kR - 1; r >= 0; --r) {
        const int pos = G * kR + r;
        if (unsafe[r] && pos > lim) myfirst = pos;
      }
      myfirst = min(myfirst, partner16_i(myfirst, lane));
      myfirst = min(myfirst, partner32_i(myfirst, lane));
      if (lane == 0 && myfirst != kInf) atomicMin(&s_first[iter & 1], myfirst);
      lds_barrier();            // A: the first sample of the round that may update
      {
        const uint64_t t2 = cyc();
        ph[1] += t2 - tt;
        tt = t2;
      }
      const int k = s_first[iter & 1];
      if (tid == 0) s_first[(iter + 1) & 1] = kInf;
      ++iter;
      if (k == kInf) break;
      const int sid = n_steps;
      if (G == k / kR) {
        // ---------------- the exact step of sample k (this group's 16 lanes)
        const int rk = k % kR;
        S t = sc[0];
        int sl[FC];
#pragma unroll
        for (int c = 0; c < FC; ++c) sl[c] = slot[0][c];
#pragma unroll
        for (int r = 1; r < kR; ++r)
          if (r == rk) {
            t = sc[r];
#pragma unroll
            for (int c = 0; c < FC; ++c) sl[c] = slot[r][c];
          }
        const int y = t.y;
        if (sub == 0) { s_nins = 0; s_upd = 0; }
        // the sample's rows not in the store yet are added first (a step
        // that then does not update leaves them with zero deltas); a full
        // bucket pair ends the segment before anything is applied
        int nnew = 0;
        bool full = false;
        if (t.nf <= NFM) {
#pragma unroll
          for (int c = 0; c < FC; ++c) {
            const bool need = t.fi[c] >= 0 && sl[c] < 0;
            nnew += __popcll(__builtin_amdgcn_ballot_w64(need));
            if (need) {
              sl[c] = cache_insert<LC>(s_key, t.fi[c]);
              full |= sl[c] < 0;
            }
          }
          full = __builtin_amdgcn_ballot_w64(full) != 0;
        }
        if (t.nf > NFM) {
          if (sub == 0) s_stop = (int)kStopDense;
        } else if (full) {
          if (sub == 0) s_stop = (int)kStopSaturated;
        } else {
          int ls = -1;
          float m = 0.f, sy = 0.f, best = 0.f, var = 0.f;
          float py[FC], pl[FC];
          bool refreshed = false;
          for (;;) {
            m = group_margin<LC>(t.s, y, act, sub, &ls, &sy, &best);
            float v = 0.f;
#pragma unroll
            for (int c = 0; c < FC; ++c) {
              py[c] = 1.f;
              pl[c] = 1.f;
              const int32_t row = t.fi[c];
              if (!use_s || row < 0) continue;
              const float* dpr = s_dp + sl[c] * LC;    // every row of the sample has a slot now
              py[c] = t.py[c] + dpr[y];
              if (ls >= 0) {
                const float p0 = ls == t.ls0 ? t.pl[c] : P[(int64_t)row * LC + ls];
                pl[c] = p0 + dpr[ls];
              }
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
            for (int c = 0; c < FC; ++c) {
#pragma unroll 1
              for (int u = 0; u < 16; ++u) {
                const int32_t ru = __shfl(t.fi[c], (lane & 48) + u, 64);
                const float xu = __shfl(t.fx[c], (lane & 48) + u, 64);
                const int su = __shfl(sl[c], (lane & 48) + u, 64);
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
          const bool up = step_coeffs(method, m, var, t.nrm, ls >= 0, C, &tau, &beta);
          if (up) {
#pragma unroll
            for (int c = 0; c < FC; ++c)
              if (t.fi[c] >= 0) { s_sst[sl[c]] = sid; s_sdy[sl[c]] = 0.f; s_sdl[sl[c]] = 0.f; }
#pragma unroll
            for (int c = 0; c < FC; ++c) {
              if (t.fi[c] < 0) continue;
              const float x = t.fx[c];
              const float a = use_s ? 1.f / py[c] : 1.f;
              const float b = (use_s && ls >= 0) ? 1.f / pl[c] : 1.f;
              const float dwy = tau * a * x;
              const float dwl = ls >= 0 ? -tau * b * x : 0.f;
              float* dwr = s_dw + sl[c] * LC;
              atomicAdd(dwr + y, dwy);
              if (ls >= 0) atomicAdd(dwr + ls, dwl);
              if (use_s) {
                float* dpr = s_dp + sl[c] * LC;
                atomicAdd(dpr + y, dprec(method, beta, x, a));
                if (ls >= 0) atomicAdd(dpr + ls, dprec(method, beta, x, b));
              }
              atomicAdd(&s_sdy[sl[c]], dwy);
              atomicAdd(&s_sdl[sl[c]], dwl);
              atomicAdd(&s_rmax[sl[c]], fmaxf(fabsf(dwy), fabsf(dwl)));
            }
          }
          if (sub == 0) {
            s_cn += nnew;
            s_nins = nnew;
            s_upd = up ? 1 : 0;
            s_yk = y;
            s_lk = ls;
            if (up) atomicAdd(&s_nupd, 1u); else atomicAdd(&s_waste, 1u);
          }
        }
      }
      lds_barrier();            // B: the step (or the stop) is visible
      {
        const uint64_t t2 = cyc();
        ph[2] += t2 - tt;
        tt = t2;
      }
      ++n_steps;
      const int sc_stop = s_stop;
      if (sc_stop >= 0) {
        rstop = k;
        why = sc_stop;
        stop = p + k;
        break;
      }
      // samples after k: the slots of rows the step added (also when it did
      // not update: a later step may write them), then the step's
      // increments of their stamped rows
      const int nins = s_nins;
      if (nins > 0 && (wv + 1) * 4 * kR - 1 > k) {
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          if (G * kR + r <= k) continue;
#pragma unroll
          for (int c = 0; c < FC; ++c)
            if (slot[r][c] < 0 && sc[r].fi[c] >= 0) slot[r][c] = cache_find<LC>(s_key, sc[r].fi[c]);
        }
      }
      if (s_upd && (wv + 1) * 4 * kR - 1 > k) {
        const int yk = s_yk, lk = s_lk;
#pragma unroll
        for (int r = 0; r < kR; ++r) {
          const int pos = G * kR + r;
          if (!alive[r] || pos <= k || sc[r].nf > NFM) continue;
          float cy = 0.f, cl = 0.f;
#pragma unroll
          for (int c = 0; c < FC; ++c) {
            const int s = slot[r][c];
            if (s >= 0 && s_sst[s] == sid) {
              cy += sc[r].fx[c] * s_sdy[s];
              cl += sc[r].fx[c] * s_sdl[s];
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
          // the margin moves by at most |cy| + |cl| (the guard band by 1e-4 of it)
          slack[r] -= (fabsf(cy) + fabsf(cl)) * (1.f + 4.f * kGuard);
          if (exact[r] && !(slack[r] > 0.f)) {
            int ls;
            float sy, best;
            const float m = group_margin<LC>(sc[r].s, sc[r].y, act, sub, &ls, &sy, &best);
            slack[r] = slack_of(method, m, sc[r].nrm, ls >= 0, C, sy, best);
          }
        }
        // samples still on S0 scores whose bounded slack ran out
        make_exact(k);
#pragma unroll
        for (int r = 0; r < kR; ++r)
          if (G * kR + r > k) unsafe[r] = (alive[r] && (sc[r].nf > NFM || !(slack[r] > 0.f))) ? 1 : 0;
      }
      lim = k;
      {
        const uint64_t t2 = cyc();
        ph[3] += t2 - tt;
        tt = t2;
      }
    }
    ++n_rounds;
    if (sub == 0) {
#pragma unroll
      for (int r = 0; r < kR; ++r)
        if (alive[r] && G * kR + r < rstop) ++n_valid;
    }
  };
  // the round loop unrolled PD times: round u of an iteration reads prefetch
  // slot u and refills it PD rounds ahead, so no slot is ever copied (a copy
  // of a register a load is still writing waits for that load)
  for (int64_t p0 = beg; p0 < end && stop == end; p0 += PD * kNS) {
#pragma unroll
    for (int u = 0; u < PD; ++u) {
      // the refill is issued whether or not the round runs: the loads then
      // leave in the same order on every path, so each round waits only for
      // its own slot (a path that skipped a refill would make the compiler
      // drain every load in flight)
      const int64_t p = p0 + u * kNS;
      const uint64_t tt = cyc();
      unpack(p, pf[u], sc);
      load_raw(p + PD * kNS, pf[u]);     // clamped: past the end it re-reads the last record
      if (p < end && stop == end) round(p, tt);
    }
  }
  __syncthreads();
  const uint64_t t_f0 = cyc();
  // ---- segment end: the deltas into the tables (the committer is their only writer)
  {
    constexpr int Q = LC / 4;
    for (int i = tid; i < NSLOT * Q; i += kT) {
      const int sl = i / Q;
      const int32_t row = s_key[sl];
      if (row < 0) continue;
      const int q = i % Q;
      float4* w4 = reinterpret_cast<float4*>(W + (int64_t)row * LC) + q;
      const float4 d = reinterpret_cast<const float4*>(s_dw + sl * LC)[q];
      float4 w = *w4;
      w.x += d.x; w.y += d.y; w.z += d.z; w.w += d.w;
      *w4 = w;
      if (use_s) {
        float4* p4 = reinterpret_cast<float4*>(P + (int64_t)row * LC) + q;
        const float4 dp = reinterpret_cast<const float4*>(s_dp + sl * LC)[q];
        float4 pv = *p4;
        pv.x += dp.x; pv.y += dp.y; pv.z += dp.z; pv.w += dp.w;
        *p4 = pv;
      }
      if (q == 0 && touched != nullptr) touched[row] = 1;
    }
  }
  if (n_valid > 0 && stats != nullptr) atomicAdd(stats + 1, (unsigned long long)n_valid);
  auto put = [&](int i, int64_t v) { tail[i] = seg == 0 ? v : tail[i] + v; };
  if (kProf && lane == 0 && tid > 0) put(12 + wv, (int64_t)wwork);
  if (tid == 0) {
    if (stop == end && end < bend) why = kStopWindow;   // the next segment takes the next window
    tail[0] = stop;
    tail[1] = bend;
    tail[kTailReason] = why;
    tail[kTailWin] = stop - beg;
    *wide = 0;                // the next segment's S0 pass sets it again
    put(2, n_steps);
    put(3, n_rounds);
    ph[4] = cyc() - t_f0;
    for (int i = 0; i < 6; ++i) put(4 + i, (int64_t)ph[i]);
    put(10, kProf ? (int64_t)(__builtin_amdgcn_s_memrealtime() - w_k0) : 0);
    put(11, (int64_t)(cyc() - t_k0));
    put(12, (int64_t)wwork);
    put(21, 1);
    put(22, (int64_t)s_waste);
    put(23, (int64_t)s_refresh);
    put(24, (int64_t)s_nupd);
    put(25, (int64_t)s_cn);
    put(26, (int64_t)s_nexact);
    put(27, (int64_t)s_nalive);
    if (stats != nullptr && s_nupd > 0) atomicAdd(stats, (unsigned long long)s_nupd);
  }
}

}  // namespace dc
}  // namespace jb

// one segment: the S0 pass, then the committers of the method (one chunk /
// two chunks per lane; the S0 pass's wide flag lets one of them run)
template <int L>
static int launch_delta(int64_t blocks, int method, const int64_t* row_ptr, const int32_t* fidx,
                        const float* fval, const int32_t* labels, const int64_t* sp, int ns, float* W,
                        float* S, float* Pp, const int32_t* active, float C, float* s0, int4* aux,
                        float2* pp0, int32_t* fi, float* fx, unsigned long long* wide,
                        unsigned long long* stats, uint8_t* touched, int64_t* tail, int seg,
                        const int64_t* why, int prof, hipStream_t stream) {
  hipLaunchKernelGGL((jb::dc::delta_s0_kernel<L>), dim3((unsigned)blocks), dim3(256), 0, stream, row_ptr, fidx,
                     fval, labels, sp, ns, W, Pp, active, method, C, s0, aux, pp0, fi, fx, wide, tail, why);
#define JB_DELTA_M(M)                                                                                     \
  hipLaunchKernelGGL((jb::dc::delta_commit_kernel<L, M, 1>), dim3(1), dim3(jb::dc::kT), 0, stream, sp, ns, \
                     W, S, active, C, s0, aux, pp0, fi, fx, wide, stats, touched, tail, seg, prof);        \
  hipLaunchKernelGGL((jb::dc::delta_commit_kernel<L, M, 2>), dim3(1), dim3(jb::dc::kT), 0, stream, sp, ns, \
                     W, S, active, C, s0, aux, pp0, fi, fx, wide, stats, touched, tail, seg, prof);        \
  break;
  switch (method) {
    case jb::PERCEPTRON: JB_DELTA_M(jb::PERCEPTRON)
    case jb::PA: JB_DELTA_M(jb::PA)
    case jb::PA1: JB_DELTA_M(jb::PA1)
    case jb::PA2: JB_DELTA_M(jb::PA2)
    case jb::CW: JB_DELTA_M(jb::CW)
    case jb::AROW: JB_DELTA_M(jb::AROW)
    case jb::NHERD: JB_DELTA_M(jb::NHERD)
    default: return -1;
  }
#undef JB_DELTA_M
  return 0;
}

// bytes of the delta committer's scratch per sample: S0 (<= 64 floats),
// PP0 (32 float2), FI / FX (32 ints / floats), AUX (int4)
extern "C" int64_t jb_delta_scratch_per_sample() { return 256 + 256 + 128 + 128 + 16; }

// Steps 1-2 of a kSerial batch for LC <= 64 (see the header); the caller
// runs the exact single-stream kernel over [tail[0], tail[1]) afterwards.
// scratch: [tail int64 x 32][S0: n_max x 64 floats][PP0: n_max x 32 float2]
// [FI: n_max x 32][FX: n_max x 32][AUX: n_max int4]; tail[28] is the wide flag.
extern "C" int jb_delta_prepare(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                                int64_t n_max, float* W, float* S, const int32_t* active, int LC,
                                int method, float C, unsigned long long* stats, uint8_t* touched,
                                void* scratch, int nseg, hipStream_t stream) {
  if (LC > 64) return -1;
  static const int prof = [] {
    const char* e = getenv("JB_COMMIT_PROF");
    return (e != nullptr && e[0] == '1') ? 1 : 0;
  }();
  int64_t* tail = (int64_t*)scratch;
  uint8_t* base = (uint8_t*)scratch + 256;
  float* s0 = (float*)base;
  float2* pp0 = (float2*)(base + 256 * n_max);
  int32_t* fi = (int32_t*)(base + 512 * n_max);
  float* fx = (float*)(base + 640 * n_max);
  int4* aux = (int4*)(base + 768 * n_max);
  unsigned long long* wide = (unsigned long long*)(tail + 28);
  if (hipMemsetAsync(wide, 0, sizeof(*wide), stream) != hipSuccess) return -2;
  float* Pp = method >= jb::CW ? S : nullptr;
  const int64_t blocks = std::min<int64_t>((n_max * 64 + 255) / 256, 2048);
  for (int seg = 0; seg < nseg; ++seg) {
    const int64_t* sp = seg == 0 ? stream_ptr : tail;
    const int ns = seg == 0 ? nstreams : 1;
    const int64_t* why = seg == 0 ? nullptr : tail + jb::dc::kTailReason;
    int rc = 0;
#define JB_DELTA_L(L)                                                                                      \
  rc = launch_delta<L>(blocks, method, row_ptr, fidx, fval, labels, sp, ns, W, S, Pp, active, C, s0, aux, \
                       pp0, fi, fx, wide, stats, touched, tail, seg, why, prof, stream);                  \
  break;
    switch (LC) {
      case 8: JB_DELTA_L(8)
      case 16: JB_DELTA_L(16)
      case 32: JB_DELTA_L(32)
      case 64: JB_DELTA_L(64)
      default: return -1;
    }
#undef JB_DELTA_L
    if (rc) return rc;
  }
  return (int)hipGetLastError();
}
