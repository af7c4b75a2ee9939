// Incremental LOF state in HBM for the native jubaanomaly: the C++ twin of
// models/lof_state.py DeviceLofState over csrc/hip/lof.hip (per-slot k
// nearest neighbour lists, k-distance, lrd, validity flags and stamps;
// insert + score of an add in one launch; staleness marks over all lists
// for moved rows and installed lists).
//
// Reference: anomaly_serv.cpp:157-244 over jubatus_core's lof_storage
// (EXTERNAL); the algorithm (Breunig et al. 2000) and its host oracle are
// documented in models/anomaly.py and models/lof_state.py.
#pragma once
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <vector>

#include "jb_server_common.hpp"

extern "C" {
int jb_lof_mark(int64_t nrows, int k, const int32_t* nb_slot, const int32_t* changed,
                const int32_t* nchanged, int clear_ok, uint8_t* ok, uint8_t* lrd_ok,
                hipStream_t stream);
int jb_lof_set_lists(int n, const int32_t* slots, const int32_t* cs, const float* cd, int kk, int k,
                     int ignore_same, int32_t* nb_slot, float* nb_dist, float* kdist, uint8_t* ok,
                     uint8_t* lrd_ok, int32_t* changed, int32_t* nchanged, hipStream_t stream);
int jb_lof_add(int p, const int32_t* cs, const float* cd, int nc, int k, int ignore_same,
               int64_t nrows, int32_t* nb_slot, float* nb_dist, float* kdist, uint8_t* ok,
               float* lrd, uint8_t* lrd_ok, int32_t* changed, int32_t* nchanged,
               uint32_t* out_host, int max_missing, hipStream_t stream);
int jb_lof_add_st(int p, const int32_t* cs, const float* cd, int nc, int k, int ignore_same, int64_t nrows,
                  int32_t* nb_slot, float* nb_dist, float* kdist, uint8_t* ok, float* lrd, uint8_t* lrd_ok,
                  int32_t* changed, int32_t* nchanged, uint32_t* kstamp, uint32_t* lstamp, uint32_t epoch,
                  uint32_t* out_host, int max_missing, hipStream_t stream);
int jb_lof_add_many(int nadd, const int32_t* ps, const int32_t* cs, const float* cd, const int32_t* nc,
                    int stride, int k, int ignore_same, int32_t* nb_slot, float* nb_dist, float* kdist,
                    uint8_t* ok, float* lrd, uint8_t* lrd_ok, int32_t* changed, int32_t* nchanged,
                    uint32_t* kstamp, uint32_t* lstamp, uint32_t epoch0, int32_t* cand, uint32_t* res,
                    uint32_t* out_host, int out_stride, int max_missing, unsigned long long* prof,
                    hipStream_t stream, int wait, uint32_t* chain);
int jb_lof_add_many_wait(int nadd, uint32_t* out_host, int out_stride, hipStream_t stream);
int jb_lof_score_st(const int32_t* ts, const float* td, int nt, int k, const int32_t* nb_slot,
                    const float* nb_dist, const float* kdist, const uint8_t* ok, float* lrd, uint8_t* lrd_ok,
                    int store_slot, const uint32_t* kstamp, uint32_t* lstamp, uint32_t epoch,
                    uint32_t* out_host, int max_missing, hipStream_t stream);
int jb_lof_score_many(int nq, const int32_t* ts, const float* td, const int32_t* nt, int stride, int k,
                      const int32_t* nb_slot, const float* nb_dist, const float* kdist, const uint8_t* ok, float* lrd,
                      uint8_t* lrd_ok, const uint32_t* kstamp, uint32_t* lstamp, uint32_t epoch, uint32_t* out_host,
                      int out_stride, int max_missing, hipStream_t stream);
int jb_lof_invalidate(const int32_t* slots, int n, int64_t nrows, uint8_t* ok, uint8_t* lrd_ok,
                      hipStream_t stream);
void* jb_host_alloc(int64_t nbytes);
int jb_host_free(void* p);
}

namespace jb {
namespace row {

using jb::srv::DevBuf;

constexpr int kLofMaxK = 64;          // lof.hip kLofMaxK
constexpr int kLofMaxChanged = 1024;  // kLofMaxChanged
constexpr int kLofMaxMissing = 1024;
constexpr int kLofArgMax = 128;       // candidates in the kernel arguments
constexpr int kLofBatchMax = 64;      // adds of one jb_lof_add_many

class LofState {
 public:
  LofState(int k, bool ignore_same, hipStream_t st) : k_(k), ignore_(ignore_same), stream_(st) {
    out_ = (uint32_t*)jb_host_alloc(4 * (4 + kLofMaxMissing));
    if (!out_) throw std::runtime_error("hipHostMalloc failed");
    changed_.get(kLofMaxChanged);
    nchanged_.get(1);
    cand_.get(2 * (size_t)kLofBatchMax * kLofArgMax);
    res_.get((size_t)kLofBatchMax * kOutStride);
    stage_ = (int32_t*)jb_host_alloc(4 * 2 * kStageWords);            // two batches in flight
    if (!stage_) throw std::runtime_error("hipHostMalloc failed");
    out_many_ = (uint32_t*)jb_host_alloc(4 * 2 * (size_t)kOutStride * kLofBatchMax);
    if (!out_many_) throw std::runtime_error("hipHostMalloc failed");
    chain_.get(1);
    HIPCHK(hipMemsetAsync(chain_.p, 0, 4, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
  }

  ~LofState() {
    for (void* q : {(void*)nb_slot_.p, (void*)nb_dist_.p, (void*)kdist_.p, (void*)lrd_.p, (void*)ok_.p,
                    (void*)lrd_ok_.p, (void*)kstamp_.p, (void*)lstamp_.p, (void*)changed_.p, (void*)nchanged_.p,
                    (void*)up_[0].p, (void*)up_[1].p, (void*)up_[2].p, (void*)cand_.p, (void*)res_.p,
                    (void*)chain_.p})
      if (q) (void)hipFree(q);
    if (out_) jb_host_free(out_);
    if (out_many_) jb_host_free(out_many_);
    if (stage_) jb_host_free(stage_);
  }
  LofState(const LofState&) = delete;
  LofState& operator=(const LofState&) = delete;

  int64_t cap() const { return cap_; }

  void ensure(int64_t n) {
    if (n <= cap_) return;
    const int64_t cap = std::max<int64_t>(std::max<int64_t>(n, 2 * cap_), 1024);
    regrow(nb_slot_, cap_ * k_, cap * k_, 0xff);          // -1
    regrow_inf(nb_dist_, cap_ * k_, cap * k_);
    regrow(kdist_, cap_, cap, 0);
    regrow(lrd_, cap_, cap, 0);
    regrow(ok_, cap_, cap, 0);
    regrow(lrd_ok_, cap_, cap, 0);
    regrow(kstamp_, cap_, cap, 0);
    regrow(lstamp_, cap_, cap, 0);
    cap_ = cap;
  }

  // DeviceLofState.add: -> true and *score, or false and the slots whose
  // lists are missing
  bool add(int32_t p, const std::vector<int32_t>& cs, const std::vector<float>& cd, float* score,
           std::vector<int32_t>* missing) {
    const int nc = (int)cs.size();     // (kLofArgMax candidates per launch inside)
    const int rc = jb_lof_add_st(p, cs.data(), cd.data(), nc, k_, ignore_ ? 1 : 0, cap_, nb_slot_.p,
                                 nb_dist_.p, kdist_.p, ok_.p, lrd_.p, lrd_ok_.p, changed_.p, nchanged_.p,
                                 kstamp_.p, lstamp_.p, ++epoch_, out_, kLofMaxMissing, stream_);
    if (rc != 0) throw std::runtime_error("lof add failed: " + std::to_string(rc));
    return result(score, missing);
  }

  // a batch of adds in order with one wait (<= kLofBatchMax, candidates <= kLofArgMax each):
  // -> the number completed (their scores in *scores); when short of all,
  // add [return] stopped on rows without a valid list (*missing) - its
  // insert is applied, its score is not (the caller scores it, as after a
  // false add()), and the later adds did not run
  size_t add_many(const std::vector<int32_t>& ps, const std::vector<std::vector<int32_t>>& cs,
                  const std::vector<std::vector<float>>& cd, std::vector<float>* scores,
                  std::vector<int32_t>* missing) {
    launch_many(ps, cs, cd);
    return finish_many(scores, missing);
  }

  // add_many in two halves: the launch returns at once, finish_many waits for
  // the oldest batch in flight and reads its results. Up to two batches in
  // flight, queued back to back on the stream (the second starts the moment
  // the first ends, no host round trip between them), each with its own
  // pinned staging and results. A batch that stops (rows without a valid
  // list) sets the chain word, so the batch queued behind it does not run:
  // finish_many then drains it (*dropped = 1: the caller reruns it) and
  // clears the word.
  void launch_many(const std::vector<int32_t>& ps, const std::vector<std::vector<int32_t>>& cs,
                   const std::vector<std::vector<float>>& cd) {
    const size_t n = ps.size();
    if (fl_.size() >= 2) throw std::logic_error("lof launch_many: two batches in flight");
    if (n == 0) return;
    if (n > (size_t)kLofBatchMax) throw std::runtime_error("lof add_many: batch too large");
    int stride = 1;
    for (const auto& c : cs) stride = std::max(stride, (int)c.size());
    if (stride > kLofArgMax) throw std::runtime_error("lof add_many: too many candidates");
    const int buf = fl_.empty() ? 0 : 1 - fl_.front().buf;
    // pinned staging the kernel reads: ps [64], nc [64], cs [n][stride], cd [n][stride]
    int32_t* hps = stage_ + (size_t)buf * kStageWords;
    int32_t* hnc = hps + kLofBatchMax;
    int32_t* hcs = hps + 2 * kLofBatchMax;
    float* hcd = reinterpret_cast<float*>(hcs + n * (size_t)stride);
    for (size_t i = 0; i < n; ++i) {
      hps[i] = ps[i];
      hnc[i] = (int32_t)cs[i].size();
      int32_t* c = hcs + (int64_t)i * stride;
      float* d = hcd + (int64_t)i * stride;
      std::copy(cs[i].begin(), cs[i].end(), c);
      std::copy(cd[i].begin(), cd[i].end(), d);
      std::fill(c + cs[i].size(), c + stride, -1);
      std::fill(d + cd[i].size(), d + stride, INFINITY);
    }
    const uint32_t epoch0 = epoch_ + 1;
    epoch_ += (uint32_t)n;            // (adds after a stop leave gaps: stamps only need to grow)
    uint32_t* out = out_many_ + (size_t)buf * kOutStride * kLofBatchMax;
    const int rc = jb_lof_add_many((int)n, hps, hcs, hcd, hnc, stride, k_, ignore_ ? 1 : 0, nb_slot_.p, nb_dist_.p,
                                   kdist_.p, ok_.p, lrd_.p, lrd_ok_.p, changed_.p, nchanged_.p, kstamp_.p, lstamp_.p,
                                   epoch0, cand_.p, res_.p, out, kOutStride, kLofMaxMissing, nullptr, stream_, 0,
                                   chain_.p);
    if (rc != 0) throw std::runtime_error("lof add_many failed: " + std::to_string(rc));
    fl_.push_back({n, buf});
  }
  bool in_flight() const { return !fl_.empty(); }
  size_t finish_many(std::vector<float>* scores, std::vector<int32_t>* missing, size_t* dropped = nullptr) {
    if (dropped) *dropped = 0;
    scores->clear();
    if (fl_.empty()) return 0;
    const Flight f = fl_.front();
    fl_.pop_front();
    const uint32_t* out = out_many_ + (size_t)f.buf * kOutStride * kLofBatchMax;
    const int rc = jb_lof_add_many_wait((int)f.n, const_cast<uint32_t*>(out), kOutStride, stream_);
    if (rc != 0) {
      fl_.clear();
      throw std::runtime_error("lof add_many failed: " + std::to_string(rc));
    }
    for (size_t i = 0; i < f.n; ++i) {
      const uint32_t* o = out + i * kOutStride;
      const uint32_t st = ((volatile const uint32_t*)o)[0];
      if (st == 1) {
        float sc;
        memcpy(&sc, &o[1], 4);
        scores->push_back(sc);
        continue;
      }
      if (st != 2) throw std::runtime_error("lof add_many: kernel did not complete");
      missing->clear();
      const uint32_t nm = std::min<uint32_t>(o[3], kLofMaxMissing);
      for (uint32_t j = 0; j < nm; ++j) {
        const int32_t s = (int32_t)o[4 + j];
        if (std::find(missing->begin(), missing->end(), s) == missing->end()) missing->push_back(s);
      }
      // the batches queued behind did not run: wait for them, clear the word
      while (!fl_.empty()) {
        const Flight g = fl_.front();
        fl_.pop_front();
        const int rw = jb_lof_add_many_wait((int)g.n, out_many_ + (size_t)g.buf * kOutStride * kLofBatchMax,
                                            kOutStride, stream_);
        if (rw != 0) throw std::runtime_error("lof add_many failed: " + std::to_string(rw));
        if (dropped) ++*dropped;
      }
      HIPCHK(hipMemsetAsync(chain_.p, 0, 4, stream_));
      return i;
    }
    return f.n;
  }

  bool score(const std::vector<int32_t>& ts, const std::vector<float>& td, int32_t store, float* sc,
             std::vector<int32_t>* missing) {
    if (ts.empty()) { *sc = 1.f; return true; }
    const int rc = jb_lof_score_st(ts.data(), td.data(), (int)ts.size(), k_, nb_slot_.p, nb_dist_.p, kdist_.p,
                                   ok_.p, lrd_.p, lrd_ok_.p, store, kstamp_.p, lstamp_.p, epoch_, out_,
                                   kLofMaxMissing, stream_);
    if (rc != 0) throw std::runtime_error("lof score failed: " + std::to_string(rc));
    return result(sc, missing);
  }

  // independent scores (no store), one wait: (*done)[i] = 1 and (*scores)[i]
  // for the queries that resolved; the others found rows without a valid
  // list and are left to score() (the caller installs the lists)
  void score_many(const std::vector<std::vector<int32_t>>& ts, const std::vector<std::vector<float>>& td,
                  std::vector<float>* scores, std::vector<char>* done) {
    const size_t n = ts.size();
    scores->assign(n, 1.f);
    done->assign(n, 0);
    for (size_t b = 0; b < n; b += kLofBatchMax) {
      const size_t m = std::min<size_t>(kLofBatchMax, n - b);
      int stride = 1;
      for (size_t i = 0; i < m; ++i) stride = std::max(stride, (int)ts[b + i].size());
      if (stride > 64) return;         // (the caller scores them one by one)
      // pinned staging the kernel reads (the add path's; never in use at once):
      // ts [m][stride], td [m][stride], nt [m]
      int32_t* fts = stage_;
      float* ftd = reinterpret_cast<float*>(stage_ + m * (size_t)stride);
      int32_t* nt = stage_ + 2 * m * (size_t)stride;
      for (size_t i = 0; i < m; ++i) {
        nt[i] = (int32_t)ts[b + i].size();
        std::copy(ts[b + i].begin(), ts[b + i].end(), fts + (int64_t)i * stride);
        std::copy(td[b + i].begin(), td[b + i].end(), ftd + (int64_t)i * stride);
      }
      const int rc = jb_lof_score_many((int)m, fts, ftd, nt, stride, k_, nb_slot_.p, nb_dist_.p, kdist_.p, ok_.p,
                                       lrd_.p, lrd_ok_.p, kstamp_.p, lstamp_.p, epoch_, out_many_, kOutStride,
                                       kLofMaxMissing, stream_);
      if (rc != 0) throw std::runtime_error("lof score_many failed: " + std::to_string(rc));
      for (size_t i = 0; i < m; ++i) {
        const uint32_t* o = out_many_ + i * kOutStride;
        if (((volatile const uint32_t*)o)[0] == 1) {
          memcpy(&(*scores)[b + i], &o[1], 4);
          (*done)[b + i] = 1;
        }
      }
    }
  }

  // rows changed or removed: their lists and every list naming them invalid
  void moved(const std::vector<int32_t>& slots) {
    if (slots.empty()) return;
    ensure((int64_t)*std::max_element(slots.begin(), slots.end()) + 1);
    for (size_t i = 0; i < slots.size(); i += kLofMaxChanged) {
      const int n = (int)std::min<size_t>(kLofMaxChanged, slots.size() - i);
      int32_t* d = upload(slots.data() + i, (size_t)n);
      HIPCHK(hipMemcpyAsync(changed_.p, d, 4 * (size_t)n, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipMemcpyAsync(nchanged_.p, &n_host(n), 4, hipMemcpyHostToDevice, stream_));
      int rc = jb_lof_mark(cap_, k_, nb_slot_.p, changed_.p, nchanged_.p, 1, ok_.p, lrd_ok_.p, stream_);
      if (rc == 0) rc = jb_lof_invalidate(d, n, cap_, ok_.p, lrd_ok_.p, stream_);
      if (rc != 0) throw std::runtime_error("lof mark failed: " + std::to_string(rc));
      HIPCHK(hipStreamSynchronize(stream_));   // the staging buffers are reused
    }
  }

  // lists[i] = ascending (slot, dist) of row slots[i], itself possibly included
  void set_lists(const std::vector<int32_t>& slots,
                 const std::vector<std::vector<std::pair<int32_t, float>>>& lists) {
    size_t kk = 0;
    for (const auto& l : lists) kk = std::max(kk, l.size());
    if (!kk || slots.empty()) return;
    for (size_t i = 0; i < slots.size(); i += kLofMaxChanged) {
      const size_t n = std::min<size_t>(kLofMaxChanged, slots.size() - i);
      std::vector<int32_t> cs(n * kk, -1);
      std::vector<float> cd(n * kk, INFINITY);
      for (size_t r = 0; r < n; ++r)
        for (size_t j = 0; j < lists[i + r].size(); ++j) {
          cs[r * kk + j] = lists[i + r][j].first;
          cd[r * kk + j] = lists[i + r][j].second;
        }
      int32_t* dsl = upload(slots.data() + i, n);
      int32_t* dcs = upload(cs.data(), cs.size(), 1);
      float* dcd = (float*)upload((const int32_t*)cd.data(), cd.size(), 2);
      int rc = jb_lof_set_lists((int)n, dsl, dcs, dcd, (int)kk, k_, ignore_ ? 1 : 0, nb_slot_.p, nb_dist_.p,
                                kdist_.p, ok_.p, lrd_ok_.p, changed_.p, nchanged_.p, stream_);
      if (rc == 0) rc = jb_lof_mark(cap_, k_, nb_slot_.p, changed_.p, nchanged_.p, 0, ok_.p, lrd_ok_.p, stream_);
      if (rc != 0) throw std::runtime_error("lof set_lists failed: " + std::to_string(rc));
      HIPCHK(hipStreamSynchronize(stream_));
    }
  }

 private:
  bool result(float* score, std::vector<int32_t>* missing) {
    const uint32_t st = ((volatile uint32_t*)out_)[0];
    if (st == 2) {
      const uint32_t nm = std::min<uint32_t>(out_[3], kLofMaxMissing);
      missing->clear();
      for (uint32_t i = 0; i < nm; ++i) {
        const int32_t s = (int32_t)out_[4 + i];
        if (std::find(missing->begin(), missing->end(), s) == missing->end()) missing->push_back(s);
      }
      return false;
    }
    if (st != 1) throw std::runtime_error("lof: kernel did not complete");
    memcpy(score, &out_[1], 4);
    return true;
  }

  int32_t& n_host(int n) {
    nh_ = n;
    return nh_;
  }

  // small host array -> device (one of three staging slots), synchronous
  int32_t* upload(const int32_t* p, size_t n, int which = 0) {
    DevBuf<int32_t>& b = up_[which];
    int32_t* d = b.get(std::max<size_t>(n, 1));
    HIPCHK(hipMemcpyAsync(d, p, 4 * n, hipMemcpyHostToDevice, stream_));
    return d;
  }

  template <class T>
  void regrow(DevBuf<T>& b, int64_t old, int64_t cap, int fill) {
    T* np = nullptr;
    HIPCHK(hipMalloc((void**)&np, (size_t)cap * sizeof(T)));
    HIPCHK(hipMemsetAsync(np, fill, (size_t)cap * sizeof(T), stream_));
    if (old > 0 && b.p) HIPCHK(hipMemcpyAsync(np, b.p, (size_t)old * sizeof(T), hipMemcpyDeviceToDevice, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    if (b.p) HIPCHK(hipFree(b.p));
    b.p = np;
    b.cap = (size_t)cap;
  }
  void regrow_inf(DevBuf<float>& b, int64_t old, int64_t cap) {
    regrow(b, old, cap, 0);
    std::vector<float> inf((size_t)(cap - old), INFINITY);
    HIPCHK(hipMemcpy(b.p + old, inf.data(), 4 * inf.size(), hipMemcpyHostToDevice));
  }

  int k_;
  bool ignore_;
  hipStream_t stream_;
  int64_t cap_ = 0;
  struct Flight {
    size_t n;   // adds
    int buf;    // staging / results buffer
  };
  std::deque<Flight> fl_;   // launch_many batches in flight, oldest first
  static constexpr size_t kStageWords = 2 * (size_t)kLofBatchMax + 2 * (size_t)kLofBatchMax * kLofArgMax;
  DevBuf<uint32_t> chain_;  // set by a batch that stops (lof_add_batch_kernel)
  DevBuf<int32_t> nb_slot_;
  DevBuf<float> nb_dist_, kdist_, lrd_;
  DevBuf<uint8_t> ok_, lrd_ok_;
  // staleness stamps (lof.hip): the add epoch that last changed a row's list
  // (kstamp) and the epoch its lrd was computed at (lstamp); adds stamp
  // instead of marking every list that names a changed row
  DevBuf<uint32_t> kstamp_, lstamp_;
  uint32_t epoch_ = 0;
  DevBuf<int32_t> changed_, nchanged_;
  DevBuf<int32_t> up_[3];
  DevBuf<int32_t> cand_;          // add_many's candidates on the device
  DevBuf<uint32_t> res_;          // add_many's results before they go to the host
  int32_t* stage_ = nullptr;       // add_many's pinned staging (the kernel reads it)
  uint32_t* out_ = nullptr;
  static constexpr int kOutStride = 4 + kLofMaxMissing;
  uint32_t* out_many_ = nullptr;   // [kLofBatchMax][kOutStride] pinned
  int32_t nh_ = 0;
};

}  // namespace row
}  // namespace jb
