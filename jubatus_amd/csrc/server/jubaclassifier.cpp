// jubaclassifier, native: the classifier server without Python.
//
// Reference: jubatus/server/server/classifier_serv.cpp (train :128-147,
// classify :149-173, labels :175-225), classifier_impl.cpp (RPC table),
// framework/server_base.cpp (save / load / status) and server_helper.hpp
// (startup). SURVEY section 7.1: server binaries must not need Python.
//
// Scope: the linear methods (perceptron, PA, PA1, PA2, CW, AROW, NHERD),
// standalone or distributed (linear and push mixers over the native MIX
// plane, csrc/native/jb_mix_group.hpp), with converters on the fixed-slot GPU
// path (fv_converter/gpu_path.py fast_eligible) or the host wide rule set
// (bigram / combination / idf, jb_linear_conv.hpp). --cpu
// and a host without /dev/kfd are handed to the Python server
// (jubatus_amd.cmd.server) by exec BEFORE anything touches the GPU. The
// nearest-neighbor methods (NN, cosine, euclidean) run on the native row
// server (jb_row_server.hpp Kind::kClassifier: rows in HBM, batched k-NN).
//
// Data path (the same kernels as the Python server, csrc/hip):
//   train    the transport copies request bodies into pinned arena slots
//            (csrc/native/jb_rpc.cpp); one jb_train_batch_submit per slot
//            (H2D, scan.hip, fv_hash.hip, hot.hip, linear.hip); the reply of
//            every request waits for the batch's scan check. A batch the
//            device scan rejects (new labels, malformed bytes, binary
//            values) is re-run one request at a time on the host path:
//            validate, commit labels, hash (jb_hostfv.hpp), one exact
//            single-stream train launch.
//   classify the batch of queued classify RPCs is hashed on the host; up to
//            32 datums / 320 slots ride in the kernel arguments
//            (classify_direct.hip), larger batches take jb_linear_classify.
// Model files are byte-compatible with the Python server's
// (framework/save_load.py container, models/classifier.py pack()).
#include <signal.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <type_traits>
#include <vector>

#include "jb_hash.hpp"
#include "jb_roctx.hpp"
#include "jb_host_linear.hpp"
#include "jb_hostfv.hpp"
#include "jb_linear_conv.hpp"
#include "jb_mix_device.hpp"
#include "jb_row_server.hpp"
#include "jb_msgpack.hpp"
#include "jb_pack.hpp"
#include "jb_rpc.hpp"
#include "jb_train_batch.hpp"
#include "jb_server_common.hpp"
#include "jb_value.hpp"

extern "C" int jb_linear_train(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                               const int32_t* labels, const int64_t* stream_ptr, int nstreams,
                               float* W, float* S, const int32_t* active, int LC, int method,
                               float C, int mode, const int32_t* hot_rows, const int32_t* hot_n,
                               float* hot_rep, int merge_every, int hot_waves,
                               unsigned long long* stats, uint8_t* touched, int64_t n_max,
                               void* scratch, int64_t scratch_bytes, hipStream_t stream);
extern "C" int64_t jb_serial_scratch_bytes_lc(int64_t n_max, int LC);
extern "C" int jb_serial_scratch_forget(void* scratch);
extern "C" int jb_linear_classify(const int64_t* row_ptr, const int32_t* fidx, const float* fval,
                                  int n_samples, const float* W, int LC, float* out,
                                  hipStream_t stream);
extern "C" int jb_classify_direct(const int32_t* idx, const float* val, const int64_t* row_ptr,
                                  int n, const float* W, int LC, float* out_host,
                                  uint32_t* done_host, hipStream_t stream);
extern "C" int jb_mix_take(uint8_t* touched, uint8_t* mark, int64_t H, hipStream_t st);
extern "C" int jb_mix_pack_bf16(const float* snap, int64_t n, int Lc, int has_s, uint16_t* wb, float* sb,
                                hipStream_t st);
extern "C" int jb_mix_unpack_bf16(const uint16_t* wb, const float* sb, int64_t n, int Lc, int has_s, float* red,
                                  hipStream_t st);
extern "C" int64_t jb_mix_compact_temp_bytes(int64_t H);
extern "C" int jb_mix_compact(const uint8_t* mark, int64_t H, int64_t* rows, int64_t* count, void* temp,
                              int64_t temp_bytes, hipStream_t st);
extern "C" int jb_mix_gather(const float* W, const float* S, int LC, const int64_t* rows, int64_t n,
                             const int32_t* map, int Lc, float* snap, hipStream_t st);
extern "C" int jb_mix_fold(float* W, float* S, int LC, const int64_t* rows, int64_t n, const int32_t* map,
                           int Lc, const float* snap, const float* red, float inv_n, hipStream_t st);
extern "C" void* jb_host_alloc(int64_t nbytes);
extern "C" int jb_host_free(void* p);
extern "C" int64_t jb_hot_rep_bytes();

namespace {

const char* const kMethods[] = {"perceptron", "PA", "PA1", "PA2", "CW", "AROW", "NHERD"};
const int kLabelCaps[] = {8, 16, 32, 64, 128, 256, 512, 1024};
constexpr int kUpdateExact = 0, kUpdateAtomic = 1, kUpdateSerial = 3;

// how concurrent train requests of one batch update the model: serial-
// equivalent (default; csrc/hip/serial.hip) or lock-free atomic streams
// (JUBATUS_UPDATE_MODE=atomic; models/classifier.py concurrent_update)
int concurrent_update_mode() {
  const char* e = getenv("JUBATUS_UPDATE_MODE");
  return (e != nullptr && strcmp(e, "atomic") == 0) ? kUpdateAtomic : kUpdateSerial;
}
constexpr int kMethodCW = 4;
constexpr int kHotMaxRows = 64, kHotEntries = 512, kHotCap = 1 << 14, kHotWaves = 8;
constexpr int kDirectMaxSamples = 32, kDirectMaxSlots = 320;
constexpr int64_t kScanLdsBytes = 27 * 1024, kScanMaxSamples = 768;   // scan.hip

using namespace jb::srv;

struct Config {
  std::string text;
  int method = -1;
  float C = 1.f;
  Rules rules;
  bool wide = false;     // the wide rule set on the host (no GPU request scan)
  WideRules wrules;
};

bool parse_config(const std::string& text, Config* c, std::string* why) {
  Value v;
  try {
    v = jb::val::parse_json(text);
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
  if (v.kind != Value::MAP) { *why = "configuration must be a JSON object"; return false; }
  const std::string m = v.str_or("method", "");
  c->method = -1;
  for (int k = 0; k < 7; ++k)
    if (m == kMethods[k]) c->method = k;
  if (c->method < 0) { *why = "method " + m + " is not a linear method"; return false; }
  const Value* p = v.get("parameter");
  const Value* rw = p ? p->get("regularization_weight") : nullptr;
  if (c->method >= 2) {
    if (!rw || !rw->is_num() || !(rw->num() > 0)) { *why = "regularization_weight"; return false; }
  }
  c->C = rw && rw->is_num() ? (float)rw->num() : 1.f;
  const Value* conv = v.get("converter");
  Value empty;
  empty.kind = Value::MAP;
  c->rules.H = device_hash_max_size();   // unless the converter names hash_max_size
  if (!build_linear_rules(conv ? *conv : empty, &c->rules, &c->wide, &c->wrules, why)) return false;
  c->text = text;
  return true;
}

// ------------------------------------------------------------------ model
class Classifier : public jb::mix::Mixable {
 public:
  std::atomic<uint64_t> update_count{0};
  std::atomic<uint64_t> train_calls{0}, train_batches{0};
  uint64_t scan_gpu = 0, scan_replayed = 0, scan_host = 0;
  int device = 0;

  Classifier(const Config& cfg, int device_index) : device(device_index) {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipStreamCreateWithFlags(&copy_, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&prep_, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking));
    int lo = 0, hi = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIPCHK(hipStreamCreateWithPriority(&prio_, hipStreamNonBlocking, hi));
    HIPCHK(hipMalloc((void**)&stats_, 2 * sizeof(unsigned long long)));
    HIPCHK(hipMemset(stats_, 0, 2 * sizeof(unsigned long long)));
    HIPCHK(hipMalloc((void**)&hash_err_, sizeof(int32_t)));
    HIPCHK(hipMemset(hash_err_, 0, sizeof(int32_t)));
    direct_out_ = (float*)jb_host_alloc((int64_t)kDirectMaxSamples * 1024 * 4);
    direct_done_ = (uint32_t*)jb_host_alloc(4 * kDirectMaxSamples);
    hot_count_host_ = (int32_t*)jb_host_alloc(4);
    if (!direct_out_ || !direct_done_ || !hot_count_host_) throw std::runtime_error("hipHostMalloc failed");
    memset(direct_done_, 0, 4 * kDirectMaxSamples);
    HIPCHK(hipEventCreateWithFlags(&hot_seen_ev_, hipEventDisableTiming));
    const size_t rep = (size_t)jb_hot_rep_bytes();
    for (Hot& h : hots_) {
      HIPCHK(hipMalloc((void**)&h.rows, kHotMaxRows * 4));
      HIPCHK(hipMemset(h.rows, 0, kHotMaxRows * 4));
      HIPCHK(hipMalloc((void**)&h.n, 4));
      HIPCHK(hipMemset(h.n, 0, 4));
      HIPCHK(hipMalloc((void**)&h.rep, rep));
      HIPCHK(hipMemset(h.rep, 0, rep));
      HIPCHK(hipMalloc((void**)&h.gkey, kHotCap * 4));
      HIPCHK(hipMemset(h.gkey, 0xff, kHotCap * 4));
      HIPCHK(hipMalloc((void**)&h.gcnt, kHotCap * 4));
      HIPCHK(hipMemset(h.gcnt, 0, kHotCap * 4));
      HIPCHK(hipEventCreateWithFlags(&h.free, hipEventDisableTiming));
    }
    // the batch threads wait on check_done; JUBATUS_SERVER_BLOCKING_WAIT=1
    // parks them (blocking-sync event) instead of spinning. Measured neutral
    // on the served path, which is bound by the transport's framing
    // (profiles/r02_served_native_sweep.jsonl), so spinning stays the default.
    const char* blk = getenv("JUBATUS_SERVER_BLOCKING_WAIT");
    const unsigned wait_flags = (blk && strcmp(blk, "1") == 0) ? (unsigned)hipEventBlockingSync : 0u;
    for (Set& s : sets_) {
      for (hipEvent_t* e : {&s.copy_done, &s.ready, &s.free})
        HIPCHK(hipEventCreateWithFlags(e, hipEventDisableTiming));
      HIPCHK(hipEventCreateWithFlags(&s.check_done, hipEventDisableTiming | wait_flags));
    }
    configure(cfg);
  }

  // (re)build the model for a configuration (set_config / load with the file's config)
  void configure(const Config& cfg) {
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipDeviceSynchronize());
    cfg_ = cfg;
    mid_ = cfg.method;
    C_ = cfg.C;
    use_s_ = mid_ >= kMethodCW;
    H_ = cfg.rules.H;
    const Rules& r = cfg.rules;
    conv_.configure(r, cfg.wide, cfg.wrules);
    const size_t rs = sizeof(jb::HostRule);
    for (void** p : {&d_srules_, &d_nrules_, (void**)&d_blob_})
      if (*p) { HIPCHK(hipFree(*p)); *p = nullptr; }
    HIPCHK(hipMalloc(&d_srules_, rs * std::max<size_t>(1, r.s.size())));
    HIPCHK(hipMalloc(&d_nrules_, rs * std::max<size_t>(1, r.n.size())));
    HIPCHK(hipMalloc((void**)&d_blob_, std::max<size_t>(1, r.blob.size())));
    if (!r.s.empty()) HIPCHK(hipMemcpy(d_srules_, r.s.data(), rs * r.s.size(), hipMemcpyHostToDevice));
    if (!r.n.empty()) HIPCHK(hipMemcpy(d_nrules_, r.n.data(), rs * r.n.size(), hipMemcpyHostToDevice));
    if (!r.blob.empty()) HIPCHK(hipMemcpy(d_blob_, r.blob.data(), r.blob.size(), hipMemcpyHostToDevice));
    labels_.clear();
    alloc_locked(kLabelCaps[0], true);
  }

  const std::string& config_text() const { return cfg_.text; }

  // pinned receive slots of the transport (H2D straight from them)
  static uint8_t* alloc_arena(size_t bytes) {
    uint8_t* p = nullptr;
    HIPCHK(hipHostMalloc((void**)&p, bytes, hipHostMallocDefault));
    return p;
  }

  // --------------------------------------------------------------- train
  // served train batch over an arena slot: -> per request sample count, -1
  // ARGUMENT_ERROR, -2 error message in msgs[k]
  void train_arena(const uint8_t* arena, const std::vector<jb::ArenaReq>& reqs,
                   std::vector<int64_t>* res, std::vector<std::string>* msgs) {
    const size_t R = reqs.size();
    res->assign(R, -1);
    msgs->assign(R, std::string());
    train_calls += R;
    train_batches += 1;
    update_count += R;
    std::vector<int64_t> counts(R);
    bool gpu_ok = R > 0 && !conv_.wide();   // the wide rule set hashes on the host
    uint64_t used = 0;
    for (size_t k = 0; k < R && gpu_ok; ++k) {
      counts[k] = body_count(arena + reqs[k].off, reqs[k].len);
      if (counts[k] < 0 || (int64_t)(reqs[k].len + (reqs[k].off & 15)) > kScanLdsBytes ||
          counts[k] > kScanMaxSamples)
        gpu_ok = false;
      used = std::max<uint64_t>(used, reqs[k].off + reqs[k].len);
    }
    if (gpu_ok) {
      int si = -1;
      const auto t0 = std::chrono::steady_clock::now();
      {
        std::unique_lock<std::mutex> g(mu_);
        // every scan set busy (more batch threads than sets): wait for one
        set_cv_.wait(g, [&] {
          for (const Set& s : sets_)
            if (!s.inflight) return true;
          return false;
        });
        if (labels_.size() > 0) si = submit_scan_locked(arena, reqs, counts, used);
      }
      if (si >= 0) {
        jb::tx::Range tr("train.scan_check_wait");
        Set& s = sets_[si];
        const auto t1 = std::chrono::steady_clock::now();
        const hipError_t we = hipEventSynchronize(s.check_done);
        if (we != hipSuccess) {   // leave the set usable for the error replies that follow
          std::lock_guard<std::mutex> g(mu_);
          s.inflight = false;
          set_cv_.notify_one();
          throw std::runtime_error(std::string("hipEventSynchronize: ") + hipGetErrorString(we));
        }
        const auto t2 = std::chrono::steady_clock::now();
        std::lock_guard<std::mutex> g(mu_);
        prof_[0] += 1;
        prof_[1] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        prof_[2] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
        const int32_t err = ((volatile int32_t*)s.host_out)[0];
        s.inflight = false;
        set_cv_.notify_one();
        if (err == 0) {
          const int32_t* hist = s.host_out + 1;
          for (int64_t l = 0; l < s.nhist; ++l)
            if (hist[l]) labels_.add_count((int)l, (uint64_t)hist[l]);
          for (size_t k = 0; k < R; ++k) (*res)[k] = counts[k];
          scan_gpu += 1;
          return;
        }
        scan_replayed += 1;
      }
    }
    std::lock_guard<std::mutex> g(mu_);
    scan_host += 1;
    for (size_t k = 0; k < R; ++k)
      host_train_locked(arena + reqs[k].off, reqs[k].len, &(*res)[k], &(*msgs)[k]);
  }

  // one request body (list<labeled_datum>) on the host path
  void train_body(const uint8_t* b, size_t n, int64_t* res, std::string* msg) {
    train_calls += 1;
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    scan_host += 1;
    host_train_locked(b, n, res, msg);
  }

  // -------------------------------------------------------------- classify
  // bodies: list<datum> each; -> per body rows of (label, score) over the
  // live labels, or an error (ok[k] false: ARGUMENT_ERROR)
  std::vector<std::string> classify(const std::vector<std::pair<const uint8_t*, size_t>>& bodies,
                                    const std::vector<uint32_t>& msgids) {
    const size_t R = bodies.size();
    std::vector<std::string> out(R);
    std::vector<int64_t> first(R + 1, 0);
    std::vector<bool> ok(R, true);
    int64_t n = 0, slots = 0;
    cidx_.get(std::max<size_t>(cidx_.cap, 1024));
    cval_.get(cidx_.cap);
    row_.get(std::max<size_t>(row_.cap, 1024));
    row_.p[0] = 0;
    for (size_t k = 0; k < R; ++k) {
      first[k] = n;
      const int64_t n0 = n, s0 = slots;
      while (true) {
        int rc = conv_.hash_body(bodies[k].first, bodies[k].second, cidx_.p, cval_.p, row_.p,
                                    (int64_t)row_.cap - 1, (int64_t)cidx_.cap, &n, &slots);
        if (rc == 2) {   // grow and re-hash this body
          n = n0;
          slots = s0;
          cidx_.get(2 * cidx_.cap);
          cval_.get(cidx_.cap);
          row_.get(2 * row_.cap);
          continue;
        }
        if (rc == 1) { ok[k] = false; n = n0; slots = s0; }
        break;
      }
    }
    first[R] = n;
    std::vector<float> scores;
    std::vector<std::string> names;
    std::vector<int> cols;
    {
      std::lock_guard<std::mutex> g(mu_);
      sync_labels_locked();
      auto nm = labels_.names();
      auto al = labels_.alive();
      for (size_t c = 0; c < nm.size(); ++c)
        if (al[c]) { cols.push_back((int)c); names.push_back(nm[c]); }
      scores.resize((size_t)n * LC_);
      if (n > 0) score_locked(n, slots, scores.data());
    }
    for (size_t k = 0; k < R; ++k) {
      if (!ok[k]) { out[k] = jb::val::response_code(msgids[k], kArgumentError); continue; }
      MsgpackWriter w;
      const int64_t nk = first[k + 1] - first[k];
      w.arr((size_t)nk);
      for (int64_t i = first[k]; i < first[k + 1]; ++i) {
        w.arr(cols.size());
        for (size_t c = 0; c < cols.size(); ++c) {
          w.arr(2);
          w.raw(names[c]);
          w.dbl((double)scores[(size_t)i * LC_ + cols[c]]);
        }
      }
      out[k] = jb::val::response_ok(msgids[k], w.out);
    }
    return out;
  }

  // ---------------------------------------------------------------- labels
  std::vector<std::pair<std::string, uint64_t>> get_labels() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::pair<std::string, uint64_t>> out;
    auto nm = labels_.names();
    auto al = labels_.alive();
    for (size_t c = 0; c < nm.size(); ++c)
      if (al[c]) out.emplace_back(nm[c], labels_.count((int)c));
    return out;
  }

  bool set_label(const std::string& l) {
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    if (labels_.lookup(l) >= 0) return false;
    if (labels_.get_or_add(l.data(), l.size()) < 0) throw std::runtime_error("label table full");
    sync_labels_locked();
    return true;
  }

  bool delete_label(const std::string& l) {
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    const int i = labels_.lookup(l);
    if (i < 0) return false;
    labels_.remove(l);
    HIPCHK(hipMemset2DAsync(W_ + i, (size_t)LC_ * 4, 0, 4, H_, compute_));
    if (S_) {
      float* ones = ones_.get(H_);
      fill_ones(ones, H_);
      HIPCHK(hipMemcpy2DAsync(S_ + i, (size_t)LC_ * 4, ones, 4, 4, H_, hipMemcpyDeviceToDevice, compute_));
    }
    HIPCHK(hipStreamSynchronize(compute_));
    sync_labels_locked();
    return true;
  }

  void clear() {
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipDeviceSynchronize());
    count_base_.clear();
    labels_.clear();
    conv_.clear();
    alloc_locked(kLabelCaps[0], true);
  }

  // ---------------------------------------------------------------- persist
  // models/classifier.py pack(): rows that differ from the initial state over
  // the live label columns
  std::string pack_user_data() {
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipDeviceSynchronize());
    std::vector<float> W((size_t)H_ * LC_), S;
    HIPCHK(hipMemcpy(W.data(), W_, W.size() * 4, hipMemcpyDeviceToHost));
    if (S_) {
      S.resize(W.size());
      HIPCHK(hipMemcpy(S.data(), S_, S.size() * 4, hipMemcpyDeviceToHost));
    }
    auto nm = labels_.names();
    auto al = labels_.alive();
    std::vector<int> cols;
    for (size_t c = 0; c < nm.size(); ++c)
      if (al[c]) cols.push_back((int)c);
    std::vector<int64_t> rows;
    std::vector<float> Wr, Sr;
    for (uint64_t h = 0; h < H_; ++h) {
      const float* w = W.data() + h * LC_;
      bool t = false;
      for (int c : cols) t |= w[c] != 0.f;
      if (S_) {
        const float* s = S.data() + h * LC_;
        for (int c : cols) t |= s[c] != 1.f;
      }
      if (!t) continue;
      rows.push_back((int64_t)h);
      for (int c : cols) Wr.push_back(w[c]);
      if (S_)
        for (int c : cols) Sr.push_back(S[h * LC_ + c]);
    }
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);   // user_data_version
    u.map(8);
    u.str("method"); u.str(kMethods[mid_]);
    u.str("H"); u.uint(H_);
    u.str("labels"); u.arr(cols.size());
    for (int c : cols) u.str(nm[c]);
    u.str("counts"); u.arr(cols.size());
    for (int c : cols) u.uint(labels_.count(c));
    u.str("rows"); u.bin(rows.data(), rows.size() * 8);
    u.str("W"); u.bin(Wr.data(), Wr.size() * 4);
    u.str("P"); u.bin(Sr.data(), Sr.size() * 4);
    u.str("weights");
    conv_.pack(u);
    return std::move(u.out);
  }

  // models/classifier.py unpack()
  void unpack(const Value& obj) {
    if (obj.kind != Value::MAP) throw std::runtime_error("broken model data: driver pack");
    const Value* H = obj.get("H");
    if (!H || !H->is_num() || (uint64_t)H->num() != H_)
      throw std::runtime_error("model hash_max_size differs from the configuration");
    const Value* lv = obj.get("labels");
    const Value* cv = obj.get("counts");
    const Value* rv = obj.get("rows");
    const Value* wv = obj.get("W");
    const Value* pv = obj.get("P");
    if (!lv || lv->kind != Value::ARR || !cv || cv->kind != Value::ARR || !rv || !wv)
      throw std::runtime_error("broken model data: classifier tables");
    const size_t L = lv->a.size();
    const size_t nr = rv->s.size() / 8;
    if (wv->s.size() != nr * L * 4) throw std::runtime_error("broken model data: W rows");
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipDeviceSynchronize());
    labels_.clear();
    int cap = -1;
    for (int c : kLabelCaps)
      if ((size_t)c >= std::max<size_t>(1, L)) { cap = c; break; }
    if (cap < 0) throw std::runtime_error("at most 1024 labels are supported");
    alloc_locked(cap, true);
    for (size_t k = 0; k < L; ++k) {
      labels_.get_or_add(lv->a[k].s.data(), lv->a[k].s.size());
      labels_.set_count((int)k, k < cv->a.size() ? (uint64_t)cv->a[k].num() : 0);
    }
    sync_labels_locked();
    std::vector<float> W((size_t)H_ * LC_, 0.f), S;
    const int64_t* rows = (const int64_t*)rv->s.data();
    const float* wr = (const float*)wv->s.data();
    for (size_t k = 0; k < nr; ++k) {
      if (rows[k] < 0 || (uint64_t)rows[k] >= H_) throw std::runtime_error("broken model data: row index");
      memcpy(&W[(size_t)rows[k] * LC_], wr + k * L, L * 4);
    }
    HIPCHK(hipMemcpy(W_, W.data(), W.size() * 4, hipMemcpyHostToDevice));
    if (S_) {
      S.assign((size_t)H_ * LC_, 1.f);
      if (pv && pv->s.size() == nr * L * 4) {
        const float* sr = (const float*)pv->s.data();
        for (size_t k = 0; k < nr; ++k) memcpy(&S[(size_t)rows[k] * LC_], sr + k * L, L * 4);
      }
      HIPCHK(hipMemcpy(S_, S.data(), S.size() * 4, hipMemcpyHostToDevice));
    }
    conv_.unpack(obj.get("weights"));
  }

  // ------------------------------------------------------------ MIX
  // distributed mode: the train kernels mark the rows they write (touched_)
  // and the linear mixer (jb_mix_group.hpp) runs mix() / hand_over() on its
  // thread. Python twin: models/classifier.py mix_begin / mix_end /
  // broadcast_from over parallel/table_mix.py.
  void enable_mix() {
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipStreamCreateWithFlags(&mixs_, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&mix_ev_, hipEventDisableTiming));
    HIPCHK(hipMalloc((void**)&touched_, H_));
    HIPCHK(hipMemset(touched_, 1, H_));   // the first MIX is dense
    count_host_ = (int64_t*)jb_host_alloc(8);
    if (!count_host_) throw std::runtime_error("hipHostMalloc failed");
  }

  std::unique_ptr<jb::mix::Plane> make_plane(jb::mix::Star& star, double dl) {
    return jb::mix::make_device_plane(star, device, mixs_, dl);
  }

  uint64_t mix(jb::mix::Group& grp) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    // 1. label agreement: the canonical order is rank 0's labels, then the
    //    labels only later ranks have, in rank order
    std::string mine;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto nm = labels_.names();
      auto al = labels_.alive();
      for (size_t c = 0; c < nm.size(); ++c)
        if (al[c]) put_name(&mine, nm[c]);
    }
    const auto parts = star.allgather(mine, grp.deadline());
    std::vector<std::string> canon;
    {
      std::set<std::string> seen;
      for (const auto& p : parts)
        for (auto& n : get_names(p))
          if (seen.insert(n).second) canon.push_back(n);
    }
    const int Lc = (int)canon.size();
    std::vector<int32_t> map((size_t)std::max(Lc, 1), 0);
    std::vector<int64_t> delta((size_t)std::max(Lc, 1), 0);
    std::vector<uint64_t> cur_at((size_t)std::max(Lc, 1), 0);
    uint64_t gen;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& n : canon)
        if (labels_.lookup(n) < 0 && labels_.get_or_add(n.data(), n.size()) < 0)
          throw std::runtime_error("label table full");
      sync_labels_locked();
      for (int c = 0; c < Lc; ++c) {
        const int col = labels_.lookup(canon[c]);
        map[c] = col;
        cur_at[c] = labels_.count(col);
        delta[c] = (int64_t)cur_at[c] - (int64_t)count_base_[canon[c]];
      }
      mark_.get(H_);
      // the touched rows so far, in stream order behind the queued training
      if (jb_mix_take(touched_, mark_.p, (int64_t)H_, compute_) != 0) throw std::runtime_error("jb_mix_take failed");
      HIPCHK(hipEventRecord(mix_ev_, compute_));
      HIPCHK(hipStreamWaitEvent(mixs_, mix_ev_, 0));
      gen = gen_;
    }
    // 2. label counts: base + the cluster's summed deltas since the last MIX
    star.allreduce_sum(delta.data(), (size_t)Lc, grp.deadline());
    uint64_t bytes = 8ull * Lc;
    // 3. the union of the touched rows (MAX all-reduce of the bitmaps)
    pl.allreduce_max(mark_.p, H_, grp.deadline());
    bytes += H_;
    const int64_t tb = jb_mix_compact_temp_bytes((int64_t)H_);
    if (tb < 0) throw std::runtime_error("jb_mix_compact_temp_bytes failed");
    rows_.get(H_);
    count_dev_.get(1);
    temp_.get((size_t)std::max<int64_t>(tb, 1));
    if (jb_mix_compact(mark_.p, (int64_t)H_, rows_.p, count_dev_.p, temp_.p, tb, mixs_) != 0)
      throw std::runtime_error("jb_mix_compact failed");
    HIPCHK(hipMemcpyAsync(count_host_, count_dev_.p, 8, hipMemcpyDeviceToHost, mixs_));
    jb::mix::wait_stream(mixs_, grp.deadline());
    const int64_t nu = *(volatile int64_t*)count_host_;
    const bool dense = (uint64_t)nu * 2 > H_;
    const int64_t* rows = dense ? nullptr : rows_.p;
    const int64_t n = dense ? (int64_t)H_ : nu;
    last_rows_ = (uint64_t)n;
    last_dense_ = dense;
    bool applied = true;
    if (n > 0 && Lc > 0) {
      const size_t width = (size_t)(use_s_ ? 2 : 1) * Lc;
      const size_t elems = (size_t)n * width;
      // 4. snapshot of the union rows (behind the queued training), then the
      //    SUM all-reduce while training goes on
      {
        std::lock_guard<std::mutex> g(mu_);
        if (gen != gen_) {
          applied = false;
        } else {
          HIPCHK(hipMemcpyAsync(map_dev_.get((size_t)Lc), map.data(), 4 * (size_t)Lc, hipMemcpyHostToDevice,
                                compute_));
          if (jb_mix_gather(W_, S_, LC_, rows, n, map_dev_.p, Lc, snap_.get(elems), compute_) != 0)
            throw std::runtime_error("jb_mix_gather failed");
          HIPCHK(hipMemcpyAsync(red_.get(elems), snap_.p, elems * 4, hipMemcpyDeviceToDevice, compute_));
          HIPCHK(hipEventRecord(mix_ev_, compute_));
          HIPCHK(hipStreamWaitEvent(mixs_, mix_ev_, 0));
        }
      }
      int64_t ok[1] = {applied ? 0 : 1};
      star.allreduce_max(ok, 1, grp.deadline());   // a rank whose tables changed: nobody folds
      if (ok[0] == 0) {
        // JUBATUS_MIX_DTYPE=bf16: the weight columns travel as bf16 (half the
        // bytes; each hop of the ring SUM rounds to bf16, ~2^-9 relative), the
        // precisions fp32; members agree on the wire over the control plane
        int64_t wire[1] = {mix_bf16() && std::string(pl.name()) == "rccl" ? 0 : 1};
        star.allreduce_max(wire, 1, grp.deadline());
        last_wire_bf16_ = wire[0] == 0;
        if (last_wire_bf16_) {
          const int has_s = use_s_ ? 1 : 0;
          const size_t nl = (size_t)n * (size_t)Lc;
          uint16_t* wb = (uint16_t*)wire_.get(nl * 2 + (has_s ? nl * 4 : 0) + 16);
          float* sb = (float*)((uint8_t*)wb + ((nl * 2 + 15) & ~(size_t)15));
          if (jb_mix_pack_bf16(snap_.p, n, Lc, has_s, wb, sb, mixs_) != 0) throw std::runtime_error("jb_mix_pack_bf16");
          pl.allreduce_sum_bf16(wb, nl, grp.deadline());
          if (has_s) pl.allreduce_sum(sb, nl, grp.deadline());
          if (jb_mix_unpack_bf16(wb, sb, n, Lc, has_s, red_.p, mixs_) != 0)
            throw std::runtime_error("jb_mix_unpack_bf16");
          bytes += nl * 2 + (has_s ? nl * 4 : 0);
        } else {
          pl.allreduce_sum(red_.p, elems, grp.deadline());
          bytes += elems * 4;
        }
        // 5. fold: T += mean(snapshot) - snapshot (updates made meanwhile stay)
        std::lock_guard<std::mutex> g(mu_);
        HIPCHK(hipEventRecord(mix_ev_, mixs_));
        HIPCHK(hipStreamWaitEvent(compute_, mix_ev_, 0));
        if (gen == gen_) {
          if (jb_mix_fold(W_, S_, LC_, rows, n, map_dev_.p, Lc, snap_.p, red_.p, 1.f / (float)grp.world(),
                          compute_) != 0)
            throw std::runtime_error("jb_mix_fold failed");
        } else {
          applied = false;
        }
      } else {
        applied = false;
      }
      if (!applied) {   // every row of the next MIX: the union is dense again
        std::lock_guard<std::mutex> g(mu_);
        HIPCHK(hipMemsetAsync(touched_, 1, H_, compute_));
      }
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int c = 0; c < Lc; ++c) {
        const uint64_t nb = (uint64_t)((int64_t)count_base_[canon[c]] + delta[c]);
        const int col = labels_.lookup(canon[c]);
        if (col >= 0) labels_.set_count(col, nb + (labels_.count(col) - cur_at[c]));
        count_base_[canon[c]] = nb;
      }
      HIPCHK(hipStreamSynchronize(compute_));
    }
    // 6. the document statistics of idf / bm25 converters (the reference
    //    mixes the weight manager with the model)
    if (conv_.global()) {
      std::string dm;
      {
        std::lock_guard<std::mutex> g(mu_);
        dm = conv_.get_diff();
      }
      const auto parts = pl.allgather_bytes(star, dm, grp.deadline());
      std::lock_guard<std::mutex> g(mu_);
      conv_.put_diffs(parts);
      bytes += dm.size();
    }
    last_applied_ = applied;
    return bytes;
  }

  // ------------------------------------------------------------ push MIX
  // random / broadcast / skip mixers (push_mixer.cpp:335-408): a round
  // exchanges with one peer and both keep the pairwise mean over the rows
  // either of them touched since this MIX began; rows a round brought in go
  // on to the next round's peer. Python twin: models/classifier.py pair_mix
  // (whole tables). Label counts stay per server, as there.
  bool push_mixable() const override { return true; }
  void push_begin() override {
    std::lock_guard<std::mutex> g(mu_);
    mark_.get(H_);
    if (jb_mix_take(touched_, mark_.p, (int64_t)H_, compute_) != 0) throw std::runtime_error("jb_mix_take failed");
    HIPCHK(hipStreamSynchronize(compute_));
    push_dirty_ = false;
  }
  void push_end() override {
    {
      std::lock_guard<std::mutex> g(mu_);
      conv_.clear_diff();              // the own statistics went to every partner of this MIX
    }
    if (!push_dirty_) return;
    std::lock_guard<std::mutex> g(mu_);   // a round that could not fold: the next MIX is dense
    HIPCHK(hipMemsetAsync(touched_, 1, H_, compute_));
  }

  uint64_t pair_mix(jb::mix::Group& grp, int peer) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    const double dl = grp.deadline();
    std::string mine;
    if (peer >= 0) {
      std::lock_guard<std::mutex> g(mu_);
      auto nm = labels_.names();
      auto al = labels_.alive();
      for (size_t c = 0; c < nm.size(); ++c)
        if (al[c]) put_name(&mine, nm[c]);
    }
    // every call below is one of the round's collectives: a rank without a
    // peer makes them too, with nothing
    const std::string theirs = pl.exchange_bytes(star, peer, mine, dl);
    if (peer < 0) {
      pl.pair_max(star, nullptr, 0, -1, dl);
      pl.exchange_bytes(star, -1, std::string(), dl);
      pl.pair_sum(star, nullptr, 0, -1, dl);
      if (conv_.global()) pl.exchange_bytes(star, -1, std::string(), dl);
      return 0;
    }
    // 1. label agreement: the lower rank's labels, then the other's new ones
    std::vector<std::string> canon;
    {
      std::set<std::string> seen;
      const std::string& first = grp.rank() < peer ? mine : theirs;
      const std::string& second = grp.rank() < peer ? theirs : mine;
      for (const std::string* p : {&first, &second})
        for (auto& n : get_names(*p))
          if (seen.insert(n).second) canon.push_back(n);
    }
    const int Lc = (int)canon.size();
    std::vector<int32_t> map((size_t)std::max(Lc, 1), 0);
    uint64_t gen;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& n : canon)
        if (labels_.lookup(n) < 0 && labels_.get_or_add(n.data(), n.size()) < 0)
          throw std::runtime_error("label table full");
      sync_labels_locked();
      for (int c = 0; c < Lc; ++c) map[c] = labels_.lookup(canon[c]);
      gen = gen_;
    }
    // 2. the pair's row union (it stays marked for the MIX's later rounds)
    pl.pair_max(star, mark_.p, H_, peer, dl);
    uint64_t bytes = H_;
    const int64_t tb = jb_mix_compact_temp_bytes((int64_t)H_);
    if (tb < 0) throw std::runtime_error("jb_mix_compact_temp_bytes failed");
    rows_.get(H_);
    count_dev_.get(1);
    temp_.get((size_t)std::max<int64_t>(tb, 1));
    if (jb_mix_compact(mark_.p, (int64_t)H_, rows_.p, count_dev_.p, temp_.p, tb, mixs_) != 0)
      throw std::runtime_error("jb_mix_compact failed");
    HIPCHK(hipMemcpyAsync(count_host_, count_dev_.p, 8, hipMemcpyDeviceToHost, mixs_));
    jb::mix::wait_stream(mixs_, dl);
    const int64_t nu = *(volatile int64_t*)count_host_;
    const bool dense = (uint64_t)nu * 2 > H_;
    const int64_t* rows = dense ? nullptr : rows_.p;
    const int64_t n = dense ? (int64_t)H_ : nu;
    last_rows_ = (uint64_t)n;
    last_dense_ = dense;
    const size_t width = (size_t)(use_s_ ? 2 : 1) * Lc;
    const size_t elems = (size_t)std::max<int64_t>(n, 0) * width;
    // 3. snapshot of the union rows behind the queued training
    bool applied = gen == gen_;
    if (applied && elems > 0) {
      std::lock_guard<std::mutex> g(mu_);
      if (gen != gen_) {
        applied = false;
      } else {
        HIPCHK(hipMemcpyAsync(map_dev_.get((size_t)Lc), map.data(), 4 * (size_t)Lc, hipMemcpyHostToDevice, compute_));
        if (jb_mix_gather(W_, S_, LC_, rows, n, map_dev_.p, Lc, snap_.get(elems), compute_) != 0)
          throw std::runtime_error("jb_mix_gather failed");
        HIPCHK(hipMemcpyAsync(red_.get(elems), snap_.p, elems * 4, hipMemcpyDeviceToDevice, compute_));
        HIPCHK(hipEventRecord(mix_ev_, compute_));
        HIPCHK(hipStreamWaitEvent(mixs_, mix_ev_, 0));
      }
    }
    // 4. both sides fold, or neither
    const std::string ok = pl.exchange_bytes(star, peer, applied ? "1" : "0", dl);
    const bool both = applied && ok == "1";
    pl.pair_sum(star, both ? red_.p : nullptr, both ? elems : 0, both ? peer : -1, dl);
    if (both && elems > 0) {
      bytes += elems * 4;
      // 5. fold: T += (mine + theirs) / 2 - snapshot (updates made meanwhile stay)
      std::lock_guard<std::mutex> g(mu_);
      HIPCHK(hipEventRecord(mix_ev_, mixs_));
      HIPCHK(hipStreamWaitEvent(compute_, mix_ev_, 0));
      if (gen == gen_) {
        if (jb_mix_fold(W_, S_, LC_, rows, n, map_dev_.p, Lc, snap_.p, red_.p, 0.5f, compute_) != 0)
          throw std::runtime_error("jb_mix_fold failed");
      } else {
        applied = false;
      }
      HIPCHK(hipStreamSynchronize(compute_));
    }
    // a side that could not fold after the exchange (its labels re-laid out
    // meanwhile) differs from a peer that did: its next MIX is dense, which
    // re-marks every row (both sides fold, or the rows return)
    if (!both || !applied) push_dirty_ = true;
    // 6. the document statistics of idf / bm25 converters
    if (conv_.global()) {
      std::string dm;
      {
        std::lock_guard<std::mutex> g(mu_);
        dm = conv_.get_diff();
      }
      const std::string td = pl.exchange_bytes(star, peer, dm, dl);
      std::lock_guard<std::mutex> g(mu_);
      conv_.put_diffs(grp.rank() < peer ? std::vector<std::string>{dm, td} : std::vector<std::string>{td, dm},
                      true);
      bytes += dm.size();
    }
    last_applied_ = applied && both;
    return bytes;
  }

  // obsolete protocol: rank src sends its tables and labels; apply = take them
  void hand_over(jb::mix::Group& grp, int src, bool apply) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    std::string meta;
    int LC = 0;
    if (grp.rank() == src) {
      std::lock_guard<std::mutex> g(mu_);
      HIPCHK(hipStreamSynchronize(compute_));
      LC = LC_;
      auto nm = labels_.names();
      auto al = labels_.alive();
      meta.append((const char*)&LC, 4);
      for (size_t c = 0; c < nm.size(); ++c) {
        put_name(&meta, nm[c]);
        const uint64_t cnt = labels_.count((int)c);
        meta.append((const char*)&cnt, 8);
        meta.push_back(al[c] ? 1 : 0);
      }
      HIPCHK(hipMemcpyAsync(hw_.get(H_ * LC), W_, H_ * LC * 4, hipMemcpyDeviceToDevice, compute_));
      if (S_) HIPCHK(hipMemcpyAsync(hs_.get(H_ * LC), S_, H_ * LC * 4, hipMemcpyDeviceToDevice, compute_));
      HIPCHK(hipStreamSynchronize(compute_));
    }
    meta = star.bcast_str(src, meta, grp.deadline());
    if (meta.size() < 4) throw std::runtime_error("hand-over: broken label table");
    memcpy(&LC, meta.data(), 4);
    const size_t tb = H_ * (size_t)LC;
    pl.bcast(hw_.get(tb), tb * 4, src, grp.deadline());
    if (use_s_) pl.bcast(hs_.get(tb), tb * 4, src, grp.deadline());
    if (!apply || grp.rank() == src) return;
    std::lock_guard<std::mutex> g(mu_);
    HIPCHK(hipDeviceSynchronize());
    labels_.clear();
    alloc_locked(LC, true);
    size_t o = 4;
    std::vector<std::pair<std::string, bool>> dead;
    count_base_.clear();
    while (o < meta.size()) {
      std::string nm = take_name(meta, &o);
      uint64_t cnt;
      memcpy(&cnt, meta.data() + o, 8);
      const bool alive = meta[o + 8] != 0;
      o += 9;
      const int id = labels_.get_or_add(nm.data(), nm.size());
      labels_.set_count(id, cnt);
      count_base_[nm] = cnt;
      if (!alive) labels_.remove(nm);
    }
    HIPCHK(hipMemcpy(W_, hw_.p, tb * 4, hipMemcpyDeviceToDevice));
    if (S_) HIPCHK(hipMemcpy(S_, hs_.p, tb * 4, hipMemcpyDeviceToDevice));
    sync_labels_locked();
  }

  bool distributed() const { return touched_ != nullptr; }

  void status(std::vector<std::pair<std::string, std::string>>* st) {
    std::lock_guard<std::mutex> g(mu_);
    unsigned long long sv[2] = {0, 0};
    HIPCHK(hipMemcpy(sv, stats_, sizeof sv, hipMemcpyDeviceToHost));
    int live = 0;
    for (bool a : labels_.alive()) live += a;
    size_t fr = 0, total = 0;
    if (hipMemGetInfo(&fr, &total) != hipSuccess) fr = total = 0;
    auto add = [&](const char* k, const std::string& v) { st->emplace_back(k, v); };
    add("num_classes", std::to_string(live));
    add("num_features", std::to_string(H_));
    add("label_capacity", std::to_string(LC_));
    add("method", kMethods[mid_]);
    add("storage", "hbm");
    add("fv_path", "gpu");
    add("server_runtime", "native");
    add("train_scan.gpu", std::to_string(scan_gpu));
    add("train_scan.replayed", std::to_string(scan_replayed));
    add("train_scan.host", std::to_string(scan_host));
    add("train_scan.replay_failed", "0");
    add("train.samples_updated", std::to_string(sv[0]));
    add("train.samples_trained", std::to_string(sv[1]));
    add("train.update_mode", update_mode_ == kUpdateSerial ? "exact" : "atomic");
    add("batching.train.calls", std::to_string(train_calls.load()));
    add("batching.train.launches", std::to_string(train_batches.load()));
    if (prof_[0]) {   // GPU-scan batches: submit (lock + set wait + launch) / scan-check wait
      add("served.batches", std::to_string(prof_[0]));
      add("served.submit_us_per_batch", std::to_string(prof_[1] / prof_[0] / 1000));
      add("served.check_wait_us_per_batch", std::to_string(prof_[2] / prof_[0] / 1000));
    }
    add("device", "cuda:" + std::to_string(device));
    add("hbm_used_bytes", std::to_string(total - fr));
    if (touched_) {
      add("mix.last_rows", std::to_string(last_rows_));
      add("mix.last_mode", last_dense_ ? "dense" : "sparse");
      add("mix.last_applied", last_applied_ ? "1" : "0");
      add("mix.wire_dtype", last_wire_bf16_ ? "bf16" : "fp32");
    }
  }

 private:
  struct Set {
    DevBuf<uint8_t> buf;
    DevBuf<int64_t> meta, off, row, slots;
    DevBuf<int32_t> len, lab, idx, err;
    DevBuf<float> val;
    DevBuf<uint32_t> hist;
    DevBuf<uint8_t> serial;        // kSerial scratch (tail range + slack per sample)
    void* serial_seen = nullptr;   // the buffer jb_serial_scratch_forget last saw
    PinBuf<int64_t> meta_host;
    int32_t* host_out = nullptr;   // fine-grained: [err | hist nhist]
    int64_t nhist = 0, host_cap = 0;
    hipEvent_t copy_done, check_done, ready, free;
    bool used = false, inflight = false;
    JbTrainBatch a;
  };
  struct Hot {
    int32_t *rows, *n, *gkey, *gcnt;
    float* rep;
    hipEvent_t free;
    bool free_used = false;
  };

  template <class T>
  struct HostBuf {
    T* p = nullptr;
    size_t cap = 0;
    T* get(size_t n) {
      if (n > cap) {
        T* np = (T*)realloc(p, n * sizeof(T));
        if (!np) throw std::bad_alloc();
        p = np;
        cap = n;
      }
      return p;
    }
  };

  void fill_ones(float* d, size_t n) {
    uint32_t one;
    const float f = 1.f;
    memcpy(&one, &f, 4);
    HIPCHK(hipMemsetD32Async((hipDeviceptr_t)d, (int)one, n, compute_));
  }

  // (re)allocate the tables for LC label columns (copy: keep old columns)
  void alloc_locked(int LC, bool fresh) {
    float* W = nullptr;
    float* S = nullptr;
    HIPCHK(hipMalloc((void**)&W, (size_t)H_ * LC * 4));
    HIPCHK(hipMemsetAsync(W, 0, (size_t)H_ * LC * 4, compute_));
    if (use_s_) {
      HIPCHK(hipMalloc((void**)&S, (size_t)H_ * LC * 4));
      fill_ones(S, (size_t)H_ * LC);
    }
    if (!fresh && LC_ && W_) {
      HIPCHK(hipMemcpy2DAsync(W, (size_t)LC * 4, W_, (size_t)LC_ * 4, (size_t)LC_ * 4, H_,
                              hipMemcpyDeviceToDevice, compute_));
      if (S && S_)
        HIPCHK(hipMemcpy2DAsync(S, (size_t)LC * 4, S_, (size_t)LC_ * 4, (size_t)LC_ * 4, H_,
                                hipMemcpyDeviceToDevice, compute_));
    }
    HIPCHK(hipStreamSynchronize(compute_));
    HIPCHK(hipDeviceSynchronize());      // nothing in flight reads the old tables
    if (W_) HIPCHK(hipFree(W_));
    if (S_) HIPCHK(hipFree(S_));
    if (active_) HIPCHK(hipFree(active_));
    W_ = W;
    S_ = S;
    HIPCHK(hipMalloc((void**)&active_, (size_t)LC * 4));
    HIPCHK(hipMemset(active_, 0, (size_t)LC * 4));
    LC_ = LC;
    label_version_ = ~0ull;
    ++gen_;   // an in-flight MIX must not fold into the new tables
  }

  // grow the tables / refresh the active mask and the device label table
  void sync_labels_locked() {
    const uint64_t v = labels_.version();
    if (v == label_version_) return;
    const int n = labels_.size();
    if (n > LC_) {
      int cap = -1;
      for (int c : kLabelCaps)
        if (c >= n) { cap = c; break; }
      if (cap < 0) throw std::runtime_error("at most 1024 labels are supported");
      alloc_locked(cap, false);
    }
    auto names = labels_.names();
    auto alive = labels_.alive();
    std::vector<int32_t> mask(LC_, 0);
    for (size_t i = 0; i < alive.size(); ++i) mask[i] = alive[i] ? 1 : 0;
    // device label table of scan.hip: open addressing on FNV-1a 64,
    // meta = [blob offset, length, id] (feature_pipeline.label_table_arrays)
    int cap = 16;
    size_t live = 0;
    for (bool a : alive) live += a;
    while ((size_t)cap < 2 * live) cap *= 2;
    std::vector<uint64_t> th(cap, 0);
    std::vector<int32_t> tm(3 * (size_t)cap, -1);
    std::string blob;
    for (size_t i = 0; i < names.size(); ++i) {
      if (!alive[i]) continue;
      const uint64_t h = fnv1a64(names[i]);
      size_t j = h & (uint64_t)(cap - 1);
      while (tm[3 * j + 2] >= 0) j = (j + 1) & (size_t)(cap - 1);
      th[j] = h;
      tm[3 * j] = (int32_t)blob.size();
      tm[3 * j + 1] = (int32_t)names[i].size();
      tm[3 * j + 2] = (int32_t)i;
      blob += names[i];
    }
    if (blob.empty()) blob.push_back('\0');
    HIPCHK(hipDeviceSynchronize());      // in-flight scans read the old table
    HIPCHK(hipMemcpy(active_, mask.data(), mask.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(lt_hash_.get(th.size()), th.data(), th.size() * 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(lt_meta_.get(tm.size()), tm.data(), tm.size() * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(lt_blob_.get(blob.size()), blob.data(), blob.size(), hipMemcpyHostToDevice));
    lt_cap_ = cap;
    lt_blob_len_ = (int64_t)blob.size();
    label_version_ = v;
  }

  // models/classifier.py _hot_wanted
  bool hot_wanted(int64_t nstreams) {
    if (!(hot_rows_ && LC_ <= 64 && nstreams >= 16)) return false;
    ++hot_batches_;
    if (hot_seen_pending_ && hipEventQuery(hot_seen_ev_) == hipSuccess) {
      hot_last_ = ((volatile int32_t*)hot_count_host_)[0];
      hot_seen_pending_ = false;
    }
    return hot_last_ != 0 || hot_batches_ % 8 == 0;
  }

  // one GPU-scan batch (feature_pipeline.scan_batch_args + classifier._submit_scan)
  int submit_scan_locked(const uint8_t* arena, const std::vector<jb::ArenaReq>& reqs,
                         const std::vector<int64_t>& counts, uint64_t used) {
    jb::tx::Range tr("train.submit_h2d_scan_hash_train");
    sync_labels_locked();
    const int64_t R = (int64_t)reqs.size();
    int64_t n = 0;
    for (int64_t c : counts) n += c;
    int si = -1;
    for (int t = 0; t < 4; ++t) {
      const int k = (next_set_ + t) % 4;
      if (!sets_[k].inflight) { si = k; break; }
    }
    if (si < 0) return -1;
    next_set_ = (si + 1) % 4;
    Set& s = sets_[si];
    if (s.used) HIPCHK(hipEventSynchronize(s.free));
    s.used = true;
    const int64_t empty_off = (int64_t)((used + 15) & ~15ull) + 16;
    const int64_t buf_need = empty_off + 16;
    const int64_t sps = (int64_t)cfg_.rules.s.size(), spn = (int64_t)cfg_.rules.n.size();
    const int64_t slot_cap = (int64_t)(used / 3 + 1) * std::max<int64_t>(1, std::max(sps, spn));
    int64_t* mh = s.meta_host.get(3 * R + 1);
    mh[2 * R] = 0;
    for (int64_t k = 0; k < R; ++k) {
      mh[k] = (int64_t)reqs[k].off;
      mh[R + k] = (int64_t)reqs[k].len;
      mh[2 * R + 1 + k] = mh[2 * R + k] + counts[k];
    }
    const int64_t nhist = std::max<int64_t>(64, 2 * labels_.size());
    if (s.host_cap < 1 + nhist) {
      if (s.host_out) jb_host_free(s.host_out);
      s.host_out = (int32_t*)jb_host_alloc(4 * (1 + nhist));
      if (!s.host_out) throw std::runtime_error("hipHostMalloc failed");
      s.host_cap = 1 + nhist;
    }
    s.nhist = nhist;
    JbTrainBatch& a = s.a;
    memset(&a, 0, sizeof a);
    a.copy_stream = copy_;
    a.prep_stream = prep_;
    a.compute_stream = compute_;
    a.copy_done = s.copy_done;
    a.check_done = s.check_done;
    a.ready = s.ready;
    a.set_free = s.free;
    a.arena = arena;
    a.used = (int64_t)used;
    a.meta_host = mh;
    a.R = R;
    a.n = n;
    a.d_buf = s.buf.get(buf_need);
    a.buf_cap = (int64_t)s.buf.cap;
    a.empty_off = empty_off;
    a.d_meta = s.meta.get(3 * R + 1);
    a.d_off = s.off.get(std::max<int64_t>(n, 1));
    a.d_len = s.len.get(std::max<int64_t>(n, 1));
    a.d_lab = s.lab.get(std::max<int64_t>(n, 1));
    a.d_row = s.row.get(n + 1);
    a.d_slots = s.slots.get(R);
    a.d_hist = s.hist.get(nhist);
    a.nhist = nhist;
    a.d_err = s.err.get(1);
    a.host_out = s.host_out;
    a.lt_hash = lt_hash_.p;
    a.lt_meta = lt_meta_.p;
    a.lt_cap = lt_cap_;
    a.lt_blob = lt_blob_.p;
    a.lt_blob_len = lt_blob_len_;
    a.sps = sps;
    a.spn = spn;
    a.srules = d_srules_;
    a.nrules = d_nrules_;
    a.n_srules = sps;
    a.n_nrules = spn;
    a.blob = d_blob_;
    a.blob_len = (int64_t)std::max<size_t>(1, cfg_.rules.blob.size());
    a.H = (int64_t)H_;
    a.d_idx = s.idx.get(slot_cap);
    a.d_val = s.val.get(slot_cap);
    a.slot_cap = slot_cap;
    a.hash_err = hash_err_;
    a.W = W_;
    a.S = S_;
    a.active = active_;
    a.LC = LC_;
    a.method = mid_;
    a.C = C_;
    a.mode = R > 1 ? update_mode_ : kUpdateExact;
    if (a.mode == kUpdateSerial) {
      const int64_t sb = jb_serial_scratch_bytes_lc(std::max<int64_t>(n, 1), LC_);
      a.serial_scratch = s.serial.get((size_t)sb);
      a.serial_bytes = sb;
      if (a.serial_scratch != s.serial_seen) {     // a new buffer: no inherited segment history
        jb_serial_scratch_forget(a.serial_scratch);
        s.serial_seen = a.serial_scratch;
      }
    }
    a.merge_every = 1;
    a.hot_waves = kHotWaves;
    a.stats = stats_;
    a.touched = touched_;
    if (n > 0 && a.mode == kUpdateAtomic && hot_wanted(R)) {
      Hot& h = hots_[hot_turn_];
      hot_turn_ ^= 1;
      a.hot_rows = h.rows;
      a.hot_n = h.n;
      a.hot_rep = h.rep;
      a.gkey = h.gkey;
      a.gcnt = h.gcnt;
      a.gcap = kHotCap;
      a.block_min = 8;
      a.min_count = std::max<int64_t>(1024, n / 128);
      a.max_rows = std::min(kHotMaxRows, kHotEntries / LC_);
      a.hot_free = h.free;
      a.hot_free_valid = h.free_used ? 1 : 0;
      h.free_used = true;
      if (!hot_seen_pending_) {
        a.hot_count_host = hot_count_host_;
        a.hot_seen = hot_seen_ev_;
        hot_seen_pending_ = true;
      }
    }
    const int rc = jb_train_batch_submit(&a);
    if (rc != 0) {
      HIPCHK(hipDeviceSynchronize());
      throw std::runtime_error("jb_train_batch_submit failed: " + std::to_string(rc));
    }
    s.inflight = true;
    return si;
  }

  // host path of one request: validate the whole body, then commit labels
  // and counts, hash, one exact single-stream train launch
  void host_train_locked(const uint8_t* b, size_t len, int64_t* res, std::string* msg) {
    jb::tx::Range tr("train.host_path");
    jb::Cursor c{b, b + len};
    uint32_t cnt;
    if (!c.array(&cnt) || cnt > len) { *res = -1; return; }
    std::vector<std::pair<const uint8_t*, uint32_t>> labs;
    labs.reserve(cnt);
    int64_t slots = 0;
    HostBuf<int64_t>& row = hrow_;
    row.get((size_t)cnt + 1)[0] = 0;
    // the document statistics this request counts are undone if it fails
    // (the wide converter's idf / bm25); out of slots: grow, hash it again
    const jb::Cursor start = c;
    conv_.begin();
    for (uint32_t k = 0; k < cnt; ++k) {
      uint32_t two;
      const uint8_t* ls;
      uint32_t ln;
      if (!c.array(&two) || two != 2 || !c.raw(&ls, &ln)) { conv_.rollback(); *res = -1; return; }
      labs.emplace_back(ls, ln);
      const int64_t cap = (int64_t)std::max<size_t>(hidx_.cap, 256);
      int rc = conv_.hash_datum(c, hidx_.get(cap), hval_.get(cap), cap, &slots, true);
      if (rc == 2) {
        conv_.rollback();
        hidx_.get(2 * cap);
        hval_.get(2 * cap);
        c = start;
        labs.clear();
        slots = 0;
        k = (uint32_t)-1;   // restart the request
        conv_.begin();
        continue;
      }
      if (rc != 0) { conv_.rollback(); *res = -1; return; }
      row.p[k + 1] = slots;
    }
    if (c.p != c.end) { conv_.rollback(); *res = -1; return; }
    int32_t* lab = hlab_.get(std::max<uint32_t>(cnt, 1));
    for (uint32_t k = 0; k < cnt; ++k) {
      const int id = labels_.get_or_add((const char*)labs[k].first, labs[k].second);
      if (id < 0) { conv_.rollback(); *res = -2; *msg = "label table full"; return; }
      lab[k] = id;
    }
    try {
      sync_labels_locked();
    } catch (const std::exception& e) {
      conv_.rollback();
      *res = -2;
      *msg = e.what();
      return;
    }
    for (uint32_t k = 0; k < cnt; ++k) labels_.add_count(lab[k], 1);
    *res = cnt;
    if (cnt == 0) return;
    const int64_t nnz = std::max<int64_t>(slots, 1);
    int64_t sp[2] = {0, (int64_t)cnt};
    HIPCHK(hipMemcpyAsync(d_hrow_.get(cnt + 1), row.p, 8 * ((size_t)cnt + 1), hipMemcpyHostToDevice, compute_));
    HIPCHK(hipMemcpyAsync(d_hidx_.get(nnz), hidx_.p, 4 * (size_t)std::max<int64_t>(slots, 0),
                          hipMemcpyHostToDevice, compute_));
    HIPCHK(hipMemcpyAsync(d_hval_.get(nnz), hval_.p, 4 * (size_t)std::max<int64_t>(slots, 0),
                          hipMemcpyHostToDevice, compute_));
    HIPCHK(hipMemcpyAsync(d_hlab_.get(cnt), lab, 4 * (size_t)cnt, hipMemcpyHostToDevice, compute_));
    HIPCHK(hipMemcpyAsync(d_hsp_.get(2), sp, sizeof sp, hipMemcpyHostToDevice, compute_));
    const int rc = jb_linear_train(d_hrow_.p, d_hidx_.p, d_hval_.p, d_hlab_.p, d_hsp_.p, 1, W_, S_,
                                   active_, LC_, mid_, C_, kUpdateExact, nullptr, nullptr, nullptr, 1,
                                   kHotWaves, stats_, touched_, 0, nullptr, 0, compute_);
    if (rc != 0) throw std::runtime_error("jb_linear_train failed: " + std::to_string(rc));
    HIPCHK(hipStreamSynchronize(compute_));   // host sources are reused by the next request
  }

  // scores of the hashed classify batch (cidx_/cval_/row_) into out[n * LC]
  void score_locked(int64_t n, int64_t slots, float* out) {
    jb::tx::Range tr("classify.score");
    const int64_t* row = row_.p;
    if (n <= kDirectMaxSamples && row[n] - row[0] <= kDirectMaxSlots) {
      hipStream_t st = hipStreamQuery(compute_) == hipSuccess ? prio_ : compute_;
      const int rc = jb_classify_direct(cidx_.p, cval_.p, row, (int)n, W_, LC_, direct_out_,
                                        direct_done_, st);
      if (rc == 0) {
        memcpy(out, direct_out_, (size_t)n * LC_ * 4);
        return;
      }
      if (rc != 1) throw std::runtime_error("jb_classify_direct failed: " + std::to_string(rc));
    }
    const int64_t nnz = std::max<int64_t>(slots, 1);
    int64_t* prow = pin_row_.get(n + 1);
    int32_t* pidx = pin_idx_.get(nnz);
    float* pval = pin_val_.get(nnz);
    memcpy(prow, row, 8 * ((size_t)n + 1));
    memcpy(pidx, cidx_.p, 4 * (size_t)slots);
    memcpy(pval, cval_.p, 4 * (size_t)slots);
    HIPCHK(hipMemcpyAsync(d_crow_.get(n + 1), prow, 8 * ((size_t)n + 1), hipMemcpyHostToDevice, compute_));
    HIPCHK(hipMemcpyAsync(d_cidx_.get(nnz), pidx, 4 * (size_t)slots, hipMemcpyHostToDevice, compute_));
    HIPCHK(hipMemcpyAsync(d_cval_.get(nnz), pval, 4 * (size_t)slots, hipMemcpyHostToDevice, compute_));
    float* dout = d_cout_.get((size_t)n * LC_);
    const int rc = jb_linear_classify(d_crow_.p, d_cidx_.p, d_cval_.p, (int)n, W_, LC_, dout, compute_);
    if (rc != 0) throw std::runtime_error("jb_linear_classify failed: " + std::to_string(rc));
    float* pout = pin_out_.get((size_t)n * LC_);
    HIPCHK(hipMemcpyAsync(pout, dout, (size_t)n * LC_ * 4, hipMemcpyDeviceToHost, compute_));
    HIPCHK(hipStreamSynchronize(compute_));
    memcpy(out, pout, (size_t)n * LC_ * 4);
  }

  std::mutex mu_;
  std::condition_variable set_cv_;   // a scan set left flight
  uint64_t prof_[3] = {0, 0, 0};     // GPU-scan batches, submit ns, check-wait ns
  Config cfg_;
  int mid_ = 0;
  float C_ = 1.f;
  bool use_s_ = false;
  uint64_t H_ = 0;
  int LC_ = 0;
  float* W_ = nullptr;
  float* S_ = nullptr;
  int32_t* active_ = nullptr;
  jb::LabelTable labels_;
  uint64_t label_version_ = ~0ull;
  DevBuf<uint64_t> lt_hash_;
  DevBuf<int32_t> lt_meta_;
  DevBuf<uint8_t> lt_blob_;
  int64_t lt_cap_ = 16, lt_blob_len_ = 1;
  LinearConv conv_;
  void* d_srules_ = nullptr;
  void* d_nrules_ = nullptr;
  uint8_t* d_blob_ = nullptr;
  hipStream_t copy_, prep_, compute_, prio_;
  Set sets_[4];
  int next_set_ = 0;
  int32_t* hash_err_ = nullptr;
  Hot hots_[2];
  const int update_mode_ = concurrent_update_mode();
  // hot-row replica of the atomic mode (models/classifier.py hot_rows)
  const bool hot_rows_ = getenv("JUBATUS_HOT_ROWS") != nullptr && strcmp(getenv("JUBATUS_HOT_ROWS"), "1") == 0;
  int hot_turn_ = 0;
  int32_t* hot_count_host_ = nullptr;
  hipEvent_t hot_seen_ev_;
  bool hot_seen_pending_ = false;
  int hot_last_ = -1;
  uint64_t hot_batches_ = 0;
  unsigned long long* stats_ = nullptr;
  DevBuf<float> ones_;
  // host train path
  HostBuf<int32_t> hidx_, hlab_;
  HostBuf<float> hval_;
  HostBuf<int64_t> hrow_;
  DevBuf<int64_t> d_hrow_, d_hsp_;
  DevBuf<int32_t> d_hidx_, d_hlab_;
  DevBuf<float> d_hval_;
  // classify
  HostBuf<int32_t> cidx_;
  HostBuf<float> cval_;
  HostBuf<int64_t> row_;
  PinBuf<int64_t> pin_row_;
  PinBuf<int32_t> pin_idx_;
  PinBuf<float> pin_val_, pin_out_;
  DevBuf<int64_t> d_crow_;
  DevBuf<int32_t> d_cidx_;
  DevBuf<float> d_cval_, d_cout_;
  float* direct_out_ = nullptr;
  uint32_t* direct_done_ = nullptr;
  // distributed mode (MIX)
  uint8_t* touched_ = nullptr;
  uint64_t gen_ = 0;
  hipStream_t mixs_ = nullptr;
  hipEvent_t mix_ev_ = nullptr;
  DevBuf<uint8_t> mark_, temp_;
  DevBuf<int64_t> rows_, count_dev_;
  DevBuf<int32_t> map_dev_;
  DevBuf<float> snap_, red_, hw_, hs_;
  DevBuf<uint8_t> wire_;          // bf16 weight columns + fp32 precisions of a bf16-wire MIX
  bool last_wire_bf16_ = false;
  static bool mix_bf16() {
    static const bool v = [] {
      const char* e = getenv("JUBATUS_MIX_DTYPE");
      return e != nullptr && strcmp(e, "bf16") == 0;
    }();
    return v;
  }
  int64_t* count_host_ = nullptr;
  std::map<std::string, uint64_t> count_base_;
  uint64_t last_rows_ = 0;
  bool last_dense_ = false, last_applied_ = true;
  bool push_dirty_ = false;   // a pair round of this push MIX did not fold

  static void put_name(std::string* o, const std::string& n) {
    const uint32_t k = (uint32_t)n.size();
    o->append((const char*)&k, 4);
    *o += n;
  }
  static std::string take_name(const std::string& b, size_t* o) {
    if (*o + 4 > b.size()) throw std::runtime_error("MIX: broken label list");
    uint32_t k;
    memcpy(&k, b.data() + *o, 4);
    *o += 4;
    if (*o + k > b.size()) throw std::runtime_error("MIX: broken label list");
    std::string n = b.substr(*o, k);
    *o += k;
    return n;
  }
  static std::vector<std::string> get_names(const std::string& b) {
    std::vector<std::string> out;
    size_t o = 0;
    while (o < b.size()) out.push_back(take_name(b, &o));
    return out;
  }
};


// ------------------------------------------------------------ host backend
// GPU-less hosts (no /dev/kfd), --cpu and JUBATUS_FORCE_CPU: the same RPC
// surface, model files and MIX protocol with the tables in host memory, so a
// classifier server never needs Python (BASELINE config
// #1: pa.json standalone on the CPU). Training is the reference's loop, one
// sample after another under the model lock (classifier_serv.cpp:138-144),
// with the update rules of jb_host_linear.hpp (the host serial trainer of the
// CPU baseline); classify scores on the host; MIX runs the device tables'
// protocol over the host plane (HostPlane: the coordinator star carries the
// bytes). No HIP call is made in this mode.
class HostClassifier : public jb::mix::Mixable {
 public:
  std::atomic<uint64_t> update_count{0};
  std::atomic<uint64_t> train_calls{0}, train_batches{0};

  explicit HostClassifier(const Config& cfg) { configure(cfg); }

  static uint8_t* alloc_arena(size_t bytes) {
    void* p = nullptr;
    if (posix_memalign(&p, 4096, bytes) != 0) throw std::bad_alloc();
    return (uint8_t*)p;
  }

  void configure(const Config& cfg) {
    std::lock_guard<std::mutex> g(mu_);
    cfg_ = cfg;
    mid_ = cfg.method;
    C_ = cfg.C;
    use_s_ = mid_ >= kMethodCW;
    H_ = cfg.rules.H;
    conv_.configure(cfg.rules, cfg.wide, cfg.wrules);
    labels_.clear();
    count_base_.clear();
    alloc_locked(kLabelCaps[0], true);
    if (mixing_) touched_.assign(H_, 1);
  }

  const std::string& config_text() const { return cfg_.text; }

  void train_arena(const uint8_t* arena, const std::vector<jb::ArenaReq>& reqs, std::vector<int64_t>* res,
                   std::vector<std::string>* msgs) {
    const size_t R = reqs.size();
    res->assign(R, -1);
    msgs->assign(R, std::string());
    train_calls += R;
    train_batches += 1;
    update_count += R;
    std::lock_guard<std::mutex> g(mu_);
    for (size_t k = 0; k < R; ++k) train_locked(arena + reqs[k].off, reqs[k].len, &(*res)[k], &(*msgs)[k]);
  }

  void train_body(const uint8_t* b, size_t n, int64_t* res, std::string* msg) {
    train_calls += 1;
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    train_locked(b, n, res, msg);
  }

  std::vector<std::string> classify(const std::vector<std::pair<const uint8_t*, size_t>>& bodies,
                                    const std::vector<uint32_t>& msgids) {
    const size_t R = bodies.size();
    std::vector<std::string> out(R);
    std::vector<int32_t> idx(1024);
    std::vector<float> val(1024);
    std::vector<int64_t> row(1024);
    std::vector<float> sc;
    std::lock_guard<std::mutex> g(mu_);
    sync_labels_locked();
    auto nm = labels_.names();
    auto al = labels_.alive();
    std::vector<int> cols;
    for (size_t c = 0; c < nm.size(); ++c)
      if (al[c]) cols.push_back((int)c);
    for (size_t k = 0; k < R; ++k) {
      int64_t n = 0, slots = 0;
      row[0] = 0;
      int rc;
      while ((rc = conv_.hash_body(bodies[k].first, bodies[k].second, idx.data(), val.data(), row.data(),
                                   (int64_t)row.size() - 1, (int64_t)idx.size(), &n, &slots)) == 2) {
        n = slots = 0;
        idx.resize(2 * idx.size());
        val.resize(idx.size());
        row.resize(2 * row.size());
      }
      if (rc != 0) { out[k] = jb::val::response_code(msgids[k], kArgumentError); continue; }
      MsgpackWriter w;
      w.arr((size_t)n);
      sc.resize((size_t)LC_);
      for (int64_t i = 0; i < n; ++i) {
        jb::hl::scores(W_.data(), LC_, idx.data() + row[i], val.data() + row[i], (int)(row[i + 1] - row[i]),
                       sc.data());
        w.arr(cols.size());
        for (int c : cols) {
          w.arr(2);
          w.raw(nm[c]);
          w.dbl((double)sc[(size_t)c]);
        }
      }
      out[k] = jb::val::response_ok(msgids[k], w.out);
    }
    return out;
  }

  std::vector<std::pair<std::string, uint64_t>> get_labels() {
    std::lock_guard<std::mutex> g(mu_);
    std::vector<std::pair<std::string, uint64_t>> out;
    auto nm = labels_.names();
    auto al = labels_.alive();
    for (size_t c = 0; c < nm.size(); ++c)
      if (al[c]) out.emplace_back(nm[c], labels_.count((int)c));
    return out;
  }

  bool set_label(const std::string& l) {
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    if (labels_.lookup(l) >= 0) return false;
    if (labels_.get_or_add(l.data(), l.size()) < 0) throw std::runtime_error("label table full");
    sync_labels_locked();
    return true;
  }

  bool delete_label(const std::string& l) {
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    const int i = labels_.lookup(l);
    if (i < 0) return false;
    labels_.remove(l);
    for (uint64_t h = 0; h < H_; ++h) {
      W_[h * LC_ + i] = 0.f;
      if (use_s_) S_[h * LC_ + i] = 1.f;
    }
    sync_labels_locked();
    return true;
  }

  void clear() {
    update_count += 1;
    std::lock_guard<std::mutex> g(mu_);
    count_base_.clear();
    labels_.clear();
    conv_.clear();
    alloc_locked(kLabelCaps[0], true);
    if (mixing_) touched_.assign(H_, 1);
  }

  // the same user data as the device tables (models/classifier.py pack())
  std::string pack_user_data() {
    std::lock_guard<std::mutex> g(mu_);
    auto nm = labels_.names();
    auto al = labels_.alive();
    std::vector<int> cols;
    for (size_t c = 0; c < nm.size(); ++c)
      if (al[c]) cols.push_back((int)c);
    std::vector<int64_t> rows;
    std::vector<float> Wr, Sr;
    for (uint64_t h = 0; h < H_; ++h) {
      const float* w = W_.data() + h * LC_;
      bool t = false;
      for (int c : cols) t |= w[c] != 0.f;
      if (use_s_) {
        const float* s = S_.data() + h * LC_;
        for (int c : cols) t |= s[c] != 1.f;
      }
      if (!t) continue;
      rows.push_back((int64_t)h);
      for (int c : cols) Wr.push_back(w[c]);
      if (use_s_)
        for (int c : cols) Sr.push_back(S_[h * LC_ + c]);
    }
    MsgpackWriter u;
    u.arr(2);
    u.uint(1);
    u.map(8);
    u.str("method"); u.str(kMethods[mid_]);
    u.str("H"); u.uint(H_);
    u.str("labels"); u.arr(cols.size());
    for (int c : cols) u.str(nm[c]);
    u.str("counts"); u.arr(cols.size());
    for (int c : cols) u.uint(labels_.count(c));
    u.str("rows"); u.bin(rows.data(), rows.size() * 8);
    u.str("W"); u.bin(Wr.data(), Wr.size() * 4);
    u.str("P"); u.bin(Sr.data(), Sr.size() * 4);
    u.str("weights");
    conv_.pack(u);
    return std::move(u.out);
  }

  void unpack(const Value& obj) {
    if (obj.kind != Value::MAP) throw std::runtime_error("broken model data: driver pack");
    const Value* H = obj.get("H");
    if (!H || !H->is_num() || (uint64_t)H->num() != H_)
      throw std::runtime_error("model hash_max_size differs from the configuration");
    const Value* lv = obj.get("labels");
    const Value* cv = obj.get("counts");
    const Value* rv = obj.get("rows");
    const Value* wv = obj.get("W");
    const Value* pv = obj.get("P");
    if (!lv || lv->kind != Value::ARR || !cv || cv->kind != Value::ARR || !rv || !wv)
      throw std::runtime_error("broken model data: classifier tables");
    const size_t L = lv->a.size();
    const size_t nr = rv->s.size() / 8;
    if (wv->s.size() != nr * L * 4) throw std::runtime_error("broken model data: W rows");
    std::lock_guard<std::mutex> g(mu_);
    labels_.clear();
    int cap = -1;
    for (int c : kLabelCaps)
      if ((size_t)c >= std::max<size_t>(1, L)) { cap = c; break; }
    if (cap < 0) throw std::runtime_error("at most 1024 labels are supported");
    alloc_locked(cap, true);
    for (size_t k = 0; k < L; ++k) {
      labels_.get_or_add(lv->a[k].s.data(), lv->a[k].s.size());
      labels_.set_count((int)k, k < cv->a.size() ? (uint64_t)cv->a[k].num() : 0);
    }
    sync_labels_locked();
    const int64_t* rows = (const int64_t*)rv->s.data();
    const float* wr = (const float*)wv->s.data();
    const bool has_p = use_s_ && pv && pv->s.size() == nr * L * 4;
    for (size_t k = 0; k < nr; ++k) {
      if (rows[k] < 0 || (uint64_t)rows[k] >= H_) throw std::runtime_error("broken model data: row index");
      memcpy(&W_[(size_t)rows[k] * LC_], wr + k * L, L * 4);
      if (has_p) memcpy(&S_[(size_t)rows[k] * LC_], (const float*)pv->s.data() + k * L, L * 4);
    }
    conv_.unpack(obj.get("weights"));
    if (mixing_) touched_.assign(H_, 1);
  }

  void status(std::vector<std::pair<std::string, std::string>>* st) {
    std::lock_guard<std::mutex> g(mu_);
    int live = 0;
    for (bool a : labels_.alive()) live += a;
    auto add = [&](const char* k, const std::string& v) { st->emplace_back(k, v); };
    add("num_classes", std::to_string(live));
    add("num_features", std::to_string(H_));
    add("label_capacity", std::to_string(LC_));
    add("method", kMethods[mid_]);
    add("storage", "host");
    add("fv_path", "host");
    add("server_runtime", "native");
    add("backend", "host");
    add("train.samples_updated", std::to_string(n_upd_));
    add("train.samples_trained", std::to_string(n_valid_));
    add("train.update_mode", "exact");
    add("batching.train.calls", std::to_string(train_calls.load()));
    add("batching.train.launches", std::to_string(train_batches.load()));
    add("host_model_bytes", std::to_string((W_.size() + S_.size()) * 4));
    if (mixing_) {
      add("mix.last_rows", std::to_string(last_rows_));
      add("mix.last_mode", last_dense_ ? "dense" : "sparse");
      add("mix.last_applied", last_applied_ ? "1" : "0");
      add("mix.wire_dtype", "fp32");
    }
  }

  // ------------------------------------------------------------ MIX (host)
  void enable_mix() {
    std::lock_guard<std::mutex> g(mu_);
    mixing_ = true;
    touched_.assign(H_, 1);   // the first MIX is dense
  }
  std::unique_ptr<jb::mix::Plane> make_plane(jb::mix::Star& star, double) {
    return std::unique_ptr<jb::mix::Plane>(new jb::mix::HostPlane(&star));
  }

  uint64_t mix(jb::mix::Group& grp) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    std::string mine;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto nm = labels_.names();
      auto al = labels_.alive();
      for (size_t c = 0; c < nm.size(); ++c)
        if (al[c]) put_name(&mine, nm[c]);
    }
    const auto parts = star.allgather(mine, grp.deadline());
    std::vector<std::string> canon;
    {
      std::set<std::string> seen;
      for (const auto& p : parts)
        for (auto& n : get_names(p))
          if (seen.insert(n).second) canon.push_back(n);
    }
    const int Lc = (int)canon.size();
    std::vector<int32_t> map((size_t)std::max(Lc, 1), 0);
    std::vector<int64_t> delta((size_t)std::max(Lc, 1), 0);
    std::vector<uint64_t> cur_at((size_t)std::max(Lc, 1), 0);
    std::vector<uint8_t> mark;
    uint64_t gen;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& n : canon)
        if (labels_.lookup(n) < 0 && labels_.get_or_add(n.data(), n.size()) < 0)
          throw std::runtime_error("label table full");
      sync_labels_locked();
      for (int c = 0; c < Lc; ++c) {
        const int col = labels_.lookup(canon[c]);
        map[c] = col;
        cur_at[c] = labels_.count(col);
        delta[c] = (int64_t)cur_at[c] - (int64_t)count_base_[canon[c]];
      }
      mark.swap(touched_);
      touched_.assign(H_, 0);
      gen = gen_;
    }
    star.allreduce_sum(delta.data(), (size_t)Lc, grp.deadline());
    uint64_t bytes = 8ull * Lc;
    pl.allreduce_max(mark.data(), H_, grp.deadline());
    bytes += H_;
    std::vector<int64_t> rows;
    for (uint64_t h = 0; h < H_; ++h)
      if (mark[h]) rows.push_back((int64_t)h);
    const bool dense = rows.size() * 2 > H_;
    if (dense) {
      rows.resize(H_);
      for (uint64_t h = 0; h < H_; ++h) rows[h] = (int64_t)h;
    }
    last_rows_ = rows.size();
    last_dense_ = dense;
    bool applied = true;
    if (!rows.empty() && Lc > 0) {
      const size_t width = (size_t)(use_s_ ? 2 : 1) * Lc;
      std::vector<float> snap(rows.size() * width), red;
      {
        std::lock_guard<std::mutex> g(mu_);
        if (gen != gen_) applied = false;
        else gather_locked(rows, map, Lc, snap.data());
      }
      int64_t ok[1] = {applied ? 0 : 1};
      star.allreduce_max(ok, 1, grp.deadline());
      if (ok[0] == 0) {
        int64_t wire[1] = {1};   // fp32 on the wire (the device tables' agreement call)
        star.allreduce_max(wire, 1, grp.deadline());
        red = snap;
        pl.allreduce_sum(red.data(), red.size(), grp.deadline());
        bytes += red.size() * 4;
        std::lock_guard<std::mutex> g(mu_);
        if (gen == gen_) fold_locked(rows, map, Lc, snap.data(), red.data(), 1.f / (float)grp.world());
        else applied = false;
      } else {
        applied = false;
      }
      if (!applied) {
        std::lock_guard<std::mutex> g(mu_);
        touched_.assign(H_, 1);
      }
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      for (int c = 0; c < Lc; ++c) {
        const uint64_t nb = (uint64_t)((int64_t)count_base_[canon[c]] + delta[c]);
        const int col = labels_.lookup(canon[c]);
        if (col >= 0) labels_.set_count(col, nb + (labels_.count(col) - cur_at[c]));
        count_base_[canon[c]] = nb;
      }
    }
    if (conv_.global()) {
      std::string dm;
      {
        std::lock_guard<std::mutex> g(mu_);
        dm = conv_.get_diff();
      }
      const auto dparts = pl.allgather_bytes(star, dm, grp.deadline());
      std::lock_guard<std::mutex> g(mu_);
      conv_.put_diffs(dparts);
      bytes += dm.size();
    }
    last_applied_ = applied;
    return bytes;
  }

  bool push_mixable() const override { return true; }
  void push_begin() override {
    std::lock_guard<std::mutex> g(mu_);
    pmark_.swap(touched_);
    touched_.assign(H_, 0);
    push_dirty_ = false;
  }
  void push_end() override {
    std::lock_guard<std::mutex> g(mu_);
    conv_.clear_diff();
    if (push_dirty_) touched_.assign(H_, 1);
  }

  uint64_t pair_mix(jb::mix::Group& grp, int peer) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    const double dl = grp.deadline();
    std::string mine;
    if (peer >= 0) {
      std::lock_guard<std::mutex> g(mu_);
      auto nm = labels_.names();
      auto al = labels_.alive();
      for (size_t c = 0; c < nm.size(); ++c)
        if (al[c]) put_name(&mine, nm[c]);
    }
    const std::string theirs = pl.exchange_bytes(star, peer, mine, dl);
    if (peer < 0) {
      pl.pair_max(star, nullptr, 0, -1, dl);
      pl.exchange_bytes(star, -1, std::string(), dl);
      pl.pair_sum(star, nullptr, 0, -1, dl);
      if (conv_.global()) pl.exchange_bytes(star, -1, std::string(), dl);
      return 0;
    }
    std::vector<std::string> canon;
    {
      std::set<std::string> seen;
      const std::string& first = grp.rank() < peer ? mine : theirs;
      const std::string& second = grp.rank() < peer ? theirs : mine;
      for (const std::string* p : {&first, &second})
        for (auto& n : get_names(*p))
          if (seen.insert(n).second) canon.push_back(n);
    }
    const int Lc = (int)canon.size();
    std::vector<int32_t> map((size_t)std::max(Lc, 1), 0);
    uint64_t gen;
    {
      std::lock_guard<std::mutex> g(mu_);
      for (const auto& n : canon)
        if (labels_.lookup(n) < 0 && labels_.get_or_add(n.data(), n.size()) < 0)
          throw std::runtime_error("label table full");
      sync_labels_locked();
      for (int c = 0; c < Lc; ++c) map[c] = labels_.lookup(canon[c]);
      gen = gen_;
    }
    if (pmark_.size() != H_) pmark_.assign(H_, 1);
    pl.pair_max(star, pmark_.data(), H_, peer, dl);
    uint64_t bytes = H_;
    std::vector<int64_t> rows;
    for (uint64_t h = 0; h < H_; ++h)
      if (pmark_[h]) rows.push_back((int64_t)h);
    last_rows_ = rows.size();
    last_dense_ = rows.size() * 2 > H_;
    const size_t width = (size_t)(use_s_ ? 2 : 1) * Lc;
    const size_t elems = rows.size() * width;
    std::vector<float> snap(elems), red;
    bool applied = gen == gen_;
    if (applied && elems > 0) {
      std::lock_guard<std::mutex> g(mu_);
      if (gen != gen_) applied = false;
      else gather_locked(rows, map, Lc, snap.data());
    }
    const std::string ok = pl.exchange_bytes(star, peer, applied ? "1" : "0", dl);
    const bool both = applied && ok == "1";
    red = snap;
    pl.pair_sum(star, both ? red.data() : nullptr, both ? elems : 0, both ? peer : -1, dl);
    if (both && elems > 0) {
      bytes += elems * 4;
      std::lock_guard<std::mutex> g(mu_);
      if (gen == gen_) fold_locked(rows, map, Lc, snap.data(), red.data(), 0.5f);
      else applied = false;
    }
    if (!both || !applied) push_dirty_ = true;
    if (conv_.global()) {
      std::string dm;
      {
        std::lock_guard<std::mutex> g(mu_);
        dm = conv_.get_diff();
      }
      const std::string td = pl.exchange_bytes(star, peer, dm, dl);
      std::lock_guard<std::mutex> g(mu_);
      conv_.put_diffs(grp.rank() < peer ? std::vector<std::string>{dm, td} : std::vector<std::string>{td, dm},
                      true);
      bytes += dm.size();
    }
    last_applied_ = applied && both;
    return bytes;
  }

  void hand_over(jb::mix::Group& grp, int src, bool apply) override {
    jb::mix::Star& star = grp.star();
    jb::mix::Plane& pl = grp.plane();
    std::string meta;
    int LC = 0;
    std::vector<float> hw, hs;
    if (grp.rank() == src) {
      std::lock_guard<std::mutex> g(mu_);
      LC = LC_;
      auto nm = labels_.names();
      auto al = labels_.alive();
      meta.append((const char*)&LC, 4);
      for (size_t c = 0; c < nm.size(); ++c) {
        put_name(&meta, nm[c]);
        const uint64_t cnt = labels_.count((int)c);
        meta.append((const char*)&cnt, 8);
        meta.push_back(al[c] ? 1 : 0);
      }
      hw = W_;
      hs = S_;
    }
    meta = star.bcast_str(src, meta, grp.deadline());
    if (meta.size() < 4) throw std::runtime_error("hand-over: broken label table");
    memcpy(&LC, meta.data(), 4);
    const size_t tb = H_ * (size_t)LC;
    hw.resize(tb);
    pl.bcast(hw.data(), tb * 4, src, grp.deadline());
    if (use_s_) {
      hs.resize(tb);
      pl.bcast(hs.data(), tb * 4, src, grp.deadline());
    }
    if (!apply || grp.rank() == src) return;
    std::lock_guard<std::mutex> g(mu_);
    labels_.clear();
    alloc_locked(LC, true);
    size_t o = 4;
    count_base_.clear();
    while (o < meta.size()) {
      std::string nm = take_name(meta, &o);
      uint64_t cnt;
      if (o + 9 > meta.size()) throw std::runtime_error("hand-over: broken label table");
      memcpy(&cnt, meta.data() + o, 8);
      const bool alive = meta[o + 8] != 0;
      o += 9;
      const int id = labels_.get_or_add(nm.data(), nm.size());
      labels_.set_count(id, cnt);
      count_base_[nm] = cnt;
      if (!alive) labels_.remove(nm);
    }
    W_ = std::move(hw);
    if (use_s_) S_ = std::move(hs);
    sync_labels_locked();
  }

 private:
  // one request body on the host: validate it whole, commit labels and
  // counts, hash, then its samples one after another
  void train_locked(const uint8_t* b, size_t len, int64_t* res, std::string* msg) {
    jb::Cursor c{b, b + len};
    uint32_t cnt;
    if (!c.array(&cnt) || cnt > len) { *res = -1; return; }
    std::vector<std::pair<const uint8_t*, uint32_t>> labs;
    labs.reserve(cnt);
    int64_t slots = 0;
    row_.assign((size_t)cnt + 1, 0);
    const jb::Cursor start = c;
    conv_.begin();
    for (uint32_t k = 0; k < cnt; ++k) {
      uint32_t two;
      const uint8_t* ls;
      uint32_t ln;
      if (!c.array(&two) || two != 2 || !c.raw(&ls, &ln)) { conv_.rollback(); *res = -1; return; }
      labs.emplace_back(ls, ln);
      if (idx_.size() < 256) { idx_.resize(256); val_.resize(256); }
      const int rc = conv_.hash_datum(c, idx_.data(), val_.data(), (int64_t)idx_.size(), &slots, true);
      if (rc == 2) {   // out of slots: grow and hash the request again
        conv_.rollback();
        idx_.resize(2 * idx_.size());
        val_.resize(idx_.size());
        c = start;
        labs.clear();
        slots = 0;
        k = (uint32_t)-1;
        conv_.begin();
        continue;
      }
      if (rc != 0) { conv_.rollback(); *res = -1; return; }
      row_[k + 1] = slots;
    }
    if (c.p != c.end) { conv_.rollback(); *res = -1; return; }
    std::vector<int32_t> lab(cnt);
    for (uint32_t k = 0; k < cnt; ++k) {
      const int id = labels_.get_or_add((const char*)labs[k].first, labs[k].second);
      if (id < 0) { conv_.rollback(); *res = -2; *msg = "label table full"; return; }
      lab[k] = id;
    }
    try {
      sync_labels_locked();
    } catch (const std::exception& e) {
      conv_.rollback();
      *res = -2;
      *msg = e.what();
      return;
    }
    for (uint32_t k = 0; k < cnt; ++k) labels_.add_count(lab[k], 1);
    *res = cnt;
    jb::hl::Trainer tr(mid_, C_, LC_, active_.data(), W_.data(), use_s_ ? S_.data() : nullptr);
    for (uint32_t k = 0; k < cnt; ++k) {
      const int y = lab[k];
      if (y < 0 || y >= LC_) continue;
      ++n_valid_;
      const int32_t* ix = idx_.data() + row_[k];
      const int n = (int)(row_[k + 1] - row_[k]);
      if (k + 1 < cnt) tr.prefetch(idx_.data() + row_[k + 1], (int)(row_[k + 2] - row_[k + 1]));
      if (tr.step(ix, val_.data() + row_[k], n, y, nullptr)) {
        ++n_upd_;
        if (mixing_)
          for (int f = 0; f < n; ++f)
            if (ix[f] >= 0) touched_[(size_t)ix[f]] = 1;
      }
    }
  }

  void alloc_locked(int LC, bool fresh) {
    std::vector<float> W((size_t)H_ * LC, 0.f), S;
    if (use_s_) S.assign((size_t)H_ * LC, 1.f);
    if (!fresh && LC_ > 0 && !W_.empty())
      for (uint64_t h = 0; h < H_; ++h) {
        memcpy(&W[h * LC], &W_[h * LC_], (size_t)LC_ * 4);
        if (use_s_) memcpy(&S[h * LC], &S_[h * LC_], (size_t)LC_ * 4);
      }
    W_.swap(W);
    S_.swap(S);
    LC_ = LC;
    active_.assign((size_t)LC, 0);
    label_version_ = ~0ull;
    ++gen_;
  }

  void sync_labels_locked() {
    const uint64_t v = labels_.version();
    if (v == label_version_) return;
    const int n = labels_.size();
    if (n > LC_) {
      int cap = -1;
      for (int c : kLabelCaps)
        if (c >= n) { cap = c; break; }
      if (cap < 0) throw std::runtime_error("at most 1024 labels are supported");
      alloc_locked(cap, false);
    }
    auto alive = labels_.alive();
    active_.assign((size_t)LC_, 0);
    for (size_t i = 0; i < alive.size() && i < (size_t)LC_; ++i) active_[i] = alive[i] ? 1 : 0;
    label_version_ = v;
  }

  // [W columns | S columns] of the union rows, in canonical label order
  void gather_locked(const std::vector<int64_t>& rows, const std::vector<int32_t>& map, int Lc, float* snap) {
    const size_t width = (size_t)(use_s_ ? 2 : 1) * Lc;
    for (size_t i = 0; i < rows.size(); ++i) {
      const float* w = W_.data() + (size_t)rows[i] * LC_;
      for (int c = 0; c < Lc; ++c) snap[i * width + c] = w[map[c]];
      if (use_s_) {
        const float* s = S_.data() + (size_t)rows[i] * LC_;
        for (int c = 0; c < Lc; ++c) snap[i * width + Lc + c] = s[map[c]];
      }
    }
  }
  // T += sum * scale - snapshot (updates made during the MIX stay)
  void fold_locked(const std::vector<int64_t>& rows, const std::vector<int32_t>& map, int Lc, const float* snap,
                   const float* red, float scale) {
    const size_t width = (size_t)(use_s_ ? 2 : 1) * Lc;
    for (size_t i = 0; i < rows.size(); ++i) {
      float* w = W_.data() + (size_t)rows[i] * LC_;
      for (int c = 0; c < Lc; ++c) w[map[c]] += red[i * width + c] * scale - snap[i * width + c];
      if (use_s_) {
        float* s = S_.data() + (size_t)rows[i] * LC_;
        for (int c = 0; c < Lc; ++c) s[map[c]] += red[i * width + Lc + c] * scale - snap[i * width + Lc + c];
      }
    }
  }

  static void put_name(std::string* o, const std::string& n) {
    const uint32_t k = (uint32_t)n.size();
    o->append((const char*)&k, 4);
    *o += n;
  }
  static std::string take_name(const std::string& b, size_t* o) {
    if (*o + 4 > b.size()) throw std::runtime_error("MIX: broken label list");
    uint32_t k;
    memcpy(&k, b.data() + *o, 4);
    *o += 4;
    if (*o + k > b.size()) throw std::runtime_error("MIX: broken label list");
    std::string n = b.substr(*o, k);
    *o += k;
    return n;
  }
  static std::vector<std::string> get_names(const std::string& b) {
    std::vector<std::string> out;
    size_t o = 0;
    while (o < b.size()) out.push_back(take_name(b, &o));
    return out;
  }

  std::mutex mu_;
  Config cfg_;
  int mid_ = 0, LC_ = 0;
  float C_ = 1.f;
  bool use_s_ = false;
  uint64_t H_ = 0;
  std::vector<float> W_, S_;
  std::vector<uint8_t> active_;
  jb::LabelTable labels_;
  uint64_t label_version_ = ~0ull, gen_ = 0;
  LinearConv conv_;
  std::vector<int32_t> idx_;
  std::vector<float> val_;
  std::vector<int64_t> row_;
  uint64_t n_upd_ = 0, n_valid_ = 0;
  // distributed mode
  bool mixing_ = false;
  std::vector<uint8_t> touched_, pmark_;
  std::map<std::string, uint64_t> count_base_;
  uint64_t last_rows_ = 0;
  bool last_dense_ = false, last_applied_ = true, push_dirty_ = false;
};

// ----------------------------------------------------------------- server
// M: Classifier (device tables) or HostClassifier (host tables)
template <class M>
class Server {
 public:
  Server(const Args& a, std::unique_ptr<M> clf) : a_(a), clf_(std::move(clf)) { cs_.start_time = time(nullptr); }

  void load_file(const std::string& path) { load_impl(path, true); }

  int run() {
    rpc_.reset(new jb::RpcServer([this](const jb::RpcRequest& r) { return dispatch(r); }, a_.threads,
                                 (double)0));
    rpc_->set_io_threads(std::max(1, a_.threads / 4));
    rpc_->set_batch({"classify", "train"},
                    [this](const std::string& m, std::vector<jb::RpcRequest>& reqs) {
                      return batch(m, reqs);
                    },
                    4096);
    const char* mb = getenv("JUBATUS_TRAIN_ARENA_MB");
    const size_t slot_bytes = (size_t)atoll(mb ? mb : "32") << 20;
    const int nbatch = atoi(getenv("JUBATUS_ARENA_THREADS") ? getenv("JUBATUS_ARENA_THREADS") : "2");
    for (int k = 0; k < std::max(1, nbatch) + 2; ++k) slots_.push_back(M::alloc_arena(slot_bytes));
    rpc_->set_arena_batch("train", slots_, slot_bytes,
                          [this](int slot, const std::vector<jb::ArenaReq>& reqs) {
                            return arena(slot, reqs);
                          });
    rpc_->set_batch_threads(std::max(1, nbatch));
    int port;
    try {
      port = rpc_->listen(a_.bind, a_.port);
    } catch (const std::exception& e) {
      logf_("FATAL", "server failed to start: any process using port %d? (%s)", a_.port, e.what());
      return 1;
    }
    a_.port = port;
    logf_("INFO", "start listening at port %d", port);
    cs_.start_time = time(nullptr);
    rpc_->start();
    if (node_) {   // distributed mode: register, then the mixer thread
      node_->register_actor(a_.eth, a_.port);
      jb::mix::MixerArgs ma;
      ma.type = "classifier";
      ma.name = a_.name;
      ma.eth = a_.eth;
      ma.port = a_.port;
      ma.interval_sec = a_.interval_sec;
      ma.interval_count = a_.interval_count;
      ma.interconnect_timeout = a_.ic_timeout;
      M* c = clf_.get();
      mixer_.reset(new jb::mix::LinearMixer(node_->coord(), ma, c, [c](jb::mix::Group& g, double dl) {
        return c->make_plane(g.star(), dl);
      }));
      mixer_->start();
      logf_("INFO", "registered group membership as %s (native linear_mixer)", ident().c_str());
    }
    logf_("INFO", "jubaclassifier RPC server startup (native%s)",
          std::is_same<M, HostClassifier>::value ? ", host" : "");
    wait_for_term();
    if (mixer_) {
      logf_("INFO", "stopping mixer thread");
      mixer_->stop();
    }
    if (node_) node_->leave();
    logf_("INFO", "stopping RPC server");
    rpc_->stop();
    return 0;
  }

  // distributed mode (-z): coordinator session, config lock, MIX state
  void join_cluster(std::unique_ptr<jb::mix::ClusterNode> node) {
    node_ = std::move(node);
    a_.connected_zookeeper = node_->connected();
    if (!node_->config_rlock()) throw std::runtime_error("failed to get config lock");
    clf_->enable_mix();
  }

 private:
  std::string ident() const { return a_.eth + "_" + std::to_string(a_.port); }

  std::vector<std::string> arena(int slot, const std::vector<jb::ArenaReq>& reqs) {
    // JB_RPC_NULL_TRAIN=1 (measurement only): answer every train request of
    // the batch without training - the RPC layer's own ceiling (loopback TCP,
    // framing, the copies into the arena) at the same load (tools/rpc_ceiling.py)
    static const bool null_train = [] {
      const char* e = getenv("JB_RPC_NULL_TRAIN");
      return e != nullptr && e[0] == '1';
    }();
    std::vector<std::string> out(reqs.size());
    if (null_train) {
      rpc_->release_slot(slot);
      for (size_t k = 0; k < reqs.size(); ++k) {
        MsgpackWriter w;
        w.uint(0);
        out[k] = jb::val::response_ok(reqs[k].msgid, w.out);
      }
      return out;
    }
    if (mixer_) mixer_->updated(reqs.size());
    std::vector<int64_t> res;
    std::vector<std::string> msgs;
    try {
      clf_->train_arena(slots_[slot], reqs, &res, &msgs);
    } catch (const std::exception& e) {
      res.assign(reqs.size(), -2);
      msgs.assign(reqs.size(), e.what());
    }
    rpc_->release_slot(slot);
    for (size_t k = 0; k < reqs.size(); ++k) {
      if (res[k] >= 0) {
        MsgpackWriter w;
        w.uint((uint64_t)res[k]);
        out[k] = jb::val::response_ok(reqs[k].msgid, w.out);
      } else if (res[k] == -1) {
        out[k] = jb::val::response_code(reqs[k].msgid, kArgumentError);
      } else {
        out[k] = jb::val::response_msg(reqs[k].msgid, msgs[k]);
      }
    }
    return out;
  }

  // params [cluster name, body]: the body's span, or false
  static bool name_and_body(const std::string& params, const uint8_t** b, size_t* n) {
    jb::Cursor c{(const uint8_t*)params.data(), (const uint8_t*)params.data() + params.size()};
    uint32_t two;
    const uint8_t* s;
    uint32_t sn;
    if (!c.array(&two) || two != 2 || !c.raw(&s, &sn)) return false;
    *b = c.p;
    *n = (size_t)(c.end - c.p);
    return true;
  }

  std::vector<std::string> batch(const std::string& method, std::vector<jb::RpcRequest>& reqs) {
    std::vector<std::string> out(reqs.size());
    if (method == "classify") {
      std::vector<std::pair<const uint8_t*, size_t>> bodies;
      std::vector<uint32_t> ids;
      std::vector<size_t> where;
      for (size_t k = 0; k < reqs.size(); ++k) {
        const uint8_t* b;
        size_t n;
        if (!name_and_body(reqs[k].params, &b, &n)) {
          out[k] = jb::val::response_code(reqs[k].msgid, kArgumentError);
          continue;
        }
        bodies.emplace_back(b, n);
        ids.push_back(reqs[k].msgid);
        where.push_back(k);
      }
      try {
        auto res = clf_->classify(bodies, ids);
        for (size_t j = 0; j < where.size(); ++j) out[where[j]] = std::move(res[j]);
      } catch (const std::exception& e) {
        for (size_t j = 0; j < where.size(); ++j) out[where[j]] = jb::val::response_msg(ids[j], e.what());
      }
    } else {   // train requests that found no arena room
      if (mixer_) mixer_->updated(reqs.size());
      for (size_t k = 0; k < reqs.size(); ++k) {
        const uint8_t* b;
        size_t n;
        if (!name_and_body(reqs[k].params, &b, &n)) {
          out[k] = jb::val::response_code(reqs[k].msgid, kArgumentError);
          continue;
        }
        int64_t res = -1;
        std::string msg;
        try {
          clf_->train_body(b, n, &res, &msg);
        } catch (const std::exception& e) {
          res = -2;
          msg = e.what();
        }
        if (res >= 0) {
          MsgpackWriter w;
          w.uint((uint64_t)res);
          out[k] = jb::val::response_ok(reqs[k].msgid, w.out);
        } else if (res == -1) {
          out[k] = jb::val::response_code(reqs[k].msgid, kArgumentError);
        } else {
          out[k] = jb::val::response_msg(reqs[k].msgid, msg);
        }
      }
    }
    for (size_t k = 0; k < reqs.size(); ++k)
      if (reqs[k].notify) out[k].clear();
    return out;
  }

  std::string dispatch(const jb::RpcRequest& r) {
    std::string out;
    Value args;
    try {
      args = MsgpackReader((const uint8_t*)r.params.data(), r.params.size()).read();
    } catch (const std::exception&) {
      return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    }
    if (args.kind != Value::ARR) return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    const std::string& m = r.method;
    static const std::vector<std::pair<std::string, size_t>> arity = {
        {"get_config", 1}, {"save", 2}, {"load", 2}, {"get_status", 1}, {"get_labels", 1},
        {"set_label", 2}, {"clear", 1}, {"delete_label", 2}, {"train", 2}, {"classify", 2}};
    size_t want = 0;
    for (const auto& x : arity)
      if (x.first == m) want = x.second;
    if (m == "do_mix" && mixer_) want = 1;
    if (want == 0) return r.notify ? std::string() : jb::val::response_code(r.msgid, kNoMethodError);
    if (args.a.size() != want || (want == 2 && m != "train" && m != "classify" && !args.a[1].is_str()))
      return r.notify ? std::string() : jb::val::response_code(r.msgid, kArgumentError);
    MsgpackWriter w;
    try {
      if (m == "get_config") {
        w.raw(clf_->config_text());
      } else if (m == "get_labels") {
        auto l = clf_->get_labels();
        w.map(l.size());
        for (auto& kv : l) { w.raw(kv.first); w.uint(kv.second); }
      } else if (m == "set_label") {
        if (mixer_) mixer_->updated(1);
        w.boolean(clf_->set_label(args.a[1].s));
      } else if (m == "delete_label") {
        w.boolean(clf_->delete_label(args.a[1].s));
      } else if (m == "clear") {
        clf_->clear();
        logf_("INFO", "model cleared: %s", a_.name.c_str());
        w.boolean(true);
      } else if (m == "save") {
        auto p = save(args.a[1].s);
        w.map(1);
        w.raw(ident());
        w.raw(p);
      } else if (m == "load") {
        if (args.a[1].s.empty()) throw std::runtime_error("empty id is not allowed");
        load_impl(local_path(args.a[1].s), false);
        w.boolean(true);
      } else if (m == "get_status") {
        status(&w);
      } else if (m == "do_mix") {
        w.boolean(mixer_->do_mix());
      } else {   // train / classify outside the batch path (not reached: batched methods)
        std::vector<jb::RpcRequest> one{r};
        return batch(m, one)[0];
      }
    } catch (const std::exception& e) {
      return r.notify ? std::string() : jb::val::response_msg(r.msgid, e.what());
    }
    return r.notify ? std::string() : jb::val::response_ok(r.msgid, w.out);
  }

  std::string local_path(const std::string& id) const {
    return a_.datadir + "/" + a_.eth + "_" + std::to_string(a_.port) + "_classifier_" + id + ".jubatus";
  }

  std::string save(const std::string& id) {
    if (id.empty()) throw std::runtime_error("empty id is not allowed");
    const std::string path = local_path(id);
    logf_("INFO", "starting save to %s", path.c_str());
    std::string user;
    try {
      user = clf_->pack_user_data();
    } catch (const std::exception& e) {
      throw std::runtime_error("cannot write output file: " + path + ": " + e.what());
    }
    write_model_file(path, "classifier", id, clf_->config_text(), user);
    std::lock_guard<std::mutex> g(st_mu_);
    cs_.last_saved = time(nullptr);
    cs_.last_saved_path = path;
    logf_("INFO", "saved to %s", path.c_str());
    return path;
  }

  void load_impl(const std::string& path, bool overwrite_config) {
    logf_("INFO", "starting load from %s", path.c_str());
    std::string bytes;
    if (!read_file(path, &bytes)) throw std::runtime_error("cannot open input file: " + path + ": " + strerror(errno));
    ModelFile mf;
    std::string err = read_model_file(bytes, &mf);
    if (!err.empty()) throw std::runtime_error(err);
    if (mf.type != "classifier")
      throw std::runtime_error("invalid model type: saved type: " + mf.type + ", expected type: classifier");
    const std::string current = clf_->config_text();
    if (!overwrite_config && !jb::val::same_config(mf.config, current))
      throw std::runtime_error("model config mismatched with the running config");
    if (mf.user_version != 1)
      throw std::runtime_error("user data version mismatched: " + std::to_string(mf.user_version) +
                               ", current version: 1");
    if (overwrite_config && !jb::val::same_config(mf.config, current)) {
      Config cfg;
      std::string why;
      if (!parse_config(mf.config, &cfg, &why))
        throw std::runtime_error("model config is not served natively: " + why);
      clf_->configure(cfg);
    }
    clf_->unpack(mf.user);
    std::lock_guard<std::mutex> g(st_mu_);
    cs_.last_loaded = time(nullptr);
    cs_.last_loaded_path = path;
    logf_("INFO", "loaded from %s", path.c_str());
  }

  void status(MsgpackWriter* w) {
    std::vector<std::pair<std::string, std::string>> st;
    {
      std::lock_guard<std::mutex> g(st_mu_);
      common_status(a_, cs_, clf_->update_count.load(), &st);
    }
    clf_->status(&st);
    if (mixer_) mixer_->status(&st);
    if (rpc_) st.emplace_back("rpc.batches", std::to_string(rpc_->batches()));
    w->map(1);
    w->raw(ident());
    w->map(st.size());
    for (auto& kv : st) { w->raw(kv.first); w->raw(kv.second); }
  }

  Args a_;
  std::unique_ptr<M> clf_;
  std::unique_ptr<jb::mix::ClusterNode> node_;
  std::unique_ptr<jb::mix::LinearMixer> mixer_;
  std::unique_ptr<jb::RpcServer> rpc_;
  std::vector<uint8_t*> slots_;
  std::mutex st_mu_;
  CommonStatus cs_;
};

}  // namespace

int main(int argc, char** argv) {
  set_engine("classifier");
  Args a;
  std::string text;
  Config cfg;
  jb::rowsrv::Config ncfg;   // NN / cosine / euclidean: the row server (jb_row_server.hpp)
  bool nn = false;
  const int rc = startup(argc, argv, &a, &text, [&](const std::string& t, std::string* why) {
    std::string wn;
    if (jb::rowsrv::parse_config(jb::rowsrv::Kind::kClassifier, t, &ncfg, &wn)) {
      nn = true;
      return true;
    }
    nn = false;
    if (parse_config(t, &cfg, why)) return true;
    if (jb::rowsrv::is_nn_classifier(ncfg.outer)) *why = wn;
    return false;
  }, true, /*native_dist=*/true, /*native_push=*/true, /*host_ok=*/true);
  if (rc >= 0) return rc;
  // a GPU-less host (or --cpu / JUBATUS_FORCE_CPU): the linear methods run on
  // the native host backend; the nearest-neighbor methods need the device
  const bool host = a.cpu || getenv("JUBATUS_FORCE_CPU") != nullptr || access("/dev/kfd", R_OK | W_OK) != 0;
  if (nn && host) exec_python(argc, argv, "nearest-neighbor classifier without a GPU");
  if (nn) return jb::rowsrv::row_serve(jb::rowsrv::Kind::kClassifier, a, ncfg);
  if (host) {
    try {
      block_signals();
      logf_("INFO", "starting jubaclassifier %s RPC server at %s:%d (native, host backend)", kVersion,
            a.eth.c_str(), a.port);
      Server<HostClassifier> srv(a, std::unique_ptr<HostClassifier>(new HostClassifier(cfg)));
      if (!a.zookeeper.empty()) {
        srv.join_cluster(std::unique_ptr<jb::mix::ClusterNode>(
            new jb::mix::ClusterNode(a.zookeeper, std::max(1, a.zk_timeout), "classifier", a.name)));
      } else if (!a.model_file.empty()) {
        srv.load_file(a.model_file);
      }
      logf_("INFO", "config loaded: %s", kMethods[cfg.method]);
      return srv.run();
    } catch (const std::exception& e) {
      logf_("FATAL", "failed to start classifier: %s", e.what());
      return 1;
    }
  }
  // below this line the process owns the GPU: no exec
  try {
    const int device = device_and_signals(a);
    logf_("INFO", "starting jubaclassifier %s RPC server at %s:%d (native, device %d)", kVersion,
          a.eth.c_str(), a.port, device);
    Server<Classifier> srv(a, std::unique_ptr<Classifier>(new Classifier(cfg, device)));
    if (!a.zookeeper.empty()) {
      srv.join_cluster(std::unique_ptr<jb::mix::ClusterNode>(
          new jb::mix::ClusterNode(a.zookeeper, std::max(1, a.zk_timeout), "classifier", a.name)));
    } else if (!a.model_file.empty()) {
      srv.load_file(a.model_file);
    }
    logf_("INFO", "config loaded: %s", kMethods[cfg.method]);
    return srv.run();
  } catch (const std::exception& e) {
    logf_("FATAL", "failed to start classifier: %s", e.what());
    return 1;
  }
}
