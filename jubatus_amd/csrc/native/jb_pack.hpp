// Native request scanner: msgpack `list<labeled_datum>` / `list<datum>`
// request bodies -> device-ready batch descriptors.
//
// This is the host half of the GPU fv_converter fast path (csrc/hip/fv_hash.hip):
// the scanner validates the datum structure, counts the features each datum
// will produce, resolves label strings to model columns and copies the raw
// request bytes into a pinned staging buffer. The bytes themselves are parsed
// and hashed on the GPU. Several concurrent requests are scanned in parallel
// (one request = one update stream, cf. the reference's RPC worker threads,
// jubatus/server/framework/server_util.cpp:155-156).
#pragma once
#include <stdint.h>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "jb_msgpack.hpp"

namespace jb {

// label string <-> model column; columns of deleted labels are recycled only
// by re-adding the same label (the engine zeroes the column on delete).
class LabelTable {
 public:
  static constexpr int kMaxLabels = 1 << 16;
  LabelTable() : counts_(new std::atomic<uint64_t>[kMaxLabels]) {
    for (int i = 0; i < kMaxLabels; ++i) counts_[i].store(0);
  }
  ~LabelTable() { delete[] counts_; }

  int get_or_add(const char* s, size_t n) {
    std::lock_guard<std::mutex> g(mu_);
    std::string k(s, n);
    auto it = ids_.find(k);
    if (it != ids_.end()) {
      if (!alive_[it->second]) { alive_[it->second] = true; ++version_; }
      return it->second;
    }
    if ((int)names_.size() >= kMaxLabels) return -1;
    int id = (int)names_.size();
    ids_.emplace(k, id);
    names_.push_back(k);
    alive_.push_back(true);
    ++version_;
    return id;
  }
  int lookup(const std::string& k) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = ids_.find(k);
    if (it == ids_.end() || !alive_[it->second]) return -1;
    return it->second;
  }
  bool remove(const std::string& k) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = ids_.find(k);
    if (it == ids_.end() || !alive_[it->second]) return false;
    alive_[it->second] = false;
    counts_[it->second].store(0);
    ++version_;
    return true;
  }
  void clear() {
    std::lock_guard<std::mutex> g(mu_);
    for (size_t i = 0; i < names_.size(); ++i) counts_[i].store(0);
    ids_.clear(); names_.clear(); alive_.clear();
    ++version_;
  }
  int size() { std::lock_guard<std::mutex> g(mu_); return (int)names_.size(); }
  std::vector<std::string> names() { std::lock_guard<std::mutex> g(mu_); return names_; }
  std::vector<bool> alive() { std::lock_guard<std::mutex> g(mu_); return alive_; }
  uint64_t version() { std::lock_guard<std::mutex> g(mu_); return version_; }
  void add_count(int id, uint64_t c) { counts_[id].fetch_add(c, std::memory_order_relaxed); }
  uint64_t count(int id) const { return counts_[id].load(std::memory_order_relaxed); }
  void set_count(int id, uint64_t c) { counts_[id].store(c); }

 private:
  std::mutex mu_;
  std::unordered_map<std::string, int> ids_;
  std::vector<std::string> names_;
  std::vector<bool> alive_;
  std::atomic<uint64_t>* counts_;
  uint64_t version_ = 0;
};

struct DatumShape {
  uint32_t n_str = 0, n_num = 0, n_bin = 0;
};

// Fast paths for the common encodings, used while at least kFastSlack bytes
// remain (so no per-byte bounds checks are needed):
//   string pair  0x92, fixraw key, fixraw value
//   num pair     0x92, fixraw key, positive/negative fixint | float32 | float64
// Anything else falls back to the checked cursor.
constexpr size_t kFastSlack = 80;

inline bool skip_str_pair_fast(Cursor& c) {
  const uint8_t* p = c.p;
  if (p[0] != 0x92 || (p[1] & 0xe0) != 0xa0) return false;
  const uint8_t* q = p + 2 + (p[1] & 0x1f);
  if ((q[0] & 0xe0) != 0xa0) return false;
  c.p = q + 1 + (q[0] & 0x1f);
  return true;
}

inline bool skip_num_pair_fast(Cursor& c) {
  const uint8_t* p = c.p;
  if (p[0] != 0x92 || (p[1] & 0xe0) != 0xa0) return false;
  const uint8_t* q = p + 2 + (p[1] & 0x1f);
  const uint8_t t = q[0];
  if (t <= 0x7f || t >= 0xe0) c.p = q + 1;
  else if (t == 0xcb) c.p = q + 9;
  else if (t == 0xca) c.p = q + 5;
  else return false;
  return true;
}

// Validate one datum [sv, nv, bv] and count its pairs.
inline bool scan_datum(Cursor& c, DatumShape* d) {
  uint32_t top;
  if (!c.array(&top) || top < 2) return false;
  uint32_t ns;
  if (!c.array(&ns)) return false;
  for (uint32_t i = 0; i < ns; ++i) {
    if ((size_t)(c.end - c.p) >= kFastSlack && skip_str_pair_fast(c)) continue;
    uint32_t two; const uint8_t* s; uint32_t n;
    if (!c.array(&two) || two != 2 || !c.raw(&s, &n) || !c.raw(&s, &n)) return false;
  }
  uint32_t nn;
  if (!c.array(&nn)) return false;
  for (uint32_t i = 0; i < nn; ++i) {
    if ((size_t)(c.end - c.p) >= kFastSlack && skip_num_pair_fast(c)) continue;
    uint32_t two; const uint8_t* s; uint32_t n; double x;
    if (!c.array(&two) || two != 2 || !c.raw(&s, &n) || !c.number(&x)) return false;
  }
  uint32_t nb = 0;
  if (top >= 3) {
    if (!c.array(&nb)) return false;
    for (uint32_t i = 0; i < nb; ++i) {
      uint32_t two; const uint8_t* s; uint32_t n;
      if (!c.array(&two) || two != 2 || !c.raw(&s, &n) || !c.raw(&s, &n)) return false;
    }
  }
  for (uint32_t i = 3; i < top; ++i)
    if (!c.skip()) return false;
  d->n_str = ns; d->n_num = nn; d->n_bin = nb;
  return true;
}

struct RequestView {
  const uint8_t* data;
  uint64_t len;
};

struct PackOut {
  uint8_t* staging;         // pinned host buffer receiving the raw request bytes,
                            // or null: zero-copy, requests already in an arena at `base`
  const uint8_t* base;
  uint64_t staging_cap;
  int64_t* datum_off;       // [max_samples]
  int32_t* datum_len;       // [max_samples] (may be null)
  int32_t* labels;          // [max_samples] (train only, may be null)
  int64_t* row_ptr;         // [max_samples + 1]
  int64_t* stream_ptr;      // [n_requests + 1]
  int64_t max_samples;
};

struct PackResult {
  int64_t n_samples = 0;
  uint64_t n_bytes = 0;
  int64_t n_slots = 0;
  int error = 0;            // 0 ok, 1 malformed request k, 2 capacity, 3 label table full
  int64_t error_request = -1;
};

// kind 0: list<datum>; 1: list<[label, datum]> (labels -> ids); 2: list<[score, datum]>
// (scored; the float targets are written, bit-cast, into out.labels)
PackResult pack_requests(const std::vector<RequestView>& reqs, int kind, int slots_per_str,
                         int slots_per_num, LabelTable* table, const PackOut& out, int nthreads);

}  // namespace jb
