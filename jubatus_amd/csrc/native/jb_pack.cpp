// See jb_pack.hpp.
#include "jb_pack.hpp"

#include <string.h>

#include "jb_hash.hpp"
#include "jb_pool.hpp"

#include <algorithm>
#include <atomic>
#include <string>
#include <thread>
#include <unordered_map>

namespace jb {

namespace {

constexpr int kUnknownLabel = -3;

// Per-thread label cache: open addressing on FNV-1a of the label bytes,
// verified by a byte compare (labels are few and repeat on every sample).
// add = false: a label the table does not know yet is reported as
// kUnknownLabel instead of being added (the scan stays free of side effects
// until every request of the batch has validated).
class LabelCache {
 public:
  LabelCache(LabelTable* t, bool add) : table_(t), add_(add), slots_(256) {}
  int get(const uint8_t* s, uint32_t n) {
    const uint64_t h = fnv_bytes(kFnvOffset, s, n);
    size_t mask = slots_.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      Slot& sl = slots_[i];
      if (sl.id < 0) {
        int id = add_ ? table_->get_or_add((const char*)s, n)
                      : table_->lookup(std::string((const char*)s, n));
        if (id < 0) return add_ ? -1 : kUnknownLabel;
        sl.h = h; sl.key.assign((const char*)s, n); sl.id = id;
        if (++used_ * 2 > slots_.size()) rehash();
        return id;
      }
      if (sl.h == h && sl.key.size() == n && memcmp(sl.key.data(), s, n) == 0) return sl.id;
    }
  }

 private:
  struct Slot { uint64_t h = 0; std::string key; int id = -1; };
  void rehash() {
    std::vector<Slot> old;
    old.swap(slots_);
    slots_.resize(old.size() * 2);
    size_t mask = slots_.size() - 1;
    for (auto& o : old) {
      if (o.id < 0) continue;
      size_t i = o.h & mask;
      while (slots_[i].id >= 0) i = (i + 1) & mask;
      slots_[i] = std::move(o);
    }
  }
  LabelTable* table_;
  bool add_;
  std::vector<Slot> slots_;
  size_t used_ = 0;
};

// Number of elements of a request body (its top-level array header).
bool body_count(const RequestView& r, uint32_t* n) {
  Cursor c{r.data, r.data + r.len};
  return c.array(n);
}

// Scan request k straight into the final output slots [s0, s0 + n): datum
// offsets / lengths / labels, and row_ptr relative to the request (the
// request's slot base is added afterwards). Returns the request's slot total
// or -1 (malformed) / -2 (label table full). *unknown is set when a label is
// not in the table yet (lookup-only cache): its samples get label -1 and no
// count.
int64_t scan_into(const RequestView& r, int kind, int sps, int spn, LabelCache* cache,
                  const PackOut& out, uint64_t byte_base, int64_t s0, uint64_t* hist,
                  size_t hist_cap, bool* unknown) {
  Cursor c{r.data, r.data + r.len};
  uint32_t n;
  if (!c.array(&n)) return -1;
  int64_t slot = 0;
  for (uint32_t i = 0; i < n; ++i) {
    const int64_t s = s0 + i;
    if (kind == 1) {
      uint32_t two; const uint8_t* ls; uint32_t ln;
      if (!c.array(&two) || two != 2 || !c.raw(&ls, &ln)) return -1;
      const int id = cache->get(ls, ln);
      if (id == kUnknownLabel) {
        *unknown = true;
        if (out.labels) out.labels[s] = -1;
      } else {
        if (id < 0) return -2;
        if (out.labels) out.labels[s] = id;
        if ((size_t)id < hist_cap) ++hist[id];
      }
    } else if (kind == 2) {  // scored_datum [score, datum]
      uint32_t two; double score;
      if (!c.array(&two) || two != 2 || !c.number(&score)) return -1;
      const float f = (float)score;
      int32_t bits;
      memcpy(&bits, &f, 4);
      if (out.labels) out.labels[s] = bits;
    }
    const uint64_t doff = (uint64_t)(c.p - r.data);
    DatumShape d;
    if (!scan_datum(c, &d)) return -1;
    out.datum_off[s] = (int64_t)(byte_base + doff);
    if (out.datum_len) out.datum_len[s] = (int32_t)((uint64_t)(c.p - r.data) - doff);
    out.row_ptr[s] = slot;
    slot += (int64_t)d.n_str * sps + (int64_t)d.n_num * spn;
  }
  return slot;
}

}  // namespace

// Three passes, one of them over the bytes:
//   1. serial: each body's top-level array length -> sample base per request
//      (a few bytes per request);
//   2. parallel over requests: one scan writes every per-sample output at its
//      final index (row_ptr relative to the request) and counts labels into a
//      per-chunk histogram;
//   3. serial prefix of the per-request slot totals, then a parallel pass adds
//      each request's slot base to its row_ptr entries.
PackResult pack_requests(const std::vector<RequestView>& reqs, int kind, int sps, int spn,
                         LabelTable* table, const PackOut& out, int nthreads) {
  PackResult res;
  const size_t R = reqs.size();
  if (R == 0) {
    if (out.row_ptr) out.row_ptr[0] = 0;
    if (out.stream_ptr) out.stream_ptr[0] = 0;
    return res;
  }
  // ---- pass 1: sample and byte bases
  const bool copy = out.staging != nullptr;
  std::vector<uint64_t> byte_base(R);
  std::vector<int64_t> sample_base(R + 1);
  uint64_t bytes = 0;
  int64_t samples = 0;
  for (size_t k = 0; k < R; ++k) {
    uint32_t n;
    if (!body_count(reqs[k], &n)) { res.error = 1; res.error_request = (int64_t)k; return res; }
    sample_base[k] = samples;
    samples += n;
    if (copy) {
      byte_base[k] = bytes;
      bytes += reqs[k].len;
      bytes = (bytes + 15) & ~(uint64_t)15;  // keep every request 16-B aligned in staging
    } else {
      if (reqs[k].data < out.base) { res.error = 1; res.error_request = (int64_t)k; return res; }
      byte_base[k] = (uint64_t)(reqs[k].data - out.base);
      bytes = std::max<uint64_t>(bytes, byte_base[k] + reqs[k].len);
    }
  }
  sample_base[R] = samples;
  if ((copy && bytes > out.staging_cap) || samples > out.max_samples) {
    // report the sizes needed so the caller can grow its buffers and retry
    res.error = 2; res.n_samples = samples; res.n_bytes = bytes;
    return res;
  }

  // ---- pass 2: the scan
  WorkerPool& pool = global_pool(nthreads);
  const int64_t nchunks = std::min<int64_t>((int64_t)R, (int64_t)pool.size() * 4);
  auto chunk = [&](int64_t c, int64_t* b, int64_t* e) {
    *b = c * (int64_t)R / nchunks;
    *e = (c + 1) * (int64_t)R / nchunks;
  };
  std::vector<int64_t> req_slots(R, 0);
  std::vector<uint8_t> unknown(R, 0);
  std::atomic<int64_t> bad{-1};
  std::atomic<int> bad_kind{0};
  constexpr size_t kHist = 4096;  // labels beyond this are counted one by one
  const bool count = kind == 1 && table;
  std::vector<std::vector<uint64_t>> hists((size_t)nchunks);
  pool.parallel_for(nchunks, [&](int64_t c) {
    LabelCache cache(table, false);
    std::vector<uint64_t>& hist = hists[(size_t)c];
    hist.assign(count ? kHist : 0, 0);
    int64_t b, e;
    chunk(c, &b, &e);
    for (int64_t k = b; k < e; ++k) {
      if (copy) memcpy(out.staging + byte_base[k], reqs[k].data, reqs[k].len);
      bool unk = false;
      const int64_t sl = scan_into(reqs[k], kind, sps, spn, &cache, out, byte_base[k],
                                   sample_base[k], hist.data(), hist.size(), &unk);
      if (sl < 0) {
        int64_t expect = -1;
        bad.compare_exchange_strong(expect, k);
        bad_kind.store(sl == -2 ? 3 : 1);
        return;
      }
      req_slots[k] = sl;
      unknown[k] = unk ? 1 : 0;
      if (unk && out.labels) {     // its known labels were counted: the commit recounts it
        for (int64_t s = sample_base[k]; s < sample_base[k + 1]; ++s)
          if (out.labels[s] >= 0 && (size_t)out.labels[s] < hist.size()) --hist[out.labels[s]];
      }
    }
  });
  if (bad.load() >= 0) {        // nothing was added to the label table
    res.error = bad_kind.load();
    res.error_request = bad.load();
    return res;
  }
  // Every request validated: commit. Requests that carried new labels are
  // re-scanned in request order with a label-adding cache (new labels get
  // ids in the order they appear), the others' counts come from the chunk
  // histograms and the per-sample pass for ids past the histogram.
  if (count) {
    LabelCache adder(table, true);
    std::vector<uint64_t> dummy;
    for (size_t k = 0; k < R; ++k) {
      if (!unknown[k]) continue;
      bool unk = false;
      const int64_t sl = scan_into(reqs[k], kind, sps, spn, &adder, out, byte_base[k],
                                   sample_base[k], dummy.data(), 0, &unk);
      if (sl < 0) { res.error = sl == -2 ? 3 : 1; res.error_request = (int64_t)k; return res; }
      for (int64_t s = sample_base[k]; s < sample_base[k + 1]; ++s)
        if (out.labels && out.labels[s] >= 0) table->add_count(out.labels[s], 1);
    }
    for (const auto& hist : hists)
      for (size_t id = 0; id < hist.size(); ++id)
        if (hist[id]) table->add_count((int)id, hist[id]);
    if (out.labels)
      for (size_t k = 0; k < R; ++k) {
        if (unknown[k]) continue;
        for (int64_t s = sample_base[k]; s < sample_base[k + 1]; ++s)
          if ((size_t)out.labels[s] >= kHist) table->add_count(out.labels[s], 1);
      }
  }

  // ---- pass 3: slot bases
  std::vector<int64_t> slot_base(R);
  int64_t slots = 0;
  for (size_t k = 0; k < R; ++k) {
    slot_base[k] = slots;
    slots += req_slots[k];
  }
  pool.parallel_for(nchunks, [&](int64_t c) {
    int64_t b, e;
    chunk(c, &b, &e);
    for (int64_t k = b; k < e; ++k) {
      const int64_t base = slot_base[k];
      if (base == 0) continue;
      for (int64_t s = sample_base[k]; s < sample_base[k + 1]; ++s) out.row_ptr[s] += base;
    }
  });
  out.row_ptr[samples] = slots;
  if (out.stream_ptr)
    for (size_t k = 0; k <= R; ++k) out.stream_ptr[k] = sample_base[k];
  res.n_samples = samples; res.n_bytes = bytes; res.n_slots = slots;
  return res;
}

WorkerPool& global_pool(int nthreads) {
  static std::mutex mu;
  static WorkerPool* pool = nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (pool == nullptr || (nthreads > pool->size() && pool->size() < 64)) {
    // grown pools are leaked on purpose: a concurrent caller may still hold the old one
    pool = new WorkerPool(std::max(1, std::min(nthreads, 64)));
  }
  return *pool;
}

}  // namespace jb
