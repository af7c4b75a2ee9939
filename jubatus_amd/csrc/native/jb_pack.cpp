// See jb_pack.hpp.
#include "jb_pack.hpp"

#include <string.h>

#include "jb_hash.hpp"
#include "jb_pool.hpp"

#include <algorithm>
#include <string>
#include <thread>
#include <unordered_map>

namespace jb {

namespace {

struct ReqScan {
  std::vector<uint64_t> off;     // datum offset inside the request
  std::vector<uint32_t> len;     // datum byte length
  std::vector<int32_t> label;
  std::vector<int64_t> slots;
  bool ok = true;
  bool table_full = false;
};

// Per-thread label cache: open addressing on FNV-1a of the label bytes,
// verified by a byte compare (labels are few and repeat on every sample).
class LabelCache {
 public:
  explicit LabelCache(LabelTable* t) : table_(t), slots_(256) {}
  int get(const uint8_t* s, uint32_t n) {
    const uint64_t h = fnv_bytes(kFnvOffset, s, n);
    size_t mask = slots_.size() - 1;
    for (size_t i = h & mask;; i = (i + 1) & mask) {
      Slot& sl = slots_[i];
      if (sl.id < 0) {
        int id = table_->get_or_add((const char*)s, n);
        if (id < 0) return -1;
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
  std::vector<Slot> slots_;
  size_t used_ = 0;
};

void scan_one(const RequestView& r, int kind, int sps, int spn, LabelCache* cache,
              ReqScan* out) {
  Cursor c{r.data, r.data + r.len};
  uint32_t n;
  if (!c.array(&n)) { out->ok = false; return; }
  out->off.reserve(n);
  out->len.reserve(n);
  out->slots.reserve(n);
  if (kind) out->label.reserve(n);
  for (uint32_t i = 0; i < n; ++i) {
    if (kind == 1) {
      uint32_t two; const uint8_t* ls; uint32_t ln;
      if (!c.array(&two) || two != 2 || !c.raw(&ls, &ln)) { out->ok = false; return; }
      int id = cache->get(ls, ln);
      if (id < 0) { out->table_full = true; out->ok = false; return; }
      out->label.push_back(id);
    } else if (kind == 2) {  // scored_datum [score, datum]
      uint32_t two; double score;
      if (!c.array(&two) || two != 2 || !c.number(&score)) { out->ok = false; return; }
      const float f = (float)score;
      int32_t bits;
      memcpy(&bits, &f, 4);
      out->label.push_back(bits);
    }
    uint64_t doff = (uint64_t)(c.p - r.data);
    DatumShape d;
    if (!scan_datum(c, &d)) { out->ok = false; return; }
    out->off.push_back(doff);
    out->len.push_back((uint32_t)((uint64_t)(c.p - r.data) - doff));
    out->slots.push_back((int64_t)d.n_str * sps + (int64_t)d.n_num * spn);
  }
}

}  // namespace

PackResult pack_requests(const std::vector<RequestView>& reqs, int kind, int sps, int spn,
                         LabelTable* table, const PackOut& out, int nthreads) {
  PackResult res;
  const size_t R = reqs.size();
  std::vector<ReqScan> scans(R);
  if (R == 0) {
    if (out.row_ptr) out.row_ptr[0] = 0;
    if (out.stream_ptr) out.stream_ptr[0] = 0;
    return res;
  }

  WorkerPool& pool = global_pool(nthreads);
  const int64_t nchunks = std::min<int64_t>((int64_t)R, (int64_t)pool.size() * 4);
  auto chunk = [&](int64_t c, int64_t* b, int64_t* e) {
    *b = c * (int64_t)R / nchunks;
    *e = (c + 1) * (int64_t)R / nchunks;
  };
  pool.parallel_for(nchunks, [&](int64_t c) {
    LabelCache cache(table);
    int64_t b, e;
    chunk(c, &b, &e);
    for (int64_t k = b; k < e; ++k) scan_one(reqs[k], kind, sps, spn, &cache, &scans[k]);
  });

  // serial prefix over requests
  // staging == nullptr: zero-copy mode, the requests already live in one
  // pinned arena starting at out.base; offsets are taken relative to it.
  const bool copy = out.staging != nullptr;
  std::vector<uint64_t> byte_base(R);
  std::vector<int64_t> sample_base(R), slot_base(R);
  uint64_t bytes = 0; int64_t samples = 0, slots = 0;
  for (size_t k = 0; k < R; ++k) {
    if (!scans[k].ok) {
      res.error = scans[k].table_full ? 3 : 1;
      res.error_request = (int64_t)k;
      return res;
    }
    sample_base[k] = samples; slot_base[k] = slots;
    if (copy) {
      byte_base[k] = bytes;
      bytes += reqs[k].len;
      bytes = (bytes + 15) & ~(uint64_t)15;  // keep every request 16-B aligned in staging
    } else {
      if (reqs[k].data < out.base) { res.error = 1; res.error_request = (int64_t)k; return res; }
      byte_base[k] = (uint64_t)(reqs[k].data - out.base);
      bytes = std::max<uint64_t>(bytes, byte_base[k] + reqs[k].len);
    }
    samples += (int64_t)scans[k].off.size();
    for (int64_t s : scans[k].slots) slots += s;
  }
  if ((copy && bytes > out.staging_cap) || samples > out.max_samples) {
    // report the sizes needed so the caller can grow its buffers and retry
    res.error = 2; res.n_samples = samples; res.n_bytes = bytes; res.n_slots = slots;
    return res;
  }

  pool.parallel_for(nchunks, [&](int64_t c) {
    int64_t b, e;
    chunk(c, &b, &e);
    for (int64_t k = b; k < e; ++k) {
      if (copy) memcpy(out.staging + byte_base[k], reqs[k].data, reqs[k].len);
      const ReqScan& sc = scans[k];
      int64_t s0 = sample_base[k], slot = slot_base[k];
      for (size_t i = 0; i < sc.off.size(); ++i) {
        out.datum_off[s0 + i] = (int64_t)(byte_base[k] + sc.off[i]);
        if (out.datum_len) out.datum_len[s0 + i] = (int32_t)sc.len[i];
        out.row_ptr[s0 + i] = slot;
        slot += sc.slots[i];
        if (kind && out.labels) out.labels[s0 + i] = sc.label[i];
      }
    }
  });
  out.row_ptr[samples] = slots;
  if (out.stream_ptr) {
    for (size_t k = 0; k < R; ++k) out.stream_ptr[k] = sample_base[k];
    out.stream_ptr[R] = samples;
  }
  if (kind == 1 && table) {
    // per-chunk histograms, then one atomic add per (chunk, label)
    pool.parallel_for(nchunks, [&](int64_t c) {
      int64_t b, e;
      chunk(c, &b, &e);
      std::vector<uint64_t> hist;
      for (int64_t k = b; k < e; ++k)
        for (int32_t id : scans[k].label) {
          if ((size_t)id >= hist.size()) hist.resize((size_t)id + 1, 0);
          ++hist[id];
        }
      for (size_t id = 0; id < hist.size(); ++id)
        if (hist[id]) table->add_count((int)id, hist[id]);
    });
  }
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
