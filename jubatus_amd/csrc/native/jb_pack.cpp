// See jb_pack.hpp.
#include "jb_pack.hpp"

#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <unordered_map>

namespace jb {

namespace {

struct ReqScan {
  std::vector<uint64_t> off;     // datum offset inside the request
  std::vector<int32_t> label;
  std::vector<int64_t> slots;
  bool ok = true;
  bool table_full = false;
};

void scan_one(const RequestView& r, bool labeled, int sps, int spn, LabelTable* table,
              std::unordered_map<std::string, int>* cache, ReqScan* out) {
  Cursor c{r.data, r.data + r.len};
  uint32_t n;
  if (!c.array(&n)) { out->ok = false; return; }
  out->off.reserve(n);
  out->slots.reserve(n);
  if (labeled) out->label.reserve(n);
  std::string key;
  for (uint32_t i = 0; i < n; ++i) {
    if (labeled) {
      uint32_t two; const uint8_t* ls; uint32_t ln;
      if (!c.array(&two) || two != 2 || !c.raw(&ls, &ln)) { out->ok = false; return; }
      key.assign((const char*)ls, ln);
      auto it = cache->find(key);
      int id;
      if (it != cache->end()) id = it->second;
      else {
        id = table->get_or_add(key.data(), key.size());
        if (id < 0) { out->table_full = true; out->ok = false; return; }
        cache->emplace(key, id);
      }
      out->label.push_back(id);
    }
    uint64_t doff = (uint64_t)(c.p - r.data);
    DatumShape d;
    if (!scan_datum(c, &d)) { out->ok = false; return; }
    out->off.push_back(doff);
    out->slots.push_back((int64_t)d.n_str * sps + (int64_t)d.n_num * spn);
  }
}

}  // namespace

PackResult pack_requests(const std::vector<RequestView>& reqs, bool labeled, int sps, int spn,
                         LabelTable* table, const PackOut& out, int nthreads) {
  PackResult res;
  const size_t R = reqs.size();
  std::vector<ReqScan> scans(R);
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > R) nthreads = (int)std::max<size_t>(R, 1);

  auto worker = [&](int t) {
    std::unordered_map<std::string, int> cache;  // per-thread label cache
    for (size_t k = t; k < R; k += nthreads) scan_one(reqs[k], labeled, sps, spn, table, &cache, &scans[k]);
  };
  if (nthreads == 1) worker(0);
  else {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(worker, t);
    for (auto& x : th) x.join();
  }

  // serial prefix over requests
  std::vector<uint64_t> byte_base(R);
  std::vector<int64_t> sample_base(R), slot_base(R);
  uint64_t bytes = 0; int64_t samples = 0, slots = 0;
  for (size_t k = 0; k < R; ++k) {
    if (!scans[k].ok) {
      res.error = scans[k].table_full ? 3 : 1;
      res.error_request = (int64_t)k;
      return res;
    }
    byte_base[k] = bytes; sample_base[k] = samples; slot_base[k] = slots;
    bytes += reqs[k].len;
    bytes = (bytes + 15) & ~(uint64_t)15;  // keep every request 16-B aligned in staging
    samples += (int64_t)scans[k].off.size();
    for (int64_t s : scans[k].slots) slots += s;
  }
  if (bytes > out.staging_cap || samples > out.max_samples) {
    // report the sizes needed so the caller can grow its buffers and retry
    res.error = 2; res.n_samples = samples; res.n_bytes = bytes; res.n_slots = slots;
    return res;
  }

  auto writer = [&](int t) {
    for (size_t k = t; k < R; k += nthreads) {
      memcpy(out.staging + byte_base[k], reqs[k].data, reqs[k].len);
      const ReqScan& sc = scans[k];
      int64_t s0 = sample_base[k], slot = slot_base[k];
      for (size_t i = 0; i < sc.off.size(); ++i) {
        out.datum_off[s0 + i] = (int64_t)(byte_base[k] + sc.off[i]);
        out.row_ptr[s0 + i] = slot;
        slot += sc.slots[i];
        if (labeled && out.labels) out.labels[s0 + i] = sc.label[i];
      }
    }
  };
  if (nthreads == 1) writer(0);
  else {
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(writer, t);
    for (auto& x : th) x.join();
  }
  out.row_ptr[samples] = slots;
  if (out.stream_ptr) {
    for (size_t k = 0; k < R; ++k) out.stream_ptr[k] = sample_base[k];
    out.stream_ptr[R] = samples;
  }
  if (labeled && table) {
    for (size_t k = 0; k < R; ++k)
      for (int32_t id : scans[k].label) table->add_count(id, 1);
  }
  res.n_samples = samples; res.n_bytes = bytes; res.n_slots = slots;
  return res;
}

}  // namespace jb
