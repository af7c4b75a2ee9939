// Host twin of the GPU fv_hash emitter (csrc/hip/jb_fv.hpp emit_datum):
// msgpack list<datum> -> hashed CSR (idx, val), same rule table, same
// feature order, same hash. Used by the low-latency classify path, where a
// request of a few datums is hashed on the CPU (~0.3 us) and its (idx, val)
// pairs travel to the GPU inside the kernel arguments (csrc/hip/classify_direct.hip).
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <vector>

#include "jb_hash.hpp"
#include "jb_msgpack.hpp"

namespace jb {

struct HostRule {        // byte layout of jb::GpuRule / gpu_path._RULE
  int32_t match_kind, match_off, match_len, suffix_off, suffix_len, value_kind;
  float weight;
  int32_t pad;
};

class HostFvHasher {
 public:
  HostFvHasher(const uint8_t* srules, int n_srules, const uint8_t* nrules, int n_nrules,
               const uint8_t* blob, size_t blob_len, uint64_t H)
      : s_(n_srules), n_(n_nrules), blob_(blob, blob + blob_len), H_(H) {
    if (n_srules) memcpy(s_.data(), srules, sizeof(HostRule) * n_srules);
    if (n_nrules) memcpy(n_.data(), nrules, sizeof(HostRule) * n_nrules);
  }

  // One body = msgpack list<datum>. Appends to idx/val, row_ptr gets one
  // entry per datum (end offset). Returns 0 ok, 1 malformed, 2 capacity.
  int hash_body(const uint8_t* p, size_t len, int32_t* idx, float* val, int64_t* row_ptr,
                int64_t max_samples, int64_t max_slots, int64_t* n, int64_t* slots) const {
    Cursor c{p, p + len};
    uint32_t cnt;
    if (!c.array(&cnt)) return 1;
    for (uint32_t i = 0; i < cnt; ++i) {
      if (*n >= max_samples) return 2;
      int rc = datum(c, idx, val, max_slots, slots);
      if (rc) return rc;
      row_ptr[++*n] = *slots;
    }
    return 0;
  }

  // One datum at the cursor: appends its slots (used by the native server's
  // host train path, which parses [label, datum] pairs itself).
  int hash_datum(Cursor& c, int32_t* idx, float* val, int64_t max_slots, int64_t* slots) const {
    return datum(c, idx, val, max_slots, slots);
  }

 private:
  bool match(const HostRule& r, const uint8_t* k, uint32_t kn) const {
    if (r.match_kind == 0) return true;
    const uint8_t* m = blob_.data() + r.match_off;
    const uint32_t mn = (uint32_t)r.match_len;
    if (r.match_kind == 3 && kn != mn) return false;
    if (kn < mn) return false;
    const uint8_t* base = (r.match_kind == 2) ? (k + kn - mn) : k;
    return memcmp(base, m, mn) == 0;
  }

  int datum(Cursor& c, int32_t* idx, float* val, int64_t max_slots, int64_t* slots) const {
    uint32_t top, ns, nn;
    if (!c.array(&top) || top < 2) return 1;
    if (!c.array(&ns)) return 1;
    for (uint32_t i = 0; i < ns; ++i) {
      uint32_t two; const uint8_t *k, *v; uint32_t kn, vn;
      if (!c.array(&two) || two != 2 || !c.raw(&k, &kn) || !c.raw(&v, &vn)) return 1;
      uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
      hk = fnv_bytes(hk, (const uint8_t*)"$", 1);
      hk = fnv_bytes(hk, v, vn);
      for (const HostRule& r : s_) {
        if (*slots >= max_slots) return 2;
        if (match(r, k, kn)) {
          idx[*slots] = (int32_t)hash_to_index(fnv_bytes(hk, blob_.data() + r.suffix_off,
                                                         (size_t)r.suffix_len), H_);
          val[*slots] = r.weight;
        } else {
          idx[*slots] = -1;
          val[*slots] = 0.f;
        }
        ++*slots;
      }
    }
    if (!c.array(&nn)) return 1;
    for (uint32_t i = 0; i < nn; ++i) {
      uint32_t two; const uint8_t* k; uint32_t kn; double x;
      if (!c.array(&two) || two != 2 || !c.raw(&k, &kn) || !c.number(&x)) return 1;
      const uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
      for (const HostRule& r : n_) {
        if (*slots >= max_slots) return 2;
        if (match(r, k, kn)) {
          idx[*slots] = (int32_t)hash_to_index(fnv_bytes(hk, blob_.data() + r.suffix_off,
                                                         (size_t)r.suffix_len), H_);
          val[*slots] = r.value_kind == 1 ? logf(fmaxf(1.f, (float)x)) : (float)x;
        } else {
          idx[*slots] = -1;
          val[*slots] = 0.f;
        }
        ++*slots;
      }
    }
    for (uint32_t i = 2; i < top; ++i)   // binary values (and extras) carry no GPU-path feature
      if (!c.skip()) return 1;
    return 0;
  }

  std::vector<HostRule> s_, n_;
  std::vector<uint8_t> blob_;
  uint64_t H_;
};

}  // namespace jb
