// Device half of the GPU fv_converter: rule table + per-datum feature
// emission, shared by the batch kernel (fv_hash.hip) and the fused
// low-latency classify kernel (classify_direct.hip).
// Feature-name scheme: jubatus_amd/fv_converter/converter.py.
#pragma once
#include "jb_device.hpp"

namespace jb {

// One key matcher + one feature-name suffix. Packed by the host
// (jubatus_amd/fv_converter/gpu_path.py, GpuRuleTable).
struct GpuRule {
  int32_t match_kind;   // 0 '*', 1 prefix "abc*", 2 suffix "*abc", 3 exact
  int32_t match_off;    // offset of the matcher bytes in the rule blob
  int32_t match_len;
  int32_t suffix_off;   // offset of "@str#bin/bin" / "@num" / "@log"
  int32_t suffix_len;
  int32_t value_kind;   // string rules: 0 = constant weight; num rules: 0 num, 1 log
  float weight;         // string rules: sample_weight*global_weight for one occurrence
  int32_t pad;
};

__device__ __forceinline__ bool key_matches(const GpuRule& r, const uint8_t* blob,
                                            const uint8_t* k, int kn) {
  if (r.match_kind == 0) return true;
  const uint8_t* m = blob + r.match_off;
  int mn = r.match_len;
  if (r.match_kind == 3 && kn != mn) return false;
  if (kn < mn) return false;
  const uint8_t* base = (r.match_kind == 2) ? (k + kn - mn) : k;
  for (int i = 0; i < mn; ++i)
    if (base[i] != m[i]) return false;
  return true;
}

// Walk one datum and emit its feature slots; returns false on a structural
// error (the host scanner validated the bytes already, so this is defensive).
__device__ __forceinline__ bool emit_datum(Reader& rd, int64_t slot, const int64_t slot_end,
                                           const GpuRule* __restrict__ srules, int n_srules,
                                           const GpuRule* __restrict__ nrules, int n_nrules,
                                           const uint8_t* blob, uint64_t H,
                                           int32_t* __restrict__ out_idx,
                                           float* __restrict__ out_val) {
  int64_t top = rd.array_len();
  if (top < 2) return false;
  // ---- string_values: [[key, value], ...]
  int64_t ns = rd.array_len();
  for (int64_t i = 0; i < ns && rd.ok; ++i) {
    if (rd.array_len() != 2) return false;
    const uint8_t *k, *v; int kn, vn;
    if (!rd.raw(&k, &kn) || !rd.raw(&v, &vn)) return false;
    uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
    hk = fnv_byte(hk, '$');
    hk = fnv_bytes(hk, v, vn);
    for (int r = 0; r < n_srules; ++r) {
      const GpuRule rule = srules[r];
      if (slot >= slot_end) return false;
      if (key_matches(rule, blob, k, kn)) {
        const uint64_t h = fnv_bytes(hk, blob + rule.suffix_off, rule.suffix_len);
        out_idx[slot] = (int32_t)hash_to_index(h, H);
        out_val[slot] = rule.weight;
      } else {
        out_idx[slot] = -1;
        out_val[slot] = 0.f;
      }
      ++slot;
    }
  }
  // ---- num_values: [[key, number], ...]
  int64_t nn = rd.ok ? rd.array_len() : -1;
  for (int64_t i = 0; i < nn && rd.ok; ++i) {
    if (rd.array_len() != 2) return false;
    const uint8_t* k; int kn; double x;
    if (!rd.raw(&k, &kn) || !rd.number(&x)) return false;
    const uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
    for (int r = 0; r < n_nrules; ++r) {
      const GpuRule rule = nrules[r];
      if (slot >= slot_end) return false;
      if (key_matches(rule, blob, k, kn)) {
        const uint64_t h = fnv_bytes(hk, blob + rule.suffix_off, rule.suffix_len);
        out_idx[slot] = (int32_t)hash_to_index(h, H);
        out_val[slot] = (rule.value_kind == 1) ? logf(fmaxf(1.f, (float)x)) : (float)x;
      } else {
        out_idx[slot] = -1;
        out_val[slot] = 0.f;
      }
      ++slot;
    }
  }
  return rd.ok && slot == slot_end;
}

}  // namespace jb
