// GPU fv_converter fast path: msgpack datum bytes -> hashed sparse feature rows.
//
// Reference behaviour: jubatus_core's datum_to_fv_converter (EXTERNAL, not in
// the tree; called at jubatus/server/server/classifier_serv.cpp:111 and
// jubatus/server/cmd/jubaconv.cpp:91-96). The feature-name scheme is
// documented in jubatus_amd/fv_converter/converter.py and is byte-identical to
// the host converter (csrc/native/jb_converter.cpp):
//     string rule  : "<key>$<value>@<type>#<sample_weight>/<global_weight>"
//     num rule     : "<key>@num"  (value)   |  "<key>@log" (log(max(1,value)))
// The feature index is hash_to_index(FNV1a64(name), hash_max_size).
//
// Design (MI355X): the raw request bytes (as received by the RPC layer) are
// copied to HBM once; one lane walks one datum and emits its feature slots.
// The host has already validated the structure and computed the exact number
// of slots per datum (row_ptr), so every lane writes a disjoint CSR segment
// and no atomics/compaction are needed. Slots whose key does not match a
// rule's key matcher are emitted as idx=-1 (skipped by every consumer).
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

__global__ __launch_bounds__(256) void fv_hash_kernel(
    const uint8_t* __restrict__ buf, int64_t buf_len,
    const int64_t* __restrict__ datum_off, const int64_t* __restrict__ row_ptr, int n,
    const GpuRule* __restrict__ srules, int n_srules,
    const GpuRule* __restrict__ nrules, int n_nrules,
    const uint8_t* __restrict__ blob, uint64_t H,
    int32_t* __restrict__ out_idx, float* __restrict__ out_val, int32_t* __restrict__ err) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n) return;
  Reader rd{buf + datum_off[s], buf + buf_len, true};
  int64_t slot = row_ptr[s];
  const int64_t slot_end = row_ptr[s + 1];

  int64_t top = rd.array_len();
  if (top < 2) { atomicOr(err, 1); return; }
  // ---- string_values: [[key, value], ...]
  int64_t ns = rd.array_len();
  for (int64_t i = 0; i < ns && rd.ok; ++i) {
    if (rd.array_len() != 2) { rd.ok = false; break; }
    const uint8_t *k, *v; int kn, vn;
    if (!rd.raw(&k, &kn) || !rd.raw(&v, &vn)) break;
    uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
    hk = fnv_byte(hk, '$');
    hk = fnv_bytes(hk, v, vn);
    for (int r = 0; r < n_srules; ++r) {
      const GpuRule rule = srules[r];
      if (slot >= slot_end) { rd.ok = false; break; }
      if (key_matches(rule, blob, k, kn)) {
        uint64_t h = fnv_bytes(hk, blob + rule.suffix_off, rule.suffix_len);
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
    if (rd.array_len() != 2) { rd.ok = false; break; }
    const uint8_t* k; int kn; double x;
    if (!rd.raw(&k, &kn) || !rd.number(&x)) break;
    uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
    for (int r = 0; r < n_nrules; ++r) {
      const GpuRule rule = nrules[r];
      if (slot >= slot_end) { rd.ok = false; break; }
      if (key_matches(rule, blob, k, kn)) {
        uint64_t h = fnv_bytes(hk, blob + rule.suffix_off, rule.suffix_len);
        float val = (rule.value_kind == 1) ? logf(fmaxf(1.f, (float)x)) : (float)x;
        out_idx[slot] = (int32_t)hash_to_index(h, H);
        out_val[slot] = val;
      } else {
        out_idx[slot] = -1;
        out_val[slot] = 0.f;
      }
      ++slot;
    }
  }
  if (!rd.ok || slot != slot_end) atomicOr(err, 2);
}

}  // namespace jb

extern "C" int jb_fv_hash(const uint8_t* buf, int64_t buf_len, const int64_t* datum_off,
                          const int64_t* row_ptr, int n, const void* srules, int n_srules,
                          const void* nrules, int n_nrules, const uint8_t* blob, uint64_t H,
                          int32_t* out_idx, float* out_val, int32_t* err, hipStream_t stream) {
  if (n <= 0) return 0;
  const int threads = 256;
  const int blocks = (n + threads - 1) / threads;
  hipLaunchKernelGGL(jb::fv_hash_kernel, dim3(blocks), dim3(threads), 0, stream, buf, buf_len,
                     datum_off, row_ptr, n, (const jb::GpuRule*)srules, n_srules,
                     (const jb::GpuRule*)nrules, n_nrules, blob, H, out_idx, out_val, err);
  return (int)hipGetLastError();
}
