// GPU converter for the wide rule set (the device twin of
// csrc/native/jb_hostfv_wide.hpp): string rules with the str / space / ngram
// splitters and bin / tf / log_tf sample weights, idf / bm25 global weights
// (applied by ops/fv_wide.py against the document-frequency table in HBM),
// num / log num rules, and add / mul combinations over the finished base
// features. Feature order, names, indices and values equal the Python
// converter (fv_converter/converter.py `_convert`); slots a rule leaves
// unused are idx -1, as on the fixed-slot fast path (fv_hash.hip).
//
// Layout per datum i (row_ptr from fvw_count_kernel + a scan): a base
// region of B_i slots (upper bound: every token, every matching num rule)
// followed by ncomb x B_i (B_i - 1) / 2 combination slots (pair (a, b),
// a < b, of the base region, in the host's i < j order).
//   fvw_count_kernel   B_i and the total per datum
//   fvw_emit_kernel    base features (one lane per datum): per (string
//                      value, rule) the distinct tokens in first-occurrence
//                      order with their counts -> sample weight, name hash
//                      and name segments kept for the combination pass
//   (ops/fv_wide.py)   idf / bm25 on the slots whose rule has a global weight
//   fvw_comb_kernel    combination pairs (name matchers on the segments,
//                      FNV-1a continued from the left name's state)
#include "jb_fv.hpp"

namespace jb {

constexpr int kWideMaxBase = 4096;   // base slots per datum

struct SlotName {                    // name segments of a base slot
  int32_t key_off, key_len;          // in the datum buffer
  int32_t tok_off, tok_len;          // token (string features), -1 for num
  int32_t rule;                      // string rule r, or 1000 + num rule
};

__device__ __forceinline__ int wide_tokens(int kind, int ngram, const uint8_t* v, int vn) {
  if (kind == 0) return 1;
  if (kind == 2) {                    // space
    int c = 0, s = 0;
    for (int i = 0; i <= vn; ++i)
      if (i == vn || v[i] == ' ') { if (i > s) ++c; s = i + 1; }
    return c;
  }
  int ncp = 0;                        // ngram over code points
  for (int i = 0; i < vn; ++i) ncp += (v[i] & 0xC0) != 0x80;
  return ncp >= ngram ? ncp - ngram + 1 : 0;
}

// token t of a value: [off, off + len) within v
__device__ __forceinline__ void wide_token(int kind, int ngram, const uint8_t* v, int vn, int t,
                                           int* off, int* len) {
  if (kind == 0) { *off = 0; *len = vn; return; }
  if (kind == 2) {
    int c = 0, s = 0;
    for (int i = 0; i <= vn; ++i) {
      if (i == vn || v[i] == ' ') {
        if (i > s) {
          if (c == t) { *off = s; *len = i - s; return; }
          ++c;
        }
        s = i + 1;
      }
    }
    *off = 0; *len = 0;
    return;
  }
  int cp = 0, start = -1;
  for (int i = 0; i <= vn; ++i) {
    const bool boundary = i == vn || (v[i] & 0xC0) != 0x80;
    if (!boundary) continue;
    if (cp == t) start = i;
    if (cp == t + ngram) { *off = start; *len = i - start; return; }
    ++cp;
  }
  *off = 0; *len = 0;
}

__device__ __forceinline__ bool wide_count_datum(Reader& rd, const GpuRule* __restrict__ sr, int ns,
                                                 const GpuRule* __restrict__ nr, int nn,
                                                 const uint8_t* blob, int64_t* base) {
  int64_t top = rd.array_len();
  if (top < 2) return false;
  int64_t b = 0;
  const int64_t nsv = rd.array_len();
  for (int64_t i = 0; i < nsv && rd.ok; ++i) {
    if (rd.array_len() != 2) return false;
    const uint8_t *k, *v;
    int kn, vn;
    if (!rd.raw(&k, &kn) || !rd.raw(&v, &vn)) return false;
    for (int r = 0; r < ns; ++r)
      if (key_matches(sr[r], blob, k, kn))
        b += wide_tokens(sr[r].value_kind & 15, sr[r].pad, v, vn);
  }
  const int64_t nnv = rd.ok ? rd.array_len() : -1;
  for (int64_t i = 0; i < nnv && rd.ok; ++i) {
    if (rd.array_len() != 2) return false;
    const uint8_t* k;
    int kn;
    double x;
    if (!rd.raw(&k, &kn) || !rd.number(&x)) return false;
    for (int r = 0; r < nn; ++r) b += key_matches(nr[r], blob, k, kn);
  }
  *base = b;
  return rd.ok;
}

__global__ __launch_bounds__(256) void fvw_count_kernel(
    const uint8_t* __restrict__ buf, int64_t buf_len, const int64_t* __restrict__ datum_off,
    const int32_t* __restrict__ datum_len, int n, const GpuRule* __restrict__ sr, int ns,
    const GpuRule* __restrict__ nr, int nn, int ncomb, const uint8_t* __restrict__ blob,
    int64_t* __restrict__ base_cnt, int64_t* __restrict__ total_cnt, int32_t* __restrict__ err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t off = datum_off[i];
  const int64_t end = off + datum_len[i] < buf_len ? off + datum_len[i] : buf_len;
  Reader rd{buf + off, buf + end, true};
  int64_t b = 0;
  if (!wide_count_datum(rd, sr, ns, nr, nn, blob, &b) || b > kWideMaxBase) {
    atomicOr(err, 2);
    b = 0;
  }
  base_cnt[i] = b;
  total_cnt[i] = b + (int64_t)ncomb * (b * (b - 1) / 2);
}

__global__ __launch_bounds__(256) void fvw_emit_kernel(
    const uint8_t* __restrict__ buf, int64_t buf_len, const int64_t* __restrict__ datum_off,
    const int32_t* __restrict__ datum_len, int n, const int64_t* __restrict__ row_ptr,
    const GpuRule* __restrict__ sr, int ns, const GpuRule* __restrict__ nr, int nn,
    const uint8_t* __restrict__ blob, uint64_t H, int32_t* __restrict__ out_idx,
    float* __restrict__ out_val, uint64_t* __restrict__ out_h, SlotName* __restrict__ out_name,
    uint8_t* __restrict__ out_gw, int32_t* __restrict__ err) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t off = datum_off[i];
  const int64_t end = off + datum_len[i] < buf_len ? off + datum_len[i] : buf_len;
  Reader rd{buf + off, buf + end, true};
  int64_t slot = row_ptr[i];
  bool good = rd.array_len() >= 2;
  const int64_t nsv = good ? rd.array_len() : -1;
  for (int64_t a = 0; a < nsv && rd.ok; ++a) {
    if (rd.array_len() != 2) { good = false; break; }
    const uint8_t *k, *v;
    int kn, vn;
    if (!rd.raw(&k, &kn) || !rd.raw(&v, &vn)) { good = false; break; }
    uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
    hk = fnv_byte(hk, '$');
    for (int r = 0; r < ns; ++r) {
      const GpuRule rule = sr[r];
      if (!key_matches(rule, blob, k, kn)) continue;
      const int kind = rule.value_kind & 15, sw = rule.value_kind >> 4 & 15;
      const int gw = rule.value_kind >> 8 & 15;
      const int m = wide_tokens(kind, rule.pad, v, vn);
      const int64_t g0 = slot;
      for (int t = 0; t < m; ++t) {
        int to, tl;
        wide_token(kind, rule.pad, v, vn, t, &to, &tl);
        const uint64_t h = fnv_bytes(fnv_bytes(hk, v + to, tl), blob + rule.suffix_off,
                                     rule.suffix_len);
        // a repeated token counts toward its first occurrence (tf)
        int64_t first = -1;
        for (int64_t s = g0; s < slot; ++s) {
          if (out_idx[s] >= 0 && out_h[s] == h) { first = s; break; }
        }
        if (first >= 0) {
          out_val[first] += 1.f;
          out_idx[slot] = -1;
          out_val[slot] = 0.f;
          out_gw[slot] = 0;
        } else {
          out_idx[slot] = (int32_t)hash_to_index(h, H);
          out_val[slot] = 1.f;                       // occurrences; weighted below
          out_h[slot] = h;
          out_gw[slot] = (uint8_t)gw;
          out_name[slot] = SlotName{(int32_t)(k - buf), kn, (int32_t)(v + to - buf), tl, r};
        }
        ++slot;
      }
      for (int64_t s = g0; s < slot; ++s) {          // counts -> sample weight
        if (out_idx[s] < 0) continue;
        const float c = out_val[s];
        out_val[s] = sw == 0 ? 1.f : sw == 1 ? c : (float)log(1.0 + (double)c);
      }
    }
  }
  const int64_t nnv = (good && rd.ok) ? rd.array_len() : -1;
  for (int64_t a = 0; a < nnv && rd.ok; ++a) {
    if (rd.array_len() != 2) { good = false; break; }
    const uint8_t* k;
    int kn;
    double x;
    if (!rd.raw(&k, &kn) || !rd.number(&x)) { good = false; break; }
    const uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
    for (int r = 0; r < nn; ++r) {
      const GpuRule rule = nr[r];
      if (!key_matches(rule, blob, k, kn)) continue;
      const uint64_t h = fnv_bytes(hk, blob + rule.suffix_off, rule.suffix_len);
      out_idx[slot] = (int32_t)hash_to_index(h, H);
      out_val[slot] = (float)(rule.value_kind == 1 ? log(x > 1.0 ? x : 1.0) : x);
      out_h[slot] = h;
      out_gw[slot] = 0;
      out_name[slot] = SlotName{(int32_t)(k - buf), kn, -1, 0, 1000 + r};
      ++slot;
    }
  }
  if (!good || !rd.ok) atomicOr(err, 2);
}

// byte `pos` of a base slot's name: key | '$' token | suffix
__device__ __forceinline__ uint8_t name_byte(const SlotName& nm, const uint8_t* buf,
                                             const uint8_t* blob, const GpuRule* sr,
                                             const GpuRule* nr, int pos) {
  if (pos < nm.key_len) return buf[nm.key_off + pos];
  pos -= nm.key_len;
  if (nm.tok_off >= 0) {
    if (pos == 0) return '$';
    pos -= 1;
    if (pos < nm.tok_len) return buf[nm.tok_off + pos];
    pos -= nm.tok_len;
  }
  const GpuRule& r = nm.rule >= 1000 ? nr[nm.rule - 1000] : sr[nm.rule];
  return blob[r.suffix_off + pos];
}

__device__ __forceinline__ int name_len(const SlotName& nm, const GpuRule* sr, const GpuRule* nr) {
  const GpuRule& r = nm.rule >= 1000 ? nr[nm.rule - 1000] : sr[nm.rule];
  return nm.key_len + (nm.tok_off >= 0 ? 1 + nm.tok_len : 0) + r.suffix_len;
}

__device__ bool name_matches(const GpuRule& m, const uint8_t* blob, const SlotName& nm,
                             const uint8_t* buf, const GpuRule* sr, const GpuRule* nr) {
  if (m.match_kind == 0) return true;
  const int L = name_len(nm, sr, nr), mn = m.match_len;
  if (m.match_kind == 3 && L != mn) return false;
  if (L < mn) return false;
  const int base = m.match_kind == 2 ? L - mn : 0;
  for (int i = 0; i < mn; ++i)
    if (name_byte(nm, buf, blob, sr, nr, base + i) != blob[m.match_off + i]) return false;
  return true;
}

__global__ __launch_bounds__(256) void fvw_comb_kernel(
    const uint8_t* __restrict__ buf, int n, const int64_t* __restrict__ row_ptr,
    const int64_t* __restrict__ base_cnt, const GpuRule* __restrict__ sr,
    const GpuRule* __restrict__ nr, const GpuRule* __restrict__ cr, int ncomb,
    const uint8_t* __restrict__ blob, uint64_t H, int32_t* __restrict__ idx,
    float* __restrict__ val, const uint64_t* __restrict__ hs, const SlotName* __restrict__ names) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t b0 = row_ptr[i];
  const int64_t B = base_cnt[i];
  int64_t out = b0 + B;
  for (int c = 0; c < ncomb; ++c) {
    const GpuRule L = cr[2 * c], R = cr[2 * c + 1];
    for (int64_t a = 0; a < B; ++a) {
      const bool la = idx[b0 + a] >= 0 && name_matches(L, blob, names[b0 + a], buf, sr, nr);
      const uint64_t ha = fnv_byte(hs[b0 + a], '&');
      for (int64_t b = a + 1; b < B; ++b, ++out) {
        idx[out] = -1;
        val[out] = 0.f;
        if (!la || idx[b0 + b] < 0) continue;
        const SlotName nb = names[b0 + b];
        if (!name_matches(R, blob, nb, buf, sr, nr)) continue;
        uint64_t h = ha;
        const int ln = name_len(nb, sr, nr);
        for (int p = 0; p < ln; ++p) h = fnv_byte(h, name_byte(nb, buf, blob, sr, nr, p));
        h = fnv_bytes(h, blob + L.suffix_off, L.suffix_len);
        idx[out] = (int32_t)hash_to_index(h, H);
        const float x = val[b0 + a], y = val[b0 + b];
        val[out] = L.value_kind == 1 ? x * y : x + y;
      }
    }
  }
}

}  // namespace jb

extern "C" int jb_fvw_count(const uint8_t* buf, int64_t buf_len, const int64_t* datum_off,
                            const int32_t* datum_len, int n, const void* sr, int ns, const void* nr,
                            int nn, int ncomb, const uint8_t* blob, int64_t* base_cnt,
                            int64_t* total_cnt, int32_t* err, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(jb::fvw_count_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, buf,
                     buf_len, datum_off, datum_len, n, (const jb::GpuRule*)sr, ns,
                     (const jb::GpuRule*)nr, nn, ncomb, blob, base_cnt, total_cnt, err);
  return (int)hipGetLastError();
}

extern "C" int jb_fvw_emit(const uint8_t* buf, int64_t buf_len, const int64_t* datum_off,
                           const int32_t* datum_len, int n, const int64_t* row_ptr, const void* sr,
                           int ns, const void* nr, int nn, const uint8_t* blob, uint64_t H,
                           int32_t* out_idx, float* out_val, uint64_t* out_h, void* out_name,
                           uint8_t* out_gw, int32_t* err, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(jb::fvw_emit_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, buf,
                     buf_len, datum_off, datum_len, n, row_ptr, (const jb::GpuRule*)sr, ns,
                     (const jb::GpuRule*)nr, nn, blob, H, out_idx, out_val, out_h,
                     (jb::SlotName*)out_name, out_gw, err);
  return (int)hipGetLastError();
}

extern "C" int jb_fvw_comb(const uint8_t* buf, int n, const int64_t* row_ptr,
                           const int64_t* base_cnt, const void* sr, const void* nr, const void* cr,
                           int ncomb, const uint8_t* blob, uint64_t H, int32_t* idx, float* val,
                           const uint64_t* hs, const void* names, hipStream_t stream) {
  if (n <= 0 || ncomb <= 0) return 0;
  hipLaunchKernelGGL(jb::fvw_comb_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, buf, n,
                     row_ptr, base_cnt, (const jb::GpuRule*)sr, (const jb::GpuRule*)nr,
                     (const jb::GpuRule*)cr, ncomb, blob, H, idx, val, hs,
                     (const jb::SlotName*)names);
  return (int)hipGetLastError();
}

extern "C" int64_t jb_fvw_name_bytes() { return (int64_t)sizeof(jb::SlotName); }
