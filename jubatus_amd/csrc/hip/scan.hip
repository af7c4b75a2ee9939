// GPU request scanner for train batches: the device twin of the host scanner
// (csrc/native/jb_pack.{hpp,cpp}, pack_requests kind 1) for bodies that are
// already in HBM.
//
// Reference behaviour: the train RPC decodes list<labeled_datum>
// (jubatus/server/server/classifier_serv.cpp:129-145; labels are added on
// first use). The host scanner walks every request on the CPU before the
// H2D copy; at 196 B/sample that walk is a chain of dependent byte loads and
// bounds the headline step (profiles/r01_train_step_breakdown.jsonl). Here
// the raw arena goes to HBM first and the walk runs on the GPU - in parallel,
// because a single GPU lane walking a request is slower than a CPU core:
//
//   scan_train_kernel, one 256-thread workgroup per request, request bytes
//   staged in LDS:
//   1. speculative chunk walks: the request is cut into 256 chunks; thread t
//      walks msgpack tokens from the start of chunk t as if a token began
//      there, marking the token starts it visits (LDS bitmap).
//   2. convergence: thread t continues from where its walk left chunk t
//      until it lands on a start marked by a later chunk's walk. msgpack
//      re-synchronises within a few tokens (ASCII bytes decode as 1-byte
//      fixints), so these extensions are short.
//   3. the true walk is the chain chunk 0 -> its convergence chunk -> ...;
//      walks off that chain are discarded, the chain's extensions are marked
//      again: the bitmap now holds exactly the real token starts.
//   4. depth scan: with d = (container arity - 1) per token, the samples
//      (children of the top-level array) start where the running sum of d
//      reaches a new minimum; chunk sums / minima are combined across threads.
//   5. one thread per sample: label lookup (open addressing on FNV-1a 64 of
//      the label bytes), datum validation and string / number pair counts
//      (same rules as the host), descriptor outputs; an in-request scan of
//      the slot counts gives row_ptr relative to the request.
//   scan_fixup_kernel: adds each request's slot base to its row_ptr entries.
//
// Anything the device path does not take (a label not in the table, binary
// values, extra datum elements, malformed bytes, a request larger than the
// LDS stage or with more than kMaxSamples samples, a walk that does not
// re-synchronise) sets a bit in *err and the fixup kernel turns every sample
// of the batch into a no-op (label -1, empty datum): the caller re-runs the
// batch through the host scanner, which adds labels and reports malformed
// requests exactly as before.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jb_device.hpp"

namespace jb {
namespace {

constexpr int kThreads = 256;                 // chunks per request
constexpr int kScanBytes = 27 * 1024;         // request bytes staged in LDS
constexpr int kBitWords = kScanBytes / 32;    // token-start bitmap
constexpr int kMaxSamples = 768;              // samples per request (their slot counts overlay the bitmap)
constexpr int kLabCap = 32;                   // label-table entries staged in LDS
constexpr int kLabBlob = 512;
constexpr int kHist = 64;                     // labels counted in LDS per request
constexpr int kExtMax = 512;                  // tokens a convergence walk may take
static_assert(kMaxSamples * 4 <= kBitWords * 4, "slot overlay");

enum : int { kErrMalformed = 1, kErrLabel = 2, kErrTooBig = 4 };

// byte at p of a request staged at q (bytes past len read as 0)
__device__ __forceinline__ uint32_t byte_at(const uint8_t* q, int p, int len) {
  return p < len ? q[p] : 0u;
}

// Header byte(s) read without the len check: q points into the LDS stage,
// whose bytes past the request are stale but in bounds (`lim` = readable
// positions from q). A token decoded from them runs past len, which ends
// the walk; positions >= len are never marked.
__device__ __forceinline__ uint32_t byte_fast(const uint8_t* q, int p, int lim) {
  return q[min(p, lim - 1)];
}

// (arity - 1) of the token at p, the only quantity the depth scan needs:
// containers give their element count - 1, everything else -1
__device__ __forceinline__ int token_d(const uint8_t* q, int p, int lim) {
  const uint32_t t = byte_fast(q, p, lim);
  if ((t & 0xe0) == 0x80) return (t <= 0x8f ? 2 * (int)(t & 0x0f) : (int)(t & 0x0f)) - 1;
  if (t < 0xdc || t > 0xdf) return -1;
  const uint32_t b1 = byte_fast(q, p + 1, lim), b2 = byte_fast(q, p + 2, lim);
  if (t == 0xdc) return (int)((b1 << 8) | b2) - 1;
  if (t == 0xde) return 2 * (int)((b1 << 8) | b2) - 1;
  uint32_t n = (b1 << 24) | (b2 << 16) | (byte_fast(q, p + 3, lim) << 8) | byte_fast(q, p + 4, lim);
  if (n > 0x3fffffffu) n = 0x3fffffffu;
  return (t == 0xdd ? (int)n : 2 * (int)n) - 1;
}

// size of the token at p (containers: header only), unchecked reads
__device__ __forceinline__ int token_size(const uint8_t* q, int p, int lim) {
  const uint32_t t = byte_fast(q, p, lim);
  if (t <= 0x9f || t >= 0xe0) return 1;              // fixint, fixmap, fixarray, negative fixint
  if (t <= 0xbf) return 1 + (int)(t & 0x1f);          // fixraw
  const uint32_t b1 = byte_fast(q, p + 1, lim);
  switch (t) {
    case 0xc4: case 0xd9: case 0xc7: return (t == 0xc7 ? 3 : 2) + (int)b1;
    case 0xc5: case 0xda: case 0xc8:
      return (t == 0xc8 ? 4 : 3) + (int)((b1 << 8) | byte_fast(q, p + 2, lim));
    case 0xc6: case 0xdb: case 0xc9: {
      uint32_t n = (b1 << 24) | (byte_fast(q, p + 2, lim) << 16) |
                   (byte_fast(q, p + 3, lim) << 8) | byte_fast(q, p + 4, lim);
      if (n > 0x3fffffffu) n = 0x3fffffffu;
      return (t == 0xc9 ? 6 : 5) + (int)n;
    }
    case 0xca: case 0xce: case 0xd2: case 0xdd: case 0xdf: return 5;
    case 0xcb: case 0xcf: case 0xd3: return 9;
    case 0xcc: case 0xd0: case 0xd4: return t == 0xd4 ? 3 : 2;
    case 0xcd: case 0xd1: case 0xdc: case 0xde: return 3;
    case 0xd5: return 4;
    case 0xd6: return 6;
    case 0xd7: return 10;
    case 0xd8: return 18;
    default: return 1;                                  // nil, false, true, 0xc1
  }
}

// size of the token at p if one starts there (containers: header only) and
// its element count (arrays / maps; 0 otherwise)
__device__ __forceinline__ int token(const uint8_t* q, int p, int len, int* arity) {
  const uint32_t t = byte_at(q, p, len);
  *arity = 0;
  if (t <= 0x7f || t >= 0xe0 || t == 0xc0 || t == 0xc2 || t == 0xc3 || t == 0xc1) return 1;
  if (t <= 0x8f) { *arity = 2 * (int)(t & 0x0f); return 1; }
  if (t <= 0x9f) { *arity = (int)(t & 0x0f); return 1; }
  if (t <= 0xbf) return 1 + (int)(t & 0x1f);
  const uint32_t b1 = byte_at(q, p + 1, len), b2 = byte_at(q, p + 2, len);
  const uint32_t be16 = (b1 << 8) | b2;
  const uint32_t be32 = (b1 << 24) | (b2 << 16) | (byte_at(q, p + 3, len) << 8) | byte_at(q, p + 4, len);
  const int big = be32 > 0x3fffffffu ? 0x3fffffff : (int)be32;   // clamp: walks past len stop anyway
  switch (t) {
    case 0xc4: case 0xd9: return 2 + (int)b1;
    case 0xc5: case 0xda: return 3 + (int)be16;
    case 0xc6: case 0xdb: return 5 + big;
    case 0xc7: return 3 + (int)b1;
    case 0xc8: return 4 + (int)be16;
    case 0xc9: return 6 + big;
    case 0xca: return 5;
    case 0xcb: return 9;
    case 0xcc: case 0xd0: return 2;
    case 0xcd: case 0xd1: return 3;
    case 0xce: case 0xd2: return 5;
    case 0xcf: case 0xd3: return 9;
    case 0xd4: return 3;
    case 0xd5: return 4;
    case 0xd6: return 6;
    case 0xd7: return 10;
    case 0xd8: return 18;
    case 0xdc: *arity = (int)be16; return 3;
    case 0xdd: *arity = big; return 5;
    case 0xde: *arity = 2 * (int)be16; return 3;
    default: *arity = 2 * big; return 5;   // 0xdf
  }
}

__device__ __forceinline__ bool bit(const uint32_t* bits, int p) {
  return (bits[p >> 5] >> (p & 31)) & 1u;
}

// bits of word w that fall in [b, e)
__device__ __forceinline__ uint32_t range_mask(int w, int b, int e) {
  const int lo = max(b - 32 * w, 0), hi = min(e - 32 * w, 32);
  if (hi <= lo) return 0u;
  const uint32_t upto = hi == 32 ? 0xffffffffu : ((1u << hi) - 1u);
  return upto & ~((1u << lo) - 1u);
}

// exclusive prefix sum / min over the 256 threads (tmp: 4 ints of LDS)
__device__ __forceinline__ int block_excl_sum(int v, int* tmp, int* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) tmp[w] = x;
  __syncthreads();
  int base = 0;
  for (int i = 0; i < w; ++i) base += tmp[i];
  *total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
  __syncthreads();
  return base + x - v;
}
__device__ __forceinline__ int block_excl_min(int v, int* tmp) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x = min(x, y);
  }
  if (lane == 63) tmp[w] = x;
  const int prev = __shfl_up(x, 1, 64);
  __syncthreads();
  int base = 0x7fffffff;
  for (int i = 0; i < w; ++i) base = min(base, tmp[i]);
  __syncthreads();
  return lane == 0 ? base : min(base, prev);
}

// label bytes -> column id, -1 if absent (meta = [blob offset, length, id])
__device__ __forceinline__ int label_lookup(const uint8_t* s, int n, const uint64_t* th,
                                            const int32_t* tm, int cap, const uint8_t* blob) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (int i = 0; i < n; ++i) {
    h ^= s[i];
    h *= 0x100000001b3ull;
  }
  const int mask = cap - 1;
  for (int i = (int)(h & (uint64_t)mask), probes = 0; probes < cap; i = (i + 1) & mask, ++probes) {
    const int id = tm[3 * i + 2];
    if (id < 0) return -1;
    if (th[i] != h || tm[3 * i + 1] != n) continue;
    const uint8_t* k = blob + tm[3 * i];
    bool eq = true;
    for (int j = 0; j < n && eq; ++j) eq = k[j] == s[j];
    if (eq) return id;
  }
  return -1;
}

// Validate one sample [label, datum] spanning exactly [p, e) and count its
// pairs (the host scanner's rules, jb_pack.hpp scan_datum).
__device__ __forceinline__ int sample_walk(const uint8_t* q, int p, int e, const uint64_t* th,
                                           const int32_t* tm, int cap, const uint8_t* blob,
                                           int* id, int* doff, int* ns_out, int* nn_out) {
  Reader c{q + p, q + e, true};
  if (c.array_len() != 2) return kErrMalformed;
  const uint8_t* ls;
  int ln;
  if (!c.raw(&ls, &ln)) return kErrMalformed;
  *id = label_lookup(ls, ln, th, tm, cap, blob);
  if (*id < 0) return kErrLabel;
  *doff = (int)(c.p - q);
  const int64_t top = c.array_len();
  if (top < 2 || top > 3) return kErrMalformed;   // extra elements: host path
  const int64_t ns = c.array_len();
  if (ns < 0) return kErrMalformed;
  for (int64_t j = 0; j < ns; ++j) {
    const uint8_t* k;
    int kn;
    if (c.array_len() != 2 || !c.raw(&k, &kn) || !c.raw(&k, &kn)) return kErrMalformed;
  }
  const int64_t nn = c.array_len();
  if (nn < 0) return kErrMalformed;
  for (int64_t j = 0; j < nn; ++j) {
    const uint8_t* k;
    int kn;
    double x;
    if (c.array_len() != 2 || !c.raw(&k, &kn) || !c.number(&x)) return kErrMalformed;
  }
  if (top == 3 && c.array_len() != 0) return kErrMalformed;   // binary values: host path
  if (!c.ok || c.p != q + e) return kErrMalformed;
  *ns_out = (int)ns;
  *nn_out = (int)nn;
  return 0;
}

__global__ __launch_bounds__(kThreads) void scan_train_kernel(
    const uint8_t* __restrict__ buf, const int64_t* __restrict__ req_off,
    const int64_t* __restrict__ req_len, const int64_t* __restrict__ sample_base, int R,
    const uint64_t* __restrict__ lt_hash, const int32_t* __restrict__ lt_meta, int lt_cap,
    const uint8_t* __restrict__ lt_blob, int lt_blob_len, int sps, int spn,
    int64_t* __restrict__ datum_off, int32_t* __restrict__ datum_len,
    int32_t* __restrict__ labels, int64_t* __restrict__ row_ptr,
    int64_t* __restrict__ req_slots, uint32_t* __restrict__ hist, int nhist,
    int32_t* __restrict__ err, long long* __restrict__ prof) {
  __shared__ __attribute__((aligned(16))) uint8_t s_req[kScanBytes];
  __shared__ uint32_t s_bits[kBitWords];      // token starts; later the per-sample slot counts
  __shared__ uint16_t s_exit[kThreads];       // where chunk t's walk left the chunk
  __shared__ uint16_t s_conv[kThreads];       // where chunk t's extension met a later walk
  __shared__ uint16_t s_tc[kThreads];         // ... in that chunk (kThreads: reached the end)
  __shared__ uint16_t s_from[kThreads];       // chunk t on the true chain: its entry point
  __shared__ uint8_t s_valid[kThreads];
  __shared__ int32_t s_jump[kThreads];        // chain pointer doubling
  __shared__ int32_t s_red[4];                // block scans
  __shared__ uint16_t s_start[kMaxSamples + 1];
  __shared__ uint64_t s_th[kLabCap];
  __shared__ int32_t s_tm[3 * kLabCap];
  __shared__ uint8_t s_blob[kLabBlob];
  __shared__ uint32_t s_hist[kHist];
  __shared__ int32_t s_err;

  const int k = blockIdx.x;
  const int t = threadIdx.x;
  if (k >= R) return;
  if (prof && t == 0) prof[8 * k + 6] = (long long)__builtin_amdgcn_s_memtime();
  const int64_t off = req_off[k];
  const int64_t len64 = req_len[k];
  const int64_t s0 = sample_base[k], nsamples = sample_base[k + 1] - s0;
  const int64_t a0 = off & ~(int64_t)15;
  const int rel = (int)(off - a0);
  if (len64 + rel > kScanBytes || nsamples > kMaxSamples) {   // host path
    if (t == 0) {
      req_slots[k] = 0;
      atomicOr(err, kErrTooBig);
    }
    return;
  }
  const int len = (int)len64;
  const uint8_t* q = s_req + rel;             // the request, position 0 = its first byte

  // ---- stage the request, the label table; clear the bitmap / histogram
  {
    const int nvec = (rel + len + 15) >> 4;
    const uint4* src = reinterpret_cast<const uint4*>(buf + a0);
    uint4* dst = reinterpret_cast<uint4*>(s_req);
    for (int i = t; i < nvec; i += kThreads) dst[i] = src[i];
  }
  const bool lab_lds = lt_cap <= kLabCap && lt_blob_len <= kLabBlob;
  if (lab_lds) {
    for (int i = t; i < lt_cap; i += kThreads) {
      s_th[i] = lt_hash[i];
      s_tm[3 * i] = lt_meta[3 * i];
      s_tm[3 * i + 1] = lt_meta[3 * i + 1];
      s_tm[3 * i + 2] = lt_meta[3 * i + 2];
    }
    for (int i = t; i < lt_blob_len; i += kThreads) s_blob[i] = lt_blob[i];
  }
  for (int i = t; i < kBitWords; i += kThreads) s_bits[i] = 0u;
  for (int i = t; i < kHist; i += kThreads) s_hist[i] = 0u;
  if (t == 0) s_err = 0;
  __syncthreads();

  if (prof && t == 0) prof[8 * k + 0] = (long long)__builtin_amdgcn_s_memtime();
  // ---- 1. speculative walk of chunk t (bits gathered per word, one LDS
  // atomic per 32 positions)
  const int C = (len + kThreads - 1) / kThreads;
  const int cb = min(t * C, len), ce = min(cb + C, len);
  const int lim = kScanBytes - rel;
  {
    int p = cb, word = cb >> 5;
    uint32_t acc = 0;
    while (p < ce) {
      if ((p >> 5) != word) {
        if (acc) atomicOr(&s_bits[word], acc);
        word = p >> 5;
        acc = 0;
      }
      acc |= 1u << (p & 31);
      p += token_size(q, p, lim);
    }
    if (acc) atomicOr(&s_bits[word], acc);
    s_exit[t] = (uint16_t)min(p, len);
  }
  __syncthreads();

  if (prof && t == 0) prof[8 * k + 1] = (long long)__builtin_amdgcn_s_memtime();
  // ---- 2. extension of chunk t's walk until it meets a later chunk's walk
  {
    int p = s_exit[t], steps = 0;   // p >= the end of chunk t: any marked p is a later chunk's
    int tc = kThreads;
    while (p < len) {
      if (bit(s_bits, p)) { tc = p / C; break; }
      p += token_size(q, p, lim);
      if (++steps > kExtMax) { tc = -1; break; }
    }
    s_tc[t] = (uint16_t)(tc < 0 ? 0xffff : tc);
    s_conv[t] = (uint16_t)min(p, len);
  }
  __syncthreads();

  if (prof && t == 0) prof[8 * k + 2] = (long long)__builtin_amdgcn_s_memtime();
  // ---- 3. the true chain: chunk 0 -> its convergence chunk -> ... (reach
  // from chunk 0 by pointer doubling, 8 rounds for 256 chunks)
  {
    const int tc = s_tc[t];
    s_jump[t] = tc == 0xffff ? kThreads + 1 : tc;
    s_valid[t] = t == 0;
    __syncthreads();
#pragma unroll 1
    for (int r = 0; r < 8; ++r) {
      const int j = s_jump[t];
      const bool rc = s_valid[t];
      const int jj = j < kThreads ? s_jump[j] : j;
      __syncthreads();
      if (rc && j < kThreads) s_valid[j] = 1;
      s_jump[t] = jj;
      __syncthreads();
    }
    if (s_valid[t]) {
      if (tc == 0xffff) atomicOr(&s_err, kErrMalformed);   // a walk that did not re-synchronise
      else if (tc < kThreads) s_from[tc] = s_conv[t];
    }
    if (t == 0) s_from[0] = 0;
  }
  __syncthreads();
  if (s_err) {
    if (t == 0) { req_slots[k] = 0; atomicOr(err, s_err); }
    return;
  }
  // drop the walks off the chain (and the false prefix of chain chunks) ...
  {
    const int drop_end = s_valid[t] ? min((int)s_from[t], ce) : ce;
    if (cb < drop_end)
      for (int w = cb >> 5; w <= (drop_end - 1) >> 5; ++w)
        atomicAnd(&s_bits[w], ~range_mask(w, cb, drop_end));
  }
  __syncthreads();
  // ... and mark the chain's extensions
  if (s_valid[t]) {
    int p = s_exit[t];
    const int stop = s_conv[t];
    while (p < stop) {
      atomicOr(&s_bits[p >> 5], 1u << (p & 31));
      p += token_size(q, p, lim);
    }
  }
  __syncthreads();

  if (prof && t == 0) prof[8 * k + 3] = (long long)__builtin_amdgcn_s_memtime();
  // ---- 4. depth scan: samples start where sum(arity - 1) hits a new minimum
  int lsum = 0, lmin = 0x7fffffff;
  if (cb < ce)
    for (int w = cb >> 5; w <= (ce - 1) >> 5; ++w) {
      uint32_t m = s_bits[w] & range_mask(w, max(cb, 1), ce);
      while (m) {
        const int p = 32 * w + __builtin_ctz(m);
        m &= m - 1;
        lmin = min(lmin, lsum);
        lsum += token_d(q, p, lim);
      }
    }
  int total;
  const int pre = block_excl_sum(lsum, s_red, &total);
  const int seen = block_excl_min(lmin == 0x7fffffff ? 0x7fffffff : pre + lmin, s_red);
  if (t == 0) {
    // root: an array of nsamples elements at position 0
    int a0n;
    const uint32_t b0 = byte_at(q, 0, len);
    token(q, 0, len, &a0n);
    const bool root_ok = len > 0 && ((b0 & 0xf0) == 0x90 || b0 == 0xdc || b0 == 0xdd) &&
                         a0n == nsamples;
    if (!root_ok || total != -(int)nsamples) atomicOr(&s_err, kErrMalformed);
    s_start[nsamples] = (uint16_t)len;
  }
  {
    int h = pre, mn = min(1, seen);   // H before this chunk; minimum of H seen so far
    if (cb < ce)
      for (int w = cb >> 5; w <= (ce - 1) >> 5; ++w) {
        uint32_t m = s_bits[w] & range_mask(w, max(cb, 1), ce);
        while (m) {
          const int p = 32 * w + __builtin_ctz(m);
          m &= m - 1;
          if (h < mn) {               // a new minimum: sample -h starts here
            if (-h < nsamples) s_start[-h] = (uint16_t)p;
            else atomicOr(&s_err, kErrMalformed);
            mn = h;
          }
          h += token_d(q, p, lim);
        }
      }
  }
  __syncthreads();
  if (s_err) {
    if (t == 0) { req_slots[k] = 0; atomicOr(err, s_err); }
    return;
  }

  if (prof && t == 0) prof[8 * k + 4] = (long long)__builtin_amdgcn_s_memtime();
  // ---- 5. one thread per sample
  uint32_t* s_slots = s_bits;                 // the bitmap is no longer needed
  int my_err = 0;
  for (int m = t; m < nsamples; m += kThreads) {
    int id = -1, doff = 0, ns = 0, nn = 0;
    // two call sites so each inlined copy keeps its table's address space
    // (LDS loads for the staged table instead of flat loads)
    const int e = lab_lds
        ? sample_walk(q, s_start[m], s_start[m + 1], s_th, s_tm, lt_cap, s_blob, &id, &doff, &ns, &nn)
        : sample_walk(q, s_start[m], s_start[m + 1], lt_hash, lt_meta, lt_cap, lt_blob, &id, &doff,
                      &ns, &nn);
    if (e) { my_err |= e; s_slots[m] = 0; continue; }
    const int64_t s = s0 + m;
    labels[s] = id;
    datum_off[s] = off + doff;
    datum_len[s] = s_start[m + 1] - doff;
    s_slots[m] = (uint32_t)(ns * sps + nn * spn);
    if (id < kHist) atomicAdd(&s_hist[id], 1u);
    else if (id < nhist) atomicAdd(&hist[id], 1u);
  }
  if (my_err) atomicOr(&s_err, my_err);
  __syncthreads();
  {   // row_ptr relative to the request: exclusive scan of the slot counts
    const int per = (kMaxSamples + kThreads - 1) / kThreads;
    const int m0 = t * per;
    int mine = 0;
    for (int m = m0; m < min(m0 + per, (int)nsamples); ++m) mine += (int)s_slots[m];
    int total_slots;
    int acc = block_excl_sum(mine, s_red, &total_slots);
    for (int m = m0; m < min(m0 + per, (int)nsamples); ++m) {
      row_ptr[s0 + m] = acc;
      acc += (int)s_slots[m];
    }
    if (t == 0) {
      req_slots[k] = total_slots;
      if (s_err) atomicOr(err, s_err);
    }
  }
  if (prof && t == 0) prof[8 * k + 5] = (long long)__builtin_amdgcn_s_memtime();
  if (s_err) return;
  const int top = nhist < kHist ? nhist : kHist;
  for (int i = t; i < top; i += kThreads)
    if (s_hist[i]) atomicAdd(&hist[i], s_hist[i]);
  if (prof && t == 0) prof[8 * k + 7] = (long long)__builtin_amdgcn_s_memtime();
}

__global__ __launch_bounds__(64) void scan_fixup_kernel(
    const int64_t* __restrict__ sample_base, int R, const int64_t* __restrict__ req_slots,
    int64_t* __restrict__ row_ptr, int64_t* __restrict__ datum_off,
    int32_t* __restrict__ datum_len, int32_t* __restrict__ labels, uint8_t* __restrict__ empty_at,
    int64_t empty_off, const int32_t* __restrict__ err, const uint32_t* __restrict__ hist, int nhist,
    int32_t* __restrict__ host_out) {
  const int k = blockIdx.x;
  const int lane = threadIdx.x;
  if (k >= R) return;
  if (k == 0) {   // the batch's check, straight into coherent host memory
    // system-scope stores (past the L2), the error word after the counts
    // are acknowledged; the host reads the record after the batch's event.
    // (A system-scope fence here wrote back the whole L2 every batch.)
    for (int i = lane; i < nhist; i += 64) sys_store(host_out + 1 + i, (int32_t)hist[i]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) sys_store(host_out, *err);
  }
  const int64_t s0 = sample_base[k], s1 = sample_base[k + 1];
  if (*err) {   // the batch goes to the host path: every sample becomes a no-op
    if (k == 0 && lane == 0) {
      empty_at[0] = 0x92;   // [[], []]
      empty_at[1] = 0x90;
      empty_at[2] = 0x90;
    }
    for (int64_t s = s0 + lane; s < s1; s += 64) {
      row_ptr[s] = 0;
      datum_off[s] = empty_off;
      datum_len[s] = 3;
      labels[s] = -1;
    }
    if (k == R - 1 && lane == 0) row_ptr[s1] = 0;
    return;
  }
  long long acc = 0;
  for (int j = lane; j < k; j += 64) acc += req_slots[j];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  for (int64_t s = s0 + lane; s < s1; s += 64) row_ptr[s] += acc;
  if (k == R - 1 && lane == 0) row_ptr[s1] = acc + req_slots[k];
}

}  // namespace
}  // namespace jb

// Scan R train requests already in `buf` (device). sample_base[R+1] comes
// from the host's header pass (element count of each body). Outputs are the
// device arrays of a DeviceBatch; hist[nhist] (label counts of the batch)
// and *err are zeroed here. empty_at = buf + empty_off must have 3 writable
// bytes (the stand-in datum of a rejected batch). host_out (fine-grained
// host memory, 1 + nhist ints) receives [err, hist...] when the batch's
// fixup kernel completes. Returns 0, or 1 on bad arguments.
extern "C" int jb_scan_train(const uint8_t* buf, const int64_t* req_off, const int64_t* req_len,
                             const int64_t* sample_base, int R, const uint64_t* lt_hash,
                             const int32_t* lt_meta, int lt_cap, const uint8_t* lt_blob,
                             int lt_blob_len, int sps, int spn, int64_t* datum_off,
                             int32_t* datum_len, int32_t* labels, int64_t* row_ptr,
                             int64_t* req_slots, uint32_t* hist, int nhist, int32_t* err,
                             uint8_t* empty_at, int64_t empty_off, int32_t* host_out,
                             hipStream_t stream) {
  if (R <= 0) return 0;
  if (lt_cap <= 0 || (lt_cap & (lt_cap - 1)) != 0 || nhist < 0) return 1;
  if (hipMemsetAsync(err, 0, sizeof(int32_t), stream) != hipSuccess) return 1;
  if (nhist > 0 && hipMemsetAsync(hist, 0, sizeof(uint32_t) * (size_t)nhist, stream) != hipSuccess)
    return 1;
  hipLaunchKernelGGL(jb::scan_train_kernel, dim3(R), dim3(jb::kThreads), 0, stream, buf, req_off, req_len,
                     sample_base, R, lt_hash, lt_meta, lt_cap, lt_blob, lt_blob_len, sps, spn,
                     datum_off, datum_len, labels, row_ptr, req_slots, hist, nhist, err,
                     (long long*)nullptr);
  hipLaunchKernelGGL(jb::scan_fixup_kernel, dim3(R), dim3(64), 0, stream, sample_base, R,
                     req_slots, row_ptr, datum_off, datum_len, labels, empty_at, empty_off, err,
                     hist, nhist, host_out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Same as jb_scan_train's first kernel, recording s_memtime at the phase
// boundaries of every workgroup into prof[8 * R] (tools/bench_scan_gpu.py).
extern "C" int jb_scan_train_profile(const uint8_t* buf, const int64_t* req_off,
                                     const int64_t* req_len, const int64_t* sample_base, int R,
                                     const uint64_t* lt_hash, const int32_t* lt_meta, int lt_cap,
                                     const uint8_t* lt_blob, int lt_blob_len, int sps, int spn,
                                     int64_t* datum_off, int32_t* datum_len, int32_t* labels,
                                     int64_t* row_ptr, int64_t* req_slots, uint32_t* hist,
                                     int nhist, int32_t* err, long long* prof, hipStream_t stream) {
  if (R <= 0 || lt_cap <= 0 || (lt_cap & (lt_cap - 1)) != 0) return 1;
  hipLaunchKernelGGL(jb::scan_train_kernel, dim3(R), dim3(jb::kThreads), 0, stream, buf, req_off,
                     req_len, sample_base, R, lt_hash, lt_meta, lt_cap, lt_blob, lt_blob_len, sps,
                     spn, datum_off, datum_len, labels, row_ptr, req_slots, hist, nhist, err, prof);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
