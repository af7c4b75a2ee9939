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
#include "jb_fv.hpp"

namespace jb {

constexpr int kBlobCap = 1024;   // rule blob staged in LDS when it fits
constexpr int kWin = 16384;      // per-wave LDS window of datum bytes

// One lane per datum. The 64 datums of a wave are consecutive samples, so
// their bytes form one contiguous window of the request arena: the wave
// stages that window into LDS with 16-B loads (coalesced), then every lane
// parses its datum out of LDS instead of issuing ~200 dependent byte loads
// to global memory. Windows larger than kWin fall back to global parsing.
__global__ __launch_bounds__(256) void fv_hash_kernel(
    const uint8_t* __restrict__ buf, int64_t buf_len, int64_t buf_cap,
    const int64_t* __restrict__ datum_off, const int32_t* __restrict__ datum_len,
    const int64_t* __restrict__ row_ptr, int n,
    const GpuRule* __restrict__ srules, int n_srules,
    const GpuRule* __restrict__ nrules, int n_nrules,
    const uint8_t* __restrict__ blob, int blob_len, uint64_t H,
    int32_t* __restrict__ out_idx, float* __restrict__ out_val, int32_t* __restrict__ err) {
  __shared__ __attribute__((aligned(16))) uint8_t s_blob[kBlobCap];
  __shared__ __attribute__((aligned(16))) uint8_t s_win[4][kWin];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const bool blob_lds = blob_len <= kBlobCap;
  if (blob_lds)
    for (int i = threadIdx.x; i < blob_len; i += blockDim.x) s_blob[i] = blob[i];
  __syncthreads();
  const uint8_t* bl = blob_lds ? (const uint8_t*)s_blob : blob;

  const int s0 = (blockIdx.x * blockDim.x) + wv * 64;
  if (s0 >= n) return;
  const int s = s0 + lane;
  const bool live = s < n;
  const int64_t off = live ? datum_off[s] : datum_off[s0];
  const int64_t dend = live ? off + datum_len[s] : off;
  // window [lo, hi) covering every datum of the wave
  int64_t lo = off, hi = dend;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t olo = __shfl_xor(lo, o, 64);
    const int64_t ohi = __shfl_xor(hi, o, 64);
    lo = olo < lo ? olo : lo;
    hi = ohi > hi ? ohi : hi;
  }
  const int64_t lo16 = lo & ~(int64_t)15;
  const int64_t span = ((hi + 15) & ~(int64_t)15) - lo16;
  bool ok = true;
  if (span <= kWin && lo16 + span <= buf_cap) {
    for (int64_t b = (int64_t)lane * 16; b < span; b += 64 * 16)
      *reinterpret_cast<uint4*>(&s_win[wv][b]) = *reinterpret_cast<const uint4*>(buf + lo16 + b);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    if (live) {
      const uint8_t* base = &s_win[wv][off - lo16];
      Reader rd{base, base + (dend - off), true};
      ok = emit_datum(rd, row_ptr[s], row_ptr[s + 1], srules, n_srules, nrules, n_nrules, bl, H,
                      out_idx, out_val);
    }
  } else if (live) {
    Reader rd{buf + off, buf + (dend < buf_len ? dend : buf_len), true};
    ok = emit_datum(rd, row_ptr[s], row_ptr[s + 1], srules, n_srules, nrules, n_nrules, bl, H,
                    out_idx, out_val);
  }
  if (!ok) atomicOr(err, 2);
}

}  // namespace jb

extern "C" int jb_fv_hash(const uint8_t* buf, int64_t buf_len, int64_t buf_cap,
                          const int64_t* datum_off, const int32_t* datum_len,
                          const int64_t* row_ptr, int n, const void* srules, int n_srules,
                          const void* nrules, int n_nrules, const uint8_t* blob, int blob_len,
                          uint64_t H, int32_t* out_idx, float* out_val, int32_t* err,
                          hipStream_t stream) {
  if (n <= 0) return 0;
  const int threads = 256;
  const int blocks = (n + threads - 1) / threads;
  hipLaunchKernelGGL(jb::fv_hash_kernel, dim3(blocks), dim3(threads), 0, stream, buf, buf_len,
                     buf_cap, datum_off, datum_len, row_ptr, n, (const jb::GpuRule*)srules,
                     n_srules, (const jb::GpuRule*)nrules, n_nrules, blob, blob_len, H, out_idx,
                     out_val, err);
  return (int)hipGetLastError();
}
