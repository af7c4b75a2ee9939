// Device-side helpers shared by every jubatus_amd HIP kernel (gfx950 / CDNA4).
//
//  * FNV-1a/64 feature hashing, identical to the host implementation in
//    csrc/native/jb_hash.hpp (the host converter and the GPU converter must
//    produce the same feature index for the same feature name).
//  * A bounds-checked msgpack reader for the datum wire layout
//    [[ [k,v]... ], [ [k,num]... ], [ [k,raw]... ]]
//    (reference: jubatus/client/common/datum.hpp:42-46).
//  * wave64 reductions.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jb {

constexpr uint64_t kFnvOffset = 0xcbf29ce484222325ull;
constexpr uint64_t kFnvPrime = 0x100000001b3ull;

__device__ __forceinline__ uint64_t fnv_bytes(uint64_t h, const uint8_t* p, int n) {
  for (int i = 0; i < n; ++i) {
    h ^= (uint64_t)p[i];
    h *= kFnvPrime;
  }
  return h;
}

__device__ __forceinline__ uint64_t fnv_byte(uint64_t h, uint8_t b) {
  h ^= (uint64_t)b;
  return h * kFnvPrime;
}

// Range reduction of a 64-bit hash into [0, H): multiply-high (fast, unbiased
// enough for feature hashing). Host twin: jb::hash_to_index.
__device__ __forceinline__ int64_t hash_to_index(uint64_t h, uint64_t H) {
  h ^= h >> 29;
  h *= 0xbf58476d1ce4e5b9ull;
  h ^= h >> 32;
  return (int64_t)__umul64hi(h, H);
}

// ---------------------------------------------------------------- msgpack ---
struct Reader {
  const uint8_t* p;
  const uint8_t* end;
  bool ok;
  __device__ __forceinline__ bool need(int64_t n) {
    if (!ok || end - p < n) { ok = false; return false; }
    return true;
  }
  __device__ __forceinline__ uint32_t be16() { uint32_t v = ((uint32_t)p[0] << 8) | p[1]; p += 2; return v; }
  __device__ __forceinline__ uint32_t be32() {
    uint32_t v = ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
    p += 4; return v;
  }
  __device__ __forceinline__ uint64_t be64() { uint64_t hi = be32(); uint64_t lo = be32(); return (hi << 32) | lo; }

  // array header -> element count, -1 on type error
  __device__ int64_t array_len() {
    if (!need(1)) return -1;
    uint8_t t = *p++;
    if ((t & 0xf0) == 0x90) return t & 0x0f;
    if (t == 0xdc) { if (!need(2)) return -1; return be16(); }
    if (t == 0xdd) { if (!need(4)) return -1; return be32(); }
    ok = false; return -1;
  }
  // raw/str/bin -> (ptr,len); accepts old-spec RAW (fixraw/raw16/raw32) and new str8/bin
  __device__ bool raw(const uint8_t** s, int* n) {
    if (!need(1)) return false;
    uint8_t t = *p++;
    int64_t len;
    if ((t & 0xe0) == 0xa0) len = t & 0x1f;
    else if (t == 0xd9 || t == 0xc4) { if (!need(1)) return false; len = *p++; }
    else if (t == 0xda || t == 0xc5) { if (!need(2)) return false; len = be16(); }
    else if (t == 0xdb || t == 0xc6) { if (!need(4)) return false; len = be32(); }
    else { ok = false; return false; }
    if (!need(len)) return false;
    *s = p; *n = (int)len; p += len;
    return true;
  }
  __device__ bool number(double* out) {
    if (!need(1)) return false;
    uint8_t t = *p++;
    if (t <= 0x7f) { *out = (double)t; return true; }
    if (t >= 0xe0) { *out = (double)(int8_t)t; return true; }
    switch (t) {
      case 0xcc: if (!need(1)) return false; *out = (double)(*p++); return true;
      case 0xcd: if (!need(2)) return false; *out = (double)be16(); return true;
      case 0xce: if (!need(4)) return false; *out = (double)be32(); return true;
      case 0xcf: if (!need(8)) return false; *out = (double)be64(); return true;
      case 0xd0: if (!need(1)) return false; *out = (double)(int8_t)(*p++); return true;
      case 0xd1: if (!need(2)) return false; *out = (double)(int16_t)be16(); return true;
      case 0xd2: if (!need(4)) return false; *out = (double)(int32_t)be32(); return true;
      case 0xd3: if (!need(8)) return false; *out = (double)(int64_t)be64(); return true;
      case 0xca: { if (!need(4)) return false; uint32_t u = be32(); *out = (double)__uint_as_float(u); return true; }
      case 0xcb: {
        if (!need(8)) return false;
        uint64_t u = be64();
        *out = __longlong_as_double((long long)u);
        return true;
      }
      default: ok = false; return false;
    }
  }
};

// ------------------------------------------------------------- reductions ---
// Results into fine-grained (coherent) pinned host memory, then the flag a
// host thread polls. System-scope stores go past the L2 to the host, so
// waiting for their acknowledgements (vmcnt) orders them before the flag; a
// system-scope release fence instead writes back the whole L2 of the XCD
// (measured ~15 us on the top-k merge, more than its work).
template <class T>
__device__ __forceinline__ void sys_store(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// every thread of the block, after its sys_store()s: then one thread may
// publish the flag with sys_store
__device__ __forceinline__ void sys_stores_block_done() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Register-only cross-lane moves (no LDS round trip): DPP inside a 16-lane
// row, v_permlane16/32_swap (gfx950) across rows. A ds_bpermute costs an LDS
// latency (~50+ cycles) per step of a dependent chain; these are VALU ops.
enum : int {
  kDppXor1 = 0xB1,        // quad_perm [1,0,3,2]
  kDppXor2 = 0x4E,        // quad_perm [2,3,0,1]
  kDppRowRor8 = 0x128,    // lane i <- lane (i+8) mod 16 within the row
  kDppHalfMirror = 0x141, // lane i <- lane 7-i within each half row
  kDppMirror = 0x140,     // lane i <- lane 15-i within the row
};

template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}

// value of lane ^ 16 / lane ^ 32
__device__ __forceinline__ float partner16_f(float v, int lane) {
  auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(((lane >> 4) & 1) ? r[0] : r[1]);
}
__device__ __forceinline__ int partner16_i(int v, int lane) {
  auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  return (int)(((lane >> 4) & 1) ? r[0] : r[1]);
}
__device__ __forceinline__ float partner32_f(float v, int lane) {
  auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(lane >= 32 ? r[0] : r[1]);
}
__device__ __forceinline__ int partner32_i(int v, int lane) {
  auto r = __builtin_amdgcn_permlane32_swap((unsigned)v, (unsigned)v, false, false);
  return (int)(lane >= 32 ? r[0] : r[1]);
}

// sum over the 16 lanes of each row (every lane gets its row's sum)
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<kDppXor1>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  v += dpp_f<kDppMirror>(v);
  return v;
}

// full-wave sum, every lane gets it, no LDS
__device__ __forceinline__ float wave_sum_fast(float v, int lane) {
  v = row16_sum(v);
  v += partner16_f(v, lane);
  v += partner32_f(v, lane);
  return v;
}

}  // namespace jb
