// Device side of the native linear MIX (csrc/native/jb_mix_group.hpp, the
// classifier's Mixable in csrc/server/jubaclassifier.cpp): the touched-row
// union compaction, the snapshot gather of the touched rows in the group's
// canonical label order, and the fold of the cluster mean.
//
// Reference: the reference MIX ships whole diffs over msgpack-RPC
// (linear_mixer.cpp:358-544, get_diff / put_diff of the storage's rows); here
// only the rows some rank touched move, and they move as one dense
// [rows x 2 * labels] fp32 block per all-reduce (RCCL over xGMI).
//
// Layout: W, S are [H][LC] (row-major, LC label columns); map[c] is the local
// column of canonical label c (c < Lc). snap / red are [n][2 * Lc] (W columns
// then S columns; [n][Lc] when S is null).
#include <hip/hip_runtime.h>
#include <hipcub/device/device_select.hpp>
#include <hipcub/iterator/counting_input_iterator.hpp>

#include "jb_device.hpp"

namespace jb {

// bf16 wire (JUBATUS_MIX_DTYPE=bf16): the W columns of a [n][w] snapshot
// (w = 2 Lc: W then S columns; Lc without S) to bf16 with round-to-nearest-
// even, the S columns (precisions) stay fp32 - and back after the SUM
__global__ __launch_bounds__(256) void mix_pack_bf16_kernel(const float* __restrict__ snap, int64_t n, int Lc,
                                                            int has_s, uint16_t* __restrict__ wb,
                                                            float* __restrict__ sb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * Lc) return;
  const int64_t r = i / Lc;
  const int c = (int)(i - r * Lc);
  const int64_t w = (has_s ? 2 : 1) * (int64_t)Lc;
  const uint32_t u = __float_as_uint(snap[r * w + c]);
  // RNE; NaN stays NaN
  wb[i] = (u & 0x7fffffffu) > 0x7f800000u ? (uint16_t)((u >> 16) | 0x40u)
                                            : (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  if (has_s) sb[i] = snap[r * w + Lc + c];
}
__global__ __launch_bounds__(256) void mix_unpack_bf16_kernel(const uint16_t* __restrict__ wb,
                                                              const float* __restrict__ sb, int64_t n, int Lc,
                                                              int has_s, float* __restrict__ red) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * Lc) return;
  const int64_t r = i / Lc;
  const int c = (int)(i - r * Lc);
  const int64_t w = (has_s ? 2 : 1) * (int64_t)Lc;
  red[r * w + c] = __uint_as_float((uint32_t)wb[i] << 16);
  if (has_s) red[r * w + Lc + c] = sb[i];
}

// rows == nullptr: row r is r (dense MIX)
__global__ __launch_bounds__(256) void mix_gather_kernel(const float* __restrict__ W, const float* __restrict__ S,
                                                         int LC, const int64_t* __restrict__ rows, int64_t n,
                                                         const int32_t* __restrict__ map, int Lc,
                                                         float* __restrict__ snap) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t w = (S != nullptr ? 2 : 1) * (int64_t)Lc;
  if (i >= n * w) return;
  const int64_t r = i / w;
  const int c = (int)(i - r * w);
  const int64_t row = rows ? rows[r] : r;
  const int col = map[c < Lc ? c : c - Lc];
  snap[i] = c < Lc ? W[row * LC + col] : S[row * LC + col];
}

// T += red * inv_n - snap (updates made meanwhile are kept)
__global__ __launch_bounds__(256) void mix_fold_kernel(float* __restrict__ W, float* __restrict__ S, int LC,
                                                       const int64_t* __restrict__ rows, int64_t n,
                                                       const int32_t* __restrict__ map, int Lc,
                                                       const float* __restrict__ snap,
                                                       const float* __restrict__ red, float inv_n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t w = (S != nullptr ? 2 : 1) * (int64_t)Lc;
  if (i >= n * w) return;
  const int64_t r = i / w;
  const int c = (int)(i - r * w);
  const int64_t row = rows ? rows[r] : r;
  const int col = map[c < Lc ? c : c - Lc];
  const float d = red[i] * inv_n - snap[i];
  if (c < Lc) W[row * LC + col] += d;
  else S[row * LC + col] += d;
}

// mark[i] = touched[i]; touched[i] = 0 (stream-ordered with the train kernels)
__global__ __launch_bounds__(256) void mix_take_kernel(uint8_t* __restrict__ touched, uint8_t* __restrict__ mark,
                                                       int64_t H) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= H) return;
  mark[i] = touched[i];
  touched[i] = 0;
}

// push mixers' pair round: p += q (float tables) / p = max(p, q) (bitmaps),
// q being what the peer sent (16 B per lane)
__global__ __launch_bounds__(256) void mix_pair_sum_kernel(float* __restrict__ p, const float* __restrict__ q,
                                                           int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * i + 3 < n) {
    float4 a = reinterpret_cast<float4*>(p)[i];
    const float4 b = reinterpret_cast<const float4*>(q)[i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    reinterpret_cast<float4*>(p)[i] = a;
  } else {
    for (int64_t j = 4 * i; j < n; ++j) p[j] += q[j];
  }
}
__global__ __launch_bounds__(256) void mix_pair_max_kernel(uint8_t* __restrict__ p, const uint8_t* __restrict__ q,
                                                           int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] > q[i] ? p[i] : q[i];
}

}  // namespace jb

namespace {
inline unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }
}  // namespace

extern "C" int jb_mix_take(uint8_t* touched, uint8_t* mark, int64_t H, hipStream_t st) {
  if (H <= 0) return 0;
  hipLaunchKernelGGL(jb::mix_take_kernel, dim3(blocks_for(H)), dim3(256), 0, st, touched, mark, H);
  return (int)hipGetLastError();
}

// bytes of the compaction's temporary storage for H rows
extern "C" int64_t jb_mix_compact_temp_bytes(int64_t H) {
  size_t bytes = 0;
  hipcub::CountingInputIterator<int64_t> it(0);
  if (hipcub::DeviceSelect::Flagged(nullptr, bytes, it, (const uint8_t*)nullptr, (int64_t*)nullptr,
                                    (int64_t*)nullptr, (int)H) != hipSuccess)
    return -1;
  return (int64_t)bytes;
}

// rows[0 .. *count) = ascending indices i with mark[i] != 0 (the same order
// on every rank: the union map is identical after the MAX all-reduce)
extern "C" int jb_mix_compact(const uint8_t* mark, int64_t H, int64_t* rows, int64_t* count, void* temp,
                              int64_t temp_bytes, hipStream_t st) {
  if (H <= 0) return 0;
  if (H > INT32_MAX) return -2;
  size_t bytes = (size_t)temp_bytes;
  hipcub::CountingInputIterator<int64_t> it(0);
  const hipError_t e = hipcub::DeviceSelect::Flagged(temp, bytes, it, mark, rows, count, (int)H, st);
  return (int)e;
}

extern "C" int jb_mix_gather(const float* W, const float* S, int LC, const int64_t* rows, int64_t n,
                             const int32_t* map, int Lc, float* snap, hipStream_t st) {
  if (n <= 0 || Lc <= 0) return 0;
  hipLaunchKernelGGL(jb::mix_gather_kernel, dim3(blocks_for(n * (S ? 2 : 1) * Lc)), dim3(256), 0, st, W, S, LC,
                     rows, n, map, Lc, snap);
  return (int)hipGetLastError();
}

extern "C" int jb_mix_fold(float* W, float* S, int LC, const int64_t* rows, int64_t n, const int32_t* map,
                           int Lc, const float* snap, const float* red, float inv_n, hipStream_t st) {
  if (n <= 0 || Lc <= 0) return 0;
  hipLaunchKernelGGL(jb::mix_fold_kernel, dim3(blocks_for(n * (S ? 2 : 1) * Lc)), dim3(256), 0, st, W, S, LC,
                     rows, n, map, Lc, snap, red, inv_n);
  return (int)hipGetLastError();
}

// p += q over n floats (p, q device memory, 16-byte aligned)
extern "C" int jb_mix_pair_sum(float* p, const float* q, int64_t n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(jb::mix_pair_sum_kernel, dim3(blocks_for((n + 3) / 4)), dim3(256), 0, st, p, q, n);
  return (int)hipGetLastError();
}

// p = max(p, q) over n bytes
extern "C" int jb_mix_pair_max(uint8_t* p, const uint8_t* q, int64_t n, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(jb::mix_pair_max_kernel, dim3(blocks_for(n)), dim3(256), 0, st, p, q, n);
  return (int)hipGetLastError();
}

extern "C" int jb_mix_pack_bf16(const float* snap, int64_t n, int Lc, int has_s, uint16_t* wb, float* sb,
                                hipStream_t st) {
  if (n <= 0 || Lc <= 0) return 0;
  hipLaunchKernelGGL(jb::mix_pack_bf16_kernel, dim3(blocks_for(n * Lc)), dim3(256), 0, st, snap, n, Lc, has_s,
                     wb, sb);
  return (int)hipGetLastError();
}

extern "C" int jb_mix_unpack_bf16(const uint16_t* wb, const float* sb, int64_t n, int Lc, int has_s, float* red,
                                  hipStream_t st) {
  if (n <= 0 || Lc <= 0) return 0;
  hipLaunchKernelGGL(jb::mix_unpack_bf16_kernel, dim3(blocks_for(n * Lc)), dim3(256), 0, st, wb, sb, n, Lc,
                     has_s, red);
  return (int)hipGetLastError();
}
