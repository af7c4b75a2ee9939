// Global feature weights (idf / bm25) of a converted batch against the
// document-frequency table in HBM, with the converter's sequential semantics
// inside the batch: datum i of a training batch sees the document counts
// after datums 0..i were added, then the table advances by the whole batch.
//
// Reference: jubatus_core's weight_manager (EXTERNAL; the semantics are
// pinned by the Python converter, fv_converter/converter.py _convert, and its
// host twin csrc/native/jb_hostfv_wide.hpp). Used by the wide device
// converter (ops/fv_wide.py) - jubaweight, and every engine whose converter
// has idf / bm25 rules.
//
// One launch chain, no host round trip before the weights are final:
//   1. per datum: the (feature, datum) key of every global-weighted slot and
//      the datum's weighted length;
//   2. radix sort of (key, slot) (hipCUB);
//   3. rank of each (feature, datum) pair among the distinct pairs of its
//      feature: inclusive sum of "new pair" flags minus the sum at the
//      feature's first pair (max-scan) -> df seen by that datum = df + rank + 1;
//   4. the table advances by one per distinct pair (update only);
//   5. per datum: idf / bm25 of its slots in double (as the Python path).
#include <hip/hip_runtime.h>
#include <hipcub/device/device_radix_sort.hpp>
#include <hipcub/device/device_scan.hpp>

#include "jb_device.hpp"

namespace jb {

constexpr uint64_t kNoKey = ~0ull;

__global__ __launch_bounds__(256) void df_keys_kernel(const int64_t* __restrict__ row_ptr, int n,
                                                      const int32_t* __restrict__ idx,
                                                      const uint8_t* __restrict__ gw,
                                                      uint64_t* __restrict__ key, int32_t* __restrict__ slot,
                                                      int64_t* __restrict__ lens) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  int64_t len = 0;
  for (int64_t s = row_ptr[d]; s < row_ptr[d + 1]; ++s) {
    const bool sel = gw[s] > 0 && idx[s] >= 0;
    key[s] = sel ? (((uint64_t)(uint32_t)idx[s] << 32) | (uint32_t)d) : kNoKey;
    slot[s] = (int32_t)s;
    len += sel;
  }
  lens[d] = len;
}

// sorted order: newpair flags (the scan input) and the feature-start marks
__global__ __launch_bounds__(256) void df_flags_kernel(const uint64_t* __restrict__ key, int64_t total,
                                                       int32_t* __restrict__ newpair) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint64_t k = key[i];
  newpair[i] = (k != kNoKey && (i == 0 || key[i - 1] != k)) ? 1 : 0;
}

__global__ __launch_bounds__(256) void df_segstart_kernel(const uint64_t* __restrict__ key, int64_t total,
                                                          const int32_t* __restrict__ cum,
                                                          int32_t* __restrict__ seg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint64_t k = key[i];
  const bool start = k != kNoKey && (i == 0 || (key[i - 1] >> 32) != (k >> 32));
  seg[i] = start ? cum[i] : 0;
}

// df seen by each selected slot; the table advances (update) one per pair
__global__ __launch_bounds__(256) void df_rank_kernel(const uint64_t* __restrict__ key,
                                                      const int32_t* __restrict__ slot, int64_t total,
                                                      const int32_t* __restrict__ cum,
                                                      const int32_t* __restrict__ first,
                                                      const int64_t* __restrict__ df,
                                                      double* __restrict__ dfat) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const uint64_t k = key[i];
  if (k == kNoKey) return;
  const int32_t f = (int32_t)(k >> 32);
  dfat[slot[i]] = (double)(df[f] + (int64_t)(cum[i] - first[i]) + 1);
}

__global__ __launch_bounds__(256) void df_advance_kernel(const uint64_t* __restrict__ key, int64_t total,
                                                         const int32_t* __restrict__ newpair,
                                                         unsigned long long* __restrict__ df,
                                                         unsigned long long* __restrict__ diff) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total || !newpair[i]) return;
  const int32_t f = (int32_t)(key[i] >> 32);
  atomicAdd(df + f, 1ull);
  atomicAdd(diff + f, 1ull);
}

__global__ __launch_bounds__(256) void df_weigh_kernel(const int64_t* __restrict__ row_ptr, int n,
                                                       const int32_t* __restrict__ idx,
                                                       const uint8_t* __restrict__ gw, float* __restrict__ val,
                                                       const double* __restrict__ dfat,
                                                       const int64_t* __restrict__ df,
                                                       const int64_t* __restrict__ lens,
                                                       const int64_t* __restrict__ cumlen, int64_t N0,
                                                       int64_t L0, int update) {
  const int d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d >= n) return;
  const double docs = update ? (double)(N0 + 1 + d) : (double)N0;
  const double clen = update ? (double)(L0 + cumlen[d]) : (double)L0;
  const double avg = docs > 0 ? clen / fmax(docs, 1.0) : 1.0;
  const double len = (double)lens[d];
  const double k1 = 1.2, b = 0.75;
  for (int64_t s = row_ptr[d]; s < row_ptr[d + 1]; ++s) {
    const int g = gw[s];
    if (g == 0 || idx[s] < 0) continue;
    const double dfa = update ? dfat[s] : (double)df[idx[s]];
    const double idf = (dfa > 0 && docs > 0) ? log(docs / fmax(dfa, 1.0)) : 0.0;
    const double w = (double)val[s];
    const double out = g == 1 ? w * idf
                              : idf * (w * (k1 + 1)) / (w + k1 * (1 - b + b * len / fmax(avg, 1e-9)));
    val[s] = (float)out;
  }
}

}  // namespace jb

namespace {

inline unsigned nb(int64_t n) { return (unsigned)((n + 255) / 256); }
inline size_t align(size_t x) { return (x + 255) & ~(size_t)255; }

struct DfPlan {
  size_t sort_tmp = 0, scan_tmp = 0, max_tmp = 0, lens_tmp = 0;
  size_t total_bytes(int64_t total, int64_t n) const {
    const size_t t = (size_t)std::max<int64_t>(total, 1), m = (size_t)std::max<int64_t>(n, 1);
    return align(t * 8) * 2 + align(t * 4) * 2 + align(t * 4) * 4 + align(t * 8) + align(m * 8) * 2 +
           align(std::max(std::max(sort_tmp, scan_tmp), std::max(max_tmp, lens_tmp)));
  }
};

struct MaxOp {
  __host__ __device__ int32_t operator()(const int32_t& a, const int32_t& b) const { return a > b ? a : b; }
};

DfPlan plan(int64_t total, int64_t n) {
  DfPlan p;
  const int T = (int)std::max<int64_t>(total, 1);
  hipcub::DeviceRadixSort::SortPairs(nullptr, p.sort_tmp, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, T);
  hipcub::DeviceScan::InclusiveSum(nullptr, p.scan_tmp, (const int32_t*)nullptr, (int32_t*)nullptr, T);
  hipcub::DeviceScan::InclusiveScan(nullptr, p.max_tmp, (const int32_t*)nullptr, (int32_t*)nullptr, MaxOp(), T);
  hipcub::DeviceScan::InclusiveSum(nullptr, p.lens_tmp, (const int64_t*)nullptr, (int64_t*)nullptr,
                                   (int)std::max<int64_t>(n, 1));
  return p;
}

}  // namespace

// scratch bytes of jb_df_weigh for `total` slots over `n` datums
extern "C" int64_t jb_df_scratch_bytes(int64_t total, int64_t n) {
  return (int64_t)plan(total, n).total_bytes(total, n);
}

// idf / bm25 of the global-weighted slots (gw 1 idf, 2 bm25; 0 none) of a
// converted batch, in place in val. update: the batch is added to the table
// (df, diff += one per distinct (feature, datum)) with the sequential
// semantics; sel_len (device int64, nullable) receives the batch's weighted
// length (the host's average-length counter).
extern "C" int jb_df_weigh(const int64_t* row_ptr, int n, int64_t total, const int32_t* idx, float* val,
                           const uint8_t* gw, int64_t* df, int64_t* diff, int64_t N0, int64_t L0, int update,
                           void* scratch, int64_t scratch_bytes, int64_t* sel_len, hipStream_t st) {
  if (n <= 0) return 0;
  if (total > INT32_MAX) return -2;
  const DfPlan p = plan(total, n);
  if (scratch == nullptr || scratch_bytes < (int64_t)p.total_bytes(total, n)) return -3;
  const size_t t = (size_t)std::max<int64_t>(total, 1), m = (size_t)n;
  uint8_t* q = (uint8_t*)scratch;
  auto take = [&](size_t bytes) { uint8_t* r = q; q += align(bytes); return (void*)r; };
  uint64_t* key = (uint64_t*)take(t * 8);
  uint64_t* key2 = (uint64_t*)take(t * 8);
  int32_t* slot = (int32_t*)take(t * 4);
  int32_t* slot2 = (int32_t*)take(t * 4);
  int32_t* newpair = (int32_t*)take(t * 4);
  int32_t* cum = (int32_t*)take(t * 4);
  int32_t* seg = (int32_t*)take(t * 4);
  int32_t* first = (int32_t*)take(t * 4);
  double* dfat = (double*)take(t * 8);
  int64_t* lens = (int64_t*)take(m * 8);
  int64_t* cumlen = (int64_t*)take(m * 8);
  void* tmp = take(std::max(std::max(p.sort_tmp, p.scan_tmp), std::max(p.max_tmp, p.lens_tmp)));
  hipLaunchKernelGGL(jb::df_keys_kernel, dim3(nb(n)), dim3(256), 0, st, row_ptr, n, idx, gw, key, slot, lens);
  size_t tb = p.lens_tmp;
  if (hipcub::DeviceScan::InclusiveSum(tmp, tb, lens, cumlen, n, st) != hipSuccess) return -4;
  if (sel_len != nullptr)
    (void)hipMemcpyAsync(sel_len, cumlen + (n - 1), 8, hipMemcpyDeviceToDevice, st);
  if (update && total > 0) {
    tb = p.sort_tmp;
    if (hipcub::DeviceRadixSort::SortPairs(tmp, tb, key, key2, slot, slot2, (int)total, 0, 64, st) != hipSuccess)
      return -5;
    hipLaunchKernelGGL(jb::df_flags_kernel, dim3(nb(total)), dim3(256), 0, st, key2, total, newpair);
    tb = p.scan_tmp;
    if (hipcub::DeviceScan::InclusiveSum(tmp, tb, newpair, cum, (int)total, st) != hipSuccess) return -6;
    hipLaunchKernelGGL(jb::df_segstart_kernel, dim3(nb(total)), dim3(256), 0, st, key2, total, cum, seg);
    tb = p.max_tmp;
    if (hipcub::DeviceScan::InclusiveScan(tmp, tb, seg, first, MaxOp(), (int)total, st) != hipSuccess) return -7;
    hipLaunchKernelGGL(jb::df_rank_kernel, dim3(nb(total)), dim3(256), 0, st, key2, slot2, total, cum, first, df,
                       dfat);
    hipLaunchKernelGGL(jb::df_advance_kernel, dim3(nb(total)), dim3(256), 0, st, key2, total, newpair,
                       (unsigned long long*)df, (unsigned long long*)diff);
  }
  hipLaunchKernelGGL(jb::df_weigh_kernel, dim3(nb(n)), dim3(256), 0, st, row_ptr, n, idx, gw, val, dfat,
                     (const int64_t*)df, lens, cumlen, N0, L0, update);
  return (int)hipGetLastError();
}
