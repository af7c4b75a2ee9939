// Hot-row detection for the concurrent train kernels (csrc/hip/linear.hip).
//
// A row is hot when a large share of a batch's samples carry it (an
// always-present numeric key, a bias feature): with one update stream per
// request, every stream then adds to the same cache lines every sample and
// the memory-side atomics serialise. The train kernel keeps such rows in a
// block-shared LDS replica that it merges into the table every few samples
// (linear.hip, "Hot rows"); this file finds them, per batch, on the device:
//
//   hot_count_kernel  one block per 2048 feature slots (at most 256 chunks,
//                     evenly spread: a sample of larger batches): exact
//                     counts of the block's rows in an LDS hash table; rows seen at least
//                     `block_min` times are added to a global candidate
//                     table (one atomic per row and block, not per slot)
//   hot_select_kernel one block: candidates with a total count >= `min_count`
//                     become the hot list (at most `max_rows`); the candidate
//                     table is emptied for the next batch
//
// Reference context: the per-sample train loop of
// jubatus/server/server/classifier_serv.cpp:138-144 has no concurrency; the
// hot-row replica is what keeps many concurrent GPU streams on one model
// cheap.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jb {

constexpr int kHotTab = 4096;       // LDS slots per block (2x the slots of a chunk:
constexpr int kHotChunk = 2048;     // feature slots per block   every row fits, load <= 1/2)
constexpr int kHotMaxBlocks = 256;  // chunks counted per batch (a sample of larger batches)

__device__ __forceinline__ uint32_t hot_hash(int32_t r) { return (uint32_t)r * 0x9E3779B1u; }

// chunks of the batch and the sampling stride: at most gridDim.x chunks are
// counted, evenly spread over the batch (every stride-th chunk)
__device__ __forceinline__ int64_t hot_stride(int64_t nnz, int blocks) {
  const int64_t chunks = (nnz + kHotChunk - 1) / kHotChunk;
  return chunks <= blocks ? 1 : (chunks + blocks - 1) / blocks;
}

__global__ __launch_bounds__(256) void hot_count_kernel(const int64_t* __restrict__ row_ptr, int n,
                                                        const int32_t* __restrict__ fidx,
                                                        int block_min, int32_t* __restrict__ gkey,
                                                        int32_t* __restrict__ gcnt, int gcap) {
  __shared__ int32_t key[kHotTab];
  __shared__ int32_t cnt[kHotTab];
  const int64_t nnz = row_ptr[n];
  const int64_t beg = (int64_t)blockIdx.x * hot_stride(nnz, gridDim.x) * kHotChunk;
  if (beg >= nnz) return;                      // uniform over the block
  for (int i = threadIdx.x; i < kHotTab; i += blockDim.x) { key[i] = -1; cnt[i] = 0; }
  __syncthreads();
  const int64_t end = beg + kHotChunk < nnz ? beg + kHotChunk : nnz;
  for (int64_t i = beg + threadIdx.x; i < end; i += blockDim.x) {
    const int32_t r = fidx[i];
    if (r < 0) continue;
    uint32_t h = hot_hash(r) >> 20;            // 12 bits
    for (int p = 0; p < 64; ++p) {
      const int32_t k = key[h];
      if (k == r) { atomicAdd(&cnt[h], 1); break; }
      if (k < 0) {
        const int32_t old = atomicCAS(&key[h], -1, r);
        if (old == -1 || old == r) { atomicAdd(&cnt[h], 1); break; }
      }
      h = (h + 1) & (kHotTab - 1);
    }
  }
  __syncthreads();
  const uint32_t gmask = (uint32_t)gcap - 1;
  for (int i = threadIdx.x; i < kHotTab; i += blockDim.x) {
    const int c = cnt[i];
    if (c < block_min) continue;
    const int32_t r = key[i];
    uint32_t h = hot_hash(r) & gmask;
    for (int p = 0; p < gcap; ++p) {
      const int32_t old = atomicCAS(&gkey[h], -1, r);
      if (old == -1 || old == r) { atomicAdd(&gcnt[h], c); break; }
      h = (h + 1) & gmask;
    }
  }
}

__global__ __launch_bounds__(1024) void hot_select_kernel(const int64_t* __restrict__ row_ptr,
                                                          int nsamp, int count_blocks,
                                                          int32_t* __restrict__ gkey,
                                                          int32_t* __restrict__ gcnt, int gcap,
                                                          int min_count, int max_rows,
                                                          int32_t* __restrict__ hot_rows,
                                                          int32_t* __restrict__ hot_n) {
  __shared__ int n;
  if (threadIdx.x == 0) n = 0;
  // the counts cover 1 / stride of the batch
  if (nsamp > 0 && count_blocks > 0) {
    const int64_t st = hot_stride(row_ptr[nsamp], count_blocks);
    min_count = (int)((min_count + st - 1) / st);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < gcap; i += blockDim.x) {
    const int32_t r = gkey[i];
    if (r < 0) continue;
    if (gcnt[i] >= min_count) {
      const int k = atomicAdd(&n, 1);
      if (k < max_rows) hot_rows[k] = r;
    }
    gkey[i] = -1;
    gcnt[i] = 0;
  }
  __syncthreads();
  if (threadIdx.x == 0) *hot_n = n < max_rows ? n : max_rows;
}

}  // namespace jb

// gkey / gcnt: device candidate table of gcap (power of two) slots, keys -1
// and counts 0 on entry; left in that state. row_ptr[n] (device) bounds the
// feature slots scanned. max_slots: upper bound of row_ptr[n] known to the
// host (grid size).
extern "C" int jb_hot_detect(const int64_t* row_ptr, int n, const int32_t* fidx, int64_t max_slots,
                             int block_min, int min_count, int max_rows, int32_t* gkey,
                             int32_t* gcnt, int gcap, int32_t* hot_rows, int32_t* hot_n,
                             hipStream_t stream) {
  if (gcap <= 0 || (gcap & (gcap - 1)) || max_rows <= 0) return -1;
  int64_t blocks = 0;
  if (n > 0 && max_slots > 0) {
    blocks = (max_slots + jb::kHotChunk - 1) / jb::kHotChunk;
    if (blocks > jb::kHotMaxBlocks) blocks = jb::kHotMaxBlocks;
    hipLaunchKernelGGL(jb::hot_count_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, row_ptr,
                       n, fidx, block_min, gkey, gcnt, gcap);
  }
  hipLaunchKernelGGL(jb::hot_select_kernel, dim3(1), dim3(1024), 0, stream, row_ptr, n,
                     (int)blocks, gkey, gcnt, gcap, min_count, max_rows, hot_rows, hot_n);
  return (int)hipGetLastError();
}
