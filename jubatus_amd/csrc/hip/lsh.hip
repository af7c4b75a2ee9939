// Similarity-search kernels for nearest_neighbor / recommender / anomaly.
//
// Reference: the nearest_neighbor / recommender engines (EXTERNAL
// jubatus_core; call sites jubatus/server/server/nearest_neighbor_serv.cpp:129-178,
// recommender_serv.cpp:136-224, anomaly_serv.cpp:157-244). Methods:
//   lsh         random-hyperplane sign bits (hash_num bits)
//   euclid_lsh  the same bits + the row norm (approximate euclidean distance)
//   minhash     1-bit min-wise hashing of the nonzero features
//
// Projections are never materialised: the hyperplane coefficient of feature
// index i, bit j is a standard normal drawn from splitmix64(seed, i, j)
// (Box-Muller), so a signature costs f x hash_num hash evaluations and no
// HBM traffic. One wave per datum; lane j owns bit j of each 64-bit word and
// a __ballot packs the 64 sign bits of a word in one instruction.
//
// The scans are bandwidth kernels over the signature table (XOR + popcount)
// and over CSR rows (exact cosine / euclid for inverted_index), writing a
// score per row; top-k selection then runs on the score vector.
#include "jb_device.hpp"
#include "jb_host_wait.hpp"

#include <cstring>

namespace jb {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t feat_hash(uint64_t seed, uint32_t idx, uint32_t j) {
  return splitmix64(seed ^ splitmix64(((uint64_t)idx << 20) ^ (uint64_t)j));
}

// standard normal from one 64-bit hash (Box-Muller on its two halves)
__device__ __forceinline__ float gauss(uint64_t h) {
  const float u1 = ((float)(uint32_t)(h >> 40) + 1.0f) * (1.0f / 16777217.0f);
  const float u2 = (float)(uint32_t)(h & 0xffffffu) * (1.0f / 16777216.0f);
  return sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853f * u2);
}

// Signature of one sample (one wave): mode 0 sign-of-projection bits (lsh,
// euclid_lsh), 1 minhash bits; lane j owns bit j of each 64-bit word.
__device__ __forceinline__ void signature_one(const int32_t* fidx, const float* fval, int64_t beg,
                                              int nf, int hash_num, uint64_t seed, int mode,
                                              uint64_t* __restrict__ bits, float* norm, int lane) {
  const int words = (hash_num + 63) / 64;
  float nrm = 0.f;
  for (int j = lane; j < nf; j += 64) {
    const float x = fval[beg + j];
    if (fidx[beg + j] >= 0) nrm += x * x;
  }
  nrm = wave_sum(nrm);
  for (int w = 0; w < words; ++w) {
    const int j = w * 64 + lane;
    bool bit = false;
    if (mode == 0) {
      float acc = 0.f;
      for (int i = 0; i < nf; ++i) {
        const int32_t idx = fidx[beg + i];
        if (idx < 0) continue;
        acc += fval[beg + i] * gauss(feat_hash(seed, (uint32_t)idx, (uint32_t)j));
      }
      bit = acc > 0.f;
    } else {
      uint64_t mn = ~0ull;
      for (int i = 0; i < nf; ++i) {
        const int32_t idx = fidx[beg + i];
        if (idx < 0 || fval[beg + i] == 0.f) continue;
        const uint64_t h = feat_hash(seed, (uint32_t)idx, (uint32_t)j);
        mn = h < mn ? h : mn;
      }
      bit = (mn & 1ull) != 0;
    }
    if (j >= hash_num) bit = false;
    const uint64_t word = __ballot(bit);
    if (lane == 0) bits[w] = word;
  }
  if (lane == 0 && norm != nullptr) *norm = sqrtf(nrm);
}

__global__ __launch_bounds__(256) void signature_kernel(
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ fidx,
    const float* __restrict__ fval, int n, int hash_num, uint64_t seed, int mode,
    uint64_t* __restrict__ bits, float* __restrict__ norms) {
  const int lane = threadIdx.x & 63;
  const int s = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (s >= n) return;
  const int64_t beg = row_ptr[s];
  const int words = (hash_num + 63) / 64;
  signature_one(fidx, fval, beg, (int)(row_ptr[s + 1] - beg), hash_num, seed, mode,
                bits + (int64_t)s * words, norms != nullptr ? norms + s : nullptr, lane);
}

// Query signatures from the kernel arguments (latency path: no H2D copy).
constexpr int kQueryMax = 8;
constexpr int kQuerySlots = 256;
struct alignas(16) QueryArgs {
  int32_t n;
  int32_t slot[kQueryMax + 1];
  int32_t pad[2];
  int64_t dst[kQueryMax];   // destination row of each signature (-1: row q of the output)
  int32_t idx[kQuerySlots];
  float val[kQuerySlots];
};

// valid != nullptr: the rows are table slots (set_row) and become valid
__global__ __launch_bounds__(64) void signature_query_kernel(const QueryArgs a, int hash_num,
                                                             uint64_t seed, int mode,
                                                             uint64_t* __restrict__ bits,
                                                             float* __restrict__ norms,
                                                             uint8_t* __restrict__ valid) {
  const int q = blockIdx.x;
  if (q >= a.n) return;
  const int words = (hash_num + 63) / 64;
  const int64_t row = a.dst[q] >= 0 ? a.dst[q] : q;
  signature_one(a.idx, a.val, a.slot[q], a.slot[q + 1] - a.slot[q], hash_num, seed, mode,
                bits + row * words, norms + row, threadIdx.x);
  if (valid != nullptr && threadIdx.x == 0) valid[row] = 1;
}

// a batch of table rows from a device CSR (the row server's batched writes):
// one wave per row, row q of the CSR into table slot slots[q]
__global__ __launch_bounds__(64) void signature_rows_kernel(const int64_t* __restrict__ rp,
                                                            const int64_t* __restrict__ slots,
                                                            const int32_t* __restrict__ idx,
                                                            const float* __restrict__ val, int n, int hash_num,
                                                            uint64_t seed, int mode, uint64_t* __restrict__ bits,
                                                            float* __restrict__ norms, uint8_t* __restrict__ valid) {
  const int q = blockIdx.x;
  if (q >= n) return;
  const int words = (hash_num + 63) / 64;
  const int64_t row = slots[q];
  signature_one(idx, val, rp[q], (int)(rp[q + 1] - rp[q]), hash_num, seed, mode, bits + row * words, norms + row,
                threadIdx.x);
  if (threadIdx.x == 0) valid[row] = 1;
}

namespace {
int fill_query_args(QueryArgs* a, const int32_t* idx, const float* val, const int64_t* row_ptr,
                    int n, const int64_t* dst) {
  if (n > kQueryMax || row_ptr[n] - row_ptr[0] > kQuerySlots) return 1;
  a->n = n;
  const int64_t base = row_ptr[0];
  for (int i = 0; i <= n; ++i) a->slot[i] = (int32_t)(row_ptr[i] - base);
  for (int i = 0; i < n; ++i) a->dst[i] = dst ? dst[i] : -1;
  const int ns = a->slot[n];
  std::memcpy(a->idx, idx + base, sizeof(int32_t) * (size_t)ns);
  std::memcpy(a->val, val + base, sizeof(float) * (size_t)ns);
  return 0;
}
}  // namespace

// metric: 0 lsh (distance = hamming / hash_num), 1 euclid_lsh (approximate
// euclidean distance from norms + angle), 2 minhash (distance = 1 - matching
// fraction). Writes a *distance* per (query, row); invalid rows get +inf.
__global__ __launch_bounds__(256) void hamming_scan_kernel(
    const uint64_t* __restrict__ qbits, const float* __restrict__ qnorm, int nq,
    const uint64_t* __restrict__ tbits, const float* __restrict__ tnorm,
    const uint8_t* __restrict__ valid, int64_t nrows, int words, int hash_num, int metric,
    float* __restrict__ out) {
  const int q = blockIdx.y;
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= nq || r >= nrows) return;
  float d;
  if (!valid[r]) {
    d = INFINITY;
  } else {
    int ham = 0;
    for (int w = 0; w < words; ++w) ham += __popcll(qbits[(int64_t)q * words + w] ^ tbits[r * words + w]);
    const float frac = (float)ham / (float)hash_num;
    if (metric == 0) d = frac;
    else if (metric == 2) d = frac;
    else {
      const float a = qnorm[q], b = tnorm[r];
      const float c = __cosf(3.14159265f * frac);
      d = sqrtf(fmaxf(0.f, a * a + b * b - 2.f * a * b * c));
    }
  }
  out[(int64_t)q * nrows + r] = d;
}

// Exact sparse similarity of one query against every CSR row (inverted_index
// family). The query (sorted feature indices) is staged in LDS; one thread
// per row walks its nonzeros with a binary search into the query.
// metric 0: cosine similarity; 1: euclidean distance.
constexpr int kMaxQuery = 4096;

__global__ __launch_bounds__(256) void sparse_scan_kernel(
    const int32_t* __restrict__ qidx, const float* __restrict__ qval, int qn, float qnorm2,
    const int64_t* __restrict__ row_ptr, const int32_t* __restrict__ ridx,
    const float* __restrict__ rval, const float* __restrict__ rnorm2,
    const uint8_t* __restrict__ valid, int64_t nrows, int metric, float* __restrict__ out) {
  __shared__ int32_t s_idx[kMaxQuery];
  __shared__ float s_val[kMaxQuery];
  for (int i = threadIdx.x; i < qn; i += blockDim.x) { s_idx[i] = qidx[i]; s_val[i] = qval[i]; }
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  if (!valid[r]) { out[r] = metric == 0 ? -INFINITY : INFINITY; return; }
  float dot = 0.f;
  for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) {
    const int32_t f = ridx[k];
    int lo = 0, hi = qn - 1;
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      const int32_t v = s_idx[mid];
      if (v == f) { dot += rval[k] * s_val[mid]; break; }
      if (v < f) lo = mid + 1; else hi = mid - 1;
    }
  }
  const float b2 = rnorm2[r];
  if (metric == 0) {
    const float den = sqrtf(qnorm2) * sqrtf(b2);
    out[r] = den > 0.f ? dot / den : 0.f;
  } else {
    out[r] = sqrtf(fmaxf(0.f, qnorm2 + b2 - 2.f * dot));
  }
}

}  // namespace jb

extern "C" int jb_signature(const int64_t* row_ptr, const int32_t* fidx, const float* fval, int n,
                            int hash_num, uint64_t seed, int mode, uint64_t* bits, float* norms,
                            hipStream_t stream) {
  if (n <= 0) return 0;
  const int threads = 256, blocks = (n * 64 + threads - 1) / threads;
  hipLaunchKernelGGL(jb::signature_kernel, dim3(blocks), dim3(threads), 0, stream, row_ptr, fidx,
                     fval, n, hash_num, seed, mode, bits, norms);
  return (int)hipGetLastError();
}

extern "C" int jb_hamming_scan(const uint64_t* qbits, const float* qnorm, int nq,
                               const uint64_t* tbits, const float* tnorm, const uint8_t* valid,
                               int64_t nrows, int words, int hash_num, int metric, float* out,
                               hipStream_t stream) {
  if (nq <= 0 || nrows <= 0) return 0;
  const int threads = 256;
  dim3 grid((unsigned)((nrows + threads - 1) / threads), (unsigned)nq);
  hipLaunchKernelGGL(jb::hamming_scan_kernel, grid, dim3(threads), 0, stream, qbits, qnorm, nq,
                     tbits, tnorm, valid, nrows, words, hash_num, metric, out);
  return (int)hipGetLastError();
}

extern "C" int jb_sparse_scan(const int32_t* qidx, const float* qval, int qn, float qnorm2,
                              const int64_t* row_ptr, const int32_t* ridx, const float* rval,
                              const float* rnorm2, const uint8_t* valid, int64_t nrows, int metric,
                              float* out, hipStream_t stream) {
  if (nrows <= 0) return 0;
  if (qn > jb::kMaxQuery) return -2;
  const int threads = 256;
  const unsigned blocks = (unsigned)((nrows + threads - 1) / threads);
  hipLaunchKernelGGL(jb::sparse_scan_kernel, dim3(blocks), dim3(threads), 0, stream, qidx, qval, qn,
                     qnorm2, row_ptr, ridx, rval, rnorm2, valid, nrows, metric, out);
  return (int)hipGetLastError();
}

extern "C" int jb_topk_direct_query(const uint64_t* qbits, const float* qnorm, int nq,
                                    const uint64_t* tbits, const float* tnorm,
                                    const uint8_t* valid, int64_t nrows, int words, int hash_num,
                                    int metric, int k, float* scratch_d, int32_t* scratch_i,
                                    float* out_d_host, int32_t* out_i_host, uint32_t* done_host,
                                    hipStream_t stream);

// Latency path of similar_row / neighbor_row (lsh family): the host-hashed
// query CSR (row_ptr[nq+1] host, idx / val host) rides in the kernel
// arguments of the signature kernel; the fused scan + top-k follows and its
// merge writes (distance, row) straight into pinned host memory. Three
// back-to-back launches, no copy, one host spin. Returns 1 when the query
// does not fit (nq > 8 or > 256 feature slots): the caller uses the batch path.
extern "C" int jb_lsh_query_direct(const int32_t* idx, const float* val, const int64_t* row_ptr,
                                   int nq, int hash_num, uint64_t seed, int mode, int metric,
                                   const uint64_t* tbits, const float* tnorm,
                                   const uint8_t* valid, int64_t nrows, int k,
                                   uint64_t* qbits_scratch, float* qnorm_scratch,
                                   float* scratch_d, int32_t* scratch_i, float* out_d_host,
                                   int32_t* out_i_host, uint32_t* done_host, hipStream_t stream) {
  if (nq <= 0 || nrows <= 0 || k <= 0) return 0;
  jb::QueryArgs a;
  if (jb::fill_query_args(&a, idx, val, row_ptr, nq, nullptr)) return 1;
  hipLaunchKernelGGL(jb::signature_query_kernel, dim3(nq), dim3(64), 0, stream, a, hash_num,
                     seed, mode, qbits_scratch, qnorm_scratch, (uint8_t*)nullptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return jb_topk_direct_query(qbits_scratch, qnorm_scratch, nq, tbits, tnorm, valid, nrows,
                              (hash_num + 63) / 64, hash_num, metric, k, scratch_d, scratch_i,
                              out_d_host, out_i_host, done_host, stream);
}

// set_row latency path: signatures of n host-hashed rows computed from the
// kernel arguments straight into their table slots (bits / norms / valid);
// asynchronous, no copy. Returns 1 when the rows do not fit (caller: bulk path).
extern "C" int jb_lsh_set_rows_direct(const int32_t* idx, const float* val, const int64_t* row_ptr,
                                      int n, const int64_t* slots, int hash_num, uint64_t seed,
                                      int mode, uint64_t* tbits, float* tnorm, uint8_t* valid,
                                      hipStream_t stream) {
  if (n <= 0) return 0;
  jb::QueryArgs a;
  if (jb::fill_query_args(&a, idx, val, row_ptr, n, slots)) return 1;
  hipLaunchKernelGGL(jb::signature_query_kernel, dim3(n), dim3(64), 0, stream, a, hash_num, seed,
                     mode, tbits, tnorm, valid);
  return (int)hipGetLastError();
}

// n table rows at once from a device CSR ([rp: n + 1][slots: n] int64, idx /
// val of rp[n] entries), each into its slot (distinct slots)
extern "C" int jb_lsh_set_rows_staged(const int64_t* rp, const int64_t* slots, const int32_t* idx, const float* val,
                                      int n, int hash_num, uint64_t seed, int mode, uint64_t* tbits, float* tnorm,
                                      uint8_t* valid, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(jb::signature_rows_kernel, dim3(n), dim3(64), 0, stream, rp, slots, idx, val, n, hash_num,
                     seed, mode, tbits, tnorm, valid);
  return (int)hipGetLastError();
}
