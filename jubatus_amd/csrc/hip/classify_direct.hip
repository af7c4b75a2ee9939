// Low-latency classify: one launch per classify RPC, no copies.
//
// Reference: classifier_serv::classify (jubatus/server/server/classifier_serv.cpp:149-173),
// called once per RPC with a short list of datums; its latency is the
// "p50 classify latency" half of the headline metric (BASELINE.json).
//
// The batch path (host scan -> H2D copies -> fv_hash -> linear_classify ->
// D2H) costs ~100 us of queue round trips for a request of one datum. For a
// small request the feature hashing is ~0.3 us of host work
// (csrc/native/jb_hostfv.hpp, bit-identical to the GPU emitter), so the
// (idx, val) pairs of up to kDirectMaxSlots features ride in the *kernel
// arguments*, delivered with the dispatch packet. One wave per datum gathers
// the W rows of its features from HBM and writes the LC scores straight
// into fine-grained pinned host memory, then publishes a per-datum
// completion flag; the host spins on the flags (an empty launch + spin is
// ~7 us on MI355X, a blocking stream sync adds ~5 us of interrupt wakeup).
// Requests that do not fit take the batch path.
#include "jb_host_wait.hpp"
#include "jb_linear.hpp"

#include <atomic>
#include <chrono>
#include <cstring>

namespace jb {

constexpr int kDirectMaxSamples = 32;
constexpr int kDirectMaxSlots = 320;

struct alignas(16) DirectArgs {
  int32_t n;
  int32_t slot[kDirectMaxSamples + 1];   // CSR row pointer
  int32_t pad[2];
  int32_t idx[kDirectMaxSlots];
  float val[kDirectMaxSlots];
};
static_assert(sizeof(DirectArgs) <= 3072, "kernarg block too large");

template <int LC, typename WT>
__global__ __launch_bounds__(64) void classify_direct_kernel(const DirectArgs a, const WT* W,
                                                             float* __restrict__ out,
                                                             volatile uint32_t* __restrict__ done,
                                                             uint32_t seq) {
  using L = Lanes<LC>;
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  if (s >= a.n) return;
  const int beg = a.slot[s];
  const int n = a.slot[s + 1] - beg;
  const int g = lane / L::LW;
  const int l0 = lane % L::LW;
  float acc[L::K];
#pragma unroll
  for (int k = 0; k < L::K; ++k) acc[k] = 0.f;
  // 4 features per lane group in flight: the W row loads of one datum are
  // independent HBM round trips, issue them together
  for (int j0 = g; j0 < n; j0 += 4 * L::G) {
    int32_t id[4];
    float x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int j = j0 + u * L::G;
      id[u] = j < n ? a.idx[beg + j] : -1;
      x[u] = j < n ? a.val[beg + j] : 0.f;
    }
    float w[4][L::K];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < L::K; ++k)
        w[u][k] = id[u] >= 0 ? ldw(W + (int64_t)id[u] * LC + l0 + 64 * k) : 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < L::K; ++k) acc[k] += x[u] * w[u][k];
  }
#pragma unroll
  for (int off = L::LW; off < 64; off <<= 1) {
#pragma unroll
    for (int k = 0; k < L::K; ++k) acc[k] += __shfl_xor(acc[k], off, 64);
  }
  // scores into the pinned host buffer by system-scope stores, then the
  // completion flag once this wave's stores are acknowledged (one wave per
  // datum). A system-scope release fence would write back the whole L2
  // instead, a cost that follows how much of it is dirty (the 18-28 us
  // spread of classify over RPC between boxes)
  if (lane < L::LW) {
#pragma unroll
    for (int k = 0; k < L::K; ++k) sys_store(out + (int64_t)s * LC + lane + 64 * k, acc[k]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) sys_store(const_cast<uint32_t*>(done) + s, seq);
}

__global__ void empty_flag_kernel(volatile uint32_t* done, uint32_t seq) {
  if (threadIdx.x == 0) sys_store(const_cast<uint32_t*>(done), seq);
}

}  // namespace jb

// Scores of n hashed datums (host CSR: row_ptr[n+1], idx/val) into
// out_host[n*LC]. Returns 0 on success, 1 when the request does not fit the
// direct path (caller uses the batch path), a HIP error code otherwise.
// Blocks until the scores landed.
template <typename WT>
static int classify_direct_impl(const int32_t* idx, const float* val, const int64_t* row_ptr,
                                int n, const WT* W, int LC, float* out_host,
                                uint32_t* done_host, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > jb::kDirectMaxSamples || row_ptr[n] - row_ptr[0] > jb::kDirectMaxSlots) return 1;
  jb::DirectArgs a;
  a.n = n;
  const int64_t base = row_ptr[0];
  for (int i = 0; i <= n; ++i) a.slot[i] = (int32_t)(row_ptr[i] - base);
  const int ns = a.slot[n];
  std::memcpy(a.idx, idx + base, sizeof(int32_t) * (size_t)ns);
  std::memcpy(a.val, val + base, sizeof(float) * (size_t)ns);
  const uint32_t seq = jb::next_seq();
#define JB_DIRECT(L)                                                                           \
  hipLaunchKernelGGL((jb::classify_direct_kernel<L, WT>), dim3(n), dim3(64), 0, stream, a, W, \
                     out_host, done_host, seq);
  JB_LC_DISPATCH(LC, JB_DIRECT)
#undef JB_DIRECT
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return jb::wait_flags(done_host, n, seq, stream);
}

extern "C" int jb_classify_direct(const int32_t* idx, const float* val, const int64_t* row_ptr,
                                  int n, const float* W, int LC, float* out_host,
                                  uint32_t* done_host, hipStream_t stream) {
  return classify_direct_impl<float>(idx, val, row_ptr, n, W, LC, out_host, done_host, stream);
}

// the same over a bf16 W table
extern "C" int jb_classify_direct_bf16(const int32_t* idx, const float* val,
                                       const int64_t* row_ptr, int n, const jb::bf16_t* W, int LC,
                                       float* out_host, uint32_t* done_host, hipStream_t stream) {
  return classify_direct_impl<jb::bf16_t>(idx, val, row_ptr, n, W, LC, out_host, done_host,
                                          stream);
}

// Launch-latency probe: one empty kernel that publishes a flag, then wait by
// spinning (spin=1) or by stream synchronisation (spin=0).
extern "C" int jb_diag_empty(uint32_t* done_host, int spin, hipStream_t stream) {
  const uint32_t seq = jb::next_seq();
  hipLaunchKernelGGL(jb::empty_flag_kernel, dim3(1), dim3(64), 0, stream, done_host, seq);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  if (!spin) return (int)hipStreamSynchronize(stream);
  return jb::wait_flags(done_host, 1, seq, stream);
}

// Fine-grained (coherent) pinned host memory the GPU writes into directly.
extern "C" void* jb_host_alloc(int64_t nbytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, (size_t)nbytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return nullptr;
  return p;
}

extern "C" int jb_host_free(void* p) { return (int)hipHostFree(p); }
