// Low-latency classify: one fused launch per classify RPC.
//
// Reference: classifier_serv::classify (jubatus/server/server/classifier_serv.cpp:149-173),
// called once per RPC with a short list of datums; its latency is the
// "p50 classify latency" half of the headline metric (BASELINE.json).
//
// The batch path (fv_hash -> linear_classify) needs ~6 H2D descriptor copies,
// two launches and a D2H copy: ~100 us of queue round trips for a request of
// one datum. Here the whole request rides in the *kernel arguments*: the
// descriptors and the raw msgpack bytes of up to kDirectMaxSamples datums
// (kDirectArgBytes in total) are copied by the host into the kernarg block,
// which the command processor delivers with the dispatch packet. One wave per
// datum stages its bytes into LDS, lane 0 parses and hashes the features into
// LDS, then the wave gathers the W rows of those features (HBM) and writes
// the LC scores straight into fine-grained pinned host memory. The host waits
// for that single dispatch by spinning on per-datum completion flags the
// kernel publishes after its scores. No copy engine, no second launch.
//
// Requests that do not fit the kernarg block take the batch path.
#include "jb_fv.hpp"
#include "jb_linear.hpp"

#include <atomic>
#include <chrono>
#include <cstring>

namespace jb {

constexpr int kDirectMaxSamples = 32;
constexpr int kDirectArgBytes = 2816;
constexpr int kDirectMaxSlots = 1024;   // feature slots per datum held in LDS

struct alignas(16) DirectArgs {
  int32_t n;
  int32_t nbytes;
  int32_t pad[2];
  int32_t off[kDirectMaxSamples];       // datum byte offset in `bytes`
  int32_t len[kDirectMaxSamples];
  int32_t slot[kDirectMaxSamples + 1];  // CSR slot pointer (relative)
  int32_t pad2[3];
  uint8_t bytes[kDirectArgBytes];
};
static_assert(sizeof(DirectArgs) <= 3584, "kernarg block too large");

template <int LC>
__global__ __launch_bounds__(64) void classify_direct_kernel(
    const DirectArgs a, const GpuRule* __restrict__ srules, int n_srules,
    const GpuRule* __restrict__ nrules, int n_nrules, const uint8_t* __restrict__ blob, uint64_t H,
    const float* W, float* __restrict__ out, int32_t* __restrict__ err,
    volatile uint32_t* __restrict__ done, uint32_t seq) {
  using L = Lanes<LC>;
  __shared__ __attribute__((aligned(16))) uint8_t s_bytes[kDirectArgBytes];
  __shared__ int32_t s_idx[kDirectMaxSlots];
  __shared__ float s_val[kDirectMaxSlots];
  __shared__ int s_ok;
  const int lane = threadIdx.x;
  const int s = blockIdx.x;
  if (s >= a.n) return;
  const int off = a.off[s], len = a.len[s];
  const int nslots = a.slot[s + 1] - a.slot[s];
  // stage this datum's bytes (kernarg -> LDS), 16-B aligned window
  const int lo = off & ~15;
  const int hi = (off + len + 15) & ~15;
  for (int b = lo + lane * 16; b < hi; b += 64 * 16)
    *reinterpret_cast<uint4*>(&s_bytes[b]) = *reinterpret_cast<const uint4*>(&a.bytes[b]);
  __syncthreads();
  if (lane == 0) {
    Reader rd{&s_bytes[off], &s_bytes[off] + len, true};
    s_ok = emit_datum(rd, 0, nslots, srules, n_srules, nrules, n_nrules, blob, H, s_idx, s_val);
  }
  __syncthreads();
  if (s_ok) {
    float acc[L::K];
    sample_scores<LC>(s_idx, s_val, 0, nslots, W, lane, acc);
    if (lane < L::LW) {
#pragma unroll
      for (int k = 0; k < L::K; ++k) out[(int64_t)s * LC + lane + 64 * k] = acc[k];
    }
  } else if (lane == 0) {
    *err = 2;
  }
  // completion flag of this datum, published after the scores at system
  // scope: the host spins on it instead of a stream synchronisation
  __threadfence_system();
  if (lane == 0) done[s] = seq;
}

}  // namespace jb

// Returns 0 on success (scores in out_host[n*LC], err_host[0] != 0 on a parse
// error), 1 when the request does not fit the direct path (caller uses the
// batch path), <0 / HIP error code otherwise. Blocks until the scores landed.
extern "C" int jb_classify_direct(const uint8_t* bytes, int64_t nbytes, const int64_t* datum_off,
                                  const int32_t* datum_len, const int64_t* row_ptr, int n,
                                  const void* srules, int n_srules, const void* nrules,
                                  int n_nrules, const uint8_t* blob, uint64_t H, const float* W,
                                  int LC, float* out_host, int32_t* err_host,
                                  uint32_t* done_host, hipStream_t stream) {
  if (n <= 0) return 0;
  if (n > jb::kDirectMaxSamples || nbytes > jb::kDirectArgBytes) return 1;
  jb::DirectArgs a;
  a.n = n;
  a.nbytes = (int32_t)nbytes;
  a.slot[0] = 0;
  for (int i = 0; i < n; ++i) {
    const int64_t ns = row_ptr[i + 1] - row_ptr[i];
    if (ns > jb::kDirectMaxSlots || datum_off[i] < 0 || datum_off[i] + datum_len[i] > nbytes)
      return 1;
    a.off[i] = (int32_t)datum_off[i];
    a.len[i] = datum_len[i];
    a.slot[i + 1] = (int32_t)(row_ptr[i + 1] - row_ptr[0]);
  }
  std::memcpy(a.bytes, bytes, (size_t)nbytes);
  *err_host = 0;
  static std::atomic<uint32_t> g_seq{0};
  const uint32_t seq = g_seq.fetch_add(1, std::memory_order_relaxed) + 1;
#define JB_DIRECT(L)                                                                       \
  hipLaunchKernelGGL((jb::classify_direct_kernel<L>), dim3(n), dim3(64), 0, stream, a,    \
                     (const jb::GpuRule*)srules, n_srules, (const jb::GpuRule*)nrules,     \
                     n_nrules, blob, H, W, out_host, err_host, done_host, seq);
  JB_LC_DISPATCH(LC, JB_DIRECT)
#undef JB_DIRECT
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  // spin on the per-datum completion flags (a blocking stream sync costs an
  // interrupt + wakeup); after ~2 ms of spinning fall back to the sync,
  // which also surfaces any asynchronous launch error
  volatile uint32_t* done = done_host;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n;) {
    if (done[i] == seq) { ++i; continue; }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2))
      return (int)hipStreamSynchronize(stream);
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return 0;
}

// Fine-grained (coherent) pinned host memory the GPU writes into directly.
extern "C" void* jb_host_alloc(int64_t nbytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, (size_t)nbytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
    return nullptr;
  return p;
}

extern "C" int jb_host_free(void* p) { return (int)hipHostFree(p); }
