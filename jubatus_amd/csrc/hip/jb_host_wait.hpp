// Host-side completion wait for the latency paths (classify_direct.hip,
// lsh.hip): kernels publish a per-item flag (seq) into fine-grained pinned
// host memory after their results; the host spins on it (an interrupt-driven
// stream sync costs ~5 us more on MI355X) and falls back to a stream sync
// after ~2 ms, which also surfaces asynchronous launch errors.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <chrono>

namespace jb {

inline int wait_flags(volatile uint32_t* done, int n, uint32_t seq, hipStream_t stream) {
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

// as wait_flags, but a flag may also carry `mark` (seq | mark): reported
// through *marked (e.g. "retry on the exact path")
inline int wait_flags_status(volatile uint32_t* done, int n, uint32_t seq, uint32_t mark,
                             hipStream_t stream, bool* marked) {
  const auto t0 = std::chrono::steady_clock::now();
  *marked = false;
  for (int i = 0; i < n;) {
    const uint32_t v = done[i];
    if (v == seq || v == (seq | mark)) {
      *marked = *marked || v != seq;
      ++i;
      continue;
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
      const int rc = (int)hipStreamSynchronize(stream);
      if (rc != 0) return rc;
      for (int x = 0; x < n; ++x) *marked = *marked || done[x] != seq;
      return 0;
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return 0;
}

// spin until *flag != 0 (a kernel's final status store), then acquire
inline int wait_nonzero(volatile uint32_t* flag, hipStream_t stream) {
  const auto t0 = std::chrono::steady_clock::now();
  while (*flag == 0) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2))
      return (int)hipStreamSynchronize(stream);
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return 0;
}

inline uint32_t next_seq() {
  static std::atomic<uint32_t> g_seq{0};
  return g_seq.fetch_add(1, std::memory_order_relaxed) + 1;
}

}  // namespace jb
