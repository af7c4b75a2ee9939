// roctx ranges around the native hot paths, behind a switch (SURVEY section
// 5.1: per-RPC and per-kernel-group trace spans next to the reference's MIX
// timing log, linear_mixer.cpp:538-543).
//
// JUBATUS_ROCTX=1 loads the ROCm marker library at the first range
// (librocprofiler-sdk-roctx, dlopen: no link-time dependency, nothing loaded
// when the switch is off); `rocprofv3 --marker-trace` then records the ranges
// beside the kernel dispatches. Off (the default) a range costs one branch on
// a cached flag.
//
//   { jb::tx::Range r("rpc.batch.train"); ... }     // push / pop on this thread
//   jb::tx::mark("mix.begin");
#pragma once
#include <dlfcn.h>
#include <stdlib.h>

#include <atomic>

namespace jb {
namespace tx {

struct Api {
  int (*push)(const char*) = nullptr;
  int (*pop)() = nullptr;
  void (*mark)(const char*) = nullptr;
  bool on = false;
};

inline const Api& api() {
  static const Api a = [] {
    Api r;
    const char* e = getenv("JUBATUS_ROCTX");
    if (e == nullptr || e[0] != '1') return r;
    void* h = dlopen("librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) h = dlopen("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) h = dlopen("libroctx64.so.4", RTLD_NOW | RTLD_GLOBAL);
    if (h == nullptr) return r;
    r.push = (int (*)(const char*))dlsym(h, "roctxRangePushA");
    r.pop = (int (*)())dlsym(h, "roctxRangePop");
    r.mark = (void (*)(const char*))dlsym(h, "roctxMarkA");
    r.on = r.push != nullptr && r.pop != nullptr;
    return r;
  }();
  return a;
}

inline bool enabled() { return api().on; }

inline void mark(const char* what) {
  const Api& a = api();
  if (a.on && a.mark != nullptr) a.mark(what);
}

class Range {
 public:
  explicit Range(const char* what) : on_(api().on) {
    if (on_) api().push(what);
  }
  ~Range() {
    if (on_) api().pop();
  }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;

 private:
  bool on_;
};

}  // namespace tx
}  // namespace jb
