// Native loader of fv_converter plug-ins ("method": "dynamic"): the servers
// and tools load them with dlopen, no Python on the way.
//
// Reference: jubatus/server/fv_converter/so_factory.cpp:41-106 (the six
// extension points, a factory symbol called with the type's other
// parameters) and dynamic_loader.cpp:44-94 (the library lookup and the
// version() log line). The ABI is the C one of csrc/plugins/jb_plugin.h (the
// Python twin is jubatus_amd/fv_converter/plugin.py). Lookup order of a
// "path": an absolute path or one that exists relative to the working
// directory, then $JUBATUS_PLUGIN_PATH/<path>, then the in-tree plug-in
// directory (jubatus_amd/plugins, found next to the executable's native_bin/).
#pragma once
#include <dlfcn.h>
#include <limits.h>
#include <stdio.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../plugins/jb_plugin.h"

namespace jb {
namespace plug {

inline bool file_exists(const std::string& p) {
  struct stat s;
  return stat(p.c_str(), &s) == 0 && S_ISREG(s.st_mode);
}

// the in-tree plug-in directory: <dir of the executable>/../plugins
// (jubatus_amd/native_bin/<tool> -> jubatus_amd/plugins); JUBATUS_AMD_PLUGIN_DIR overrides
inline std::string default_dir() {
  if (const char* e = getenv("JUBATUS_AMD_PLUGIN_DIR")) return e;
  char buf[PATH_MAX];
  const ssize_t n = readlink("/proc/self/exe", buf, sizeof(buf) - 1);
  if (n <= 0) return "";
  std::string exe(buf, (size_t)n);
  const size_t s = exe.rfind('/');
  if (s == std::string::npos) return "";
  return exe.substr(0, s) + "/../plugins";
}

// dynamic_loader.cpp:44-94 search order; "" when not found
inline std::string resolve(const std::string& path, std::string* searched) {
  if (path.empty()) return "";
  if (path[0] == '/' || file_exists(path)) return file_exists(path) ? path : "";
  std::vector<std::string> bases;
  if (const char* e = getenv("JUBATUS_PLUGIN_PATH"))
    if (*e) bases.push_back(e);
  bases.push_back(default_dir());
  for (const std::string& b : bases) {
    if (b.empty()) continue;
    if (searched) *searched += (searched->empty() ? "" : ", ") + b;
    const std::string c = b + "/" + path;
    if (file_exists(c)) return c;
  }
  return "";
}

enum Kind : int {
  kStringFeature = JB_STRING_FEATURE,
  kStringFilter = JB_STRING_FILTER,
  kNumFeature = JB_NUM_FEATURE,
  kNumFilter = JB_NUM_FILTER,
  kBinaryFeature = JB_BINARY_FEATURE,
  kCombination = JB_COMBINATION_FEATURE
};

inline const char* kind_name(int k) {
  switch (k) {
    case kStringFeature: return "string_feature";
    case kStringFilter: return "string_filter";
    case kNumFeature: return "num_feature";
    case kNumFilter: return "num_filter";
    case kBinaryFeature: return "binary_feature";
    case kCombination: return "combination_feature";
    default: return "?";
  }
}

// one loaded library (kept open for the process: plug-in instances point into it)
struct Library {
  void* h = nullptr;
  std::string path;
};

inline Library* open_library(const std::string& path) {
  static std::mutex mu;
  static std::map<std::string, std::unique_ptr<Library>> libs;
  std::string searched;
  const std::string found = resolve(path, &searched);
  if (found.empty())
    throw std::runtime_error("cannot load dynamic library: " + path + " (searched " +
                             (searched.empty() ? std::string("the working directory") : searched) + ")");
  char real[PATH_MAX];
  const std::string key = realpath(found.c_str(), real) ? std::string(real) : found;
  std::lock_guard<std::mutex> g(mu);
  auto it = libs.find(key);
  if (it != libs.end()) return it->second.get();
  void* h = dlopen(key.c_str(), RTLD_NOW | RTLD_LOCAL);
  if (!h) throw std::runtime_error("cannot load dynamic library: " + key + ": " + dlerror());
  using VerFn = const char* (*)();
  if (auto ver = (VerFn)dlsym(h, "version")) {
    const char* v = ver();
    fprintf(stderr, "plugin loaded: %s version: %s\n", key.c_str(), v ? v : "?");
  } else {
    fprintf(stderr, "plugin %s has no version() symbol\n", key.c_str());
  }
  auto lib = std::make_unique<Library>();
  lib->h = h;
  lib->path = key;
  Library* out = lib.get();
  libs.emplace(key, std::move(lib));
  return out;
}

// one plug-in instance; calls are serialised (a plug-in keeps its output
// buffers in the instance, as the reference's plug-ins may)
class Plugin {
 public:
  Plugin(const std::string& path, const std::string& function, int kind,
         const std::vector<std::pair<std::string, std::string>>& params)
      : kind_(kind) {
    if (path.empty() || function.empty())
      throw std::runtime_error(std::string("dynamic ") + kind_name(kind) + ": 'path' and 'function' are required");
    Library* lib = open_library(path);
    auto factory = (jb_plugin_factory)dlsym(lib->h, function.c_str());
    if (!factory) throw std::runtime_error("cannot find symbol " + function + " in " + path);
    std::vector<const char*> k, v;
    for (const auto& kv : params) {
      k.push_back(kv.first.c_str());
      v.push_back(kv.second.c_str());
    }
    p_ = factory(k.data(), v.data(), (int)k.size());
    if (!p_) throw std::runtime_error(function + " in " + path + " returned no plug-in");
    if (p_->abi != JB_PLUGIN_ABI) {
      destroy();
      throw std::runtime_error(function + ": plug-in ABI mismatch");
    }
    if (p_->kind != kind) {
      destroy();
      throw std::runtime_error(function + " is not a " + kind_name(kind) + " plug-in");
    }
  }
  ~Plugin() { destroy(); }
  Plugin(const Plugin&) = delete;
  Plugin& operator=(const Plugin&) = delete;

  int kind() const { return kind_; }

  // text -> tokens (the token bytes copied into *out)
  void split(const char* text, size_t len, std::vector<std::string>* out) {
    std::lock_guard<std::mutex> g(mu_);
    out->clear();
    int cap = 64;
    for (;;) {
      tok_.resize((size_t)cap);
      const int n = p_->string_feature(p_->self, text, (int64_t)len, tok_.data(), cap);
      if (n < 0) throw std::runtime_error("string_feature plug-in failed");
      if (n > cap) { cap = n; continue; }
      for (int i = 0; i < n; ++i) {
        const jb_token& t = tok_[(size_t)i];
        if (t.value) out->emplace_back(t.value, (size_t)t.value_len);
        else if (t.begin >= 0 && t.length >= 0 && (size_t)(t.begin + t.length) <= len)
          out->emplace_back(text + t.begin, (size_t)t.length);
        else throw std::runtime_error("string_feature plug-in: token out of range");
      }
      return;
    }
  }
  std::string filter_string(const char* in, size_t len) {
    std::lock_guard<std::mutex> g(mu_);
    int64_t cap = (int64_t)std::max<size_t>(64, 2 * len);
    for (;;) {
      buf_.resize((size_t)cap);
      const int64_t n = p_->string_filter(p_->self, in, (int64_t)len, buf_.data(), cap);
      if (n < 0) throw std::runtime_error("string_filter plug-in failed");
      if (n <= cap) return std::string(buf_.data(), (size_t)n);
      cap = n;
    }
  }
  double filter_num(double x) {
    std::lock_guard<std::mutex> g(mu_);
    return p_->num_filter(p_->self, x);
  }
  void num_feature(const std::string& key, double x, std::vector<std::pair<std::string, double>>* out) {
    std::lock_guard<std::mutex> g(mu_);
    named(out, [&](jb_named* b, int cap) { return p_->num_feature(p_->self, key.c_str(), x, b, cap); });
  }
  void binary_feature(const std::string& key, const char* data, size_t len,
                      std::vector<std::pair<std::string, double>>* out) {
    std::lock_guard<std::mutex> g(mu_);
    named(out, [&](jb_named* b, int cap) {
      return p_->binary_feature(p_->self, key.c_str(), data, (int64_t)len, b, cap);
    });
  }
  double combine(double a, double b) {
    std::lock_guard<std::mutex> g(mu_);
    return p_->combination(p_->self, a, b);
  }

 private:
  template <class F>
  void named(std::vector<std::pair<std::string, double>>* out, F call) {
    out->clear();
    int cap = 16;
    for (;;) {
      nam_.resize((size_t)cap);
      const int n = call(nam_.data(), cap);
      if (n < 0) throw std::runtime_error(std::string(kind_name(kind_)) + " plug-in failed");
      if (n > cap) { cap = n; continue; }
      for (int i = 0; i < n; ++i)
        out->emplace_back(nam_[(size_t)i].name ? nam_[(size_t)i].name : "", nam_[(size_t)i].value);
      return;
    }
  }
  void destroy() {
    if (p_ && p_->destroy) p_->destroy(p_->self);
    p_ = nullptr;
  }

  int kind_;
  jb_plugin* p_ = nullptr;
  std::mutex mu_;
  std::vector<jb_token> tok_;
  std::vector<char> buf_;
  std::vector<jb_named> nam_;
};

}  // namespace plug
}  // namespace jb
