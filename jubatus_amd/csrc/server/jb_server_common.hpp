// Common parts of the native engine servers (csrc/server/juba*.cpp): the
// reference's server flags (framework/server_util.cpp:146-225), the
// fixed-slot GPU converter rule tables (fv_converter/gpu_path.py), the model
// file container (framework/save_load.py, reference framework/save_load.cpp),
// device / pinned buffers and the hand-over to the Python server.
//
// Every server names itself once (set_engine) before anything else runs.
#pragma once
#include "jb_coord_client.hpp"
#include <arpa/inet.h>
#include <errno.h>
#include <fcntl.h>
#include <getopt.h>
#include <ifaddrs.h>
#include <limits.h>
#include <math.h>
#include <netinet/in.h>
#include <pwd.h>
#include <signal.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/file.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <vector>

#include "jb_hash.hpp"
#include "jb_hostfv.hpp"
#include "jb_value.hpp"

namespace jb {
namespace srv {

using jb::val::MsgpackReader;
using jb::val::MsgpackWriter;
using jb::val::Value;

inline std::string& engine_ref() {
  static std::string e;
  return e;
}
inline std::string& prog_ref() {
  static std::string p;
  return p;
}
inline void set_engine(const char* e) {
  engine_ref() = e;
  prog_ref() = std::string("juba") + e;
}
inline const char* engine_name() { return engine_ref().c_str(); }
inline const char* prog_name() { return prog_ref().c_str(); }

inline const char* const kVersion = "0.9.2";
const uint32_t kVersionParts[3] = {0, 9, 2};
constexpr int kArgumentError = 2, kNoMethodError = 1;

#define HIPCHK(x)                                                                    \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess)                                                            \
      throw std::runtime_error(std::string(#x) + ": " + hipGetErrorString(e_));      \
  } while (0)

void logf_(const char* level, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline void logf_(const char* level, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  jb::jlog::write(level, prog_name(), buf);
}

// ------------------------------------------------------------------ argv
struct Args {
  int port = 9199;
  std::string listen_addr, listen_if, bind = "0.0.0.0", eth;
  int threads = 2, timeout = 10, zk_timeout = 10, ic_timeout = 10;
  bool daemon = false, version = false, cpu = false;
  bool native_check = false;   // print whether the config is served natively, exit
  std::string logdir, log_config, datadir = "/tmp", configpath, model_file, zookeeper, name,
      mixer = "linear_mixer";
  int interval_sec = 16, interval_count = 512;
  int gpu = -1;
  std::string connected_zookeeper;   // distributed mode: the coordinator in use
};

inline std::string real_path(const std::string& p) {
  char buf[PATH_MAX];
  return realpath(p.c_str(), buf) ? std::string(buf) : p;
}

inline std::string default_v4() {
  std::string out = "127.0.0.1";
  struct ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) != 0) return out;
  for (auto* p = ifa; p; p = p->ifa_next) {
    if (!p->ifa_addr || p->ifa_addr->sa_family != AF_INET) continue;
    char b[INET_ADDRSTRLEN];
    inet_ntop(AF_INET, &((struct sockaddr_in*)p->ifa_addr)->sin_addr, b, sizeof b);
    if (strncmp(b, "127.", 4) != 0) { out = b; break; }
  }
  freeifaddrs(ifa);
  return out;
}

inline std::string if_v4(const std::string& nic) {
  std::string out;
  struct ifaddrs* ifa = nullptr;
  if (getifaddrs(&ifa) != 0) return out;
  for (auto* p = ifa; p; p = p->ifa_next)
    if (p->ifa_addr && p->ifa_addr->sa_family == AF_INET && nic == p->ifa_name) {
      char b[INET_ADDRSTRLEN];
      inet_ntop(AF_INET, &((struct sockaddr_in*)p->ifa_addr)->sin_addr, b, sizeof b);
      out = b;
      break;
    }
  freeifaddrs(ifa);
  return out;
}

inline std::string user_name() {
  struct passwd* pw = getpwuid(getuid());
  return pw ? std::string(pw->pw_name) : std::to_string(getuid());
}

inline const char* const kUsageFlags =
    "[-p port] [-b listen_addr] [-B listen_if] [-c thread] [-t timeout]\n"
    "                      [-d datadir] [-l logdir] [-g log_config] [-f configpath]\n"
    "                      [-m model_file] [-z zookeeper] [-n name] [-x mixer] [-s interval_sec]\n"
    "                      [-i interval_count] [-Z zookeeper_timeout] [-I interconnect_timeout]\n"
    "                      [-D] [-v] [--gpu N] [--cpu]\n";

inline void usage(FILE* f) { fprintf(f, "usage: %s %s", prog_name(), kUsageFlags); }

// 0 ok, >0 exit code
inline int parse_args(int argc, char** argv, Args* a) {
  static const struct option opts[] = {
      {"rpc-port", required_argument, nullptr, 'p'}, {"listen_addr", required_argument, nullptr, 'b'},
      {"listen_if", required_argument, nullptr, 'B'}, {"thread", required_argument, nullptr, 'c'},
      {"timeout", required_argument, nullptr, 't'}, {"zookeeper_timeout", required_argument, nullptr, 'Z'},
      {"interconnect_timeout", required_argument, nullptr, 'I'}, {"daemon", no_argument, nullptr, 'D'},
      {"logdir", required_argument, nullptr, 'l'}, {"log_config", required_argument, nullptr, 'g'},
      {"version", no_argument, nullptr, 'v'}, {"datadir", required_argument, nullptr, 'd'},
      {"configpath", required_argument, nullptr, 'f'}, {"model_file", required_argument, nullptr, 'm'},
      {"zookeeper", required_argument, nullptr, 'z'}, {"name", required_argument, nullptr, 'n'},
      {"mixer", required_argument, nullptr, 'x'}, {"interval_sec", required_argument, nullptr, 's'},
      {"interval_count", required_argument, nullptr, 'i'}, {"gpu", required_argument, nullptr, 1000},
      {"cpu", no_argument, nullptr, 1001}, {"help", no_argument, nullptr, 'h'},
      {"native-check", no_argument, nullptr, 1002},
      {nullptr, 0, nullptr, 0}};
  auto num = [](const char* s, long lo, long hi, int* out) {
    char* e = nullptr;
    long v = strtol(s, &e, 10);
    if (!*s || *e || v < lo || v > hi) return false;
    *out = (int)v;
    return true;
  };
  int c;
  optind = 1;
  while ((c = getopt_long(argc, argv, "p:b:B:c:t:Z:I:Dl:g:vd:f:m:z:n:x:s:i:h", opts, nullptr)) != -1) {
    bool ok = true;
    switch (c) {
      case 'p': ok = num(optarg, 1, 65535, &a->port); break;
      case 'b': a->listen_addr = optarg; break;
      case 'B': a->listen_if = optarg; break;
      case 'c': ok = num(optarg, 1, INT_MAX, &a->threads); break;
      case 't': ok = num(optarg, 0, INT_MAX, &a->timeout); break;
      case 'Z': ok = num(optarg, INT_MIN, INT_MAX, &a->zk_timeout); break;
      case 'I': ok = num(optarg, INT_MIN, INT_MAX, &a->ic_timeout); break;
      case 'D': a->daemon = true; break;
      case 'l': a->logdir = optarg; break;
      case 'g': a->log_config = optarg; break;
      case 'v': a->version = true; break;
      case 'd': a->datadir = optarg; break;
      case 'f': a->configpath = optarg; break;
      case 'm': a->model_file = optarg; break;
      case 'z': a->zookeeper = optarg; break;
      case 'n': a->name = optarg; break;
      case 'x': a->mixer = optarg; break;
      case 's': ok = num(optarg, 0, INT_MAX, &a->interval_sec); break;
      case 'i': ok = num(optarg, 0, INT_MAX, &a->interval_count); break;
      case 1000: ok = num(optarg, 0, 1023, &a->gpu); break;
      case 1001: a->cpu = true; break;
      case 1002: a->native_check = true; break;
      case 'h': usage(stdout); return -1;
      default: ok = false;
    }
    if (!ok) {
      usage(stderr);
      return 2;
    }
  }
  if (optind < argc) {
    usage(stderr);
    return 2;
  }
  return 0;
}

// ---------------------------------------------------------------- config
struct Rules {
  std::vector<jb::HostRule> s, n;
  std::string blob;
  uint64_t H = 1ull << 20;
};

// Feature-table height of the GPU linear models (classifier, regression)
// when the configuration gives no hash_max_size (JUBATUS_DEVICE_HASH_BITS=24:
// AROW at 64 labels is 8 GiB of W + P on a 288 GB device). Python twin:
// fv_converter/converter.py device_hash_max_size (both servers pick the same
// height, so their model files interchange).
inline uint64_t device_hash_max_size() {
  // one default on every backend (the host servers' 2^20): a model file saved
  // by a GPU server loads on a --cpu one and back, and mixed members agree on
  // the height; JUBATUS_DEVICE_HASH_BITS opts into an HBM-sized table (rows
  // are int32 feature indices, so at most 2^31)
  int bits = 20;
  if (const char* e = getenv("JUBATUS_DEVICE_HASH_BITS")) {
    const int b = atoi(e);
    if (b >= 10 && b <= 31) bits = b;
  }
  return 1ull << bits;
}

inline int matcher_kind(const std::string& spec, std::string* arg) {
  if (spec.empty() || spec == "*") { arg->clear(); return 0; }
  if (spec.size() >= 2 && spec.front() == '/' && spec.back() == '/') return -1;   // regex
  if (spec.back() == '*') { *arg = spec.substr(0, spec.size() - 1); return 1; }
  if (spec.front() == '*') { *arg = spec.substr(1); return 2; }
  *arg = spec;
  return 3;
}

inline bool nonempty_list(const Value& conv, const char* key) {
  const Value* v = conv.get(key);
  return v && v->kind == Value::ARR && !v->a.empty();
}

// the fixed-slot GPU converter (fv_converter/gpu_path.py fast_eligible +
// GpuRuleTable): false with a reason when the config needs the host converter
inline bool build_rules(const Value& conv, Rules* r, std::string* why) {
  if (conv.kind != Value::MAP) { *why = "converter is not an object"; return false; }
  for (const char* k : {"string_filter_rules", "num_filter_rules", "binary_rules", "combination_rules"})
    if (nonempty_list(conv, k)) { *why = std::string(k) + " need the host converter"; return false; }
  const Value* st = conv.get("string_types");
  const Value* nt = conv.get("num_types");
  if (const Value* h = conv.get("hash_max_size")) {
    if (h->kind == Value::INT && h->i > 0) r->H = (uint64_t)h->i;
    else if (h->kind != Value::NIL) { *why = "hash_max_size"; return false; }
  }
  auto put = [&](const std::string& b, int32_t* off, int32_t* len) {
    *off = (int32_t)r->blob.size();
    *len = (int32_t)b.size();
    r->blob += b;
  };
  if (const Value* sr = conv.get("string_rules")) {
    if (sr->kind != Value::ARR) { *why = "string_rules"; return false; }
    for (const Value& x : sr->a) {
      const std::string type = x.str_or("type", "");
      const std::string sw = x.str_or("sample_weight", "bin");
      const std::string gw = x.str_or("global_weight", "bin");
      if (type != "str" || (st && st->get("str"))) { *why = "string type " + type; return false; }
      if (gw != "bin") { *why = "global_weight " + gw; return false; }
      float w;
      if (sw == "bin" || sw == "tf") w = 1.f;
      else if (sw == "log_tf") w = logf(2.f);
      else { *why = "sample_weight " + sw; return false; }
      std::string arg;
      const int kind = matcher_kind(x.str_or("key", ""), &arg);
      if (kind < 0) { *why = "regex key matcher"; return false; }
      jb::HostRule h{};
      h.match_kind = kind;
      put(arg, &h.match_off, &h.match_len);
      put("@str#" + sw + "/" + gw, &h.suffix_off, &h.suffix_len);
      h.weight = w;
      r->s.push_back(h);
    }
  }
  if (const Value* nr = conv.get("num_rules")) {
    if (nr->kind != Value::ARR) { *why = "num_rules"; return false; }
    for (const Value& x : nr->a) {
      const std::string type = x.str_or("type", "");
      if ((type != "num" && type != "log") || (nt && nt->get(type))) { *why = "num type " + type; return false; }
      std::string arg;
      const int kind = matcher_kind(x.str_or("key", ""), &arg);
      if (kind < 0) { *why = "regex key matcher"; return false; }
      jb::HostRule h{};
      h.match_kind = kind;
      put(arg, &h.match_off, &h.match_len);
      put("@" + type, &h.suffix_off, &h.suffix_len);
      h.value_kind = type == "log" ? 1 : 0;
      r->n.push_back(h);
    }
  }
  return true;
}

inline bool read_file(const std::string& path, std::string* out) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) return false;
  char buf[1 << 16];
  size_t n;
  out->clear();
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out->append(buf, n);
  fclose(f);
  return true;
}

// ------------------------------------------------------------ model file
// framework/save_load.py: 48-byte big-endian header, CRC32 over header[0:28]
// ++ header[32:48] ++ system ++ user; system = [1, ts, type, id, config]
// (old-spec raw strings), user = [1, driver pack] (bin types).
inline uint64_t rd_be(const uint8_t* p, int n) {
  uint64_t x = 0;
  for (int k = 0; k < n; ++k) x = (x << 8) | p[k];
  return x;
}

inline void wr_be(uint8_t* p, uint64_t x, int n) {
  for (int k = n - 1; k >= 0; --k) { p[k] = (uint8_t)x; x >>= 8; }
}

struct ModelFile {
  std::string type, id, config;
  Value user;      // the driver pack
  int64_t user_version = 0;
};

inline std::string read_model_file(const std::string& bytes, ModelFile* mf) {
  if (bytes.size() < 48) return "failed to read header: truncated file";
  const uint8_t* h = (const uint8_t*)bytes.data();
  if (memcmp(h, "jubatus\0", 8) != 0) return "invalid file format";
  if (rd_be(h + 8, 8) != 1) return "invalid format version: " + std::to_string(rd_be(h + 8, 8)) + ", expected 1";
  const uint32_t maj = (uint32_t)rd_be(h + 16, 4), min = (uint32_t)rd_be(h + 20, 4),
                 mnt = (uint32_t)rd_be(h + 24, 4);
  if (maj != kVersionParts[0] || min != kVersionParts[1] || mnt != kVersionParts[2])
    return std::string("jubatus version mismatched: current version: ") + kVersion +
           ", saved version: " + std::to_string(maj) + "." + std::to_string(min) + "." + std::to_string(mnt);
  const uint32_t crc = (uint32_t)rd_be(h + 28, 4);
  const uint64_t ssz = rd_be(h + 32, 8), usz = rd_be(h + 40, 8);
  if (bytes.size() < 48 + ssz + usz || ssz > bytes.size() || usz > bytes.size()) return "model file truncated";
  uint32_t c = jb::crc32_update(0, h, 28);
  c = jb::crc32_update(c, h + 32, 16);
  c = jb::crc32_update(c, h + 48, ssz);
  c = jb::crc32_update(c, h + 48 + ssz, usz);
  if (c != crc) {
    char b[96];
    snprintf(b, sizeof b, "invalid crc32 checksum: %#x, read %#x", c, crc);
    return b;
  }
  try {
    Value sys = MsgpackReader(h + 48, ssz).read();
    Value usr = MsgpackReader(h + 48 + ssz, usz).read();
    if (sys.kind != Value::ARR || sys.a.size() != 5) return "invalid system data";
    if (usr.kind != Value::ARR || usr.a.size() != 2) return "invalid user data";
    if (sys.a[0].kind != Value::INT || sys.a[0].i != 1)
      return "invalid system data version: saved version: " + std::to_string(sys.a[0].i) + ", expected version: 1";
    mf->type = sys.a[2].s;
    mf->id = sys.a[3].s;
    mf->config = sys.a[4].s;
    mf->user_version = usr.a[0].kind == Value::INT ? usr.a[0].i : -1;
    mf->user = std::move(usr.a[1]);
  } catch (const std::exception& e) {
    return std::string("broken model data: ") + e.what();
  }
  return "";
}

// --------------------------------------------------------------- buffers
template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t cap = 0;
  T* get(size_t n) {
    if (n > cap) {
      if (p) HIPCHK(hipFree(p));
      size_t c = cap ? cap : 1024;
      while (c < n) c *= 2;
      HIPCHK(hipMalloc((void**)&p, c * sizeof(T)));
      cap = c;
    }
    return p;
  }
};

template <class T>
struct PinBuf {   // page-locked host memory (H2D staging)
  T* p = nullptr;
  size_t cap = 0;
  T* get(size_t n) {
    if (n > cap) {
      if (p) HIPCHK(hipHostFree(p));
      size_t c = cap ? cap : 1024;
      while (c < n) c *= 2;
      HIPCHK(hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault));
      cap = c;
    }
    return p;
  }
};

inline uint64_t fnv1a64(const std::string& s) {
  return jb::fnv_bytes(jb::kFnvOffset, (const uint8_t*)s.data(), s.size());
}

// element count of a body's top-level array header (-1: none)
inline int64_t body_count(const uint8_t* b, uint64_t n) {
  if (n < 1) return -1;
  const uint8_t t = b[0];
  if ((t & 0xf0) == 0x90) return t & 0x0f;
  if (t == 0xdc && n >= 3) return ((int64_t)b[1] << 8) | b[2];
  if (t == 0xdd && n >= 5) return (int64_t)rd_be(b + 1, 4);
  return -1;
}

// hand the server to the Python implementation (before any HIP call)
[[noreturn]] inline void exec_python(int argc, char** argv, const char* why) {
  fprintf(stderr, "%s: %s: starting the Python server\n", prog_name(), why);
  char exe[PATH_MAX];
  ssize_t n = readlink("/proc/self/exe", exe, sizeof exe - 1);
  std::string root = ".";
  if (n > 0) {
    exe[n] = 0;
    std::string p(exe);   // <root>/jubatus_amd/native_bin/juba<engine>
    for (int k = 0; k < 3; ++k) p = p.substr(0, p.rfind('/'));
    root = p;
  }
  const char* pp = getenv("PYTHONPATH");
  std::string path = root + (pp && *pp ? std::string(":") + pp : std::string());
  setenv("PYTHONPATH", path.c_str(), 1);
  std::vector<char*> av;
  static char py[] = "python3", m[] = "-m", mod[] = "jubatus_amd.cmd.server";
  static std::string eng;
  eng = engine_name();
  av.push_back(py);
  av.push_back(m);
  av.push_back(mod);
  av.push_back(&eng[0]);
  for (int k = 1; k < argc; ++k) av.push_back(argv[k]);
  av.push_back(nullptr);
  execvp("python3", av.data());
  perror("execvp python3");
  _exit(127);
}


// write a model file (the container of read_model_file); throws on error
inline void write_model_file(const std::string& path, const std::string& type, const std::string& id,
                             const std::string& config, const std::string& user) {
  const int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) throw std::runtime_error("cannot open output file: " + path + ": " + strerror(errno));
  if (flock(fd, LOCK_EX | LOCK_NB) != 0) {
    close(fd);
    throw std::runtime_error("cannot get the lock of file; any RPC is saving to same file?: " + path);
  }
  MsgpackWriter sys;
  sys.arr(5);
  sys.uint(1);
  sys.uint((uint64_t)time(nullptr));
  sys.raw(type);
  sys.raw(id);
  sys.raw(config);
  uint8_t head[48];
  memcpy(head, "jubatus\0", 8);
  wr_be(head + 8, 1, 8);
  for (int k = 0; k < 3; ++k) wr_be(head + 16 + 4 * k, kVersionParts[k], 4);
  wr_be(head + 28, 0, 4);
  wr_be(head + 32, sys.out.size(), 8);
  wr_be(head + 40, user.size(), 8);
  uint32_t c = jb::crc32_update(0, head, 28);
  c = jb::crc32_update(c, head + 32, 16);
  c = jb::crc32_update(c, (const uint8_t*)sys.out.data(), sys.out.size());
  c = jb::crc32_update(c, (const uint8_t*)user.data(), user.size());
  wr_be(head + 28, c, 4);
  auto write_all = [fd](const void* p, size_t n) {
    const char* q = (const char*)p;
    while (n) {
      ssize_t w = write(fd, q, n);
      if (w <= 0) {
        if (w < 0 && errno == EINTR) continue;
        return false;
      }
      q += w;
      n -= (size_t)w;
    }
    return true;
  };
  const bool ok = write_all(head, 48) && write_all(sys.out.data(), sys.out.size()) &&
                  write_all(user.data(), user.size());
  close(fd);
  if (!ok) {
    unlink(path.c_str());
    throw std::runtime_error("cannot write output file: " + path);
  }
}

// the status keys every server reports (framework/server_helper.py get_status)
struct CommonStatus {
  time_t start_time = 0, last_saved = 0, last_loaded = 0;
  std::string last_saved_path, last_loaded_path;
};

// the engines whose requests route by consistent hashing (the reference's
// server_helper<...>(a, true): anomaly, bandit, burst, graph,
// nearest_neighbor, recommender and stat *_impl.cpp:20)
inline bool engine_uses_cht() {
  static const char* const kCht[] = {"jubaanomaly", "jubabandit", "jubaburst", "jubagraph",
                                     "jubanearest_neighbor", "jubarecommender", "jubastat"};
  std::string n = prog_name();
  const size_t s = n.rfind('/');
  if (s != std::string::npos) n = n.substr(s + 1);
  for (const char* k : kCht)
    if (n == k) return true;
  return false;
}

inline void common_status(const Args& a, const CommonStatus& cs, uint64_t update_count,
                          std::vector<std::pair<std::string, std::string>>* st) {
  const time_t now = time(nullptr);
  long vsz = 0, rss = 0, shr = 0;
  if (FILE* f = fopen("/proc/self/statm", "r")) {
    if (fscanf(f, "%ld %ld %ld", &vsz, &rss, &shr) != 3) vsz = rss = shr = 0;
    fclose(f);
  }
  const long kb = sysconf(_SC_PAGESIZE) / 1024;
  auto add = [&](const char* k, const std::string& v) { st->emplace_back(k, v); };
  add("clock_time", std::to_string(now));
  add("start_time", std::to_string(cs.start_time));
  add("uptime", std::to_string(now - cs.start_time));
  add("VIRT", std::to_string(vsz * kb));
  add("RSS", std::to_string(rss * kb));
  add("SHR", std::to_string(shr * kb));
  add("timeout", std::to_string(a.timeout));
  add("threadnum", std::to_string(a.threads));
  add("datadir", a.datadir);
  add("is_standalone", a.zookeeper.empty() ? "1" : "0");
  add("VERSION", kVersion);
  add("PROGNAME", prog_name());
  add("type", engine_name());
  add("logdir", a.logdir);
  add("log_config", a.log_config);
  add("configpath",
      a.zookeeper.empty() ? a.configpath : std::string("/jubatus/config/") + engine_name() + "/" + a.name);
  add("pid", std::to_string(getpid()));
  add("user", user_name());
  add("update_count", std::to_string(update_count));
  add("last_saved", std::to_string(cs.last_saved));
  add("last_saved_path", cs.last_saved_path);
  add("last_loaded", std::to_string(cs.last_loaded));
  add("last_loaded_path", cs.last_loaded_path);
  add("gpu", a.gpu >= 0 ? std::to_string(a.gpu) : std::string());
  if (!a.zookeeper.empty()) {   // distributed mode (server_helper.py get_status)
    add("zk", a.zookeeper);
    add("name", a.name);
    add("interval_sec", std::to_string(a.interval_sec));
    add("interval_count", std::to_string(a.interval_count));
    add("zookeeper_timeout", std::to_string(a.zk_timeout));
    add("interconnect_timeout", std::to_string(a.ic_timeout));
    add("connected_zookeeper", a.connected_zookeeper);
    add("use_cht", engine_uses_cht() ? "1" : "0");
    add("mixer", a.mixer);
  }
}

// Startup shared by the servers, before any GPU call: flags, the decision
// native vs Python (exec), paths, addresses and the configuration text
// (the model file's wins over -f, server_helper.hpp). Returns -1 to go on,
// otherwise the exit code. check(text, why) says whether the config is
// served natively; --native-check prints that decision and exits.
// config text of a distributed server: /jubatus/config/<engine>/<name> on
// the coordinator (server_util.py get_conf); false when absent/unreachable
inline bool config_from_coordinator(const Args& a, std::string* text, std::string* why) {
  try {
    jb::cc::Coord c(a.zookeeper, std::max(1, a.zk_timeout), "config");
    const bool ok = c.read(std::string("/jubatus/config/") + engine_name() + "/" + a.name, text);
    c.close();
    if (!ok) *why = std::string("config is not found: /jubatus/config/") + engine_name() + "/" + a.name;
    return ok;
  } catch (const std::exception& e) {
    *why = e.what();
    return false;
  }
}

// native_dist: the engine serves distributed mode (-z) natively with the
// linear mixer (csrc/native/jb_mix_group.hpp); other mixers and engines are
// handed to the Python server
// host_ok: the engine serves on a GPU-less host natively (its host backend);
// otherwise --cpu / no /dev/kfd hand the configuration to the Python server
template <class Check>
int startup(int argc, char** argv, Args* a, std::string* text, Check check, bool needs_gpu = true,
            bool native_dist = false, bool native_push = false, bool host_ok = false) {
  int rc = parse_args(argc, argv, a);
  if (rc == -1) return 0;
  if (rc) return rc;
  if (a->version) {
    printf("jubatus-%s (mi355x, native)\n", kVersion);
    return 0;
  }
  const char* force = a->native_check ? nullptr : getenv("JUBATUS_NATIVE_SERVER");
  if (force && strcmp(force, "0") == 0) exec_python(argc, argv, "JUBATUS_NATIVE_SERVER=0");
  const bool dist = !a->zookeeper.empty();
  if (!a->native_check) {
    if (dist && !native_dist) exec_python(argc, argv, "distributed mode");
    const bool push = a->mixer == "random_mixer" || a->mixer == "broadcast_mixer" || a->mixer == "skip_mixer";
    if (dist && a->mixer != "linear_mixer" && !(push && native_push))
      exec_python(argc, argv, "distributed mode with a push mixer");
    if (needs_gpu && !host_ok && (a->cpu || getenv("JUBATUS_FORCE_CPU")))
      exec_python(argc, argv, "host backend requested");
    if (needs_gpu && !host_ok && access("/dev/kfd", R_OK | W_OK) != 0) exec_python(argc, argv, "no GPU (/dev/kfd)");
  }
  if (dist && a->name.empty()) {
    fprintf(stderr, "can't start multinode mode without name specified\n");
    usage(stderr);
    return 1;
  }
  if (!dist && a->configpath.empty() && a->model_file.empty()) {
    fprintf(stderr, "config path or model file must be specified for standalone mode\n");
    usage(stderr);
    return 1;
  }
  if (!a->configpath.empty()) a->configpath = real_path(a->configpath);
  if (!a->model_file.empty()) a->model_file = real_path(a->model_file);
  if (!a->datadir.empty()) {
    a->datadir = real_path(a->datadir);
    if (access(a->datadir.c_str(), W_OK) != 0) {
      fprintf(stderr, "can't use datadir: %s\n", a->datadir.c_str());
      usage(stderr);
      return 1;
    }
  }
  if (!a->listen_addr.empty()) {
    a->bind = a->eth = a->listen_addr;
  } else if (!a->listen_if.empty()) {
    a->bind = a->eth = if_v4(a->listen_if);
  } else {
    a->eth = default_v4();
  }
  if (!a->native_check) {
    // logging (server_util.cpp:236-242,305-311; server_helper.cpp:34-44)
    std::string err;
    if (!a->logdir.empty()) {
      a->logdir = real_path(a->logdir);
      if (access(a->logdir.c_str(), W_OK) != 0) {
        fprintf(stderr, "can't create log file in logdir: %s\n", a->logdir.c_str());
        usage(stderr);
        return 1;
      }
    }
    if (!a->log_config.empty()) a->log_config = real_path(a->log_config);
    jb::jlog::set_parameters(prog_name(), a->eth, a->port);
    if (!jb::jlog::configure(a->log_config, &err)) {
      fprintf(stderr, "failed to configure logger: %s\n", err.c_str());
      exit(1);
    }
    if (dist && !a->logdir.empty() && !jb::jlog::set_zk_log(a->logdir, prog_name(), a->eth, a->port, &err)) {
      fprintf(stderr, "%s\n", err.c_str());
      exit(1);
    }
    if (a->daemon) {
      // daemon mode keeps the process in the foreground and ignores SIGHUP
      // (server_util.cpp:379-388)
      if (a->logdir.empty() && a->log_config.empty() && isatty(fileno(stderr)))
        logf_("WARN", "logs may be lost because started in daemon mode without log directory");
      jb::jlog::sink().daemon = true;
      logf_("INFO", "set daemon mode (SIGHUP is now ignored)");
    }
  }
  if (dist) {
    std::string why;
    if (!config_from_coordinator(*a, text, &why)) {
      if (a->native_check) {
        printf("python: %s\n", why.c_str());
        return 0;
      }
      fprintf(stderr, "%s: %s\n", prog_name(), why.c_str());
      return 1;
    }
  } else if (!a->model_file.empty()) {
    // the reference rejects what it cannot load and exits
    // (server_helper.hpp:81-113: load_file throws; save_load.cpp:169-285)
    std::string bytes;
    ModelFile mf;
    if (!read_file(a->model_file, &bytes)) {
      fprintf(stderr, "%s: cannot open input file: %s: %s\n", prog_name(), a->model_file.c_str(), strerror(errno));
      return 1;
    }
    const std::string err = read_model_file(bytes, &mf);
    if (!err.empty()) {
      fprintf(stderr, "%s: %s: %s\n", prog_name(), a->model_file.c_str(), err.c_str());
      return 1;
    }
    *text = mf.config;
  } else if (!read_file(a->configpath, text)) {
    // config.cpp:39-48 config_fromlocal: "can't read <path> ."
    fprintf(stderr, "%s: can't read %s .\n", prog_name(), a->configpath.c_str());
    return 1;
  }
  std::string why;
  if (a->native_check) {   // the config check alone (tests, operators): no GPU, no exec
    const bool ok = check(*text, &why);
    printf("%s\n", ok ? "native" : ("python: " + why).c_str());
    return 0;
  }
  if (!check(*text, &why)) exec_python(argc, argv, why.c_str());
  return -1;
}

// block the signals the main thread waits on (every thread inherits it)
inline void block_signals() {
  sigset_t set;
  sigemptyset(&set);
  sigaddset(&set, SIGTERM);
  sigaddset(&set, SIGINT);
  sigaddset(&set, SIGHUP);
  pthread_sigmask(SIG_BLOCK, &set, nullptr);
  signal(SIGPIPE, SIG_IGN);
}

// the HIP device of this process (--gpu, else LOCAL_RANK); blocks the signals
inline int device_and_signals(const Args& a) {
  int device = a.gpu;
  if (device < 0) {
    const char* lr = getenv("LOCAL_RANK");
    device = lr ? atoi(lr) : 0;
  }
  block_signals();
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (ndev <= 0) throw std::runtime_error("no HIP device");
  return device % ndev;
}

// the main thread's signal loop (signals.cpp:98-181): TERM / INT return (the
// caller shuts down), HUP reloads the log configuration unless in daemon mode
inline void wait_for_term() {
  sigset_t set;
  sigemptyset(&set);
  sigaddset(&set, SIGTERM);
  sigaddset(&set, SIGINT);
  sigaddset(&set, SIGHUP);
  int sig = 0;
  while (true) {
    if (sigwait(&set, &sig) != 0) continue;
    if (sig == SIGTERM || sig == SIGINT) return;
    if (sig == SIGHUP && !jb::jlog::sink().daemon) jb::jlog::reload(prog_name());
  }
}

}  // namespace srv
}  // namespace jb
