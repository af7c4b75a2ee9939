// Native logger of the C++ servers, proxies and tools (reference C16,
// jubatus/server/common/logger/logger.{hpp,cpp}; flags and reload from
// framework/server_util.cpp:68-92,236-242 and server_helper.cpp:34-44).
//
//  * Line format "<date time> <pid> <LEVEL> [<tag>] <message>" on stderr, or
//    in the file a log configuration names (-g / --log_config): a JSON file
//    {"file": ..., "level": ...} or the reference's log4cxx XML (a file
//    appender's <param name="File" value="..."/> and <level value="..."/>).
//    The file name may use ${JUBATUS_PROCESS}, ${JUBATUS_HOST},
//    ${JUBATUS_PORT} and ${JUBATUS_PID} (log4cxx.xml:12-18). Python twin:
//    jubatus_amd/utils/logger.py.
//  * SIGHUP reloads the configuration and reopens the files (the servers'
//    sigwait loop calls reload()); in daemon mode (-D) SIGHUP is ignored.
//  * -l <logdir>: the coordination session's log goes to
//    <logdir>/<program>.<eth>_<port>.zklog.<pid> (the reference's ZooKeeper
//    log, server_helper.cpp:34-44).
#pragma once
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <fstream>
#include <mutex>
#include <sstream>
#include <string>

namespace jb {
namespace jlog {

enum Level : int { kTrace = 0, kDebug = 1, kInfo = 2, kWarn = 3, kError = 4, kFatal = 5 };

inline int level_of(const char* s) {
  if (!s) return kInfo;
  if (!strcasecmp(s, "TRACE")) return kTrace;
  if (!strcasecmp(s, "DEBUG")) return kDebug;
  if (!strcasecmp(s, "WARN") || !strcasecmp(s, "WARNING")) return kWarn;
  if (!strcasecmp(s, "ERROR")) return kError;
  if (!strcasecmp(s, "FATAL")) return kFatal;
  return kInfo;
}

struct Sink {
  std::mutex mu;
  FILE* fp = nullptr;        // nullptr: stderr
  FILE* zk = nullptr;        // coordination log (-l), nullptr: the main log
  int level = kInfo;
  std::string config;        // -g path ("" : stderr at INFO)
  std::string file;          // the file the configuration named
  std::string zk_path;
  bool daemon = false;
};
inline Sink& sink() {
  static Sink s;
  return s;
}

inline void write_line(FILE* f, const char* level, const char* tag, const char* msg) {
  char ts[32];
  time_t t = time(nullptr);
  struct tm tmv;
  localtime_r(&t, &tmv);
  strftime(ts, sizeof ts, "%Y-%m-%d %H:%M:%S", &tmv);
  fprintf(f, "%s %d %-5s [%s] %s\n", ts, (int)getpid(), level, tag, msg);
  fflush(f);
}

inline void write(const char* level, const char* tag, const char* msg) {
  Sink& s = sink();
  std::lock_guard<std::mutex> g(s.mu);
  if (level_of(level) < s.level) return;
  write_line(s.fp ? s.fp : stderr, level, tag, msg);
}

// the coordination session's log (the reference's ZooKeeper client log)
inline void zk(const char* level, const char* tag, const std::string& msg) {
  Sink& s = sink();
  std::lock_guard<std::mutex> g(s.mu);
  if (level_of(level) < s.level) return;
  write_line(s.zk ? s.zk : (s.fp ? s.fp : stderr), level, tag, msg.c_str());
}

inline void set_parameters(const std::string& prog, const std::string& host, int port) {
  const char* slash = strrchr(prog.c_str(), '/');
  setenv("JUBATUS_PROCESS", slash ? slash + 1 : prog.c_str(), 1);
  setenv("JUBATUS_HOST", host.c_str(), 1);
  setenv("JUBATUS_PORT", std::to_string(port).c_str(), 1);
  setenv("JUBATUS_PID", std::to_string((int)getpid()).c_str(), 1);
}

inline std::string expand(const std::string& in) {
  std::string out;
  size_t i = 0;
  while (i < in.size()) {
    if (in[i] == '$' && i + 1 < in.size() && in[i + 1] == '{') {
      const size_t e = in.find('}', i + 2);
      if (e != std::string::npos) {
        const char* v = getenv(in.substr(i + 2, e - i - 2).c_str());
        out += v ? v : "";
        i = e + 1;
        continue;
      }
    }
    out += in[i++];
  }
  return out;
}

// value of `attr="..."` in the first tag that starts with `open` and
// contains `must` (log4cxx XML)
inline std::string xml_attr(const std::string& text, const std::string& open, const std::string& must,
                            const std::string& attr) {
  size_t p = 0;
  while ((p = text.find(open, p)) != std::string::npos) {
    const size_t e = text.find('>', p);
    if (e == std::string::npos) break;
    const std::string tag = text.substr(p, e - p);
    p = e;
    if (!must.empty() && tag.find(must) == std::string::npos) continue;
    const size_t a = tag.find(attr + "=\"");
    if (a == std::string::npos) continue;
    const size_t b = a + attr.size() + 2;
    const size_t c = tag.find('"', b);
    if (c != std::string::npos) return tag.substr(b, c - b);
  }
  return "";
}
// value of "key": "..." (JSON configuration)
inline std::string json_str(const std::string& text, const std::string& key) {
  const size_t k = text.find("\"" + key + "\"");
  if (k == std::string::npos) return "";
  size_t c = text.find(':', k);
  if (c == std::string::npos) return "";
  const size_t a = text.find('"', c);
  if (a == std::string::npos) return "";
  const size_t b = text.find('"', a + 1);
  return b == std::string::npos ? "" : text.substr(a + 1, b - a - 1);
}

inline bool parse_config(const std::string& path, std::string* file, int* level, std::string* err) {
  std::ifstream f(path);
  if (!f) {
    *err = "cannot read log configuration " + path;
    return false;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string text = ss.str();
  std::string lv, fl;
  if (text.find('<') != std::string::npos) {
    fl = xml_attr(text, "<param", "\"File\"", "value");
    lv = xml_attr(text, "<level", "", "value");
  } else {
    fl = json_str(text, "file");
    lv = json_str(text, "level");
  }
  *file = fl.empty() ? "" : expand(fl);
  *level = lv.empty() ? kInfo : level_of(lv.c_str());
  return true;
}

// (re)configure from `config` ("" : stderr); false (with *err) if the
// configuration or its file cannot be used - the previous sink stays
inline bool configure(const std::string& config, std::string* err) {
  std::string file;
  int level = kInfo;
  if (!config.empty() && !parse_config(config, &file, &level, err)) return false;
  FILE* nf = nullptr;
  if (!file.empty()) {
    nf = fopen(file.c_str(), "a");
    if (!nf) {
      *err = "cannot open log file " + file;
      return false;
    }
  }
  Sink& s = sink();
  std::lock_guard<std::mutex> g(s.mu);
  if (s.fp) fclose(s.fp);
  s.fp = nf;
  s.level = level;
  s.config = config;
  s.file = file;
  if (!s.zk_path.empty()) {   // reopen the coordination log as well
    if (s.zk) fclose(s.zk);
    s.zk = fopen(s.zk_path.c_str(), "a");
  }
  return true;
}

// -l: the coordination log file
inline bool set_zk_log(const std::string& logdir, const std::string& prog, const std::string& eth,
                       int port, std::string* err) {
  const char* slash = strrchr(prog.c_str(), '/');
  const std::string path = logdir + "/" + (slash ? slash + 1 : prog.c_str()) + "." + eth + "_" +
                           std::to_string(port) + ".zklog." + std::to_string((int)getpid());
  FILE* f = fopen(path.c_str(), "a");
  if (!f) {
    *err = "cannot open coordination log " + path;
    return false;
  }
  Sink& s = sink();
  std::lock_guard<std::mutex> g(s.mu);
  if (s.zk) fclose(s.zk);
  s.zk = f;
  s.zk_path = path;
  return true;
}

// SIGHUP (not in daemon mode): reload the configuration
inline void reload(const char* tag) {
  std::string cfg, err;
  {
    Sink& s = sink();
    std::lock_guard<std::mutex> g(s.mu);
    cfg = s.config;
  }
  if (!cfg.empty()) write("INFO", tag, ("reloading log configuration: " + cfg).c_str());
  if (!configure(cfg, &err)) write("ERROR", tag, ("log reload failed: " + err).c_str());
  else if (!cfg.empty()) write("INFO", tag, ("log configuration reloaded: " + cfg).c_str());
}

}  // namespace jlog
}  // namespace jb
