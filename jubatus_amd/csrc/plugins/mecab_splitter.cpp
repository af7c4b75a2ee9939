// MeCab morphological splitter plug-in (string_feature).
//
// Reference: plugin/src/fv_converter/mecab_splitter.cpp:49-225 - parameters
//   arg               MeCab tagger arguments (e.g. "-d /path/to/dic")
//   ngram             n of the word n-grams (positive, default 1)
//   base              "true": use the base form (7th CSV field of the node
//                     feature, the surface when it is "*"), "false": surface
//   include_features  '|'-separated key matchers over the node feature CSV
//                     (default "*"); exclude_features likewise (default none)
// Each emitted token is the n words joined by ',' with the byte span of the
// n surfaces in the input and weight 1.0.
//
// MeCab is not linked at build time: the plug-in binds libmecab's C API
// (mecab.h) with dlopen at create() - parameter "libmecab" or env
// JUBATUS_MECAB_LIB, else "libmecab.so.2" - so it builds everywhere and
// fails with a clear error where MeCab is not installed.
#include <dlfcn.h>

#include <cstdio>
#include <cstring>
#include <regex>
#include <string>
#include <vector>

#include "jb_plugin.h"

namespace {

// ---- the parts of MeCab's C ABI used here (mecab.h, MeCab 0.99x)
struct mecab_node_t {
  mecab_node_t* prev;
  mecab_node_t* next;
  mecab_node_t* enext;
  mecab_node_t* bnext;
  void* rpath;
  void* lpath;
  const char* surface;
  const char* feature;
  unsigned int id;
  unsigned short length;
  unsigned short rlength;
  unsigned short rcAttr;
  unsigned short lcAttr;
  unsigned short posid;
  unsigned char char_type;
  unsigned char stat;
  unsigned char isbest;
  float alpha;
  float beta;
  float prob;
  short wcost;
  long cost;
};
enum { MECAB_BOS_NODE = 2, MECAB_EOS_NODE = 3 };

struct MecabApi {
  void* lib = nullptr;
  void* (*model_new2)(const char*) = nullptr;
  void (*model_destroy)(void*) = nullptr;
  void* (*model_new_tagger)(void*) = nullptr;
  void* (*model_new_lattice)(void*) = nullptr;
  void (*destroy)(void*) = nullptr;
  void (*lattice_destroy)(void*) = nullptr;
  void (*lattice_set_sentence2)(void*, const char*, size_t) = nullptr;
  int (*parse_lattice)(void*, void*) = nullptr;
  const mecab_node_t* (*lattice_get_bos_node)(void*) = nullptr;
  const char* (*strerror)(void*) = nullptr;

  bool load(const char* path, std::string* err) {
    lib = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!lib) { *err = std::string("cannot load libmecab (") + path + "): " + dlerror(); return false; }
    bool ok = true;
    auto sym = [&](const char* n) {
      void* p = dlsym(lib, n);
      if (!p) { ok = false; *err = std::string("libmecab lacks ") + n; }
      return p;
    };
    model_new2 = (void* (*)(const char*))sym("mecab_model_new2");
    model_destroy = (void (*)(void*))sym("mecab_model_destroy");
    model_new_tagger = (void* (*)(void*))sym("mecab_model_new_tagger");
    model_new_lattice = (void* (*)(void*))sym("mecab_model_new_lattice");
    destroy = (void (*)(void*))sym("mecab_destroy");
    lattice_destroy = (void (*)(void*))sym("mecab_lattice_destroy");
    lattice_set_sentence2 = (void (*)(void*, const char*, size_t))sym("mecab_lattice_set_sentence2");
    parse_lattice = (int (*)(void*, void*))sym("mecab_parse_lattice");
    lattice_get_bos_node = (const mecab_node_t* (*)(void*))sym("mecab_lattice_get_bos_node");
    strerror = (const char* (*)(void*))sym("mecab_strerror");
    return ok;
  }
};

// Jubatus key matcher over a feature string: "*", "prefix*", "*suffix",
// "/regex/", exact
struct Matcher {
  int kind = 0;   // 0 all, 1 prefix, 2 suffix, 3 exact, 4 regex
  std::string arg;
  std::regex re;
  explicit Matcher(const std::string& s) {
    if (s == "*" || s.empty()) { kind = 0; }
    else if (s.size() >= 2 && s.front() == '/' && s.back() == '/') {
      kind = 4;
      arg = s.substr(1, s.size() - 2);
      re = std::regex(arg);
    }
    else if (s.back() == '*') { kind = 1; arg = s.substr(0, s.size() - 1); }
    else if (s.front() == '*') { kind = 2; arg = s.substr(1); }
    else { kind = 3; arg = s; }
  }
  bool match(const std::string& f) const {
    switch (kind) {
      case 0: return true;
      case 1: return f.compare(0, arg.size(), arg) == 0;
      case 2: return f.size() >= arg.size() && f.compare(f.size() - arg.size(), arg.size(), arg) == 0;
      case 3: return f == arg;
      default: return std::regex_search(f, re);
    }
  }
};

std::vector<Matcher> matchers(const std::string& spec) {
  std::vector<Matcher> out;
  size_t s = 0;
  while (s <= spec.size()) {
    size_t e = spec.find('|', s);
    if (e == std::string::npos) e = spec.size();
    out.emplace_back(spec.substr(s, e - s));
    s = e + 1;
  }
  return out;
}

struct Mecab {
  jb_plugin p{};
  MecabApi api;
  void* model = nullptr;
  size_t ngram = 1;
  bool base = false;
  std::vector<Matcher> include, exclude;
  std::vector<std::string> values;   // token strings of the last call

  ~Mecab() {
    if (model) api.model_destroy(model);
    if (api.lib) dlclose(api.lib);
  }

  bool included(const std::string& f) const {
    bool in = false;
    for (const auto& m : include) if (m.match(f)) { in = true; break; }
    if (!in) return false;
    for (const auto& m : exclude) if (m.match(f)) return false;
    return true;
  }
};

int split(void* self, const char* text, int64_t len, jb_token* out, int cap) {
  Mecab* m = static_cast<Mecab*>(self);
  void* tagger = m->api.model_new_tagger(m->model);
  if (!tagger) return 0;
  void* lattice = m->api.model_new_lattice(m->model);
  if (!lattice) { m->api.destroy(tagger); return 0; }
  m->api.lattice_set_sentence2(lattice, text, (size_t)len);
  struct Word { std::string w; size_t begin, length; };
  std::vector<Word> words;
  if (m->api.parse_lattice(tagger, lattice)) {
    size_t p = 0;
    for (const mecab_node_t* n = m->api.lattice_get_bos_node(lattice); n; n = n->next) {
      if (n->stat == MECAB_BOS_NODE || n->stat == MECAB_EOS_NODE) continue;
      p += n->rlength - n->length;            // leading white space of the node
      const std::string feature = n->feature ? n->feature : "";
      if (m->included(feature)) {
        std::string w;
        if (m->base) {
          size_t b = 0;
          for (int i = 0; i < 6 && b != std::string::npos; ++i) {
            b = feature.find(',', b);
            if (b != std::string::npos) ++b;
          }
          if (b != std::string::npos) {
            const size_t e = feature.find(',', b);
            w = feature.substr(b, e == std::string::npos ? std::string::npos : e - b);
          }
          if (w.empty() || w == "*") w.assign(text + p, n->length);
        } else {
          w.assign(text + p, n->length);
        }
        words.push_back({w, p, n->length});
      }
      p += n->length;
    }
  }
  m->api.lattice_destroy(lattice);
  m->api.destroy(tagger);
  if (words.size() < m->ngram) return 0;
  const size_t nf = words.size() - m->ngram + 1;
  m->values.assign(nf, std::string());
  for (size_t i = 0; i < nf; ++i) {
    std::string& f = m->values[i];
    f = words[i].w;
    size_t length = words[i].length;
    for (size_t j = 1; j < m->ngram; ++j) {
      f += "," + words[i + j].w;
      length += words[i + j].length;
    }
    if ((int)i < cap)
      out[i] = jb_token{(int64_t)words[i].begin, (int64_t)length, f.data(), (int64_t)f.size(), 1.0};
  }
  return (int)nf;
}

void destroy(void* self) { delete static_cast<Mecab*>(self); }

}  // namespace

extern "C" {

const char* version(void) { return "jubatus_amd-mecab-splitter 1.0"; }

jb_plugin* create(const char** keys, const char** values, int n) {
  std::string arg, ngram = "1", base = "false", inc = "*", exc, lib;
  for (int i = 0; i < n; ++i) {
    const std::string k = keys[i];
    if (k == "arg") arg = values[i];
    else if (k == "ngram") ngram = values[i];
    else if (k == "base") base = values[i];
    else if (k == "include_features") inc = values[i];
    else if (k == "exclude_features") exc = values[i];
    else if (k == "libmecab") lib = values[i];
  }
  char* end = nullptr;
  const long ng = std::strtol(ngram.c_str(), &end, 10);
  if (!end || *end || ng <= 0) {
    std::fprintf(stderr, "mecab_splitter: ngram must be a positive number\n");
    return nullptr;
  }
  if (base != "true" && base != "false") {
    std::fprintf(stderr, "mecab_splitter: base must be a boolean value\n");
    return nullptr;
  }
  if (inc.empty()) { std::fprintf(stderr, "mecab_splitter: include_features must not be empty\n"); return nullptr; }
  if (lib.empty()) {
    const char* env = std::getenv("JUBATUS_MECAB_LIB");
    lib = env && *env ? env : "libmecab.so.2";
  }
  Mecab* m = new Mecab();
  std::string err;
  try {
    m->include = matchers(inc);
    if (!exc.empty()) m->exclude = matchers(exc);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "mecab_splitter: bad feature matcher: %s\n", e.what());
    delete m;
    return nullptr;
  }
  if (!m->api.load(lib.c_str(), &err)) {
    std::fprintf(stderr, "mecab_splitter: %s\n", err.c_str());
    delete m;
    return nullptr;
  }
  m->model = m->api.model_new2(arg.c_str());
  if (!m->model) {
    std::fprintf(stderr, "mecab_splitter: cannot make mecab tagger: %s\n", m->api.strerror(nullptr));
    delete m;
    return nullptr;
  }
  m->ngram = (size_t)ng;
  m->base = base == "true";
  m->p = jb_plugin{JB_PLUGIN_ABI, JB_STRING_FEATURE, m, split, nullptr, nullptr, nullptr, nullptr,
                   nullptr, destroy};
  return &m->p;
}

}  // extern "C"
