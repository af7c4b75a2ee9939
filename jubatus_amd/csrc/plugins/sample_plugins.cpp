// Sample fv_converter plug-ins, one per extension point (the counterpart of
// the reference's test fixture plug-ins: splitter_sample, filter_sample,
// num_feature_sample, num_filter_sample, binary_feature_sample -
// jubatus/server/fv_converter/wscript:40-86). Built into
// jubatus_amd/plugins/libjubatus_sample_plugins.so by build_ext.
#include <cctype>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "jb_plugin.h"

namespace {

const char* param(const char** k, const char** v, int n, const char* key, const char* dflt) {
  for (int i = 0; i < n; ++i)
    if (std::strcmp(k[i], key) == 0) return v[i];
  return dflt;
}

struct Base {
  jb_plugin p{};
  std::vector<std::string> names;  // backing store of jb_named names
  virtual ~Base() = default;
};

void destroy(void* self) { delete static_cast<Base*>(self); }

Base* make(int kind) {
  Base* b = new Base();
  b->p.abi = JB_PLUGIN_ABI;
  b->p.kind = kind;
  b->p.self = b;
  b->p.destroy = destroy;
  return b;
}

// ---- string feature: split on a delimiter character (param "delimiter",
// default ' '); tokens shorter than "min_length" are dropped
struct Splitter : Base {
  char delim = ' ';
  int64_t min_len = 1;
};

int split(void* self, const char* text, int64_t len, jb_token* out, int cap) {
  auto* s = static_cast<Splitter*>(static_cast<Base*>(self));
  int n = 0;
  int64_t i = 0;
  while (i < len) {
    while (i < len && text[i] == s->delim) ++i;
    const int64_t b = i;
    while (i < len && text[i] != s->delim) ++i;
    if (i - b >= s->min_len) {
      if (n < cap) out[n] = jb_token{b, i - b, nullptr, 0, 1.0};
      ++n;
    }
  }
  return n;
}

// ---- string filter: upper-case ASCII
int64_t upper(void*, const char* in, int64_t len, char* out, int64_t cap) {
  for (int64_t i = 0; i < len && i < cap; ++i) out[i] = (char)std::toupper((unsigned char)in[i]);
  return len;
}

// ---- num filter: x * scale + shift
struct Affine : Base {
  double scale = 1.0, shift = 0.0;
};
double affine(void* self, double x) {
  auto* a = static_cast<Affine*>(static_cast<Base*>(self));
  return x * a->scale + a->shift;
}

// ---- num feature: bucketise x into "<key>@bucket<floor(x / width)>" = 1 and
// keep the raw value as "<key>@raw"
struct Bucket : Base {
  double width = 1.0;
};
int bucket(void* self, const char* key, double x, jb_named* out, int cap) {
  auto* b = static_cast<Bucket*>(static_cast<Base*>(self));
  b->names.clear();
  b->names.push_back(std::string(key) + "@bucket" + std::to_string((long long)std::floor(x / b->width)));
  b->names.push_back(std::string(key) + "@raw");
  if (cap >= 2) {
    out[0] = jb_named{b->names[0].c_str(), 1.0};
    out[1] = jb_named{b->names[1].c_str(), x};
  }
  return 2;
}

// ---- binary feature: histogram of byte values -> "b<byte>" = count
struct ByteHist : Base {};
int byte_hist(void* self, const char*, const char* data, int64_t len, jb_named* out, int cap) {
  auto* h = static_cast<ByteHist*>(static_cast<Base*>(self));
  int cnt[256] = {0};
  for (int64_t i = 0; i < len; ++i) cnt[(unsigned char)data[i]]++;
  h->names.clear();
  std::vector<double> vals;
  for (int c = 0; c < 256; ++c)
    if (cnt[c]) {
      h->names.push_back("b" + std::to_string(c));
      vals.push_back(cnt[c]);
    }
  const int n = (int)h->names.size();
  for (int i = 0; i < n && i < cap; ++i) out[i] = jb_named{h->names[i].c_str(), vals[i]};
  return n;
}

// ---- combination: max(left, right)
double comb_max(void*, double l, double r) { return l > r ? l : r; }

}  // namespace

extern "C" {

const char* version(void) { return "jubatus_amd-sample-plugins 1.0"; }

jb_plugin* create_splitter(const char** k, const char** v, int n) {
  auto* s = new Splitter();
  s->p = jb_plugin{JB_PLUGIN_ABI, JB_STRING_FEATURE, static_cast<Base*>(s), split, nullptr, nullptr,
                   nullptr, nullptr, nullptr, destroy};
  const char* d = param(k, v, n, "delimiter", " ");
  s->delim = d[0] ? d[0] : ' ';
  s->min_len = std::atoll(param(k, v, n, "min_length", "1"));
  s->p.string_feature = split;
  return &s->p;
}

jb_plugin* create_upper_filter(const char**, const char**, int) {
  Base* b = make(JB_STRING_FILTER);
  b->p.string_filter = upper;
  return &b->p;
}

jb_plugin* create_affine_filter(const char** k, const char** v, int n) {
  auto* a = new Affine();
  a->p = jb_plugin{JB_PLUGIN_ABI, JB_NUM_FILTER, static_cast<Base*>(a), nullptr, nullptr, nullptr, affine, nullptr,
                   nullptr, destroy};
  a->scale = std::atof(param(k, v, n, "scale", "1"));
  a->shift = std::atof(param(k, v, n, "shift", "0"));
  return &a->p;
}

jb_plugin* create_bucket_feature(const char** k, const char** v, int n) {
  auto* b = new Bucket();
  b->p = jb_plugin{JB_PLUGIN_ABI, JB_NUM_FEATURE, static_cast<Base*>(b), nullptr, nullptr, bucket, nullptr, nullptr,
                   nullptr, destroy};
  b->width = std::atof(param(k, v, n, "width", "1"));
  if (!(b->width > 0)) b->width = 1.0;
  return &b->p;
}

jb_plugin* create_byte_histogram(const char**, const char**, int) {
  auto* h = new ByteHist();
  h->p = jb_plugin{JB_PLUGIN_ABI, JB_BINARY_FEATURE, static_cast<Base*>(h), nullptr, nullptr, nullptr, nullptr,
                   byte_hist, nullptr, destroy};
  return &h->p;
}

jb_plugin* create_max_combination(const char**, const char**, int) {
  Base* b = make(JB_COMBINATION_FEATURE);
  b->p.combination = comb_max;
  return &b->p;
}

}  // extern "C"
