// The wide converter's rule table built from a config's "converter" object
// in C++ (the twin of fv_converter/gpu_path.py wide_eligible + WideRuleTable):
// str / space / ngram splitters, bin / tf / log_tf sample weights, bin / idf /
// bm25 global weights, num / log rules, add / mul combinations. Shared by the
// native row-engine servers (jb_row_engine.hpp) and jubaweight.
#pragma once
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "jb_hostfv.hpp"
#include "jb_hostfv_wide.hpp"
#include "jb_value.hpp"

namespace jb {
namespace row {

using jb::val::Value;

// ---------------------------------------------------------------- converter
inline int as_int(const Value* v, int dflt) {
  if (!v) return dflt;
  if (v->is_num()) return (int)v->num();
  if (v->is_str()) return atoi(v->s.c_str());
  return dflt;
}

// Python's str() of a float (the shortest repr that reads back, ".0" on integers)
inline std::string py_float_str(double x) {
  if (std::isnan(x)) return "nan";
  if (std::isinf(x)) return x > 0 ? "inf" : "-inf";
  char b[64];
  for (int prec = 1; prec <= 17; ++prec) {
    snprintf(b, sizeof(b), "%.*g", prec, x);
    if (strtod(b, nullptr) == x) break;
  }
  std::string out = b;
  if (out.find_first_of(".en") == std::string::npos) out += ".0";
  return out;
}

// the parameters a "dynamic" type hands its plug-in factory: every key but
// "method", "path" and "function", values as strings (converter.py _params)
inline std::vector<std::pair<std::string, std::string>> plugin_params(const Value& t) {
  std::vector<std::pair<std::string, std::string>> out;
  if (t.kind != Value::MAP) return out;
  for (const auto& kv : t.o) {
    if (kv.first == "method" || kv.first == "path" || kv.first == "function") continue;
    const Value& v = kv.second;
    std::string sv;
    if (v.is_str()) sv = v.s;
    else if (v.kind == Value::INT) sv = std::to_string(v.i);
    else if (v.kind == Value::UINT) sv = std::to_string((unsigned long long)v.num());
    else if (v.is_num()) sv = py_float_str(v.num());
    else if (v.kind == Value::BOOL) sv = v.b ? "True" : "False";
    else continue;
    out.emplace_back(kv.first, sv);
  }
  return out;
}

// a "dynamic" type's plug-in (so_factory.cpp:41-106): loaded now, so a bad
// path / symbol / kind fails the configuration as the reference's does
inline int load_plugin(WideExt* ext, const Value& t, int kind, std::string* why) {
  try {
    return ext->add_plugin(std::make_unique<plug::Plugin>(t.str_or("path", ""), t.str_or("function", ""), kind,
                                                          plugin_params(t)));
  } catch (const std::exception& e) {
    *why = e.what();
    return -1;
  }
}

inline double as_double(const Value* v, double dflt, bool* ok) {
  if (!v) { *ok = false; return dflt; }
  if (v->is_num()) return v->num();
  if (v->is_str()) {
    char* end = nullptr;
    const double d = strtod(v->s.c_str(), &end);
    if (end && *end == 0 && !v->s.empty()) return d;
  }
  *ok = false;
  return dflt;
}

// fv_converter/gpu_path.py wide_eligible + WideRuleTable; with `ext` also the
// "dynamic" plug-in types, the filter rules (plug-in string filters; add /
// linear / gaussian / sigmoid / plug-in num filters), the binary rules and
// the add / str num types - the rest of the converter but regular
// expressions, which stay with the Python converter (its re semantics)
inline bool build_wide_rules(const Value& conv, std::vector<HostRule>* s, std::vector<HostRule>* n,
                             std::vector<HostRule>* c, std::string* blob, uint64_t* H, bool* global,
                             std::string* why, std::shared_ptr<WideExt>* ext_out = nullptr) {
  if (conv.kind != Value::MAP) { *why = "converter is not an object"; return false; }
  auto ext = std::make_shared<WideExt>();
  if (!ext_out) {
    for (const char* k : {"string_filter_rules", "num_filter_rules", "binary_rules"})
      if (jb::srv::nonempty_list(conv, k)) { *why = std::string(k) + " need the host converter"; return false; }
  }
  auto put_ext = [&](const std::string& b, HostRule* h) {
    h->match_off = (int32_t)ext->blob.size();
    h->match_len = (int32_t)b.size();
    ext->blob += b;
  };
  if (ext_out) {
    // string filters: plug-ins (regexp filters need Python's re)
    std::map<std::string, int> sft;
    if (const Value* t = conv.get("string_filter_types")) {
      if (t->kind != Value::MAP) { *why = "string_filter_types"; return false; }
      for (const auto& kv : t->o) {
        const std::string m = kv.second.str_or("method", "");
        if (m != "dynamic") { *why = "string filter method " + m; return false; }
        const int p = load_plugin(ext.get(), kv.second, plug::kStringFilter, why);
        if (p < 0) return false;
        sft[kv.first] = p;
      }
    }
    if (const Value* r = conv.get("string_filter_rules")) {
      if (r->kind != Value::ARR) { *why = "string_filter_rules"; return false; }
      for (const Value& x : r->a) {
        auto it = sft.find(x.str_or("type", ""));
        if (it == sft.end()) { *why = "unknown string filter type: " + x.str_or("type", ""); return false; }
        WideExt::Filter f;
        std::string arg;
        f.m.match_kind = jb::srv::matcher_kind(x.str_or("key", ""), &arg);
        if (f.m.match_kind < 0) { *why = "regex key matcher"; return false; }
        put_ext(arg, &f.m);
        f.suffix = x.str_or("suffix", "");
        f.plug = it->second;
        ext->sf.push_back(f);
      }
    }
    // num filters
    std::map<std::string, WideExt::Filter> nft;
    if (const Value* t = conv.get("num_filter_types")) {
      if (t->kind != Value::MAP) { *why = "num_filter_types"; return false; }
      for (const auto& kv : t->o) {
        const std::string m = kv.second.str_or("method", "");
        WideExt::Filter f;
        bool ok = true;
        if (m == "add") {
          f.kind = WideExt::kAdd;
          f.a = as_double(kv.second.get("value"), 0, &ok);
        } else if (m == "linear_normalization") {
          f.kind = WideExt::kLinear;
          f.a = as_double(kv.second.get("min"), 0, &ok);
          f.b = as_double(kv.second.get("max"), 0, &ok);
          std::string tr = kv.second.str_or("truncate", "true");
          for (auto& ch : tr) ch = (char)tolower(ch);
          f.trunc = tr != "false";
          if (ok && !(f.b > f.a)) { *why = "linear_normalization: max must exceed min"; return false; }
        } else if (m == "gaussian_normalization") {
          f.kind = WideExt::kGauss;
          f.a = as_double(kv.second.get("average"), 0, &ok);
          f.b = as_double(kv.second.get("standard_deviation"), 0, &ok);
          if (ok && !(f.b > 0)) { *why = "gaussian_normalization: standard_deviation must be > 0"; return false; }
        } else if (m == "sigmoid_normalization") {
          f.kind = WideExt::kSigmoid;
          f.a = as_double(kv.second.get("gain"), 0, &ok);
          f.b = as_double(kv.second.get("bias"), 0, &ok);
        } else if (m == "dynamic") {
          f.kind = WideExt::kPlug;
          f.plug = load_plugin(ext.get(), kv.second, plug::kNumFilter, why);
          if (f.plug < 0) return false;
        } else {
          *why = "num filter method " + m;
          return false;
        }
        if (!ok) { *why = "num filter " + kv.first + ": parameters"; return false; }
        nft[kv.first] = f;
      }
    }
    if (const Value* r = conv.get("num_filter_rules")) {
      if (r->kind != Value::ARR) { *why = "num_filter_rules"; return false; }
      for (const Value& x : r->a) {
        auto it = nft.find(x.str_or("type", ""));
        if (it == nft.end()) { *why = "unknown num filter type: " + x.str_or("type", ""); return false; }
        WideExt::Filter f = it->second;
        std::string arg;
        f.m = HostRule{};
        f.m.match_kind = jb::srv::matcher_kind(x.str_or("key", ""), &arg);
        if (f.m.match_kind < 0) { *why = "regex key matcher"; return false; }
        put_ext(arg, &f.m);
        f.suffix = x.str_or("suffix", "");
        ext->nf.push_back(f);
      }
    }
    // binary types: plug-ins only (binary_types: the reference has no built-in)
    std::map<std::string, int> bt;
    if (const Value* t = conv.get("binary_types")) {
      if (t->kind != Value::MAP) { *why = "binary_types"; return false; }
      for (const auto& kv : t->o) {
        if (kv.second.str_or("method", "") != "dynamic") { *why = "binary type method"; return false; }
        const int p = load_plugin(ext.get(), kv.second, plug::kBinaryFeature, why);
        if (p < 0) return false;
        bt[kv.first] = p;
      }
    }
    if (const Value* r = conv.get("binary_rules")) {
      if (r->kind != Value::ARR) { *why = "binary_rules"; return false; }
      for (const Value& x : r->a) {
        const std::string type = x.str_or("type", "");
        auto it = bt.find(type);
        if (it == bt.end()) { *why = "unknown binary type: " + type; return false; }
        WideExt::BinRule b;
        b.m = HostRule{};
        std::string arg;
        b.m.match_kind = jb::srv::matcher_kind(x.str_or("key", ""), &arg);
        if (b.m.match_kind < 0) { *why = "regex key matcher"; return false; }
        put_ext(arg, &b.m);
        b.type = "@" + type;
        b.plug = it->second;
        ext->br.push_back(b);
      }
    }
  }
  if (const Value* h = conv.get("hash_max_size")) {
    if (h->kind == Value::INT && h->i > 0) *H = (uint64_t)h->i;
    else if (h->kind != Value::NIL) { *why = "hash_max_size"; return false; }
  }
  auto put = [&](const std::string& b, int32_t* off, int32_t* len) {
    *off = (int32_t)blob->size();
    *len = (int32_t)b.size();
    *blob += b;
  };
  // string types: built-in str / space, ngram(char_num)
  std::map<std::string, std::pair<int, int>> st = {{"str", {kSplitStr, 0}}, {"space", {kSplitSpace, 0}}};
  if (const Value* t = conv.get("string_types")) {
    if (t->kind != Value::MAP) { *why = "string_types"; return false; }
    for (const auto& kv : t->o) {
      const std::string m = kv.second.str_or("method", "");
      if (m == "dynamic" && ext_out) {
        const int p = load_plugin(ext.get(), kv.second, plug::kStringFeature, why);
        if (p < 0) return false;
        st[kv.first] = {kSplitPlugin, p};
        continue;
      }
      if (m != "ngram") { *why = "string type method " + m; return false; }
      const int cn = as_int(kv.second.get("char_num"), 0);
      if (cn <= 0) { *why = "char_num"; return false; }
      st[kv.first] = {kSplitNgram, cn};
    }
  }
  *global = false;
  if (const Value* sr = conv.get("string_rules")) {
    if (sr->kind != Value::ARR) { *why = "string_rules"; return false; }
    for (const Value& x : sr->a) {
      const std::string type = x.str_or("type", "");
      auto it = st.find(type);
      if (it == st.end()) { *why = "string type " + type; return false; }
      const std::string sw = x.str_or("sample_weight", "bin"), gw = x.str_or("global_weight", "bin");
      const int swk = sw == "bin" ? kSwBin : sw == "tf" ? kSwTf : sw == "log_tf" ? kSwLogTf : -1;
      const int gwk = gw == "bin" ? kGwBin : gw == "idf" ? kGwIdf : gw == "bm25" ? kGwBm25 : -1;
      if (swk < 0 || gwk < 0) { *why = "sample / global weight"; return false; }
      if (gwk != kGwBin) *global = true;
      std::string arg;
      const int kind = jb::srv::matcher_kind(x.str_or("key", ""), &arg);
      if (kind < 0) { *why = "regex key matcher"; return false; }
      HostRule h{};
      h.match_kind = kind;
      put(arg, &h.match_off, &h.match_len);
      put("@" + type + "#" + sw + "/" + gw, &h.suffix_off, &h.suffix_len);
      h.value_kind = it->second.first | swk << 4 | gwk << 8;
      h.pad = it->second.second;
      s->push_back(h);
    }
  }
  // num types: num / log (user names map to their method); with ext also add,
  // str and plug-ins (pad: the value's / plug-in's index)
  std::map<std::string, std::pair<int, int>> nt = {{"num", {kNumNum, 0}}, {"log", {kNumLog, 0}}};
  if (ext_out) nt["str"] = {kNumStr, 0};
  if (const Value* t = conv.get("num_types")) {
    if (t->kind != Value::MAP) { *why = "num_types"; return false; }
    for (const auto& kv : t->o) {
      const std::string m = kv.second.str_or("method", "");
      if (m == "num" || m == "log") { nt[kv.first] = {m == "log" ? kNumLog : kNumNum, 0}; continue; }
      if (!ext_out) { *why = "num type method " + m; return false; }
      if (m == "str") {
        nt[kv.first] = {kNumStr, 0};
      } else if (m == "add") {
        bool ok = true;
        const double v = as_double(kv.second.get("value"), 0, &ok);
        if (!ok) { *why = "num type add: value"; return false; }
        ext->addv.push_back(v);
        nt[kv.first] = {kNumAdd, (int)ext->addv.size() - 1};
      } else if (m == "dynamic") {
        const int p = load_plugin(ext.get(), kv.second, plug::kNumFeature, why);
        if (p < 0) return false;
        nt[kv.first] = {kNumPlugin, p};
      } else {
        *why = "num type method " + m;
        return false;
      }
    }
  }
  if (const Value* nr = conv.get("num_rules")) {
    if (nr->kind != Value::ARR) { *why = "num_rules"; return false; }
    for (const Value& x : nr->a) {
      const std::string type = x.str_or("type", "");
      auto it = nt.find(type);
      if (it == nt.end()) { *why = "num type " + type; return false; }
      std::string arg;
      const int kind = jb::srv::matcher_kind(x.str_or("key", ""), &arg);
      if (kind < 0) { *why = "regex key matcher"; return false; }
      HostRule h{};
      h.match_kind = kind;
      put(arg, &h.match_off, &h.match_len);
      put("@" + type, &h.suffix_off, &h.suffix_len);
      h.value_kind = it->second.first;
      h.pad = it->second.second;
      n->push_back(h);
    }
  }
  std::map<std::string, std::pair<int, int>> ct = {{"add", {kCombAdd, 0}}, {"mul", {kCombMul, 0}}};
  if (const Value* t = conv.get("combination_types")) {
    if (t->kind != Value::MAP) { *why = "combination_types"; return false; }
    for (const auto& kv : t->o) {
      const std::string m = kv.second.str_or("method", "");
      if (m == "dynamic" && ext_out) {
        const int p = load_plugin(ext.get(), kv.second, plug::kCombination, why);
        if (p < 0) return false;
        ct[kv.first] = {kCombPlugin, p};
        continue;
      }
      if (m != "add" && m != "mul") { *why = "combination method " + m; return false; }
      ct[kv.first] = {m == "mul" ? kCombMul : kCombAdd, 0};
    }
  }
  if (const Value* cr = conv.get("combination_rules")) {
    if (cr->kind != Value::ARR) { *why = "combination_rules"; return false; }
    for (const Value& x : cr->a) {
      const std::string type = x.str_or("type", "");
      auto it = ct.find(type);
      if (it == ct.end()) { *why = "combination type " + type; return false; }
      std::string la, ra;
      const int lk = jb::srv::matcher_kind(x.str_or("key_left", ""), &la);
      const int rk = jb::srv::matcher_kind(x.str_or("key_right", ""), &ra);
      if (lk < 0 || rk < 0) { *why = "regex key matcher"; return false; }
      HostRule l{}, r{};
      l.match_kind = lk;
      put(la, &l.match_off, &l.match_len);
      put("/" + type, &l.suffix_off, &l.suffix_len);
      l.value_kind = it->second.first;
      l.pad = it->second.second;
      r.match_kind = rk;
      put(ra, &r.match_off, &r.match_len);
      c->push_back(l);
      c->push_back(r);
    }
  }
  if (ext_out) *ext_out = ext->needed() ? ext : nullptr;
  return true;
}

}  // namespace row
}  // namespace jb
