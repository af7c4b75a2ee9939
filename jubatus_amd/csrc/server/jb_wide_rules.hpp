// The wide converter's rule table built from a config's "converter" object
// in C++ (the twin of fv_converter/gpu_path.py wide_eligible + WideRuleTable):
// str / space / ngram splitters, bin / tf / log_tf sample weights, bin / idf /
// bm25 global weights, num / log rules, add / mul combinations. Shared by the
// native row-engine servers (jb_row_engine.hpp) and jubaweight.
#pragma once
#include <stdlib.h>

#include <string>
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

// fv_converter/gpu_path.py wide_eligible + WideRuleTable
inline bool build_wide_rules(const Value& conv, std::vector<HostRule>* s, std::vector<HostRule>* n,
                             std::vector<HostRule>* c, std::string* blob, uint64_t* H, bool* global,
                             std::string* why) {
  if (conv.kind != Value::MAP) { *why = "converter is not an object"; return false; }
  for (const char* k : {"string_filter_rules", "num_filter_rules", "binary_rules"})
    if (jb::srv::nonempty_list(conv, k)) { *why = std::string(k) + " need the host converter"; return false; }
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
  // num types: num / log (user names map to their method)
  std::map<std::string, int> nt = {{"num", 0}, {"log", 1}};
  if (const Value* t = conv.get("num_types")) {
    if (t->kind != Value::MAP) { *why = "num_types"; return false; }
    for (const auto& kv : t->o) {
      const std::string m = kv.second.str_or("method", "");
      if (m != "num" && m != "log") { *why = "num type method " + m; return false; }
      nt[kv.first] = m == "log" ? 1 : 0;
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
      h.value_kind = it->second;
      n->push_back(h);
    }
  }
  std::map<std::string, int> ct = {{"add", 0}, {"mul", 1}};
  if (const Value* t = conv.get("combination_types")) {
    if (t->kind != Value::MAP) { *why = "combination_types"; return false; }
    for (const auto& kv : t->o) {
      const std::string m = kv.second.str_or("method", "");
      if (m != "add" && m != "mul") { *why = "combination method " + m; return false; }
      ct[kv.first] = m == "mul" ? 1 : 0;
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
      l.value_kind = it->second;
      r.match_kind = rk;
      put(ra, &r.match_off, &r.match_len);
      c->push_back(l);
      c->push_back(r);
    }
  }
  return true;
}

}  // namespace row
}  // namespace jb
