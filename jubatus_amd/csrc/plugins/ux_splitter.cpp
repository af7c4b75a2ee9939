// Dictionary longest-prefix splitter plug-in (string_feature).
//
// Reference: plugin/src/fv_converter/ux_splitter.cpp:40-107 - reads the
// word list at "dict_path" (one word per line), then scans the text byte by
// byte: at each position the longest dictionary word starting there becomes
// a token and the scan jumps past it; positions with no match are skipped.
// The reference uses the ux succinct trie; this is a plain byte trie with
// sorted child arrays (same results, no external dependency).
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "jb_plugin.h"

namespace {

struct Trie {
  struct Node {
    std::vector<std::pair<unsigned char, int>> next;  // sorted by byte
    bool terminal = false;
  };
  std::vector<Node> nodes{Node()};

  void insert(const std::string& w) {
    int cur = 0;
    for (unsigned char ch : w) {
      auto& nx = nodes[cur].next;
      auto it = std::lower_bound(nx.begin(), nx.end(), std::make_pair(ch, -1));
      if (it == nx.end() || it->first != ch) {
        const int id = (int)nodes.size();
        it = nx.insert(it, std::make_pair(ch, id));
        nodes.emplace_back();
      }
      cur = it->second;
    }
    nodes[cur].terminal = true;
  }

  // length of the longest word that prefixes s[0, n), 0 if none
  int64_t longest(const char* s, int64_t n) const {
    int cur = 0;
    int64_t best = 0;
    for (int64_t i = 0; i < n; ++i) {
      const auto& nx = nodes[cur].next;
      const unsigned char ch = (unsigned char)s[i];
      auto it = std::lower_bound(nx.begin(), nx.end(), std::make_pair(ch, -1));
      if (it == nx.end() || it->first != ch) break;
      cur = it->second;
      if (nodes[cur].terminal) best = i + 1;
    }
    return best;
  }
};

struct Ux {
  jb_plugin p{};
  Trie trie;
  size_t words = 0;
};

int split(void* self, const char* text, int64_t len, jb_token* out, int cap) {
  const Ux* u = static_cast<const Ux*>(self);
  int n = 0;
  for (int64_t i = 0; i < len; ++i) {
    const int64_t m = u->trie.longest(text + i, len - i);
    if (m == 0) continue;
    if (n < cap) out[n] = jb_token{i, m, nullptr, 0, 1.0};
    ++n;
    i += m - 1;
  }
  return n;
}

void destroy(void* self) { delete static_cast<Ux*>(self); }

}  // namespace

extern "C" {

const char* version(void) { return "jubatus_amd-ux-splitter 1.0"; }

jb_plugin* create(const char** keys, const char** values, int n) {
  const char* path = nullptr;
  for (int i = 0; i < n; ++i)
    if (std::strcmp(keys[i], "dict_path") == 0) path = values[i];
  if (!path) {
    std::fprintf(stderr, "ux_splitter: parameter dict_path is required\n");
    return nullptr;
  }
  struct stat st;
  if (stat(path, &st) != 0 || S_ISDIR(st.st_mode)) {
    std::fprintf(stderr, "ux_splitter: cannot read dictionary %s\n", path);
    return nullptr;
  }
  std::ifstream ifs(path);
  if (!ifs) return nullptr;
  Ux* u = new Ux();
  for (std::string line; std::getline(ifs, line);) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    if (line.empty()) continue;
    u->trie.insert(line);
    ++u->words;
  }
  u->p = jb_plugin{JB_PLUGIN_ABI, JB_STRING_FEATURE, u, split, nullptr, nullptr, nullptr, nullptr,
                   nullptr, destroy};
  return &u->p;
}

}  // extern "C"
