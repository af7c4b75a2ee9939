// Test double of libmecab's C API (MeCab is not installed in this image):
// whitespace tokenizer whose node feature CSV is
//   "<POS>,*,*,*,*,*,<base>"  with POS = 動詞 for words ending in "ing"
// (base = the word without "ing"), 記号 for punctuation-only words (base
// "*"), else 名詞 (base = lower-cased word). Node layout and the
// rlength/length convention (rlength includes leading spaces) follow mecab.h.
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {
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

struct Lattice {
  std::string sentence;
  std::vector<mecab_node_t> nodes;
  std::vector<std::string> features;
};
int g_model;
int g_tagger;
}  // namespace

extern "C" {
void* mecab_model_new2(const char* arg) { return (arg && std::strstr(arg, "--fail")) ? nullptr : &g_model; }
void mecab_model_destroy(void*) {}
void* mecab_model_new_tagger(void*) { return &g_tagger; }
void* mecab_model_new_lattice(void*) { return new Lattice(); }
void mecab_destroy(void*) {}
void mecab_lattice_destroy(void* l) { delete static_cast<Lattice*>(l); }
const char* mecab_strerror(void*) { return "fake mecab error"; }
void mecab_lattice_set_sentence2(void* l, const char* s, size_t n) {
  static_cast<Lattice*>(l)->sentence.assign(s, n);
}
int mecab_parse_lattice(void*, void* lp) {
  Lattice* l = static_cast<Lattice*>(lp);
  const std::string& s = l->sentence;
  struct W { size_t lead, b, e; };
  std::vector<W> ws;
  size_t i = 0;
  while (i < s.size()) {
    size_t b = i;
    while (b < s.size() && s[b] == ' ') ++b;
    if (b >= s.size()) break;
    size_t e = b;
    while (e < s.size() && s[e] != ' ') ++e;
    ws.push_back({b - i, b, e});
    i = e;
  }
  l->nodes.assign(ws.size() + 2, mecab_node_t{});
  l->features.assign(ws.size() + 2, std::string());
  l->nodes[0].stat = 2;
  l->nodes.back().stat = 3;
  for (size_t k = 0; k < ws.size(); ++k) {
    std::string w = s.substr(ws[k].b, ws[k].e - ws[k].b);
    std::string pos, base;
    bool punct = true;
    for (char c : w) punct = punct && std::ispunct((unsigned char)c);
    if (punct) { pos = "記号"; base = "*"; }
    else if (w.size() > 3 && w.compare(w.size() - 3, 3, "ing") == 0) { pos = "動詞"; base = w.substr(0, w.size() - 3); }
    else { pos = "名詞"; base = w; for (auto& c : base) c = (char)std::tolower((unsigned char)c); }
    l->features[k + 1] = pos + ",*,*,*,*,*," + base;
    mecab_node_t& n = l->nodes[k + 1];
    n.length = (unsigned short)(ws[k].e - ws[k].b);
    n.rlength = (unsigned short)(n.length + ws[k].lead);
    n.stat = 0;
  }
  for (size_t k = 0; k < l->nodes.size(); ++k) {
    l->nodes[k].feature = l->features[k].c_str();
    l->nodes[k].next = k + 1 < l->nodes.size() ? &l->nodes[k + 1] : nullptr;
  }
  return 1;
}
const mecab_node_t* mecab_lattice_get_bos_node(void* l) { return &static_cast<Lattice*>(l)->nodes[0]; }
}
