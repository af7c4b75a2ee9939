// Host-native converter for the wide rule set: string rules with the str /
// space / ngram splitters, bin / tf / log_tf sample weights and bin / idf /
// bm25 global weights (document frequencies in the WeightManager's dense
// int64 arrays, updated in place), num rules num / log, and combination rules
// add / mul over the finished feature list. Output order and values equal the
// Python converter (jubatus_amd/fv_converter/converter.py `_convert`): per
// string value and rule the distinct tokens in first-occurrence order, then
// the num features, then for every combination rule the pairs i < j of that
// list. Values are computed in double and stored as float, as the Python path
// does. Rule tables come from fv_converter/gpu_path.py WideRuleTable; the GPU
// twin is csrc/hip/fv_wide.hip.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <deque>
#include <memory>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "jb_hash.hpp"
#include "jb_hostfv.hpp"
#include "jb_msgpack.hpp"
#include "jb_plugin_host.hpp"

namespace jb {

// string rule value_kind bit fields (fv_converter/gpu_path.py); kSplitPlugin:
// a "dynamic" splitter (pad: its plug-in in WideExt)
constexpr int kSplitStr = 0, kSplitNgram = 1, kSplitSpace = 2, kSplitPlugin = 3;
// num rule value_kind: num, log, a "dynamic" num_feature plug-in (pad: its
// index), add (pad: the value's index in WideExt::addv), str
constexpr int kNumNum = 0, kNumLog = 1, kNumPlugin = 2, kNumAdd = 3, kNumStr = 4;
// combination rule value_kind: add, mul, a "dynamic" plug-in (pad: its index)
constexpr int kCombAdd = 0, kCombMul = 1, kCombPlugin = 2;

// What the rule tables cannot carry: the plug-ins of "dynamic" types
// (jb_plugin_host.hpp), the filter rules, the binary rules and the values of
// "add" num types. Output order and names are those of the Python converter
// (fv_converter/converter.py _filtered / _convert).
struct WideExt {
  std::vector<std::unique_ptr<plug::Plugin>> plugins;
  // num filter kinds
  enum { kAdd = 0, kLinear = 1, kGauss = 2, kSigmoid = 3, kPlug = 4 };
  struct Filter {
    HostRule m;            // key matcher (its argument in blob)
    std::string suffix;
    int kind = kPlug;      // string filters: plug-ins only
    double a = 0, b = 0;
    bool trunc = true;
    int plug = -1;
  };
  std::vector<Filter> sf, nf;
  struct BinRule {
    HostRule m;
    std::string type;      // "@<type>"
    int plug;
  };
  std::vector<BinRule> br;
  std::vector<double> addv;
  std::string blob;
  int add_plugin(std::unique_ptr<plug::Plugin> p) {
    plugins.push_back(std::move(p));
    return (int)plugins.size() - 1;
  }
  bool needed() const { return !plugins.empty() || !sf.empty() || !nf.empty() || !br.empty() || !addv.empty(); }
};

// %.17g of a value, an integer without a fraction (converter.py _num_str)
inline std::string num_str(double x) {
  char b[64];
  if (x == (double)(long long)x && fabs(x) < 1e16) snprintf(b, sizeof(b), "%lld", (long long)x);
  else snprintf(b, sizeof(b), "%.17g", x);
  return b;
}
constexpr int kSwBin = 0, kSwTf = 1, kSwLogTf = 2;
constexpr int kGwBin = 0, kGwIdf = 1, kGwBm25 = 2;

struct WideName {        // a feature name as up to four byte segments
  const uint8_t* p[4];
  uint32_t n[4];
  int k;
  uint32_t len() const { uint32_t t = 0; for (int i = 0; i < k; ++i) t += n[i]; return t; }
  uint8_t at(uint32_t pos) const {
    for (int i = 0; i < k; ++i) {
      if (pos < n[i]) return p[i][pos];
      pos -= n[i];
    }
    return 0;
  }
  uint64_t fnv(uint64_t h) const {
    for (int i = 0; i < k; ++i) h = fnv_bytes(h, p[i], n[i]);
    return h;
  }
};

struct WideFeat {
  uint64_t h;       // FNV-1a/64 state of the full name
  int32_t idx;
  double w;
  int gw;
  WideName name;
};

class HostFvWide {
 public:
  HostFvWide(const uint8_t* srules, int n_srules, const uint8_t* nrules, int n_nrules,
             const uint8_t* crules, int n_crules, const uint8_t* blob, size_t blob_len, uint64_t H)
      : s_(n_srules), n_(n_nrules), c_(2 * n_crules), blob_(blob, blob + blob_len), H_(H) {
    if (n_srules) memcpy(s_.data(), srules, sizeof(HostRule) * n_srules);
    if (n_nrules) memcpy(n_.data(), nrules, sizeof(HostRule) * n_nrules);
    if (n_crules) memcpy(c_.data(), crules, sizeof(HostRule) * 2 * n_crules);
    for (const HostRule& r : s_)
      if ((r.value_kind >> 8 & 15) != kGwBin) global_ = true;
  }

  // WeightManager storage: df[H], diff[H] (int64) and counts[4] =
  // [doc_count, total_len, diff_docs, diff_len]
  void set_weights(int64_t* df, int64_t* diff, int64_t* counts) {
    df_ = df; diff_ = diff; counts_ = counts;
  }
  bool needs_weights() const { return global_; }
  // plug-ins, filters, binary rules (shared: every converter built from one
  // config may hold it)
  void set_ext(std::shared_ptr<WideExt> e) { ext_ = std::move(e); }
  // the table height of the document statistics when it differs from the
  // feature index's (clustering keys features over 2^31 - 1 while the
  // weight manager counts them in the converter's hash_max_size rows)
  void set_df_height(uint64_t H) { Hdf_ = H; }

  // Optional sinks of hash_body: the name of every emitted slot (appended to
  // *names, end offsets in *name_end) and the byte span of every datum in the
  // body (datum_span: begin / end pairs relative to the body). Engines that
  // keep named features (clustering, weight) use them; null = off.
  void set_sinks(std::string* names, std::vector<int64_t>* name_end, std::vector<int64_t>* datum_span) {
    names_ = names; name_end_ = name_end; span_ = datum_span;
  }

  // Document-statistics journal of one hash call: on an error the caller
  // rolls back every update it made (a capacity retry re-runs the batch).
  void begin() { journal_.clear(); jdocs_ = jlen_ = 0; }
  void rollback() {
    for (int32_t i : journal_) { df_[i] -= 1; if (diff_) diff_[i] -= 1; }
    counts_[0] -= jdocs_; counts_[2] -= jdocs_;
    counts_[1] -= jlen_; counts_[3] -= jlen_;
    begin();
  }

  // One body = msgpack list<datum>; same contract as HostFvHasher::hash_body.
  int hash_body(const uint8_t* p, size_t len, int32_t* idx, float* val, int64_t* row_ptr,
                int64_t max_samples, int64_t max_slots, int64_t* n, int64_t* slots,
                bool update) {
    if (global_ && (!df_ || !counts_)) return 1;
    Cursor c{p, p + len};
    uint32_t cnt;
    if (!c.array(&cnt)) return 1;
    for (uint32_t i = 0; i < cnt; ++i) {
      if (*n >= max_samples) return 2;
      const uint8_t* d0 = c.p;
      int rc = datum(c, idx, val, max_slots, slots, update);
      if (rc) return rc;
      if (span_) {
        span_->push_back((int64_t)(d0 - p));
        span_->push_back((int64_t)(c.p - p));
      }
      row_ptr[++*n] = *slots;
    }
    return 0;
  }

  // one datum at the cursor (HostFvHasher::hash_datum contract: 0 ok,
  // 1 malformed, 2 out of slots); update: count it into the statistics
  int hash_datum(Cursor& c, int32_t* idx, float* val, int64_t max_slots, int64_t* slots, bool update) {
    if (global_ && (!df_ || !counts_)) return 1;
    return datum(c, idx, val, max_slots, slots, update);
  }

 private:
  bool match_key(const HostRule& r, const uint8_t* k, uint32_t kn) const {
    if (r.match_kind == 0) return true;
    const uint8_t* m = blob_.data() + r.match_off;
    const uint32_t mn = (uint32_t)r.match_len;
    if (r.match_kind == 3 && kn != mn) return false;
    if (kn < mn) return false;
    const uint8_t* base = (r.match_kind == 2) ? (k + kn - mn) : k;
    return memcmp(base, m, mn) == 0;
  }

  bool match_name(const HostRule& r, const WideName& nm) const {
    if (r.match_kind == 0) return true;
    const uint8_t* m = blob_.data() + r.match_off;
    const uint32_t mn = (uint32_t)r.match_len, L = nm.len();
    if (r.match_kind == 3 && L != mn) return false;
    if (L < mn) return false;
    const uint32_t base = (r.match_kind == 2) ? L - mn : 0;
    for (uint32_t i = 0; i < mn; ++i)
      if (nm.at(base + i) != m[i]) return false;
    return true;
  }

  // tokens of one string value for a splitter -> tok_ (offset, length) pairs
  void split(int kind, int ngram, const uint8_t* v, uint32_t vn) {
    tok_.clear();
    if (kind == kSplitStr) {
      tok_.push_back({0, vn});
    } else if (kind == kSplitSpace) {
      uint32_t s = 0;
      for (uint32_t i = 0; i <= vn; ++i) {
        if (i == vn || v[i] == ' ') {
          if (i > s) tok_.push_back({s, i - s});
          s = i + 1;
        }
      }
    } else {                              // ngram over code points
      cp_.clear();
      for (uint32_t i = 0; i < vn; ++i)
        if ((v[i] & 0xC0) != 0x80) cp_.push_back(i);
      const int ncp = (int)cp_.size();
      cp_.push_back(vn);
      for (int i = 0; i + ngram <= ncp; ++i) tok_.push_back({cp_[i], cp_[i + ngram] - cp_[i]});
    }
  }

  bool match_ext(const HostRule& r, const uint8_t* k, uint32_t kn) const {
    if (r.match_kind == 0) return true;
    const uint8_t* m = (const uint8_t*)ext_->blob.data() + r.match_off;
    const uint32_t mn = (uint32_t)r.match_len;
    if (r.match_kind == 3 && kn != mn) return false;
    if (kn < mn) return false;
    const uint8_t* base = (r.match_kind == 2) ? (k + kn - mn) : k;
    return memcmp(base, m, mn) == 0;
  }
  // bytes that must live until the datum's features are out (filtered keys
  // and values, plug-in tokens and names): a deque never moves its strings
  const std::string& keep(std::string s) {
    store_.push_back(std::move(s));
    return store_.back();
  }
  static const uint8_t* u8(const std::string& s) { return (const uint8_t*)s.data(); }

  void add_feat(const WideName& nm, double w, int gw) {
    WideFeat f;
    f.h = nm.fnv(kFnvOffset);
    f.idx = (int32_t)hash_to_index(f.h, H_);
    f.w = w;
    f.gw = gw;
    f.name = nm;
    feats_.push_back(f);
  }

  int datum(Cursor& c, int32_t* idx, float* val, int64_t max_slots, int64_t* slots, bool update) {
    uint32_t top, ns, nn;
    if (!c.array(&top) || top < 2) return 1;
    feats_.clear();
    store_.clear();
    sv_.clear();
    nv_.clear();
    if (!c.array(&ns)) return 1;
    for (uint32_t i = 0; i < ns; ++i) {
      uint32_t two; const uint8_t *k, *v; uint32_t kn, vn;
      if (!c.array(&two) || two != 2 || !c.raw(&k, &kn) || !c.raw(&v, &vn)) return 1;
      sv_.push_back({k, kn, v, vn});
    }
    if (!c.array(&nn)) return 1;
    for (uint32_t i = 0; i < nn; ++i) {
      uint32_t two; const uint8_t* k; uint32_t kn; double x;
      if (!c.array(&two) || two != 2 || !c.raw(&k, &kn) || !c.number(&x)) return 1;
      nv_.push_back({k, kn, x});
    }
    // filters (converter.py _filtered): every filter sees the values the
    // earlier ones appended
    if (ext_) {
      for (const WideExt::Filter& f : ext_->sf) {
        const size_t n0 = sv_.size();
        for (size_t i = 0; i < n0; ++i) {
          const SV e = sv_[i];
          if (!match_ext(f.m, e.k, e.kn)) continue;
          const std::string& nk = keep(std::string((const char*)e.k, e.kn) + f.suffix);
          const std::string& nvl = keep(ext_->plugins[(size_t)f.plug]->filter_string((const char*)e.v, e.vn));
          sv_.push_back({u8(nk), (uint32_t)nk.size(), u8(nvl), (uint32_t)nvl.size()});
        }
      }
      for (const WideExt::Filter& f : ext_->nf) {
        const size_t n0 = nv_.size();
        for (size_t i = 0; i < n0; ++i) {
          const NV e = nv_[i];
          if (!match_ext(f.m, e.k, e.kn)) continue;
          double y;
          switch (f.kind) {
            case WideExt::kAdd: y = e.x + f.a; break;
            case WideExt::kLinear:
              y = (e.x - f.a) / (f.b - f.a);
              if (f.trunc) y = std::min(1.0, std::max(0.0, y));
              break;
            case WideExt::kGauss: y = (e.x - f.a) / f.b; break;
            case WideExt::kSigmoid: y = 1.0 / (1.0 + exp(-f.a * (e.x - f.b))); break;
            default: y = ext_->plugins[(size_t)f.plug]->filter_num(e.x); break;
          }
          const std::string& nk = keep(std::string((const char*)e.k, e.kn) + f.suffix);
          nv_.push_back({u8(nk), (uint32_t)nk.size(), y});
        }
      }
    }
    for (const SV& e : sv_) {
      const uint8_t *k = e.k, *v = e.v;
      const uint32_t kn = e.kn, vn = e.vn;
      uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
      hk = fnv_bytes(hk, (const uint8_t*)"$", 1);
      for (const HostRule& r : s_) {
        if (!match_key(r, k, kn)) continue;
        const int sp = r.value_kind & 15, sw = r.value_kind >> 4 & 15, gw = r.value_kind >> 8 & 15;
        const uint8_t* suf = blob_.data() + r.suffix_off;
        if (sp == kSplitPlugin) {
          // a plug-in splitter: its tokens' bytes, counted in first-occurrence order
          ext_->plugins[(size_t)r.pad]->split((const char*)v, vn, &ptok_);
          uniqs_.clear();
          for (const std::string& t : ptok_) {
            bool found = false;
            for (auto& u : uniqs_)
              if (u.first == t) { ++u.second; found = true; break; }
            if (!found) uniqs_.emplace_back(t, 1);
          }
          for (const auto& u : uniqs_) {
            const std::string& tok = keep(u.first);
            const double w = sw == kSwBin ? 1.0 : sw == kSwTf ? (double)u.second : log(1.0 + (double)u.second);
            add_feat(WideName{{k, (const uint8_t*)"$", u8(tok), suf}, {kn, 1, (uint32_t)tok.size(),
                                                                         (uint32_t)r.suffix_len}, 4},
                     w, gw);
          }
          continue;
        }
        split(sp, r.pad, v, vn);
        // distinct tokens in first-occurrence order with their counts
        uniq_.clear();
        if (tok_.size() <= 32) {
          for (const auto& t : tok_) {
            bool found = false;
            for (auto& u : uniq_) {
              if (u.len == t.len && memcmp(v + u.off, v + t.off, t.len) == 0) { ++u.cnt; found = true; break; }
            }
            if (!found) uniq_.push_back({t.off, t.len, 1});
          }
        } else {                          // long text: hash map over the token bytes
          seen_.clear();
          for (const auto& t : tok_) {
            auto it = seen_.emplace(std::string_view((const char*)v + t.off, t.len), uniq_.size());
            if (it.second) uniq_.push_back({t.off, t.len, 1});
            else ++uniq_[it.first->second].cnt;
          }
        }
        for (const auto& u : uniq_) {
          WideFeat f;
          f.h = fnv_bytes(fnv_bytes(hk, v + u.off, u.len), suf, (size_t)r.suffix_len);
          f.idx = (int32_t)hash_to_index(f.h, H_);
          f.w = sw == kSwBin ? 1.0 : sw == kSwTf ? (double)u.cnt : log(1.0 + (double)u.cnt);
          f.gw = gw;
          f.name = WideName{{k, (const uint8_t*)"$", v + u.off, suf}, {kn, 1, u.len, (uint32_t)r.suffix_len}, 4};
          feats_.push_back(f);
        }
      }
    }
    if (global_) weigh(update);
    for (const NV& e : nv_) {
      const uint8_t* k = e.k;
      const uint32_t kn = e.kn;
      const double x = e.x;
      const uint64_t hk = fnv_bytes(kFnvOffset, k, kn);
      for (const HostRule& r : n_) {
        if (!match_key(r, k, kn)) continue;
        const uint8_t* suf = blob_.data() + r.suffix_off;
        if (r.value_kind == kNumPlugin) {
          ext_->plugins[(size_t)r.pad]->num_feature(std::string((const char*)k, kn), x, &pnamed_);
          for (const auto& nv : pnamed_) {
            const std::string& nm = keep(nv.first);
            add_feat(WideName{{u8(nm), nullptr, nullptr, nullptr}, {(uint32_t)nm.size(), 0, 0, 0}, 1}, nv.second,
                     kGwBin);
          }
          continue;
        }
        if (r.value_kind == kNumStr) {      // <key>$<value>@<type>, weight 1
          const std::string& vs = keep(num_str(x));
          add_feat(WideName{{k, (const uint8_t*)"$", u8(vs), suf}, {kn, 1, (uint32_t)vs.size(),
                                                                    (uint32_t)r.suffix_len}, 4},
                   1.0, kGwBin);
          continue;
        }
        WideFeat f;
        f.h = fnv_bytes(hk, suf, (size_t)r.suffix_len);
        f.idx = (int32_t)hash_to_index(f.h, H_);
        f.w = r.value_kind == kNumLog ? log(x > 1.0 ? x : 1.0)
              : r.value_kind == kNumAdd ? x + ext_->addv[(size_t)r.pad] : x;
        f.gw = kGwBin;
        f.name = WideName{{k, suf, nullptr, nullptr}, {kn, (uint32_t)r.suffix_len, 0, 0}, 2};
        feats_.push_back(f);
      }
    }
    // binary values: plug-in features <key>$<token>@<type> (others carry none)
    if (top >= 3 && ext_ && !ext_->br.empty()) {
      uint32_t nb;
      if (!c.array(&nb)) return 1;
      for (uint32_t i = 0; i < nb; ++i) {
        uint32_t two; const uint8_t *k, *v; uint32_t kn, vn;
        if (!c.array(&two) || two != 2 || !c.raw(&k, &kn) || !c.raw(&v, &vn)) return 1;
        for (const WideExt::BinRule& r : ext_->br) {
          if (!match_ext(r.m, k, kn)) continue;
          ext_->plugins[(size_t)r.plug]->binary_feature(std::string((const char*)k, kn), (const char*)v, vn, &pnamed_);
          for (const auto& tv : pnamed_) {
            const std::string& tok = keep(tv.first);
            add_feat(WideName{{k, (const uint8_t*)"$", u8(tok), u8(r.type)},
                              {kn, 1, (uint32_t)tok.size(), (uint32_t)r.type.size()}, 4},
                     tv.second, kGwBin);
          }
        }
      }
    }
    for (uint32_t i = (top >= 3 && ext_ && !ext_->br.empty()) ? 3 : 2; i < top; ++i)   // the rest carries no feature
      if (!c.skip()) return 1;
    const size_t nb = feats_.size();
    for (size_t i = 0; i < nb; ++i) {
      if (*slots >= max_slots) return 2;
      idx[*slots] = feats_[i].idx;
      val[*slots] = (float)feats_[i].w;
      ++*slots;
      if (names_) put_name(feats_[i].name);
    }
    for (size_t r = 0; r + 1 < c_.size(); r += 2) {
      const HostRule& L = c_[r];
      const HostRule& R = c_[r + 1];
      const uint8_t* suf = blob_.data() + L.suffix_off;
      for (size_t i = 0; i < nb; ++i) {
        if (!match_name(L, feats_[i].name)) continue;
        const uint64_t hi = fnv_bytes(feats_[i].h, (const uint8_t*)"&", 1);
        for (size_t j = i + 1; j < nb; ++j) {
          if (!match_name(R, feats_[j].name)) continue;
          if (*slots >= max_slots) return 2;
          const uint64_t h = fnv_bytes(feats_[j].name.fnv(hi), suf, (size_t)L.suffix_len);
          idx[*slots] = (int32_t)hash_to_index(h, H_);
          const double a = feats_[i].w, b = feats_[j].w;
          val[*slots] = (float)(L.value_kind == kCombMul ? a * b
                                : L.value_kind == kCombPlugin ? ext_->plugins[(size_t)L.pad]->combine(a, b)
                                                              : a + b);
          ++*slots;
          if (names_) {     // left & right + the rule's suffix (the hashed bytes)
            put_name(feats_[i].name, false);
            names_->push_back('&');
            put_name(feats_[j].name, false);
            names_->append((const char*)suf, (size_t)L.suffix_len);
            name_end_->push_back((int64_t)names_->size());
          }
        }
      }
    }
    return 0;
  }

  // update the document statistics with this datum (when asked), then apply
  // the idf / bm25 weights (converter.py _convert)
  void weigh(bool update) {
    gidx_.clear();
    for (const auto& f : feats_)
      if (f.gw != kGwBin) gidx_.push_back(dfi(f));
    const int64_t dl = (int64_t)gidx_.size();
    if (update) {
      counts_[0] += 1; counts_[2] += 1;
      counts_[1] += dl; counts_[3] += dl;
      jdocs_ += 1; jlen_ += dl;
      std::sort(gidx_.begin(), gidx_.end());
      for (size_t i = 0; i < gidx_.size(); ++i) {
        if (i && gidx_[i] == gidx_[i - 1]) continue;
        df_[gidx_[i]] += 1;
        if (diff_) diff_[gidx_[i]] += 1;
        journal_.push_back(gidx_[i]);
      }
    }
    const int64_t nd = counts_[0];
    const double avg = nd ? (double)counts_[1] / (double)nd : 1.0;
    for (auto& f : feats_) {
      if (f.gw == kGwBin) continue;
      const int64_t df = df_[dfi(f)];
      const double idf = (df > 0 && nd > 0) ? log((double)nd / (double)df) : 0.0;
      if (f.gw == kGwIdf) {
        f.w *= idf;
      } else {
        const double k1 = 1.2, b = 0.75;
        f.w = idf * (f.w * (k1 + 1)) / (f.w + k1 * (1 - b + b * (double)dl / (avg > 1e-9 ? avg : 1e-9)));
      }
    }
  }

  int32_t dfi(const WideFeat& f) const { return Hdf_ ? (int32_t)hash_to_index(f.h, Hdf_) : f.idx; }

  void put_name(const WideName& nm, bool end = true) {
    for (int i = 0; i < nm.k; ++i) names_->append((const char*)nm.p[i], nm.n[i]);
    if (end) name_end_->push_back((int64_t)names_->size());
  }

  std::string* names_ = nullptr;
  std::vector<int64_t>* name_end_ = nullptr;
  std::vector<int64_t>* span_ = nullptr;

  struct Tok { uint32_t off, len; };
  struct Uniq { uint32_t off, len; int cnt; };
  std::vector<HostRule> s_, n_, c_;
  std::vector<uint8_t> blob_;
  uint64_t H_;
  uint64_t Hdf_ = 0;     // 0: the document statistics use H_
  bool global_ = false;
  int64_t *df_ = nullptr, *diff_ = nullptr, *counts_ = nullptr;
  std::vector<WideFeat> feats_;
  std::vector<Tok> tok_;
  std::vector<Uniq> uniq_;
  std::vector<uint32_t> cp_;
  std::unordered_map<std::string_view, size_t> seen_;
  std::vector<int32_t> gidx_;
  std::vector<int32_t> journal_;
  int64_t jdocs_ = 0, jlen_ = 0;
  // one datum's values (spans into the body or into store_) and extension state
  struct SV { const uint8_t* k; uint32_t kn; const uint8_t* v; uint32_t vn; };
  struct NV { const uint8_t* k; uint32_t kn; double x; };
  std::vector<SV> sv_;
  std::vector<NV> nv_;
  std::deque<std::string> store_;
  std::shared_ptr<WideExt> ext_;
  std::vector<std::string> ptok_;
  std::vector<std::pair<std::string, int>> uniqs_;
  std::vector<std::pair<std::string, double>> pnamed_;
};

}  // namespace jb
