// Host-only parts of the row engines shared by the GPU servers
// (jb_row_engine.hpp) and the CPU rehearsal of their MIX
// (csrc/tools/jb_mix_rehearsal.cpp --rows): the datum type and the row-diff
// protocol of a MIX.
//
// Row MIX (parallel/row_mix.py's protocol, natively; reference: the linear
// mixer's get_diff / mix / put_diff, linear_mixer.cpp:422-544, over row
// stores whose newest version wins, anomaly_serv.cpp:178-211): every rank
// packs the rows written since its last MIX with their versions, datums and
// hashed vectors, its removals, and its document-statistics diff into ONE
// byte string; the strings are all-gathered (RCCL over xGMI or the control
// plane); every rank folds them in rank order - newest version wins, the
// later rank on ties - and applies what it does not hold yet.
//
//   {"ids": [...], "ver": [...], "datum": [[sv, nv, bv]...], "rp": bin i64,
//    "idx": bin i32, "val": bin f32, "removed": [[id, ver]...],
//    "w": [docs, len, bin i64 idx, bin i64 count]}
#pragma once
#include <string.h>

#include <algorithm>
#include <map>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "jb_value.hpp"

namespace jb {
namespace row {

using jb::val::MsgpackWriter;
using jb::val::Value;

struct ArgError : std::runtime_error {   // -> ARGUMENT_ERROR on the wire
  explicit ArgError(const std::string& s) : std::runtime_error(s) {}
};

// ------------------------------------------------------------------ datum
// models/rows.py as_dicts: (string, num, binary) maps; a repeated key keeps
// its last value; serialised with sorted keys (dicts_wire)
struct Datum {
  std::map<std::string, std::string> sv;
  std::map<std::string, double> nv;
  std::map<std::string, std::string> bv;
};

inline void parse_datum(const Value& v, Datum* d) {
  // Datum.from_msgpack: at least [string_values, num_values]; more is ignored
  if (v.kind != Value::ARR || v.a.size() < 2) throw ArgError("malformed datum");
  for (size_t part = 0; part < std::min<size_t>(v.a.size(), 3); ++part) {
    const Value& lst = v.a[part];
    if (lst.kind != Value::ARR) throw ArgError("malformed datum");
    for (const Value& kv : lst.a) {
      if (kv.kind != Value::ARR || kv.a.size() != 2 || !kv.a[0].is_str()) throw ArgError("malformed datum");
      const Value& x = kv.a[1];
      if (part == 1) {
        if (!x.is_num()) throw ArgError("num_values value must be a number");
        d->nv[kv.a[0].s] = x.num();
      } else {
        if (!x.is_str()) throw ArgError("malformed datum");
        (part == 0 ? d->sv : d->bv)[kv.a[0].s] = x.s;
      }
    }
  }
}

inline void write_datum(MsgpackWriter& w, const Datum& d) {
  w.arr(3);
  w.arr(d.sv.size());
  for (const auto& kv : d.sv) { w.arr(2); w.raw(kv.first); w.raw(kv.second); }
  w.arr(d.nv.size());
  for (const auto& kv : d.nv) { w.arr(2); w.raw(kv.first); w.dbl(kv.second); }
  w.arr(d.bv.size());
  for (const auto& kv : d.bv) { w.arr(2); w.raw(kv.first); w.raw(kv.second); }
}

// ------------------------------------------------------------- row diff
// Store interface (RowEngine, the rehearsal's host store):
//   std::vector<std::string> mix_ids() const         written since the MIX (held rows, sorted)
//   std::vector<std::string> mix_removed() const     removed since the MIX (sorted)
//   bool version_of(const std::string&, uint64_t*) const
//   bool holds(const std::string&) const
//   void row_view(const std::string&, const Datum**, const std::vector<int32_t>**,
//                 const std::vector<float>**) const
//   int32_t slot_id(const std::string&) const        (-1: none)
//   void store_mixed(const std::string&, Datum&&, const std::vector<int32_t>&,
//                    const std::vector<float>&, uint64_t version, bool forward)
//   void remove_mixed(const std::string&, uint64_t version, bool forward)
//     (forward: a push MIX passes the row on in its later rounds - it stays
//      in the written / removed sets until the MIX ends)
//   bool weight_diff(int64_t*, int64_t*, std::vector<int64_t>*, std::vector<int64_t>*) const
//   void put_weight_diff(int64_t, int64_t, const std::vector<int64_t>&, const std::vector<int64_t>&, bool keep_own)
//   void mix_done()                                   forget the written / removed sets
template <class S>
void pack_row_diff(const S& st, MsgpackWriter& w) {
  const std::vector<std::string> ids = st.mix_ids();
  std::vector<int64_t> rp(1, 0);
  std::vector<int32_t> ci;
  std::vector<float> cv;
  w.map(8);
  w.str("ids");
  w.arr(ids.size());
  for (const auto& id : ids) w.str(id);
  w.str("ver");
  w.arr(ids.size());
  for (const auto& id : ids) {
    uint64_t v = 0;
    st.version_of(id, &v);
    w.sint((int64_t)v);
  }
  w.str("datum");
  w.arr(ids.size());
  for (const auto& id : ids) {
    const Datum* d;
    const std::vector<int32_t>* ix;
    const std::vector<float>* vx;
    st.row_view(id, &d, &ix, &vx);
    write_datum(w, *d);
    ci.insert(ci.end(), ix->begin(), ix->end());
    cv.insert(cv.end(), vx->begin(), vx->end());
    rp.push_back((int64_t)ci.size());
  }
  w.str("rp");
  w.bin(rp.data(), rp.size() * 8);
  w.str("idx");
  w.bin(ci.data(), ci.size() * 4);
  w.str("val");
  w.bin(cv.data(), cv.size() * 4);
  const std::vector<std::string> rm = st.mix_removed();
  w.str("removed");
  w.arr(rm.size());
  for (const auto& id : rm) {
    uint64_t v = 0;
    st.version_of(id, &v);
    w.arr(2);
    w.str(id);
    w.sint((int64_t)v);
  }
  int64_t docs = 0, len = 0;
  std::vector<int64_t> widx, wcnt;
  st.weight_diff(&docs, &len, &widx, &wcnt);
  w.str("w");
  w.arr(4);
  w.sint(docs);
  w.sint(len);
  w.bin(widx.data(), widx.size() * 8);
  w.bin(wcnt.data(), wcnt.size() * 8);
}

inline const std::string& diff_bin(const Value* b) {
  static const std::string empty;
  return b && (b->kind == Value::BIN || b->kind == Value::STR) ? b->s : empty;
}

// fold every rank's diff (rank order) and apply what this store does not
// hold yet; -> rows written (their slots appended to *changed, with the
// slots of removed rows). forward: one round of a push MIX (what was applied
// is shipped again in the MIX's later rounds; the caller forgets the diff
// when the MIX ends)
template <class S>
size_t apply_row_diffs(S& st, const std::vector<Value>& parts, std::vector<int32_t>* changed,
                       bool forward = false) {
  struct Win {
    uint64_t v;
    size_t p, i;
  };
  std::unordered_map<std::string, Win> win;
  std::vector<std::string> order;
  std::map<std::string, uint64_t> gone;
  for (size_t p = 0; p < parts.size(); ++p) {
    const Value& d = parts[p];
    const Value* ids = d.get("ids");
    const Value* ver = d.get("ver");
    if (!ids || !ver || ids->kind != Value::ARR || ver->kind != Value::ARR || ids->a.size() != ver->a.size())
      throw std::runtime_error("mix: malformed row diff");
    for (size_t i = 0; i < ids->a.size(); ++i) {
      const std::string& id = ids->a[i].s;
      const uint64_t v = (uint64_t)ver->a[i].num();
      auto it = win.find(id);
      if (it == win.end()) {
        win[id] = {v, p, i};
        order.push_back(id);
      } else if (v >= it->second.v) {
        it->second = {v, p, i};
      }
    }
    if (const Value* rm = d.get("removed"))
      for (const Value& x : rm->a) {
        if (x.kind != Value::ARR || x.a.size() != 2) continue;
        const uint64_t v = (uint64_t)x.a[1].num();
        auto g = gone.find(x.a[0].s);
        if (g == gone.end() || v > g->second) gone[x.a[0].s] = v;
      }
  }
  size_t written = 0;
  for (size_t p = 0; p < parts.size(); ++p) {
    const Value& d = parts[p];
    const std::string& rpb = diff_bin(d.get("rp"));
    const std::string& ib = diff_bin(d.get("idx"));
    const std::string& vb = diff_bin(d.get("val"));
    const Value* dat = d.get("datum");
    const size_t nrp = rpb.size() / 8;
    for (const auto& id : order) {
      const Win& w = win[id];
      if (w.p != p) continue;
      uint64_t have = 0;
      if (st.version_of(id, &have) && have >= w.v && st.holds(id)) continue;
      if (!dat || dat->kind != Value::ARR || w.i >= dat->a.size() || w.i + 1 >= nrp)
        throw std::runtime_error("mix: malformed row diff");
      int64_t b, e;
      memcpy(&b, rpb.data() + 8 * w.i, 8);
      memcpy(&e, rpb.data() + 8 * (w.i + 1), 8);
      if (b < 0 || e < b || (size_t)e * 4 > ib.size() || (size_t)e * 4 > vb.size())
        throw std::runtime_error("mix: malformed row diff");
      std::vector<int32_t> idx((size_t)(e - b));
      std::vector<float> val((size_t)(e - b));
      if (e > b) {
        memcpy(idx.data(), ib.data() + 4 * b, 4 * (size_t)(e - b));
        memcpy(val.data(), vb.data() + 4 * b, 4 * (size_t)(e - b));
      }
      Datum dd;
      parse_datum(dat->a[w.i], &dd);
      st.store_mixed(id, std::move(dd), idx, val, w.v, forward);
      if (changed) changed->push_back(st.slot_id(id));
      ++written;
    }
  }
  for (const auto& g : gone) {
    uint64_t have = 0;
    if (!st.version_of(g.first, &have) || have <= g.second) {
      const int32_t s = st.slot_id(g.first);
      if (s >= 0 && changed) changed->push_back(s);
      st.remove_mixed(g.first, g.second, forward);
    }
  }
  int64_t docs = 0, len = 0;
  std::map<int64_t, int64_t> acc;
  bool any_w = false;
  for (const Value& d : parts) {
    const Value* w = d.get("w");
    if (!w || w->kind != Value::ARR || w->a.size() != 4) continue;
    any_w = true;
    docs += (int64_t)w->a[0].num();
    len += (int64_t)w->a[1].num();
    const std::string& wi = diff_bin(&w->a[2]);
    const std::string& wc = diff_bin(&w->a[3]);
    const size_t n = std::min(wi.size(), wc.size()) / 8;
    for (size_t k = 0; k < n; ++k) {
      int64_t i, c;
      memcpy(&i, wi.data() + 8 * k, 8);
      memcpy(&c, wc.data() + 8 * k, 8);
      acc[i] += c;
    }
  }
  if (any_w) {
    std::vector<int64_t> ks, cs;
    for (const auto& kv : acc) {
      ks.push_back(kv.first);
      cs.push_back(kv.second);
    }
    st.put_weight_diff(docs, len, ks, cs, forward);
  }
  if (!forward) st.mix_done();
  return written;
}

}  // namespace row
}  // namespace jb
