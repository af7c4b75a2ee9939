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
// The written rows travel as flat arrays - no msgpack object per row on the
// wire or in the receiver's parse (a 100 K-row diff decodes into a dozen
// values, not a million):
//   {"n": rows, "ids": bin (id bytes, concatenated), "ido": bin u32 [n + 1]
//    offsets, "ver": bin u64 [n], "dat": bin (each row's datum, msgpack
//    [sv, nv, bv], concatenated), "dato": bin u32 [n + 1], "rp": bin i64
//    [n + 1], "idx": bin i32, "val": bin f32 (the hashed vectors, CSR),
//    "removed": [[id, ver]...], "w": [docs, len, bin i64 idx, bin i64 count]}
// A receiver parses the datum of a row only when that row wins the fold and
// is not held already.
#pragma once
#include <cmath>
#include <string.h>

#include <algorithm>
#include <map>
#include <string_view>
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
  const size_t n = ids.size();
  std::vector<uint32_t> ido(1, 0), dato(1, 0);
  std::vector<uint64_t> ver(n);
  std::vector<int64_t> rp(1, 0);
  std::vector<int32_t> ci;
  std::vector<float> cv;
  std::string idb;
  MsgpackWriter dw;   // the datums, back to back
  for (size_t r = 0; r < n; ++r) {
    const std::string& id = ids[r];
    idb += id;
    ido.push_back((uint32_t)idb.size());
    uint64_t v = 0;
    st.version_of(id, &v);
    ver[r] = v;
    const Datum* d;
    const std::vector<int32_t>* ix;
    const std::vector<float>* vx;
    st.row_view(id, &d, &ix, &vx);
    write_datum(dw, *d);
    dato.push_back((uint32_t)dw.out.size());
    ci.insert(ci.end(), ix->begin(), ix->end());
    cv.insert(cv.end(), vx->begin(), vx->end());
    rp.push_back((int64_t)ci.size());
  }
  w.map(11);
  w.str("n");
  w.uint(n);
  w.str("ids");
  w.bin(idb.data(), idb.size());
  w.str("ido");
  w.bin(ido.data(), ido.size() * 4);
  w.str("ver");
  w.bin(ver.data(), ver.size() * 8);
  w.str("dat");
  w.bin(dw.out.data(), dw.out.size());
  w.str("dato");
  w.bin(dato.data(), dato.size() * 4);
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
// one rank's diff, its flat arrays checked once
struct DiffView {
  size_t n = 0;
  const std::string *ids, *ido, *ver, *dat, *dato, *rp, *idx, *val;
  uint32_t off(const std::string& b, size_t i) const {
    uint32_t x;
    memcpy(&x, b.data() + 4 * i, 4);
    return x;
  }
  std::string_view id(size_t i) const {
    const uint32_t a = off(*ido, i), b = off(*ido, i + 1);
    return std::string_view(ids->data() + a, b - a);
  }
  uint64_t version(size_t i) const {
    uint64_t v;
    memcpy(&v, ver->data() + 8 * i, 8);
    return v;
  }
};

inline DiffView diff_view(const Value& d) {
  DiffView v;
  const Value* n = d.get("n");
  if (!n || !n->is_num()) throw std::runtime_error("mix: malformed row diff");
  // n is a peer's double: reject negative / non-integral / NaN values before
  // the cast, and compare sizes by division so no product can wrap
  const double nd = n->num();
  if (!(nd >= 0) || nd != std::floor(nd) || nd > 9.0e15) throw std::runtime_error("mix: malformed row diff");
  v.n = (size_t)nd;
  v.ids = &diff_bin(d.get("ids"));
  v.ido = &diff_bin(d.get("ido"));
  v.ver = &diff_bin(d.get("ver"));
  v.dat = &diff_bin(d.get("dat"));
  v.dato = &diff_bin(d.get("dato"));
  v.rp = &diff_bin(d.get("rp"));
  v.idx = &diff_bin(d.get("idx"));
  v.val = &diff_bin(d.get("val"));
  auto count_is = [](const std::string* b, size_t width, size_t want) {
    return b->size() % width == 0 && b->size() / width == want;
  };
  if (!count_is(v.ver, 8, v.n) || !count_is(v.ido, 4, v.n + 1) || !count_is(v.dato, 4, v.n + 1) ||
      !count_is(v.rp, 8, v.n + 1))
    throw std::runtime_error("mix: malformed row diff");
  for (size_t i = 0; i < v.n; ++i)
    if (v.off(*v.ido, i) > v.off(*v.ido, i + 1) || v.off(*v.dato, i) > v.off(*v.dato, i + 1))
      throw std::runtime_error("mix: malformed row diff");
  if (v.off(*v.ido, v.n) > v.ids->size() || v.off(*v.dato, v.n) > v.dat->size())
    throw std::runtime_error("mix: malformed row diff");
  return v;
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
    uint32_t p;
    uint32_t i;
  };
  std::vector<DiffView> views;
  size_t total = 0;
  for (const Value& d : parts) {
    views.push_back(diff_view(d));
    total += views.back().n;
  }
  // newest version wins, the later rank on ties (keys view the payloads)
  std::unordered_map<std::string_view, Win> win;
  win.reserve(total);
  std::vector<std::string_view> order;
  order.reserve(total);
  std::map<std::string, uint64_t> gone;
  for (size_t p = 0; p < parts.size(); ++p) {
    const DiffView& dv = views[p];
    for (size_t i = 0; i < dv.n; ++i) {
      const std::string_view id = dv.id(i);
      const uint64_t v = dv.version(i);
      auto it = win.find(id);
      if (it == win.end()) {
        win.emplace(id, Win{v, (uint32_t)p, (uint32_t)i});
        order.push_back(id);
      } else if (v >= it->second.v) {
        it->second = Win{v, (uint32_t)p, (uint32_t)i};
      }
    }
    if (const Value* rm = parts[p].get("removed"))
      for (const Value& x : rm->a) {
        if (x.kind != Value::ARR || x.a.size() != 2) continue;
        const uint64_t v = (uint64_t)x.a[1].num();
        auto g = gone.find(x.a[0].s);
        if (g == gone.end() || v > g->second) gone[x.a[0].s] = v;
      }
  }
  // the winners of each part, in first-seen order
  std::vector<std::vector<Win>> by_part(parts.size());
  for (const std::string_view idv : order) {
    const Win& w = win.find(idv)->second;
    by_part[w.p].push_back(w);
  }
  size_t written = 0;
  std::string id;
  std::vector<int32_t> idx;
  std::vector<float> val;
  for (size_t p = 0; p < parts.size(); ++p) {
    const DiffView& dv = views[p];
    for (const Win& w : by_part[p]) {
      const std::string_view idv = dv.id(w.i);
      id.assign(idv.data(), idv.size());
      uint64_t have = 0;
      if (st.version_of(id, &have) && have >= w.v && st.holds(id)) continue;
      int64_t b, e;
      memcpy(&b, dv.rp->data() + 8 * (size_t)w.i, 8);
      memcpy(&e, dv.rp->data() + 8 * ((size_t)w.i + 1), 8);
      if (b < 0 || e < b || (size_t)e * 4 > dv.idx->size() || (size_t)e * 4 > dv.val->size())
        throw std::runtime_error("mix: malformed row diff");
      idx.resize((size_t)(e - b));
      val.resize((size_t)(e - b));
      if (e > b) {
        memcpy(idx.data(), dv.idx->data() + 4 * b, 4 * (size_t)(e - b));
        memcpy(val.data(), dv.val->data() + 4 * b, 4 * (size_t)(e - b));
      }
      const uint32_t da = dv.off(*dv.dato, w.i), db = dv.off(*dv.dato, (size_t)w.i + 1);
      Datum dd;
      parse_datum(jb::val::MsgpackReader((const uint8_t*)dv.dat->data() + da, db - da).read(), &dd);
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
