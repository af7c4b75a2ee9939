"""Common driver of the row-oriented engines: a RowStore + a similarity
index (LSH family on the GPU, or the exact inverted index) + the converter.

MIX (the reference's versioned column table, mixed by linear_mixer): the
diff is every row changed or removed since the last MIX with its version;
diffs are folded newest-version-wins and applied everywhere, so every
server can answer random-routed queries over all rows.
"""
from __future__ import annotations

import contextlib
import gc
import threading
from typing import Any

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum, as_datum
from .rows import RowStore, Unlearner, as_dicts, datum_to_dicts, dicts_to_datum, dicts_wire
from .similarity import InvertedIndex, LshIndex

LSH_METHODS = ("lsh", "euclid_lsh", "minhash")
INDEX_METHODS = LSH_METHODS + ("inverted_index", "inverted_index_euclid")


def make_index(method: str, parameter: dict, device: Any):
    if method in LSH_METHODS:
        return LshIndex(method, int(parameter.get("hash_num", 64)),
                        int(parameter.get("seed", 1091)), device)
    if method == "inverted_index":
        return InvertedIndex(False, device)
    if method == "inverted_index_euclid":
        return InvertedIndex(True, device)
    raise ValueError(f"unknown similarity method: {method}")



@contextlib.contextmanager
def _gc_paused():
    """no cyclic-GC passes while a bulk ingest allocates millions of small
    objects (with a large live heap, collections cost more than the work)"""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()

class RowEngine:
    def __init__(self, method: str, parameter: dict | None, converter: DatumToFvConverter,
                 device: Any = None, unlearner: str | None = None,
                 unlearner_parameter: dict | None = None):
        self.method = method
        self.parameter = dict(parameter or {})
        self.conv = converter
        self.device = device
        self.gpu = device is not None
        self.index = make_index(method, self.parameter, device)
        self.rows = RowStore()
        self.unlearner = Unlearner(unlearner, unlearner_parameter)
        self._lock = threading.RLock()
        self._last_mix: dict = {}
        self._host_hasher = None

    # ------------------------------------------------------------ rows
    def fv_of(self, d: Datum, update_weight: bool = False):
        f = self.conv.convert_and_update_weight(d) if update_weight else self.conv.convert(d)
        return self.conv.hashed(f)

    def _set(self, rid: str, dicts, bump: bool = True, update_weight: bool = True) -> None:
        if self.gpu and hasattr(self.index, "set_rows_direct") and \
                self._set_direct(rid, dicts, bump, update_weight):
            pass
        else:
            fv = self.fv_of(dicts_to_datum(*dicts), update_weight)
            slot = self.rows.put(rid, dicts, fv, bump)
            self.index.set_rows([slot], [fv])
        for victim in self.unlearner.touch(rid):
            if victim != rid:
                self._remove(victim)

    def _hasher(self):
        """native host converter when the converter config allows it, else
        None: csrc/native/jb_hostfv.hpp for the plain rule set,
        csrc/native/jb_hostfv_wide.hpp for ngram / space splitters, tf /
        idf / bm25 weights (the WeightManager's arrays, updated in place) and
        combinations. No filters / plug-ins / regex matchers."""
        if self._host_hasher is None:
            from ..fv_converter.gpu_path import (GpuRuleTable, WideRuleTable, fast_eligible,
                                                 wide_eligible)
            from .._native import native
            if fast_eligible(self.conv):
                rt = GpuRuleTable(self.conv)
                self._host_hasher = native().HostFvHasher(rt.srules, rt.n_srules, rt.nrules,
                                                          rt.n_nrules, rt.blob, rt.H)
            elif wide_eligible(self.conv):
                rt = WideRuleTable(self.conv)
                h = native().HostFvWide(rt.srules, rt.n_srules, rt.nrules, rt.n_nrules, rt.crules,
                                        rt.n_crules, rt.blob, rt.H)
                if h.needs_weights():
                    df, diff, counts = self.conv.weights.arrays()
                    h.set_weights(df.ctypes.data, diff.ctypes.data, counts.ctypes.data)
                self._host_hasher = h
            else:
                self._host_hasher = False
        return self._host_hasher or None

    def _set_many(self, items: list, bump: bool = True, update_weight: bool = True) -> None:
        """set many rows at once: one native hashing pass over all datums and
        one bulk index insert (signatures of every row in one launch)."""
        with _gc_paused():
            self._set_many_impl(items, bump, update_weight)

    def _set_many_impl(self, items: list, bump: bool, update_weight: bool) -> None:
        h = self._hasher()
        if h is None or len(items) < 2 or self.unlearner.kind:
            # (the lru unlearner interleaves evictions with inserts: sequential)
            for rid, dicts in items:
                self._set(rid, dicts, bump, update_weight)
            return
        import msgpack
        import numpy as np
        body = msgpack.packb([dicts_wire(d) for _, d in items], use_bin_type=False)
        n = len(items)
        cap = max(1024, 64 * n)
        while True:
            idx = np.empty(cap, np.int32)
            val = np.empty(cap, np.float32)
            rp = np.zeros(n + 1, np.int64)
            # (a failed call rolls back its document-statistics updates)
            got, _, err = h.hash([body], idx.ctypes.data, val.ctypes.data, rp.ctypes.data, n, cap,
                                 update_weight)
            if err == 2:
                cap *= 4
                continue
            if err:
                raise ValueError("malformed datum in bulk row update")
            break
        nnz = int(rp[n])
        idx, val = idx[:nnz], val[:nnz]
        slots = self.rows.put_many(items, rp, idx, val, bump)
        # a row set twice in one batch: the last write wins (same as sequential)
        last = {}
        for i, (rid, _) in enumerate(items):
            last[rid] = i
        if len(last) == n:
            self.index.set_rows_csr(slots, rp, idx, val)
        else:
            sel = np.asarray(sorted(last.values()), np.int64)
            lens = rp[sel + 1] - rp[sel]
            rp2 = np.zeros(sel.size + 1, np.int64)
            np.cumsum(lens, out=rp2[1:])
            gather = np.repeat(rp[sel] - rp2[:-1], lens) + np.arange(int(rp2[-1]), dtype=np.int64)
            self.index.set_rows_csr(slots[sel], rp2, idx[gather], val[gather])
        for rid, _ in items:
            for victim in self.unlearner.touch(rid):
                if victim != rid:
                    self._remove(victim)

    def _set_direct(self, rid: str, dicts, bump: bool, update_weight: bool = True) -> bool:
        """native hashing + one index write into the row's slot"""
        h = self._hasher()
        if h is None:
            return False
        import msgpack
        import numpy as np
        from ..ops import hip
        body = msgpack.packb([dicts_to_datum(*dicts).to_msgpack()], use_bin_type=False)
        idx = np.empty(hip.QUERY_SLOTS, np.int32)
        val = np.empty(hip.QUERY_SLOTS, np.float32)
        rp = np.zeros(2, np.int64)
        n, _, err = h.hash([body], idx.ctypes.data, val.ctypes.data, rp.ctypes.data, 1,
                           hip.QUERY_SLOTS, update_weight)
        if err or n != 1:
            return False
        keep = idx[:rp[1]] >= 0
        fv = (idx[:rp[1]][keep].tolist(), val[:rp[1]][keep].tolist())
        slot = self.rows.put(rid, dicts, fv, bump)
        if not self.index.set_rows_direct(np.asarray([slot], np.int64), rp, idx, val):
            self.index.set_rows([slot], [fv])
        return True

    def set_rows(self, items: list) -> int:
        """bulk set_row: [(id, datum)] -> number of rows written"""
        with self._lock, _gc_paused():
            self._set_many([(rid, as_dicts(d)) for rid, d in items])
            return len(items)

    def _remove(self, rid: str, record: bool = True) -> bool:
        s = self.rows.remove(rid, record)
        if s is None:
            return False
        self.index.remove(s)
        self.unlearner.remove(rid)
        return True

    def set_row(self, rid: str, d: Any) -> bool:
        with self._lock:
            self._set(rid, datum_to_dicts(as_datum(d)))
            return True

    def update_row(self, rid: str, d: Any) -> bool:
        """merge the datum into the existing row (recommender update_row)"""
        with self._lock:
            new = datum_to_dicts(as_datum(d))
            s = self.rows.slot(rid)
            if s is not None:
                sv, nv, bv = (dict(x) for x in self.rows.datum[s])
                sv.update(new[0]); nv.update(new[1]); bv.update(new[2])
                new = (sv, nv, bv)
            self._set(rid, new)
            return True

    def clear_row(self, rid: str) -> bool:
        with self._lock:
            return self._remove(rid)

    def clear(self) -> None:
        with self._lock:
            self.rows.clear()
            self.index.clear()
            self.unlearner.clear()
            self.conv.weights.clear()

    def get_all_rows(self) -> list[str]:
        with self._lock:
            return self.rows.all_ids()

    # ------------------------------------------------------------ queries
    def _results(self, res: list[tuple[int, float]]) -> list[tuple[str, float]]:
        out = []
        for slot, score in res:
            rid = self.rows.id_of(slot)
            if rid is not None:
                out.append((rid, float(score)))
        return out

    def query_fv_slots(self, fv, k: int, similar: bool) -> list[tuple[int, float]]:
        """k nearest stored rows of a feature vector -> [(slot, score)]"""
        with self._lock:
            n = self.rows.nslots
            if n == 0 or k <= 0:
                return []
            if self.gpu and hasattr(self.index, "query_direct") and len(fv[0]) <= 256:
                import numpy as np
                idx = np.asarray(fv[0], np.int32)
                val = np.asarray(fv[1], np.float32)
                rp = np.asarray([0, idx.size], np.int64)
                r = self.index.query_direct(idx, val, rp, 1, n, k, similar)
                if r is not None:
                    return list(r[0])
            (r,) = self.index.query([fv], n, k, similar)
            return list(r)

    def query_fv(self, fv, k: int, similar: bool) -> list[tuple[str, float]]:
        with self._lock:
            return self._results(self.query_fv_slots(fv, k, similar))

    def query_datum(self, d: Any, k: int, similar: bool) -> list[tuple[str, float]]:
        d = as_datum(d)
        if self.gpu and hasattr(self.index, "query_direct") and k > 0:
            r = self._query_datum_direct(d, k, similar)
            if r is not None:
                return r
        return self.query_fv(self.fv_of(d), k, similar)

    def _query_datum_direct(self, d, k: int, similar: bool):
        r = self._query_datum_slots_direct(d, k, similar)
        return None if r is None else self._results(r)

    def _query_datum_slots_direct(self, d, k: int, similar: bool):
        """native hashing of the datum + the single-shot LSH query kernel
        -> [(slot, score)] or None (not eligible)"""
        h = self._hasher()
        if h is None:
            return None
        import msgpack
        import numpy as np
        body = msgpack.packb([d.to_msgpack()], use_bin_type=False)
        from ..ops import hip
        idx = np.empty(hip.QUERY_SLOTS, np.int32)
        val = np.empty(hip.QUERY_SLOTS, np.float32)
        rp = np.zeros(2, np.int64)
        n, _, err = h.hash([body], idx.ctypes.data, val.ctypes.data, rp.ctypes.data, 1,
                           hip.QUERY_SLOTS)
        if err or n != 1:
            return None
        with self._lock:
            nrows = self.rows.nslots
            if nrows == 0:
                return []
            r = self.index.query_direct(idx, val, rp, 1, nrows, k, similar)
            if r is None:
                return None
            return list(r[0])

    def query_id(self, rid: str, k: int, similar: bool) -> list[tuple[str, float]]:
        with self._lock:
            s = self.rows.slot(rid)
            if s is None:
                raise KeyError(f"row not found: {rid}")
            if hasattr(self.index, "query_slots") and k > 0:
                r = self.index.query_slots([s], self.rows.nslots, k, similar)
                if r is not None:
                    return self._results(r[0])
            return self.query_fv(self.rows.fv[s], k, similar)

    def query_slot_lists(self, slots: list[int], k: int, similar: bool) -> list[list[tuple[int, float]]]:
        """batched query by stored row (each row's neighbours, itself
        included) -> per row [(slot, score)]: stored signatures / pool rows,
        QUERY_MAX queries per launch on the GPU"""
        with self._lock:
            n = self.rows.nslots
            res = None
            if hasattr(self.index, "query_slots"):
                from ..ops import hip
                if len(slots) > hip.QUERY_MAX and self.gpu:
                    res = []
                    for i in range(0, len(slots), hip.QUERY_MAX):
                        part = self.index.query_slots(slots[i:i + hip.QUERY_MAX], n, k, similar)
                        if part is None:
                            res = None
                            break
                        res.extend(part)
                else:
                    res = self.index.query_slots(slots, n, k, similar)
            if res is None:
                res = self.index.query([self.rows.fv[s] for s in slots], n, k, similar)
            ids = self.rows.ids
            return [[(int(o), float(d)) for o, d in r if ids[o] is not None] for r in res]

    def query_ids(self, rids: list[str], k: int, similar: bool) -> dict[str, list[tuple[str, float]]]:
        """batched query_id (every row's neighbours, itself included)"""
        with self._lock:
            slots = [self.rows.slot(r) for r in rids]
            if any(s is None for s in slots):
                raise KeyError("row not found")
            res = self.query_slot_lists(slots, k, similar)
            return {rid: self._results(r) for rid, r in zip(rids, res)}

    # ------------------------------------------------------------ MIX
    def mix(self, group=None) -> int:
        """collective MIX over the process group (parallel/row_mix.py: one
        byte tensor per rank, RCCL / gloo all-gather, no pickling); returns
        the bytes this rank contributed"""
        from ..parallel.row_mix import row_mix
        st = row_mix(self, group)
        self._last_mix = st
        return st["bytes"]

    def pair_mix(self, peer: int, group=None) -> None:
        """symmetric MIX with one peer (push mixers)"""
        from ..parallel.row_mix import row_mix
        self._last_mix = row_mix(self, group, peer=peer)

    def _rows_changed(self, slots) -> None:
        """rows rewritten by a MIX (hook: derived state such as LOF lists)"""

    def get_diff(self) -> dict:
        return self.rows.get_diff()

    @staticmethod
    def mix_diff(a: dict, b: dict) -> dict:
        return RowStore.mix_diff(a, b)

    def put_diff(self, mixed: dict) -> bool:
        with self._lock:
            todo = [(rid, v, d) for rid, (v, d) in mixed["rows"].items()
                    if self.rows.version.get(rid, -1) < v or rid not in self.rows.slot_of]
            self._set_many([(rid, tuple(dict(x) for x in d)) for rid, _, d in todo], bump=False,
                           update_weight=False)
            for rid, v, _ in todo:
                self.rows.version[rid] = v
            for rid, v in mixed["removed"].items():
                if self.rows.version.get(rid, -1) <= v:
                    self._remove(rid, record=False)
                    self.rows.version[rid] = v
            self.rows.dirty.clear()
            self.rows.removed.clear()
            return True

    # ------------------------------------------------------------ persist
    def pack(self) -> dict:
        with self._lock:
            return {"method": self.method, "rows": self.rows.pack()["rows"],
                    "weights": self.conv.weights.pack()}

    def unpack(self, obj: dict) -> None:
        with self._lock:
            self.clear()
            if obj.get("weights"):
                self.conv.weights.unpack(obj["weights"])
            items = list(obj["rows"].items())
            self._set_many([(rid, tuple(dict(x) for x in d)) for rid, (_, d) in items], bump=False,
                           update_weight=False)
            for rid, (v, _) in items:
                self.rows.version[rid] = v

    def get_status(self) -> dict[str, str]:
        st = {"method": self.method, "num_rows": str(len(self.rows.slot_of)),
              "storage": "hbm" if self.gpu else "host",
              "unlearner": self.unlearner.kind or "none"}
        for k, v in self._last_mix.items():
            st[f"mix.last_{k}"] = str(v)
        return st
