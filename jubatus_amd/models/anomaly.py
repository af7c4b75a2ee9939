"""Anomaly detection: LOF and light_lof (Breunig et al., SIGMOD 2000).

Reference: jubatus/server/server/anomaly_serv.cpp:126-320 over jubatus_core's
lof / light_lof (EXTERNAL). ``lof`` runs on a recommender backend method
(inverted_index, inverted_index_euclid, lsh, minhash, euclid_lsh) and
``light_lof`` on a nearest_neighbor backend method (lsh, euclid_lsh,
minhash); both use the same row index here (models/row_engine.py), with the
k-nearest-neighbor search on the GPU for the LSH family.

For a point p with neighbours N_k(p) at distances d(p, o):
    kdist(o)       distance from o to its k-th neighbour
    reach(p, o)    max(kdist(o), d(p, o))
    lrd(p)         1 / mean_o reach(p, o)
    LOF(p)         mean_o lrd(o) / lrd(p)
Every stored row keeps its k-neighbour list, kdist and lrd
(models/lof_state.py; in HBM with csrc/hip/lof.hip on the GPU). An insert
queries the new row's ``reverse_nearest_neighbor_num`` nearest once, takes
the row into the lists of those neighbours it is close enough to, and marks
stale exactly the lrd values that depend on a changed list; the score then
refreshes only those. ``ignore_kth_same_point`` skips zero-distance
(duplicate) neighbours when taking the k-th distance.
"""
from __future__ import annotations

from typing import Any

import numpy as np

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import as_datum
from .lof_state import DeviceLofState, HostLofState
from .row_engine import INDEX_METHODS, LSH_METHODS, RowEngine
from .rows import datum_to_dicts


class LOF(RowEngine):
    def __init__(self, method: str, parameter: dict | None, converter: DatumToFvConverter,
                 device: Any = None):
        p = dict(parameter or {})
        if method not in ("lof", "light_lof"):
            raise ValueError(f"unsupported anomaly method: {method}")
        inner = p.get("method")
        allowed = INDEX_METHODS if method == "lof" else LSH_METHODS
        if inner not in allowed:
            raise ValueError(f"{method}: parameter.method must be one of {allowed}")
        self.k = int(p.get("nearest_neighbor_num", 10))
        self.rnn = int(p.get("reverse_nearest_neighbor_num", 30))
        if self.k <= 0 or self.rnn < self.k:
            raise ValueError("nearest_neighbor_num must be > 0 and <= reverse_nearest_neighbor_num")
        self.ignore_kth_same = bool(p.get("ignore_kth_same_point", False))

        self.outer = method
        super().__init__(inner, dict(p.get("parameter") or {}), converter, device,
                         p.get("unlearner"), p.get("unlearner_parameter"))
        self._st = None          # HostLofState / DeviceLofState (models/lof_state.py)

    # ------------------------------------------------------------ state
    def _state(self):
        if self._st is None:
            if self.gpu:
                self._st = DeviceLofState(self.k, self.ignore_kth_same, self.device)
            else:
                self._st = HostLofState(self.k, self.ignore_kth_same)
        self._st.ensure(self.rows.nslots)
        return self._st

    @staticmethod
    def _pairs(lst) -> tuple[np.ndarray, np.ndarray]:
        return (np.asarray([o for o, _ in lst], np.int32),
                np.asarray([d for _, d in lst], np.float32))

    def _score_from(self, ts: np.ndarray, td: np.ndarray, store: int = -1) -> float:
        """LOF from the k nearest (slot, distance) pairs; rows whose
        neighbour lists are missing (bulk-loaded, or next to a row that moved)
        get them from batched kNN queries first"""
        st = self._state()
        for _ in range(1 + 2 * self.k):
            sc, missing = st.score(ts, td, store)
            if sc is not None:
                return sc
            lists = self.query_slot_lists(missing, self.k + 1, similar=False)
            st.set_lists(missing, [self._pairs(lst) for lst in lists])
        raise RuntimeError("lof: neighbour lists did not converge")

    def _insert(self, rid: str, dicts) -> float:
        existed = self.rows.slot(rid) is not None
        self._set(rid, dicts)
        s = self.rows.slot(rid)
        st = self._state()
        if existed:
            st.moved([s])
        (near,) = self.query_slot_lists([s], self.rnn + 1, similar=False)
        cs, cd = self._pairs([(o, d) for o, d in near if o != s][:self.rnn])
        # insert + score in one device call; the k nearest are the head of
        # the rnn-nearest list (same query, rnn >= k): no second search
        sc, missing = st.add(s, cs, cd)
        if sc is not None:
            return sc
        return self._score_from(cs[:self.k], cd[:self.k], store=s)

    def _remove(self, rid: str, record: bool = True) -> bool:
        s = self.rows.slot(rid)
        ok = super()._remove(rid, record)
        if ok and self._st is not None:
            self._st.moved([s])
        return ok

    # a MIX / bulk write that changes at least this share of the stored rows
    # rebuilds every neighbour list (exact k-NN of the whole set); smaller ones
    # are applied incrementally
    REBUILD_ALL_FRACTION = 0.25

    def _rows_changed(self, slots) -> None:
        """rows written by a MIX (inserted, replaced or removed): applied
        incrementally, as a batch of adds - the changed rows' lists and every
        list naming them are invalidated (one device pass per 1024 rows), the
        rows among the reverse_nearest_neighbor_num nearest of a changed row
        that now have it inside their k-distance join them, and all those
        lists are rebuilt with batched k-NN queries right away, so the first
        adds and scores after the MIX find a warm state (the lists were
        wiped past 4096 rows before)."""
        if self._st is None or not len(slots):
            return
        self._apply_changed([int(s) for s in slots])

    def _set_many(self, items: list, bump: bool = True, update_weight: bool = True) -> None:
        super()._set_many(items, bump, update_weight)
        if self._st is None or not items:
            return
        self._apply_changed([self.rows.slot(rid) for rid, _ in items])

    def _apply_changed(self, slots: list, chunk: int = 1024) -> None:
        st = self._state()
        ids = self.rows.ids
        live_n = sum(1 for r in ids if r is not None)
        slots = sorted(set(s for s in slots if s is not None))
        if not slots:
            return
        st.moved(slots)
        if live_n == 0:
            return
        if len(slots) >= self.REBUILD_ALL_FRACTION * live_n:
            st.moved([s for s, r in enumerate(ids) if r is not None])
            self.build_lists(chunk)
            return
        alive = [s for s in slots if s < len(ids) and ids[s] is not None]
        kd = st.kdist[:len(ids)].cpu().numpy() if hasattr(st.kdist, "cpu") else np.asarray(st.kdist[:len(ids)])
        ok = st.ok[:len(ids)].cpu().numpy() if hasattr(st.ok, "cpu") else np.asarray(st.ok[:len(ids)])
        affected = set(alive)
        for i in range(0, len(alive), chunk):
            part = alive[i:i + chunk]
            for s, lst in zip(part, self.query_slot_lists(part, self.rnn + 1, similar=False)):
                for o, d in lst:
                    if o != s and (not ok[o] or d <= kd[o]):
                        affected.add(o)
        todo = sorted(affected)
        for i in range(0, len(todo), chunk):
            part = todo[i:i + chunk]
            st.set_lists(part, [self._pairs(lst) for lst in self.query_slot_lists(part, self.k + 1,
                                                                                   similar=False)])
        # lists invalidated because they named a changed row
        self.build_lists(chunk)

    def build_lists(self, chunk: int = 1024, progress=None) -> int:
        """compute the neighbour list of every stored row that has none
        (after a bulk load / MIX / model load) with batched kNN queries, so
        later adds and scores find a warm state; returns the rows built"""
        with self._lock:
            st = self._state()
            n = self.rows.nslots
            ok = st.ok[:n].cpu().numpy() if hasattr(st.ok, "cpu") else st.ok[:n]
            ids = self.rows.ids
            todo = [s for s in np.flatnonzero(ok == 0).tolist() if ids[s] is not None]
            for i in range(0, len(todo), chunk):
                part = todo[i:i + chunk]
                lists = self.query_slot_lists(part, self.k + 1, similar=False)
                st.set_lists(part, [self._pairs(lst) for lst in lists])
                if progress and (i // chunk) % 64 == 0:
                    progress(i + len(part), len(todo))
            return len(todo)

    # ---------------------------------------------------------------- API
    def add(self, rid: str, d) -> float:
        with self._lock:
            return self._insert(rid, datum_to_dicts(as_datum(d)))

    def update(self, rid: str, d) -> float:
        with self._lock:
            new = datum_to_dicts(as_datum(d))
            s = self.rows.slot(rid)
            if s is not None:
                sv, nv, bv = (dict(x) for x in self.rows.datum[s])
                sv.update(new[0]); nv.update(new[1]); bv.update(new[2])
                new = (sv, nv, bv)
            return self._insert(rid, new)

    def overwrite(self, rid: str, d) -> float:
        with self._lock:
            return self._insert(rid, datum_to_dicts(as_datum(d)))

    def clear_row(self, rid: str) -> bool:
        with self._lock:
            return self._remove(rid)

    def calc_score(self, d) -> float:
        with self._lock:
            d = as_datum(d)
            nb = None
            if self.gpu and hasattr(self.index, "query_direct"):
                nb = self._query_datum_slots_direct(d, self.k, similar=False)
            if nb is None:
                nb = self.query_fv_slots(self.fv_of(d), self.k, similar=False)
            ids = self.rows.ids
            ts, td = self._pairs([(o, dd) for o, dd in nb if ids[o] is not None])
            return self._score_from(ts, td)

    def clear(self) -> None:
        super().clear()
        self._st = None

    def unpack(self, obj: dict) -> None:
        self._st = None
        super().unpack(obj)

    def find_max_int_id(self) -> int:
        m = -1
        for rid in self.rows.all_ids():
            if rid.isdigit():
                m = max(m, int(rid))
        return m

    def get_status(self) -> dict[str, str]:
        st = super().get_status()
        st["method"] = self.outer
        st["backend"] = self.method
        return st
