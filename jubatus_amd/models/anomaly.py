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
kdist / lrd of stored rows are cached and invalidated for the
``reverse_nearest_neighbor_num`` rows nearest to every inserted/updated
row. ``ignore_kth_same_point`` skips zero-distance (duplicate) neighbours
when taking the k-th distance.
"""
from __future__ import annotations

import math
from typing import Any

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import as_datum
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
        self._kdist: dict[str, float] = {}
        self._lrd: dict[str, float] = {}

    # neighbours in *distance* order
    def _neighbors_fv(self, fv, k: int, exclude: str | None = None) -> list[tuple[str, float]]:
        res = self.query_fv(fv, k + (1 if exclude else 0), similar=False)
        return [(r, d) for r, d in res if r != exclude][:k]

    def _neighbors_id(self, rid: str, k: int) -> list[tuple[str, float]]:
        s = self.rows.slot(rid)
        return self._neighbors_fv(self.rows.fv[s], k, exclude=rid)

    def _kth(self, nb: list[tuple[str, float]]) -> float:
        ds = [d for _, d in nb]
        if self.ignore_kth_same:
            ds = [d for d in ds if d > 0] or [0.0]
        return ds[-1] if ds else 0.0

    def kdist(self, rid: str) -> float:
        v = self._kdist.get(rid)
        if v is None:
            v = self._kth(self._neighbors_id(rid, self.k))
            self._kdist[rid] = v
        return v

    def _lrd_of(self, nb: list[tuple[str, float]]) -> float:
        if not nb:
            return 0.0
        mean_reach = sum(max(self.kdist(o), d) for o, d in nb) / len(nb)
        return math.inf if mean_reach <= 0 else 1.0 / mean_reach

    def lrd(self, rid: str) -> float:
        v = self._lrd.get(rid)
        if v is None:
            v = self._lrd_of(self._neighbors_id(rid, self.k))
            self._lrd[rid] = v
        return v

    def _knn_many(self, rids: list[str], k: int) -> dict[str, list[tuple[str, float]]]:
        res = self.query_ids(rids, k + 1, similar=False)
        return {rid: [(o, d) for o, d in nb if o != rid][:k] for rid, nb in res.items()}

    def _prefetch(self, nb: list[tuple[str, float]]) -> None:
        """warm the lrd/kdist caches _score(nb) needs with two batched kNN
        launches (neighbours of the neighbours, then the kdist of theirs)
        instead of one query per row"""
        need = [o for o, _ in nb if o not in self._lrd]
        if not need:
            return
        lists = self._knn_many(need, self.k)
        for o, lo in lists.items():
            self._kdist.setdefault(o, self._kth(lo))
        need_k = sorted({x for lo in lists.values() for x, _ in lo if x not in self._kdist})
        if need_k:
            for x, lx in self._knn_many(need_k, self.k).items():
                self._kdist[x] = self._kth(lx)
        for o, lo in lists.items():
            self._lrd[o] = self._lrd_of(lo)

    def _score(self, nb: list[tuple[str, float]]) -> float:
        if not nb:
            return 1.0
        self._prefetch(nb)
        lp = self._lrd_of(nb)
        lo = [self.lrd(o) for o, _ in nb]
        mean_lo = sum(lo) / len(lo)
        if math.isinf(lp):
            return 1.0 if math.isinf(mean_lo) else 0.0
        if lp == 0.0:
            return math.inf
        if math.isinf(mean_lo):
            return math.inf
        return mean_lo / lp

    def _invalidate_near(self, fv, rid: str) -> list[tuple[str, float]]:
        """drop the cached kdist / lrd the change of ``rid`` can affect;
        returns its reverse_nearest_neighbor_num nearest rows"""
        self._kdist.pop(rid, None)
        self._lrd.pop(rid, None)
        near = self._neighbors_fv(fv, self.rnn, exclude=rid)
        for o, _ in near:
            self._kdist.pop(o, None)
            self._lrd.pop(o, None)
        # lrd depends on the neighbours' kdist: drop every cached lrd
        self._lrd.clear()
        return near

    def _insert(self, rid: str, dicts) -> float:
        self._set(rid, dicts)
        fv = self.rows.fv[self.rows.slot(rid)]
        near = self._invalidate_near(fv, rid)
        # the k nearest are the head of the rnn-nearest list (same query,
        # rnn >= k): no second search
        return self._score(near[:self.k])

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
            s = self.rows.slot(rid)
            if s is None:
                return False
            fv = self.rows.fv[s]
            ok = self._remove(rid)
            self._invalidate_near(fv, rid)
            return ok

    def calc_score(self, d) -> float:
        with self._lock:
            return self._score(self._neighbors_fv(self.fv_of(as_datum(d)), self.k))

    def clear(self) -> None:
        super().clear()
        self._kdist = {}
        self._lrd = {}

    def put_diff(self, mixed: dict) -> bool:
        ok = super().put_diff(mixed)
        self._kdist.clear()
        self._lrd.clear()
        return ok

    def unpack(self, obj: dict) -> None:
        super().unpack(obj)
        self._kdist.clear()
        self._lrd.clear()

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
