"""Nearest-neighbor and recommender drivers.

References: nearest_neighbor_serv.cpp:96-178 (methods lsh / euclid_lsh /
minhash) and recommender_serv.cpp:105-224 (inverted_index,
inverted_index_euclid, lsh, minhash, euclid_lsh, nearest_neighbor_recommender;
unlearner lru). Core algorithms are EXTERNAL (jubatus_core); ours:

* neighbor_row_*   -> [(id, distance)] ascending (lsh/minhash: normalised
  Hamming distance; euclid_lsh: approximate euclidean distance from the
  norms and the estimated angle; inverted_index_euclid: exact euclidean)
* similar_row_*    -> [(id, similarity)] descending (1 - distance for
  lsh/minhash, cosine for inverted_index, -distance for the euclid methods)
* complete_row_*   -> the datum's numeric values completed with the
  similarity-weighted mean of its neighbours' values (neighbours = the
  ``COMPLETE_K`` most similar rows)
* decode_row       -> the stored (merged) datum
* calc_similarity / calc_l2norm on the converted feature vectors.

Parameters ``bin_width``, ``probe_num``, ``table_num`` of the reference's
multi-table euclid_lsh are accepted; our signature scan is exhaustive over
the whole table, which makes them unnecessary.
"""
from __future__ import annotations

import math
from typing import Any

import numpy as np

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum, as_datum
from .row_engine import INDEX_METHODS, LSH_METHODS, RowEngine
from .rows import dicts_to_datum
from .similarity import LshIndex, signature_host

COMPLETE_K = 10


class NearestNeighbor(RowEngine):
    def __init__(self, method: str, parameter: dict | None, converter: DatumToFvConverter,
                 device: Any = None):
        if method not in LSH_METHODS:
            raise ValueError(f"unsupported nearest_neighbor method: {method}")
        p = dict(parameter or {})
        super().__init__(method, p, converter, device, p.get("unlearner"),
                         p.get("unlearner_parameter"))

    def neighbor_row_from_id(self, rid: str, size: int):
        return self.query_id(rid, int(size), similar=False)

    def neighbor_row_from_datum(self, d, size: int):
        return self.query_datum(d, int(size), similar=False)

    def similar_row_from_id(self, rid: str, n: int):
        return self.query_id(rid, int(n), similar=True)

    def similar_row_from_datum(self, d, n: int):
        return self.query_datum(d, int(n), similar=True)


class Recommender(RowEngine):
    def __init__(self, method: str, parameter: dict | None, converter: DatumToFvConverter,
                 device: Any = None):
        p = dict(parameter or {})
        unl, unlp = p.get("unlearner"), p.get("unlearner_parameter")
        self.outer_method = method
        if method == "nearest_neighbor_recommender":
            inner = p.get("method")
            if inner not in LSH_METHODS:
                raise ValueError("nearest_neighbor_recommender needs parameter.method in "
                                 f"{LSH_METHODS}")
            method, p = inner, dict(p.get("parameter") or {})
        elif method not in INDEX_METHODS:
            raise ValueError(f"unsupported recommender method: {method}")
        super().__init__(method, p, converter, device, unl, unlp)

    def similar_row_from_id(self, rid: str, size: int):
        return self.query_id(rid, int(size), similar=True)

    def similar_row_from_datum(self, d, size: int):
        return self.query_datum(d, int(size), similar=True)

    def decode_row(self, rid: str) -> Datum:
        with self._lock:
            s = self.rows.slot(rid)
            if s is None:
                return Datum()
            return self.rows.to_wire_datum(s)

    def _complete(self, base_nv: dict, neighbors: list[tuple[str, float]]) -> Datum:
        acc: dict[str, float] = {}
        wsum: dict[str, float] = {}
        for rid, sim in neighbors:
            s = self.rows.slot(rid)
            if s is None:
                continue
            w = sim if self.method in ("inverted_index", "lsh", "minhash") else 1.0 / (1.0 + max(0.0, -sim))
            if w <= 0:
                continue
            for k, v in self.rows.datum[s][1].items():
                acc[k] = acc.get(k, 0.0) + w * v
                wsum[k] = wsum.get(k, 0.0) + w
        nv = {k: acc[k] / wsum[k] for k in acc if wsum[k] > 0}
        nv.update(base_nv)
        return dicts_to_datum({}, nv)

    def complete_row_from_id(self, rid: str) -> Datum:
        with self._lock:
            s = self.rows.slot(rid)
            if s is None:
                return Datum()
            nb = [x for x in self.query_fv(self.rows.fv[s], COMPLETE_K + 1, True) if x[0] != rid]
            return self._complete(dict(self.rows.datum[s][1]), nb[:COMPLETE_K])

    def complete_row_from_datum(self, d) -> Datum:
        d = as_datum(d)
        with self._lock:
            nb = self.query_datum(d, COMPLETE_K, True)
            return self._complete(dict(d.num_values), nb)

    def calc_similarity(self, lhs, rhs) -> float:
        a = self.fv_of(as_datum(lhs))
        b = self.fv_of(as_datum(rhs))
        if isinstance(self.index, LshIndex):
            ix = self.index
            ba, na = signature_host(*a, ix.hash_num, ix.seed, ix.mode)
            bb, nb = signature_host(*b, ix.hash_num, ix.seed, ix.mode)
            ham = sum(bin(int(x) ^ int(y)).count("1") for x, y in zip(ba, bb))
            frac = ham / ix.hash_num
            if ix.metric == 1:
                return -math.sqrt(max(0.0, na * na + nb * nb - 2 * na * nb * math.cos(math.pi * frac)))
            return 1.0 - frac
        da = _dense(a)
        db = _dense(b)
        dot = sum(v * db.get(k, 0.0) for k, v in da.items())
        if self.method == "inverted_index_euclid":
            n2 = sum(v * v for v in da.values()) + sum(v * v for v in db.values()) - 2 * dot
            return -math.sqrt(max(0.0, n2))
        den = math.sqrt(sum(v * v for v in da.values())) * math.sqrt(sum(v * v for v in db.values()))
        return dot / den if den > 0 else 0.0

    def calc_l2norm(self, d) -> float:
        _, val = self.fv_of(as_datum(d))
        return float(np.sqrt(np.sum(np.asarray(val, np.float64) ** 2)))

    def get_status(self) -> dict[str, str]:
        st = super().get_status()
        st["method"] = self.outer_method
        return st


def _dense(fv) -> dict[int, float]:
    out: dict[int, float] = {}
    for i, v in zip(*fv):
        if i >= 0:
            out[int(i)] = out.get(int(i), 0.0) + float(v)
    return out
