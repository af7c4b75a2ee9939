"""Row store shared by the row-oriented engines (nearest_neighbor,
recommender, anomaly): id <-> slot mapping, the stored datum and its hashed
feature vector per row, row versions for MIX, and the ``lru`` unlearner
(``unlearner: "lru", unlearner_parameter: {max_size}``; reference configs
config/recommender/*_unlearn_lru.json, ChangeLog.rst:294).
"""
from __future__ import annotations

import threading
from collections import OrderedDict
from typing import Any

from ..fv_converter.datum import Datum


def datum_to_dicts(d: Datum) -> tuple[dict, dict, dict]:
    return (dict(d.string_values), dict(d.num_values), dict(d.binary_values))


def dicts_to_datum(sv: dict, nv: dict, bv: dict | None = None) -> Datum:
    d = Datum()
    d.string_values = sorted(sv.items())
    d.num_values = sorted(nv.items())
    d.binary_values = sorted((bv or {}).items())
    return d


class Unlearner:
    def __init__(self, kind: str | None, parameter: dict | None):
        if kind not in (None, "lru"):
            raise ValueError(f"unknown unlearner: {kind}")
        self.kind = kind
        p = parameter or {}
        self.max_size = int(p.get("max_size", 0)) if kind else 0
        if kind and self.max_size <= 0:
            raise ValueError("unlearner_parameter.max_size must be positive")
        self.order: OrderedDict[str, None] = OrderedDict()

    def touch(self, rid: str) -> list[str]:
        """mark rid as used; returns ids to evict"""
        if not self.kind:
            return []
        self.order.pop(rid, None)
        self.order[rid] = None
        out = []
        while len(self.order) > self.max_size:
            victim, _ = self.order.popitem(last=False)
            out.append(victim)
        return out

    def remove(self, rid: str) -> None:
        self.order.pop(rid, None)

    def clear(self) -> None:
        self.order.clear()


class RowStore:
    def __init__(self):
        self.lock = threading.RLock()
        self.clear()

    def clear(self) -> None:
        self.ids: list[str | None] = []
        self.slot_of: dict[str, int] = {}
        self.free: list[int] = []
        self.datum: dict[int, tuple[dict, dict, dict]] = {}
        self.fv: dict[int, tuple[list[int], list[float]]] = {}
        self.version: dict[str, int] = {}
        self.dirty: set[str] = set()      # rows changed since the last MIX
        self.removed: set[str] = set()

    @property
    def nslots(self) -> int:
        return len(self.ids)

    def slot(self, rid: str) -> int | None:
        return self.slot_of.get(rid)

    def assign(self, rid: str) -> int:
        s = self.slot_of.get(rid)
        if s is not None:
            return s
        if self.free:
            s = self.free.pop()
            self.ids[s] = rid
        else:
            s = len(self.ids)
            self.ids.append(rid)
        self.slot_of[rid] = s
        return s

    def put(self, rid: str, dicts: tuple[dict, dict, dict], fv, bump: bool = True) -> int:
        s = self.assign(rid)
        self.datum[s] = dicts
        self.fv[s] = fv
        if bump:
            self.version[rid] = self.version.get(rid, 0) + 1
            self.dirty.add(rid)
            self.removed.discard(rid)
        return s

    def remove(self, rid: str, record: bool = True) -> int | None:
        s = self.slot_of.pop(rid, None)
        if s is None:
            return None
        self.ids[s] = None
        self.free.append(s)
        self.datum.pop(s, None)
        self.fv.pop(s, None)
        if record:
            self.version[rid] = self.version.get(rid, 0) + 1
            self.removed.add(rid)
            self.dirty.discard(rid)
        return s

    def all_ids(self) -> list[str]:
        return [i for i in self.ids if i is not None]

    def id_of(self, slot: int) -> str | None:
        return self.ids[slot] if 0 <= slot < len(self.ids) else None

    # ---- MIX (linear_mixable protocol: row versions, newest wins)
    def get_diff(self) -> dict:
        with self.lock:
            rows = {rid: [self.version.get(rid, 0), self.datum[self.slot_of[rid]]]
                    for rid in self.dirty if rid in self.slot_of}
            dels = {rid: self.version.get(rid, 0) for rid in self.removed}
            return {"rows": rows, "removed": dels}

    @staticmethod
    def mix_diff(a: dict, b: dict) -> dict:
        rows = dict(a["rows"])
        for rid, (v, d) in b["rows"].items():
            if rid not in rows or v >= rows[rid][0]:
                rows[rid] = [v, d]
        dels = dict(a["removed"])
        for rid, v in b["removed"].items():
            dels[rid] = max(v, dels.get(rid, -1))
        return {"rows": rows, "removed": dels}

    def pack(self) -> dict:
        with self.lock:
            return {"rows": {rid: [self.version.get(rid, 0), list(map(lambda x: dict(x), self.datum[s]))]
                             for rid, s in self.slot_of.items()}}

    def to_wire_datum(self, slot: int) -> Any:
        sv, nv, bv = self.datum[slot]
        return dicts_to_datum(sv, nv, bv)
