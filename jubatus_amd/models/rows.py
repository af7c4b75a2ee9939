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

from ..common.exceptions import ArgumentError
from ..fv_converter.datum import Datum, _b, _s, as_datum


def datum_to_dicts(d: Datum) -> tuple[dict, dict, dict]:
    return (dict(d.string_values), dict(d.num_values), dict(d.binary_values))


def as_dicts(x: Any) -> tuple[dict, dict, dict]:
    """datum (Datum, {key: value} or the wire array) -> (string, num, binary)
    dicts, without building a Datum for the common input forms (the bulk
    row-ingest path; same validation as Datum.from_msgpack / Datum.add)"""
    if isinstance(x, (list, tuple)) and len(x) in (2, 3):
        try:
            sv = {_s(k): _s(v) for k, v in x[0]}
            nv = {}
            for k, v in x[1]:
                if isinstance(v, bool) or not isinstance(v, (int, float)):
                    raise ArgumentError("num_values value must be a number")
                nv[_s(k)] = float(v)
            bv = {_s(k): (v if isinstance(v, bytes) else _b(v)) for k, v in x[2]} if len(x) == 3 else {}
        except (ValueError, TypeError) as e:
            raise ArgumentError(f"malformed datum: {e}") from e
        return sv, nv, bv
    if isinstance(x, dict):
        # fast path: only str and float / int values
        sv = {k: v for k, v in x.items() if type(v) is str}
        nv = {k: float(v) for k, v in x.items() if type(v) is float or type(v) is int}
        if len(sv) + len(nv) == len(x):
            return sv, nv, {}
        sv, nv, bv = {}, {}, {}
        for k, v in x.items():
            if isinstance(v, str):
                sv[k] = v
            elif isinstance(v, (int, float)):        # bool included, as Datum.add
                nv[k] = float(v)
            elif isinstance(v, (bytes, bytearray, memoryview)):
                bv[k] = bytes(v)
            else:
                raise ArgumentError(f"unsupported datum value type {type(v)!r} for key {k!r}")
        return sv, nv, bv
    return datum_to_dicts(as_datum(x))


def dicts_wire(d: tuple[dict, dict, dict]) -> list:
    """(sv, nv, bv) -> the datum wire array with sorted keys (the feature
    order dicts_to_datum(...).to_msgpack() gives)"""
    sv, nv, bv = d
    return [sorted(sv.items()), sorted(nv.items()), sorted(bv.items()) if bv else []]


class _CsrBatch:
    __slots__ = ("rp", "idx", "val")

    def __init__(self, rp, idx, val):
        self.rp, self.idx, self.val = rp, idx, val


class FvTable:
    """slot -> hashed feature vector ([idx], [val]). Rows written in bulk keep
    a reference into their batch's CSR arrays and become Python lists only
    when read (most rows are never read back on the host: queries use the
    signatures in HBM)."""

    def __init__(self):
        self._d: dict[int, Any] = {}

    def __setitem__(self, slot: int, fv) -> None:
        self._d[slot] = fv

    def put_batch(self, slots, rp, idx, val) -> None:
        b = _CsrBatch(rp, idx, val)
        d = self._d
        for i, s in enumerate(slots.tolist()):
            d[s] = (b, i)

    def __getitem__(self, slot: int):
        fv = self._d[slot]
        if isinstance(fv[0], _CsrBatch):
            b, i = fv
            a, e = int(b.rp[i]), int(b.rp[i + 1])
            ix = b.idx[a:e]
            keep = ix >= 0
            fv = (ix[keep].tolist(), b.val[a:e][keep].tolist())
            self._d[slot] = fv
        return fv

    def get(self, slot: int, default=None):
        return self[slot] if slot in self._d else default

    def pop(self, slot: int, default=None):
        if slot not in self._d:
            return default
        v = self[slot]
        del self._d[slot]
        return v

    def __contains__(self, slot: int) -> bool:
        return slot in self._d

    def __len__(self) -> int:
        return len(self._d)


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
        self.fv = FvTable()
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

    def put_many(self, items: list, rp, idx, val, bump: bool = True):
        """bulk put: items [(rid, dicts)], their feature vectors as one CSR
        (rp / idx / val, row i = items[i]); returns the slots (int64 array)"""
        import numpy as np
        slots = np.fromiter((self.assign(rid) for rid, _ in items), np.int64, len(items))
        datum = self.datum
        for s, (_, dicts) in zip(slots.tolist(), items):
            datum[s] = dicts
        self.fv.put_batch(slots, rp, idx, val)
        if bump:
            version = self.version
            for rid, _ in items:
                version[rid] = version.get(rid, 0) + 1
            self.dirty.update(rid for rid, _ in items)
            if self.removed:
                self.removed.difference_update(rid for rid, _ in items)
        return slots

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
