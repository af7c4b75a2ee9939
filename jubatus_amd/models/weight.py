"""Feature-weight engine (jubaweight).

Reference: jubatus/server/server/weight_serv.cpp:30-110 - ``update(datum)``
converts with the global-weight statistics updated (document frequencies,
average length), ``calc_weight(datum)`` converts without touching them; both
return the weighted feature vector as ``list<feature>``. ``method`` /
``parameter`` in the config are accepted and ignored (weight_serv.cpp:33-36).
MIX exchanges the converter's weight-manager diff (df counts, document
count), exactly like every converter-backed engine.
"""
from __future__ import annotations

import threading

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import as_datum


class Weight:
    def __init__(self, converter: DatumToFvConverter):
        self.conv = converter
        self._lock = threading.RLock()

    def update(self, d) -> list[tuple[str, float]]:
        with self._lock:
            return [(k, float(v)) for k, v in self.conv.convert_and_update_weight(as_datum(d))]

    def calc_weight(self, d) -> list[tuple[str, float]]:
        with self._lock:
            return [(k, float(v)) for k, v in self.conv.convert(as_datum(d))]

    def clear(self) -> None:
        with self._lock:
            self.conv.weights.clear()

    def get_diff(self):
        return self.conv.weights.get_diff()

    @staticmethod
    def mix_diff(a, b):
        from ..fv_converter.converter import WeightManager
        return WeightManager.mix(a, b)

    def put_diff(self, mixed) -> bool:
        with self._lock:
            self.conv.weights.put_diff(mixed)
            return True

    def pack(self):
        return {"weights": self.conv.weights.pack()}

    def unpack(self, obj) -> None:
        with self._lock:
            self.conv.weights.unpack(obj["weights"])

    def get_status(self) -> dict[str, str]:
        return {"weight_manager": "df"}
