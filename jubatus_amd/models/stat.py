"""Windowed per-key statistics (jubastat).

Reference: jubatus/server/server/stat_serv.cpp:51-106 (config
``window_size``; push / sum / stddev / max / min / entropy / moment / clear)
over jubatus_core's stat (EXTERNAL). Semantics kept:
* one global window of the last ``window_size`` pushes (any key); the
  oldest push leaves the window when it overflows;
* per-key running n / sum / sum of squares; max / min are recomputed from
  the window only when the leaving value was the extreme;
* ``entropy`` ignores its key (stat_serv.cpp:89-91): the entropy of the key
  distribution inside the window, or - after a MIX - of the cluster-wide
  distribution (the mixable exchanges sum(n log n) and n);
* ``moment(key, degree, center)`` = mean over the key's window values of
  (v - center)^degree; degree 0 -> 1, negative -> error;
* unknown keys raise ``stat_error`` ("<op>: key <k> not found").
"""
from __future__ import annotations

import math
import threading
from collections import deque


class StatError(RuntimeError):
    pass


class _KeyStat:
    __slots__ = ("n", "s", "s2", "mx", "mn")

    def __init__(self):
        self.n, self.s, self.s2 = 0, 0.0, 0.0
        self.mx, self.mn = -math.inf, math.inf


class Stat:
    def __init__(self, window_size: int):
        if int(window_size) <= 0:
            raise ValueError("window_size must be positive")
        self.window_size = int(window_size)
        self._lock = threading.RLock()
        self.clear()

    def clear(self) -> None:
        with getattr(self, "_lock", threading.RLock()):
            self.window: deque[tuple[str, float]] = deque()
            self.stats: dict[str, _KeyStat] = {}
            self.mixed_e = 0.0   # cluster-wide sum n*log(n) after a MIX
            self.mixed_n = 0     # cluster-wide window population after a MIX

    def push(self, key: str, value: float) -> bool:
        with self._lock:
            value = float(value)
            self.window.append((key, value))
            st = self.stats.setdefault(key, _KeyStat())
            st.n += 1
            st.s += value
            st.s2 += value * value
            st.mx = max(st.mx, value)
            st.mn = min(st.mn, value)
            if len(self.window) > self.window_size:
                self._evict()
            return True

    def _evict(self) -> None:
        k, v = self.window.popleft()
        st = self.stats[k]
        st.n -= 1
        if st.n == 0:
            del self.stats[k]
            return
        st.s -= v
        st.s2 -= v * v
        if v >= st.mx or v <= st.mn:
            vals = [x for kk, x in self.window if kk == k]
            st.mx, st.mn = max(vals), min(vals)

    def _get(self, op: str, key: str) -> _KeyStat:
        st = self.stats.get(key)
        if st is None:
            raise StatError(f"{op}: key {key} not found")
        return st

    def sum(self, key: str) -> float:
        with self._lock:
            return self._get("sum", key).s

    def stddev(self, key: str) -> float:
        with self._lock:
            st = self._get("stddev", key)
            mean = st.s / st.n
            return math.sqrt(max(0.0, st.s2 / st.n - mean * mean))

    def max(self, key: str) -> float:
        with self._lock:
            return self._get("max", key).mx

    def min(self, key: str) -> float:
        with self._lock:
            return self._get("min", key).mn

    def _local_e(self) -> tuple[float, int]:
        return sum(st.n * math.log(st.n) for st in self.stats.values()), len(self.window)

    def entropy(self) -> float:
        with self._lock:
            e, n = (self.mixed_e, self.mixed_n) if self.mixed_n > 0 else self._local_e()
            if n == 0:
                return 0.0
            return math.log(n) - e / n

    def moment(self, key: str, degree: int, center: float) -> float:
        with self._lock:
            st = self._get("moment", key)
            if degree < 0:
                raise StatError("moment: negative degree")
            if degree == 0:
                return 1.0
            return sum((v - center) ** degree for k, v in self.window if k == key) / st.n

    # MIX (entropy across servers): diff = [sum n log n, n]
    def get_diff(self) -> list:
        with self._lock:
            e, n = self._local_e()
            return [e, n]

    @staticmethod
    def mix_diff(a: list, b: list) -> list:
        return [a[0] + b[0], a[1] + b[1]]

    def put_diff(self, mixed: list) -> bool:
        with self._lock:
            self.mixed_e, self.mixed_n = float(mixed[0]), int(mixed[1])
            return True

    def pack(self) -> dict:
        with self._lock:
            return {"window_size": self.window_size, "window": [[k, v] for k, v in self.window],
                    "mixed": [self.mixed_e, self.mixed_n]}

    def unpack(self, obj: dict) -> None:
        with self._lock:
            self.clear()
            for k, v in obj["window"]:
                self.push(k, v)
            self.mixed_e, self.mixed_n = float(obj["mixed"][0]), int(obj["mixed"][1])

    def get_status(self) -> dict[str, str]:
        return {"storage": "stat", "window_size": str(self.window_size),
                "num_keys": str(len(self.stats)), "window_population": str(len(self.window))}
