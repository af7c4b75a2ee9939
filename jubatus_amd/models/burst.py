"""Kleinberg burst detection over a sliding batch window (jubaburst).

Reference: jubatus/server/server/burst_serv.cpp:44-246 over jubatus_core's
burst (EXTERNAL); config config/burst/burst.json (window_batch_size,
batch_interval, max_reuse_batch_num, costcut_threshold,
result_window_rotate_size). Behaviour:
* the window holds ``window_batch_size`` batches of width ``batch_interval``
  aligned to multiples of the interval; a document past the window's end
  slides it forward so the document lands in the last batch; a document
  older than the window start is rejected (add_documents counts accepted
  documents, burst_serv.cpp:127-151);
* per keyword and batch: d = documents, r = documents whose text contains
  the keyword; results are recomputed after each accepted add
  (``calculate_results``) for the keywords this server processes
  (standalone: all; distributed: its two CHT owners, burst_serv.cpp:73-86);
* two-state automaton per keyword: p0 = R/D over the window,
  p1 = min(scaling_param * p0, 1 - 1e-9), emission cost
  -ln(C(d,r) p^r (1-p)^(d-r)), entering the burst state costs
  gamma * ln(n_batches); Viterbi picks the state sequence and a bursting
  batch reports burst_weight = cost(p0) - cost(p1) (0 otherwise; weights
  below a positive ``costcut_threshold`` are cut to 0). Every window is
  recomputed exactly (max_reuse_batch_num is accepted; nothing is reused);
* ``result_window_rotate_size`` past windows are kept for get_result_at.
MIX: keywords and the processed keywords' result windows are exchanged.
"""
from __future__ import annotations

import math
import threading


class BurstError(RuntimeError):
    pass


def _lgamma_binom(d: int, r: int) -> float:
    return math.lgamma(d + 1) - math.lgamma(r + 1) - math.lgamma(d - r + 1)


def _cost(d: int, r: int, p: float) -> float:
    if d == 0:
        return 0.0
    return -(_lgamma_binom(d, r) + r * math.log(p) + (d - r) * math.log1p(-p))


def detect(d: list[int], r: list[int], scaling: float, gamma: float,
           costcut: float = -1.0) -> list[float]:
    """Per-batch burst weights of one keyword (two-state Viterbi)."""
    n = len(d)
    D, R = sum(d), sum(r)
    if n == 0 or D == 0 or R == 0 or R >= D:
        return [0.0] * n
    p0 = R / D
    p1 = min(scaling * p0, 1.0 - 1e-9)
    trans = gamma * math.log(n) if n > 1 else gamma
    c0 = [_cost(di, ri, p0) for di, ri in zip(d, r)]
    c1 = [_cost(di, ri, p1) for di, ri in zip(d, r)]
    # Viterbi, start in the base state
    best = [c0[0], trans + c1[0]]
    back: list[tuple[int, int]] = []
    for i in range(1, n):
        from0 = (best[0], 0) if best[0] <= best[1] else (best[1], 1)
        to1 = (best[0] + trans, 0) if best[0] + trans <= best[1] else (best[1], 1)
        back.append((from0[1], to1[1]))
        best = [from0[0] + c0[i], to1[0] + c1[i]]
    state = 0 if best[0] <= best[1] else 1
    states = [0] * n
    for i in range(n - 1, -1, -1):
        states[i] = state
        if i > 0:
            state = back[i - 1][state]
    out = []
    for i in range(n):
        w = c0[i] - c1[i] if states[i] == 1 else 0.0
        if costcut > 0 and w < costcut:
            w = 0.0
        out.append(max(w, 0.0))
    return out


class Burst:
    def __init__(self, method: str, parameter: dict | None):
        if method != "burst":
            raise ValueError(f"unsupported burst method: {method}")
        p = dict(parameter or {})
        try:
            self.window_batch_size = int(p["window_batch_size"])
            self.batch_interval = float(p["batch_interval"])
            self.max_reuse = int(p.get("max_reuse_batch_num", 5))
            self.costcut = float(p.get("costcut_threshold", -1))
            self.rotate = int(p.get("result_window_rotate_size", 5))
        except KeyError as e:
            raise ValueError(f"burst parameter {e} is required") from e
        if self.window_batch_size <= 0 or self.batch_interval <= 0 or self.rotate <= 0:
            raise ValueError("window_batch_size, batch_interval and "
                             "result_window_rotate_size must be positive")
        self._lock = threading.RLock()
        self.keywords: dict[str, tuple[float, float]] = {}
        self.processed: set[str] = set()
        self.clear()

    def clear(self) -> None:
        with self._lock:
            self.start: float | None = None
            self.d = [0] * self.window_batch_size
            self.r: dict[str, list[int]] = {k: [0] * self.window_batch_size for k in self.keywords}
            self.results: dict[str, list[tuple[float, list]]] = {}
            self.mixed_once = False

    # ------------------------------------------------------------ keywords
    def add_keyword(self, kw: str, scaling: float, gamma: float, processed: bool = True) -> bool:
        with self._lock:
            if kw in self.keywords:
                return False
            if scaling <= 1.0 or gamma <= 0.0:
                raise BurstError("scaling_param must be > 1 and gamma > 0")
            self.keywords[kw] = (float(scaling), float(gamma))
            self.r[kw] = [0] * self.window_batch_size
            if processed:
                self.processed.add(kw)
            return True

    def remove_keyword(self, kw: str) -> bool:
        with self._lock:
            if kw not in self.keywords:
                return False
            del self.keywords[kw]
            self.r.pop(kw, None)
            self.results.pop(kw, None)
            self.processed.discard(kw)
            return True

    def remove_all_keywords(self) -> bool:
        with self._lock:
            self.keywords.clear()
            self.r.clear()
            self.results.clear()
            self.processed.clear()
            return True

    def get_all_keywords(self) -> list[tuple[str, float, float]]:
        with self._lock:
            return [(k, s, g) for k, (s, g) in self.keywords.items()]

    def set_processed_keywords(self, kws) -> None:
        with self._lock:
            self.processed = {k for k in kws if k in self.keywords}

    # ----------------------------------------------------------- documents
    def _window_end(self) -> float:
        return self.start + self.window_batch_size * self.batch_interval

    def add_document(self, text: str, pos: float) -> bool:
        with self._lock:
            pos = float(pos)
            last = math.floor(pos / self.batch_interval) * self.batch_interval
            if self.start is None:
                self.start = last - (self.window_batch_size - 1) * self.batch_interval
            if pos < self.start:
                return False
            if pos >= self._window_end():
                new_start = last - (self.window_batch_size - 1) * self.batch_interval
                shift = int(round((new_start - self.start) / self.batch_interval))
                shift = min(shift, self.window_batch_size)
                pad = [0] * shift
                self.d = self.d[shift:] + pad
                for k in self.r:
                    self.r[k] = self.r[k][shift:] + pad
                self.start = new_start
            i = min(int((pos - self.start) // self.batch_interval), self.window_batch_size - 1)
            self.d[i] += 1
            for k, rr in self.r.items():
                if k in text:
                    rr[i] += 1
            return True

    def calculate_results(self) -> None:
        with self._lock:
            if self.start is None:
                return
            for kw in self.processed:
                s, g = self.keywords[kw]
                rr = self.r[kw]
                w = detect(self.d, rr, s, g, self.costcut)
                res = (self.start, [[self.d[i], rr[i], w[i]] for i in range(self.window_batch_size)])
                hist = self.results.setdefault(kw, [])
                if hist and hist[-1][0] == self.start:
                    hist[-1] = res
                else:
                    hist.append(res)
                    del hist[:-self.rotate]

    # ------------------------------------------------------------- queries
    @staticmethod
    def _empty() -> tuple[float, list]:
        return (0.0, [])

    def get_result(self, kw: str):
        with self._lock:
            hist = self.results.get(kw)
            return hist[-1] if hist else self._empty()

    def _covers(self, start: float, pos: float) -> bool:
        return start <= pos < start + self.window_batch_size * self.batch_interval

    def get_result_at(self, kw: str, pos: float):
        with self._lock:
            for start, batches in reversed(self.results.get(kw, [])):
                if self._covers(start, pos):
                    return (start, batches)
            return self._empty()

    @staticmethod
    def _bursted(res) -> bool:
        return any(b[2] > 0 for b in res[1])

    def get_all_bursted_results(self) -> dict:
        with self._lock:
            out = {}
            for kw in self.keywords:
                res = self.get_result(kw)
                if self._bursted(res):
                    out[kw] = res
            return out

    def get_all_bursted_results_at(self, pos: float) -> dict:
        with self._lock:
            out = {}
            for kw in self.keywords:
                res = self.get_result_at(kw, pos)
                if self._bursted(res):
                    out[kw] = res
            return out

    # ----------------------------------------------------------------- MIX
    def get_diff(self) -> dict:
        with self._lock:
            return {"keywords": {k: list(v) for k, v in self.keywords.items()},
                    "results": {k: [[s, b] for s, b in self.results.get(k, [])]
                                for k in self.processed}}

    @staticmethod
    def mix_diff(a: dict, b: dict) -> dict:
        kws = dict(a["keywords"])
        kws.update(b["keywords"])
        res = dict(a["results"])
        res.update(b["results"])
        return {"keywords": kws, "results": res}

    def put_diff(self, mixed: dict) -> bool:
        with self._lock:
            for k, (s, g) in mixed["keywords"].items():
                if k not in self.keywords:
                    self.keywords[k] = (float(s), float(g))
                    self.r[k] = [0] * self.window_batch_size
            for k, hist in mixed["results"].items():
                if k in self.keywords and k not in self.processed:
                    self.results[k] = [(float(s), [list(x) for x in b]) for s, b in hist]
            self.mixed_once = True
            return True

    def pack(self) -> dict:
        with self._lock:
            return {"keywords": {k: list(v) for k, v in self.keywords.items()},
                    "processed": sorted(self.processed), "start": self.start, "d": self.d,
                    "r": self.r, "results": {k: [[s, b] for s, b in h] for k, h in self.results.items()}}

    def unpack(self, obj: dict) -> None:
        with self._lock:
            self.keywords = {k: (float(v[0]), float(v[1])) for k, v in obj["keywords"].items()}
            self.processed = set(obj["processed"])
            self.start = obj["start"]
            self.d = [int(x) for x in obj["d"]]
            self.r = {k: [int(x) for x in v] for k, v in obj["r"].items()}
            self.results = {k: [(float(s), [list(x) for x in b]) for s, b in h]
                            for k, h in obj["results"].items()}

    def get_status(self) -> dict[str, str]:
        return {"num_keywords": str(len(self.keywords)), "processed_keywords": str(len(self.processed)),
                "window_start": str(self.start), "window_batch_size": str(self.window_batch_size),
                "batch_interval": str(self.batch_interval)}
