"""Online regression driver: passive-aggressive (``method: "PA"``).

Reference surface: jubatus/server/server/regression_serv.cpp:95-156 (train,
estimate, clear) over jubatus_core's PA regression (EXTERNAL). Parameters:
``sensitivity`` (epsilon of the insensitive loss, scaled by the running
target standard deviation) and ``regularization_weight`` (C).

Rule (also the numerical oracle of csrc/hip/regression.hip):
    count, sum, sum2 of the targets; sd = sqrt(max(0, sum2/count - (sum/count)^2))
    err = y - w.x ; loss = |err| - sensitivity * sd
    loss > 0:  w += sign(err) * min(C, loss) / ||x||^2 * x

Storage: w[H] (hashed features) in HBM on a GPU, NumPy otherwise.
MIX: all-reduce mean of w and of the target statistics.
"""
from __future__ import annotations

import math
import threading
from typing import Any, Sequence

import msgpack
import numpy as np

from ..common.exceptions import ArgumentError
from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import as_datum


class RegressionConfigError(ValueError):
    pass


def train_one(w: np.ndarray, stats: np.ndarray, idx, val, y: float, C: float, eps: float) -> None:
    m = np.asarray(idx) >= 0
    idx = np.asarray(idx, np.int64)[m]
    x = np.asarray(val, np.float32)[m]
    dot = float((x * w[idx]).sum(dtype=np.float32)) if len(idx) else 0.0
    stats[0] += y
    stats[1] += y * y
    stats[2] += 1.0
    avg = stats[0] / stats[2]
    sd = math.sqrt(max(0.0, stats[1] / stats[2] - avg * avg))
    err = y - dot
    sgn = 1.0 if err > 0 else -1.0
    loss = sgn * err - eps * sd
    nrm = float((x * x).sum())
    if loss > 0 and nrm > 0:
        coeff = sgn * min(C, loss) / nrm
        w[idx] = w[idx] + np.float32(coeff) * x


class PARegression:
    def __init__(self, method: str, parameter: dict | None, converter: DatumToFvConverter,
                 device: Any = None):
        if method != "PA":
            raise RegressionConfigError(f"unsupported regression method: {method}")
        p = dict(parameter or {})
        self.eps = float(p.get("sensitivity", 0.1))
        self.C = float(p.get("regularization_weight", 3.40282e+38))
        if self.eps < 0 or not self.C > 0:
            raise RegressionConfigError("sensitivity must be >= 0 and regularization_weight > 0")
        self.method = method
        self.conv = converter
        self.H = converter.hash_max_size
        self.device = device
        self.gpu = device is not None
        self._lock = threading.RLock()
        if self.gpu:
            import torch
            from ..ops.feature_pipeline import FeaturePipeline
            self.torch = torch
            self.pipe = FeaturePipeline(converter, device)
        self.clear()

    def clear(self) -> None:
        with self._lock:
            if self.gpu:
                t = self.torch
                self.w = t.zeros(self.H, dtype=t.float32, device=self.device)
                self.stats = t.zeros(3, dtype=t.float32, device=self.device)
            else:
                self.w = np.zeros(self.H, dtype=np.float32)
                self.stats = np.zeros(3, dtype=np.float64)
            self.conv.weights.clear()

    # -------------------------------------------------------------- train
    def train_requests(self, bodies: Sequence[Any]) -> int:
        """raw msgpack list<scored_datum> bodies, one update stream each"""
        with self._lock:
            if self.gpu and self.pipe.fast:
                from ..ops import hip
                b = self.pipe.from_requests(list(bodies), 2)
                if b.n:
                    hip.regression_train(b.row_ptr, b.fidx, b.fval, b.labels.view(self.torch.float32),
                                         b.stream_ptr, b.nstreams, self.w, self.stats, self.C,
                                         self.eps, concurrent=b.nstreams > 1)
                return b.n
        n = 0
        for body in bodies:
            n += self.train(msgpack.unpackb(bytes(body), raw=False))
        return n

    def train(self, data: Sequence) -> int:
        data = list(data)
        if not data:
            return 0
        items = []
        for it in data:
            if not isinstance(it, (list, tuple)) or len(it) != 2:
                raise ArgumentError("scored_datum must be [score, datum]")
            score, d = it
            if isinstance(score, bool) or not isinstance(score, (int, float)):
                raise ArgumentError("score must be a number")
            items.append((float(score), as_datum(d)))
        if self.gpu and self.pipe.fast:
            body = msgpack.packb([[s, d.to_msgpack()] for s, d in items], use_bin_type=False)
            return self.train_requests([body])
        with self._lock:
            rows = [self.conv.hashed(self.conv.convert_and_update_weight(d)) for _, d in items]
            if self.gpu:
                from ..ops import hip
                b = self.pipe.from_rows(rows, None)
                tg = self.torch.tensor([s for s, _ in items], dtype=self.torch.float32,
                                       device=self.device)
                hip.regression_train(b.row_ptr, b.fidx, b.fval, tg, b.stream_ptr, 1, self.w,
                                     self.stats, self.C, self.eps, concurrent=False)
            else:
                for (s, _), (idx, val) in zip(items, rows):
                    train_one(self.w, self.stats, idx, val, s, self.C, self.eps)
        return len(items)

    # ----------------------------------------------------------- estimate
    def estimate(self, data: Sequence) -> list[float]:
        ds = [as_datum(d) for d in data]
        if not ds:
            return []
        rows = [self.conv.hashed(self.conv.convert(d)) for d in ds]
        with self._lock:
            if self.gpu:
                from ..ops import hip
                b = self.pipe.from_rows(rows, None)
                out = self.torch.empty(len(ds), dtype=self.torch.float32, device=self.device)
                hip.regression_estimate(b.row_ptr, b.fidx, b.fval, b.n, self.w, out)
                return [float(x) for x in out.cpu().tolist()]
            res = []
            for idx, val in rows:
                i = np.asarray(idx, np.int64)
                m = i >= 0
                res.append(float((np.asarray(val, np.float32)[m] * self.w[i[m]]).sum()))
            return res

    # ---------------------------------------------------------- persist/mix
    def _host(self) -> tuple[np.ndarray, np.ndarray]:
        if self.gpu:
            return self.w.cpu().numpy(), self.stats.cpu().numpy().astype(np.float64)
        return self.w, self.stats

    def pack(self) -> dict:
        with self._lock:
            w, st = self._host()
            rows = np.nonzero(w)[0].astype(np.int64)
            return {"method": self.method, "H": self.H, "rows": rows.tobytes(),
                    "w": w[rows].astype(np.float32).tobytes(), "stats": [float(x) for x in st],
                    "weights": self.conv.weights.pack()}

    def unpack(self, obj: dict) -> None:
        with self._lock:
            if int(obj["H"]) != self.H:
                raise ValueError("model hash_max_size differs from the configuration")
            self.clear()
            rows = np.frombuffer(obj["rows"], dtype=np.int64)
            w = np.zeros(self.H, np.float32)
            w[rows] = np.frombuffer(obj["w"], dtype=np.float32)
            st = np.asarray(obj["stats"], dtype=np.float64)
            if self.gpu:
                self.w.copy_(self.torch.from_numpy(w))
                self.stats.copy_(self.torch.from_numpy(st.astype(np.float32)))
            else:
                self.w, self.stats = w, st
            if obj.get("weights"):
                self.conv.weights.unpack(obj["weights"])

    def _tables(self):
        import torch
        if self.gpu:
            return [self.w, self.stats]
        return [torch.from_numpy(self.w), torch.from_numpy(self.stats)]

    def mix(self) -> int:
        from ..parallel import collective as coll
        with self._lock:
            ts = self._tables()
            coll.allreduce_mean_(ts)
            return sum(t.numel() * t.element_size() for t in ts)

    def broadcast_from(self, src: int, apply: bool = True) -> None:
        """model hand-over from rank ``src``; apply=False: take part in the
        collective without replacing the local model (an up-to-date member)"""
        import torch
        import torch.distributed as dist
        with self._lock:
            for t in self._tables():
                if apply or dist.get_rank() == src:
                    dist.broadcast(t, src=src)
                else:
                    dist.broadcast(torch.empty_like(t), src=src)

    def pair_mix(self, peer: int) -> None:
        import torch
        import torch.distributed as dist
        with self._lock:
            for t in self._tables():
                buf = torch.empty_like(t)
                for r in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, peer),
                                                 dist.P2POp(dist.irecv, buf, peer)]):
                    r.wait()
                t.add_(buf).mul_(0.5)

    def get_status(self) -> dict[str, str]:
        return {"num_features": str(self.H), "method": self.method,
                "storage": "hbm" if self.gpu else "host"}
