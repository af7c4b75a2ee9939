"""Online clustering over compressive coresets: k-means and GMM.

Reference: jubatus/server/server/clustering_serv.cpp:71-151 (push,
get_revision, get_core_members, get_k_center, get_nearest_center,
get_nearest_members, clear) over jubatus_core's clustering (EXTERNAL).
Parameters (config/clustering/*.json): k, compressor_method (simple,
compressive_kmeans, compressive_gmm), bucket_size, compressed_bucket_size,
bicriteria_base_size, bucket_length, forgetting_factor, forgetting_threshold,
seed.

Pipeline (our design, documented):
* pushed points (datum -> feature vector, named features) accumulate in a
  bucket; a full bucket (``bucket_size``) is compressed to a weighted coreset
  of ``compressed_bucket_size`` points (``simple``: uniform sample with
  weights scaled up; ``compressive_*``: k-means++ representatives, each
  weighted by the points it absorbs), the revision increments and the
  clusters are recomputed over every coreset point;
* more than ``bucket_length`` coresets: the two oldest merge (and recompress);
  a new coreset decays older weights by exp(-forgetting_factor) and drops
  points whose weight falls below ``forgetting_threshold``;
* clustering: weighted k-means (k-means++ seeding from ``seed``, Lloyd
  iterations) or a diagonal-covariance GMM (EM initialised from k-means).

The distance matrix of every assignment step runs on the matrix cores on a
GPU (csrc/hip/clustering.hip: fp32 MFMA Gram term), torch elsewhere.
MIX: coresets are exchanged (get_diff / mix_diff / put_diff); every server
clusters its own coresets plus the other servers' ones.
"""
from __future__ import annotations

import math
import random
import threading
import uuid
from typing import Any

import numpy as np

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum, as_datum

COMPRESSORS = ("simple", "compressive_kmeans", "compressive_gmm")


class NotPerformed(RuntimeError):
    def __init__(self):
        super().__init__("clustering is not performed yet")


class Clustering:
    def __init__(self, method: str, parameter: dict | None, converter: DatumToFvConverter,
                 device: Any = None):
        if method not in ("kmeans", "gmm"):
            raise ValueError(f"unsupported clustering method: {method}")
        p = dict(parameter or {})
        self.method = method
        self.k = int(p.get("k", 3))
        self.compressor = p.get("compressor_method", "simple")
        if self.compressor not in COMPRESSORS:
            raise ValueError(f"unknown compressor_method: {self.compressor}")
        self.bucket_size = int(p.get("bucket_size", 1000))
        self.compressed = int(p.get("compressed_bucket_size", 100))
        self.bicriteria = int(p.get("bicriteria_base_size", 10))
        self.bucket_length = int(p.get("bucket_length", 2))
        self.forgetting_factor = float(p.get("forgetting_factor", 0.0))
        self.forgetting_threshold = float(p.get("forgetting_threshold", 0.5))
        self.seed = int(p.get("seed", 0))
        if self.k <= 0 or self.bucket_size <= 0 or not 0 < self.compressed <= self.bucket_size:
            raise ValueError("invalid clustering parameter (k, bucket_size, compressed_bucket_size)")
        if self.bucket_length < 1:
            raise ValueError("bucket_length must be positive")
        self.conv = converter
        self.device = device
        self.gpu = device is not None
        self.token = uuid.uuid4().hex
        self._lock = threading.RLock()
        self.clear()

    def clear(self) -> None:
        with getattr(self, "_lock", threading.RLock()):
            self.pending: list[tuple[float, dict, Datum]] = []
            self.buckets: list[list[tuple[float, dict, Datum]]] = []
            self.others: list[tuple[float, dict, Datum]] = []
            self.revision = 0
            self.centers = None     # torch [k, D]
            self.variances = None   # gmm
            self.mix_weights = None
            self.dims: list[str] = []
            self.assign: list[int] = []
            self.core: list[tuple[float, dict, Datum]] = []
            self._rng = random.Random(self.seed)

    # ------------------------------------------------------------ tensors
    def _t(self):
        import torch
        return torch

    # with a device every coreset / Lloyd / EM step runs in HBM: the k-means++
    # draws and the Lloyd iterations of a bucket each run in ONE single-
    # workgroup launch (csrc/hip/clustering.hip), so a 1000-point bucket no
    # longer pays a host round trip per draw / iteration. (Set higher to keep
    # small problems on the host.)
    GPU_MIN_ELEMS = 0

    def _dense(self, pts: list[dict], dims: list[str], device=None):
        torch = self._t()
        pos = {n: i for i, n in enumerate(dims)}
        X = np.zeros((len(pts), len(dims)), dtype=np.float32)
        for r, fv in enumerate(pts):
            for name, v in fv.items():
                j = pos.get(name)
                if j is not None:
                    X[r, j] = v
        t = torch.from_numpy(X)
        if device is not None:
            return t.to(device)
        return t.to(self.device) if self.gpu and X.size >= self.GPU_MIN_ELEMS else t

    def _sqdist(self, X, C):
        if X.is_cuda:
            from ..ops import hip
            return hip.sqdist(X.contiguous(), C.contiguous())
        xn = (X * X).sum(1, keepdim=True)
        cn = (C * C).sum(1)[None, :]
        return (xn + cn - 2.0 * X @ C.T).clamp_min(0.0)

    # ------------------------------------------------------------ push
    def _fv(self, d: Datum) -> dict:
        out: dict[str, float] = {}
        for name, v in self.conv.convert_and_update_weight(d):
            out[name] = out.get(name, 0.0) + float(v)
        return out

    def push(self, points: list) -> bool:
        with self._lock:
            for p in points:
                d = as_datum(p)
                self.pending.append((1.0, self._fv(d), d))
                if len(self.pending) >= self.bucket_size:
                    self._close_bucket()
            return True

    def _kmeanspp(self, X, w, m: int, rng: random.Random) -> list[int]:
        torch = self._t()
        n = X.shape[0]
        m = min(m, n)
        chosen: list[int] = []
        if X.is_cuda:
            from ..ops import hip
            # one uniform per draw, as the host path's random.choices uses
            chosen, status = hip.kmeanspp(X.contiguous(), w.contiguous(),
                                          [rng.random() for _ in range(m)], m)
            if status == 0:
                return chosen
            chosen = chosen[:status - 1]      # zero mass left: finish on the host
        if not chosen:
            chosen = [rng.choices(range(n), weights=w.cpu().tolist(), k=1)[0]]
        d2 = self._sqdist(X, X[chosen])
        d2 = d2.min(1).values if d2.shape[1] > 1 else d2[:, 0]
        for _ in range(len(chosen), m):
            prob = (d2 * w).cpu().numpy().astype(np.float64)
            s = prob.sum()
            if s <= 0:
                rest = [i for i in range(n) if i not in set(chosen)]
                if not rest:
                    break
                nxt = rng.choice(rest)
            else:
                nxt = rng.choices(range(n), weights=prob.tolist(), k=1)[0]
            chosen.append(nxt)
            d2 = torch.minimum(d2, self._sqdist(X, X[nxt:nxt + 1])[:, 0])
        return chosen

    def _compress(self, pts: list[tuple[float, dict, Datum]], m: int):
        if len(pts) <= m:
            return list(pts)
        if self.compressor == "simple":
            idx = self._rng.sample(range(len(pts)), m)
            scale = sum(p[0] for p in pts) / sum(pts[i][0] for i in idx)
            return [(pts[i][0] * scale, pts[i][1], pts[i][2]) for i in idx]
        torch = self._t()
        dims = sorted({n for _, fv, _ in pts for n in fv})
        X = self._dense([fv for _, fv, _ in pts], dims)
        w = torch.tensor([p[0] for p in pts], dtype=torch.float32, device=X.device)
        reps = self._kmeanspp(X, w, m, self._rng)
        a = self._sqdist(X, X[reps]).argmin(1)
        wsum = torch.zeros(len(reps), dtype=torch.float32, device=X.device).index_add_(0, a, w)
        ws = wsum.cpu().tolist()
        return [(ws[j], pts[i][1], pts[i][2]) for j, i in enumerate(reps) if ws[j] > 0]

    def _close_bucket(self) -> None:
        core = self._compress(self.pending, self.compressed)
        self.pending = []
        if self.forgetting_factor > 0:
            f = math.exp(-self.forgetting_factor)
            self.buckets = [[(w * f, fv, d) for w, fv, d in b if w * f >= self.forgetting_threshold]
                            for b in self.buckets]
            self.buckets = [b for b in self.buckets if b]
        self.buckets.append(core)
        while len(self.buckets) > self.bucket_length:
            merged = self._compress(self.buckets[0] + self.buckets[1], self.compressed)
            self.buckets = [merged] + self.buckets[2:]
        self._recluster()

    # ------------------------------------------------------------ cluster
    def _all_core(self):
        return [p for b in self.buckets for p in b] + list(self.others)

    def _recluster(self) -> None:
        torch = self._t()
        pts = self._all_core()
        if len(pts) < self.k:
            return
        dims = sorted({n for _, fv, _ in pts for n in fv})
        X = self._dense([fv for _, fv, _ in pts], dims)
        w = torch.tensor([p[0] for p in pts], dtype=torch.float32, device=X.device)
        rng = random.Random(self.seed + self.revision)
        C = X[self._kmeanspp(X, w, self.k, rng)].clone()
        fused = None
        if X.is_cuda:
            from ..ops import hip
            C = C.contiguous()
            fused = hip.lloyd(X.contiguous(), w.contiguous(), C, 100, 1e-6, 1e-5)
        for _ in range(0 if fused is not None else 100):
            a = self._sqdist(X, C).argmin(1)
            wsum = torch.zeros(C.shape[0], dtype=torch.float32, device=X.device).index_add_(0, a, w)
            S = torch.zeros_like(C).index_add_(0, a, X * w[:, None])
            newC = torch.where(wsum[:, None] > 0, S / wsum.clamp_min(1e-12)[:, None], C)
            done = bool(torch.allclose(newC, C, atol=1e-6))
            C = newC
            if done:
                break
        if self.method == "gmm":
            C, var, pi = self._em(X, w, C)
            self.variances, self.mix_weights = var, pi
        self.centers, self.dims = C, dims
        self.core = pts
        if fused is not None and self.method == "kmeans":
            self.assign = fused[0].cpu().tolist()    # the kernel's final assignment pass
        else:
            self.assign = self._assign(X).cpu().tolist()
        self.revision += 1

    def _log_resp(self, X, C, var, pi):
        torch = self._t()
        # diagonal Gaussian log densities [n, k]
        diff2 = (X[:, None, :] - C[None, :, :]) ** 2
        lp = -0.5 * ((diff2 / var[None]).sum(-1) + torch.log(2 * math.pi * var).sum(-1)[None])
        return lp + torch.log(pi.clamp_min(1e-12))[None]

    def _em(self, X, w, C, iters: int = 50):
        torch = self._t()
        k, d = C.shape
        var = torch.ones((k, d), dtype=torch.float32, device=X.device)
        pi = torch.full((k,), 1.0 / k, dtype=torch.float32, device=X.device)
        if X.is_cuda:
            from ..ops import hip
            C = C.contiguous().clone()
            if hip.gmm_em(X.contiguous(), w.contiguous(), C, var, pi, iters):
                return C, var, pi
        for _ in range(iters):
            r = torch.softmax(self._log_resp(X, C, var, pi), dim=1) * w[:, None]
            nk = r.sum(0).clamp_min(1e-9)
            C = (r.T @ X) / nk[:, None]
            var = ((r.T @ (X * X)) / nk[:, None] - C * C).clamp_min(1e-6)
            pi = nk / nk.sum()
        return C, var, pi

    def _assign(self, X):
        if self.method == "gmm":
            return self._log_resp(X, self.centers, self.variances, self.mix_weights).argmax(1)
        return self._sqdist(X, self.centers).argmin(1)

    def _check(self) -> None:
        if self.centers is None:
            raise NotPerformed()

    def _center_datum(self, j: int) -> Datum:
        c = self.centers[j].cpu().numpy()
        d = Datum()
        d.num_values = [(n, float(v)) for n, v in zip(self.dims, c) if v != 0.0]
        return d

    # ------------------------------------------------------------ queries
    def get_revision(self) -> int:
        return self.revision

    def get_k_center(self) -> list[Datum]:
        with self._lock:
            self._check()
            return [self._center_datum(j) for j in range(self.centers.shape[0])]

    def _nearest(self, d) -> int:
        fv: dict[str, float] = {}
        for name, v in self.conv.convert(as_datum(d)):
            fv[name] = fv.get(name, 0.0) + float(v)
        X = self._dense([fv], self.dims, self.centers.device)
        return int(self._assign(X)[0])

    def get_nearest_center(self, d) -> Datum:
        with self._lock:
            self._check()
            return self._center_datum(self._nearest(d))

    def get_core_members(self) -> list[list[tuple[float, Datum]]]:
        with self._lock:
            self._check()
            out: list[list[tuple[float, Datum]]] = [[] for _ in range(self.centers.shape[0])]
            for (w, _, d), a in zip(self.core, self.assign):
                out[a].append((float(w), d))
            return out

    def get_nearest_members(self, d) -> list[tuple[float, Datum]]:
        with self._lock:
            self._check()
            j = self._nearest(d)
            return [(float(w), dd) for (w, _, dd), a in zip(self.core, self.assign) if a == j]

    # ------------------------------------------------------------ MIX/persist
    def _wire(self, pts):
        return [[w, fv, d.to_msgpack()] for w, fv, d in pts]

    def _unwire(self, pts):
        return [(float(w), {str(k): float(v) for k, v in fv.items()}, Datum.from_msgpack(d))
                for w, fv, d in pts]

    def get_diff(self) -> dict:
        with self._lock:
            return {self.token: self._wire([p for b in self.buckets for p in b])}

    @staticmethod
    def mix_diff(a: dict, b: dict) -> dict:
        out = dict(a)
        out.update(b)
        return out

    def put_diff(self, mixed: dict) -> bool:
        with self._lock:
            self.others = [p for tok, pts in mixed.items() if tok != self.token
                           for p in self._unwire(pts)]
            self._recluster()
            return True

    def pack(self) -> dict:
        with self._lock:
            return {"method": self.method, "revision": self.revision,
                    "pending": self._wire(self.pending),
                    "buckets": [self._wire(b) for b in self.buckets],
                    "others": self._wire(self.others)}

    def unpack(self, obj: dict) -> None:
        with self._lock:
            self.clear()
            self.pending = self._unwire(obj["pending"])
            self.buckets = [self._unwire(b) for b in obj["buckets"]]
            self.others = self._unwire(obj["others"])
            rev = int(obj["revision"])
            if self.buckets or self.others:
                self._recluster()
            self.revision = rev

    def get_status(self) -> dict[str, str]:
        return {"method": self.method, "k": str(self.k), "revision": str(self.revision),
                "pending": str(len(self.pending)), "buckets": str(len(self.buckets)),
                "compressor_method": self.compressor, "storage": "hbm" if self.gpu else "host"}
