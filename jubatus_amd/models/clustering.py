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

Storage (MI355X design): points never live as per-point Python objects. A
push is converted in ONE native call (csrc/native/jb_hostfv_wide.hpp
``hash_named``: the whole msgpack list<datum> -> feature keys, values, names
and datum byte spans) into a ``PointSet``: weights, a CSR of (feature key,
value) and the raw datum bytes. Feature keys are the feature names hashed
into [0, 2^31 - 1) (each distinct key's name is recorded once); converters
the native path does not reproduce, or with idf / bm25 global weights, go
through the Python converter into the same key space. A bucket becomes a
dense matrix over its features (columns in name order) with one vectorised
scatter, and every k-means++ draw, Lloyd and EM iteration runs in
single-workgroup HIP launches (csrc/hip/clustering.hip), the distance
matrices on the matrix cores.
MIX: coresets are exchanged (get_diff / mix_diff / put_diff); every server
clusters its own coresets plus the other servers' ones.
"""
from __future__ import annotations

import math
import random
import threading
import uuid
from typing import Any

import msgpack
import numpy as np

from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import Datum, as_datum

COMPRESSORS = ("simple", "compressive_kmeans", "compressive_gmm")
KEY_SPACE = (1 << 31) - 1      # feature keys: hashed names (int32)


class NotPerformed(RuntimeError):
    def __init__(self):
        super().__init__("clustering is not performed yet")


def _ranges(starts: np.ndarray, lens: np.ndarray) -> np.ndarray:
    """concatenated arange(s, s + l) for every (s, l)"""
    tot = int(lens.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    rep = np.repeat(starts - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens)
    return rep + np.arange(tot, dtype=np.int64)


class PointSet:
    """weighted points: w [m] float64, CSR rows (key int64, value float32)
    and the msgpack bytes of every point's datum"""

    __slots__ = ("w", "rp", "key", "val", "raw", "_names")

    def __init__(self, w, rp, key, val, raw: list, names: dict):
        self.w = np.asarray(w, np.float64)
        self.rp = np.asarray(rp, np.int64)
        self.key = np.asarray(key, np.int64)
        self.val = np.asarray(val, np.float32)
        self.raw = raw
        self._names = names

    @classmethod
    def empty(cls, names: dict) -> "PointSet":
        return cls(np.zeros(0), np.zeros(1, np.int64), np.zeros(0, np.int64), np.zeros(0, np.float32), [],
                   names)

    def __len__(self) -> int:
        return int(self.w.size)

    def fv(self, i: int) -> dict:
        a, b = self.rp[i], self.rp[i + 1]
        out: dict[str, float] = {}
        for k, v in zip(self.key[a:b].tolist(), self.val[a:b].tolist()):
            nm = self._names[k]
            out[nm] = out.get(nm, 0.0) + float(v)
        return out

    def datum(self, i: int) -> Datum:
        return Datum.from_msgpack(msgpack.unpackb(self.raw[i], raw=False))

    def __iter__(self):
        """(weight, feature dict, datum) per point (tests, debugging)"""
        for i in range(len(self)):
            yield float(self.w[i]), self.fv(i), self.datum(i)

    def take(self, rows, w=None) -> "PointSet":
        rows = np.asarray(rows, np.int64)
        lens = self.rp[rows + 1] - self.rp[rows] if rows.size else np.zeros(0, np.int64)
        rp = np.zeros(rows.size + 1, np.int64)
        np.cumsum(lens, out=rp[1:])
        sel = _ranges(self.rp[rows], lens) if rows.size else np.zeros(0, np.int64)
        return PointSet(self.w[rows] if w is None else w, rp, self.key[sel], self.val[sel],
                        [self.raw[r] for r in rows.tolist()], self._names)

    @staticmethod
    def concat(sets: list, names: dict) -> "PointSet":
        sets = [s for s in sets if len(s)]
        if not sets:
            return PointSet.empty(names)
        if len(sets) == 1:
            return sets[0]
        rp = [np.zeros(1, np.int64)]
        off = 0
        for s in sets:
            rp.append(s.rp[1:] + off)
            off += int(s.rp[-1])
        return PointSet(np.concatenate([s.w for s in sets]), np.concatenate(rp),
                        np.concatenate([s.key for s in sets]), np.concatenate([s.val for s in sets]),
                        [r for s in sets for r in s.raw], names)

    def split(self, m: int) -> tuple["PointSet", "PointSet"]:
        n = len(self)
        return self.take(np.arange(min(m, n))), self.take(np.arange(min(m, n), n))


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
        self._names: dict[int, str] = {}       # feature key -> name
        self._native = self._make_native()
        self.clear()

    def _make_native(self):
        """the native named converter when it reproduces this config exactly
        (not with idf / bm25: their statistics live in the converter's tables)"""
        try:
            from .._native import native
            from ..fv_converter.gpu_path import WideRuleTable, wide_eligible
            if not wide_eligible(self.conv) or self.conv.uses_global_weight:
                return None
            rt = WideRuleTable(self.conv)
            return native().HostFvWide(rt.srules, rt.n_srules, rt.nrules, rt.n_nrules, rt.crules,
                                       rt.n_crules, rt.blob, KEY_SPACE)
        except Exception:  # noqa: BLE001 - native runtime not built: the Python converter
            return None

    def clear(self) -> None:
        with getattr(self, "_lock", threading.RLock()):
            self.pending = PointSet.empty(self._names)
            self.buckets: list[PointSet] = []
            self.others = PointSet.empty(self._names)
            self.revision = 0
            self.centers = None     # torch [k, D]
            self.variances = None   # gmm
            self.mix_weights = None
            self.dims: list[str] = []
            self._dim_keys = np.zeros(0, np.int64)
            self.assign: list[int] = []
            self.core = PointSet.empty(self._names)
            self._rng = random.Random(self.seed)

    # ------------------------------------------------------------ tensors
    def _t(self):
        import torch
        return torch

    # with a device every coreset / Lloyd / EM step runs in HBM: the k-means++
    # draws, the Lloyd iterations and the EM iterations of a bucket each run
    # in ONE single-workgroup launch (csrc/hip/clustering.hip). (Set higher to
    # keep small problems on the host.)
    GPU_MIN_ELEMS = 0

    def _columns(self, ps: PointSet) -> tuple[np.ndarray, list[str]]:
        """feature keys of a point set, ordered by feature name"""
        keys = np.unique(ps.key)
        names = [self._names[k] for k in keys.tolist()]
        order = sorted(range(len(names)), key=names.__getitem__)
        return keys[order], [names[i] for i in order]

    def _dense_keys(self, ps: PointSet, keys: np.ndarray, device=None):
        """[m, len(keys)] float32 of the points over the given feature keys
        (features outside them are dropped; repeated features add up)"""
        torch = self._t()
        m, D = len(ps), keys.size
        X = np.zeros((m, D), dtype=np.float32)
        if m and D and ps.key.size:
            srt = np.argsort(keys, kind="stable")
            sk = keys[srt]
            pos = np.minimum(np.searchsorted(sk, ps.key), D - 1)
            hit = sk[pos] == ps.key
            rows = np.repeat(np.arange(m), np.diff(ps.rp))
            np.add.at(X, (rows[hit], srt[pos[hit]]), ps.val[hit])
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

    # ------------------------------------------------------------ convert
    def _convert_body(self, body: bytes, update: bool) -> PointSet:
        """one msgpack list<datum> -> PointSet (weights 1)"""
        if self._native is not None:
            err, rp, idx, val, names, name_end, spans = self._native.hash_named(body, update)
            if err:
                from ..common.exceptions import ArgumentError
                raise ArgumentError("push: malformed datum list")
            key = idx.astype(np.int64)
            if key.size:
                uk, first = np.unique(key, return_index=True)
                new = [i for i, k in zip(first.tolist(), uk.tolist()) if k not in self._names]
                if new:
                    starts = np.concatenate([[0], name_end[:-1]])
                    for i in new:
                        self._names[int(key[i])] = names[starts[i]:name_end[i]].decode("utf-8",
                                                                                        "surrogateescape")
            mv = memoryview(body)
            raw = [bytes(mv[spans[2 * i]:spans[2 * i + 1]]) for i in range(rp.size - 1)]
            return PointSet(np.ones(rp.size - 1), rp, key, val, raw, self._names)
        pts = msgpack.unpackb(body, raw=False)
        return self._convert_datums([Datum.from_msgpack(p) for p in pts], update)

    def _key(self, name: str) -> int:
        from ..fv_converter.hashing import feature_index
        k = feature_index(name, KEY_SPACE)
        self._names.setdefault(k, name)
        return k

    def _convert_datums(self, ds: list, update: bool) -> PointSet:
        """the Python converter (configs the native one does not cover)"""
        rp, key, val, raw = [0], [], [], []
        for d in ds:
            d = as_datum(d)
            fv = self.conv.convert_and_update_weight(d) if update else self.conv.convert(d)
            for name, v in fv:
                key.append(self._key(name))
                val.append(float(v))
            rp.append(len(key))
            raw.append(msgpack.packb(d.to_msgpack(), use_bin_type=True))
        return PointSet(np.ones(len(ds)), rp, key, val, raw, self._names)

    # ------------------------------------------------------------ push
    def push(self, points: list) -> bool:
        ds = [as_datum(p) for p in points]
        if self._native is not None:
            return self.push_body(msgpack.packb([d.to_msgpack() for d in ds], use_bin_type=True))
        with self._lock:
            self._take(self._convert_datums(ds, True))
            return True

    def push_body(self, body) -> bool:
        """push(list<datum>) from the request's msgpack bytes (the server's
        raw path: no per-point Python object)"""
        with self._lock:
            self._take(self._convert_body(bytes(body), True))
            return True

    def _take(self, ps: PointSet) -> None:
        pend = PointSet.concat([self.pending, ps], self._names)
        while len(pend) >= self.bucket_size:
            full, pend = pend.split(self.bucket_size)
            self.pending = PointSet.empty(self._names)
            self._close_bucket(full)
        self.pending = pend

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

    def _compress(self, ps: PointSet, m: int) -> PointSet:
        if len(ps) <= m:
            return ps
        if self.compressor == "simple":
            idx = self._rng.sample(range(len(ps)), m)
            scale = float(ps.w.sum()) / float(ps.w[idx].sum())
            return ps.take(idx, ps.w[idx] * scale)
        torch = self._t()
        keys, _ = self._columns(ps)
        X = self._dense_keys(ps, keys)
        w = torch.tensor(ps.w, dtype=torch.float32, device=X.device)
        reps = self._kmeanspp(X, w, m, self._rng)
        a = self._sqdist(X, X[reps]).argmin(1)
        wsum = torch.zeros(len(reps), dtype=torch.float32, device=X.device).index_add_(0, a, w)
        ws = wsum.cpu().numpy().astype(np.float64)
        keep = [j for j in range(len(reps)) if ws[j] > 0]
        return ps.take([reps[j] for j in keep], ws[keep])

    def _close_bucket(self, full: PointSet) -> None:
        core = self._compress(full, self.compressed)
        if self.forgetting_factor > 0:
            f = math.exp(-self.forgetting_factor)
            out = []
            for b in self.buckets:
                w = b.w * f
                keep = np.flatnonzero(w >= self.forgetting_threshold)
                if keep.size:
                    out.append(b.take(keep, w[keep]))
            self.buckets = out
        self.buckets.append(core)
        while len(self.buckets) > self.bucket_length:
            merged = self._compress(PointSet.concat(self.buckets[:2], self._names), self.compressed)
            self.buckets = [merged] + self.buckets[2:]
        self._recluster()

    # ------------------------------------------------------------ cluster
    def _all_core(self) -> PointSet:
        return PointSet.concat(self.buckets + [self.others], self._names)

    def _recluster(self) -> None:
        torch = self._t()
        pts = self._all_core()
        if len(pts) < self.k:
            return
        keys, dims = self._columns(pts)
        X = self._dense_keys(pts, keys)
        w = torch.tensor(pts.w, dtype=torch.float32, device=X.device)
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
        em_assign = None
        if self.method == "gmm":
            C, var, pi = self._em(X, w, C)
            self.variances, self.mix_weights = var, pi
            em_assign = getattr(self, "_em_assign", None)
        self.centers, self.dims, self._dim_keys = C, dims, keys
        self.core = pts
        if fused is not None and self.method == "kmeans":
            self.assign = fused[0].cpu().tolist()    # the kernel's final assignment pass
        elif em_assign is not None:
            self.assign = em_assign.cpu().tolist()   # the EM kernel's final E-step argmax
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
            self._em_assign = torch.empty(X.shape[0], dtype=torch.int32, device=X.device)
            if hip.gmm_em(X.contiguous(), w.contiguous(), C, var, pi, iters, self._em_assign):
                return C, var, pi
        self._em_assign = None
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
        d = as_datum(d)
        if self._native is not None:
            ps = self._convert_body(msgpack.packb([d.to_msgpack()], use_bin_type=True), False)
        else:
            ps = self._convert_datums([d], False)
        X = self._dense_keys(ps, self._dim_keys, self.centers.device)
        return int(self._assign(X)[0])

    def get_nearest_center(self, d) -> Datum:
        with self._lock:
            self._check()
            return self._center_datum(self._nearest(d))

    def get_core_members(self) -> list[list[tuple[float, Datum]]]:
        with self._lock:
            self._check()
            out: list[list[tuple[float, Datum]]] = [[] for _ in range(self.centers.shape[0])]
            for i, a in enumerate(self.assign):
                out[a].append((float(self.core.w[i]), self.core.datum(i)))
            return out

    def get_nearest_members(self, d) -> list[tuple[float, Datum]]:
        with self._lock:
            self._check()
            j = self._nearest(d)
            return [(float(self.core.w[i]), self.core.datum(i)) for i, a in enumerate(self.assign)
                    if a == j]

    # ------------------------------------------------------------ MIX/persist
    def _wire(self, ps: PointSet) -> list:
        return [[float(ps.w[i]), ps.fv(i), msgpack.unpackb(ps.raw[i], raw=False)] for i in range(len(ps))]

    def _unwire(self, pts) -> PointSet:
        rp, key, val, raw, w = [0], [], [], [], []
        for pw, fv, d in pts:
            w.append(float(pw))
            for nm, v in fv.items():
                key.append(self._key(str(nm)))
                val.append(float(v))
            rp.append(len(key))
            raw.append(msgpack.packb(Datum.from_msgpack(d).to_msgpack(), use_bin_type=True))
        return PointSet(np.asarray(w), rp, key, val, raw, self._names)

    def get_diff(self) -> dict:
        with self._lock:
            return {self.token: self._wire(PointSet.concat(self.buckets, self._names))}

    @staticmethod
    def mix_diff(a: dict, b: dict) -> dict:
        out = dict(a)
        out.update(b)
        return out

    def put_diff(self, mixed: dict) -> bool:
        with self._lock:
            self.others = PointSet.concat([self._unwire(pts) for tok, pts in mixed.items()
                                           if tok != self.token], self._names)
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
            if self.buckets or len(self.others):
                self._recluster()
            self.revision = rev

    def get_status(self) -> dict[str, str]:
        return {"method": self.method, "k": str(self.k), "revision": str(self.revision),
                "pending": str(len(self.pending)), "buckets": str(len(self.buckets)),
                "compressor_method": self.compressor, "storage": "hbm" if self.gpu else "host",
                "converter": "native" if self._native is not None else "python"}
