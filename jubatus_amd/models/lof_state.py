"""Incremental LOF state: per-slot neighbour lists, k-distances and lrd.

Reference: anomaly_serv.cpp:157-244 (add / update / overwrite / calc_score)
over jubatus_core's lof_storage (EXTERNAL), which keeps, per stored row, its
k nearest neighbours, k-distance and local reachability density, and
refreshes them for the reverse_nearest_neighbor_num rows around every
changed row.

Two backends with the same semantics: ``HostLofState`` (NumPy; the CPU
engine and the oracle of the kernels) and ``DeviceLofState`` (HBM arrays and
csrc/hip/lof.hip - the list insert, the staleness mark over all lists and the
fused lrd/LOF score run on the GPU; only the candidate list goes up and the
score comes back).

State per slot s: nb_slot[s, :k] / nb_dist[s, :k] (ascending (distance,
slot), -1 / inf padded), kdist[s], lrd[s], ok[s] (the list is valid),
lrd_ok[s] (lrd is current). Operations:

* ``insert(p, cand)`` - p's rnn nearest candidates (ascending, p excluded):
  nb[p] = cand[:k]; every candidate o with a valid list takes p in when p is
  closer than its k-th neighbour. Every row whose list changed, and every row
  listing one of them, gets lrd_ok = 0.
* ``moved(slots)`` - these rows changed or were removed: their lists and the
  lists of every row listing them become invalid (recomputed on demand). An
  lrd counts as current only while every row of its list has a valid list;
  re-installing a list (``set_lists``) marks the rows listing it stale.
* ``score(targets, store)`` - LOF of a point from its k nearest (slot,
  distance) pairs, refreshing the stale lrd of the targets; returns the score
  or the slots whose lists must be (re)queried first (``set_lists``).
"""
from __future__ import annotations

import math

import numpy as np

LOF_MAX_K = 64            # csrc/hip/lof.hip kLofMaxK
LOF_MAX_CHANGED = 1024    # csrc/hip/lof.hip kLofMaxChanged
LOF_MAX_MISSING = 1024


def _kth(d: np.ndarray, ignore_same: bool) -> float:
    if ignore_same:
        d = d[d > 0]
    return float(d[-1]) if d.size else 0.0


def lof_score(lp: float, mean_lo: float) -> float:
    if math.isinf(lp):
        return 1.0 if math.isinf(mean_lo) else 0.0
    if lp == 0.0 or math.isinf(mean_lo):
        return math.inf
    return mean_lo / lp


class HostLofState:
    def __init__(self, k: int, ignore_same: bool):
        if not 0 < k <= LOF_MAX_K:
            raise ValueError(f"nearest_neighbor_num must be in 1..{LOF_MAX_K}")
        self.k = k
        self.ignore_same = ignore_same
        self.cap = 0
        self.clear()

    def clear(self) -> None:
        self.cap = 0
        self.nb_slot = np.zeros((0, self.k), np.int32)
        self.nb_dist = np.zeros((0, self.k), np.float32)
        self.kdist = np.zeros(0, np.float32)
        self.lrd = np.zeros(0, np.float32)
        self.ok = np.zeros(0, np.uint8)
        self.lrd_ok = np.zeros(0, np.uint8)

    def ensure(self, n: int) -> None:
        if n <= self.cap:
            return
        cap = max(n, 2 * self.cap, 1024)
        grow = cap - self.cap
        self.nb_slot = np.concatenate([self.nb_slot, np.full((grow, self.k), -1, np.int32)])
        self.nb_dist = np.concatenate([self.nb_dist, np.full((grow, self.k), np.inf, np.float32)])
        self.kdist = np.concatenate([self.kdist, np.zeros(grow, np.float32)])
        self.lrd = np.concatenate([self.lrd, np.zeros(grow, np.float32)])
        self.ok = np.concatenate([self.ok, np.zeros(grow, np.uint8)])
        self.lrd_ok = np.concatenate([self.lrd_ok, np.zeros(grow, np.uint8)])
        self.cap = cap

    def _set_list(self, s: int, sl: np.ndarray, dl: np.ndarray) -> None:
        m = sl.size
        self.nb_slot[s, :m] = sl
        self.nb_slot[s, m:] = -1
        self.nb_dist[s, :m] = dl
        self.nb_dist[s, m:] = np.inf
        self.kdist[s] = _kth(self.nb_dist[s, :m], self.ignore_same)
        self.ok[s] = 1
        self.lrd_ok[s] = 0

    def _mark(self, changed, clear_ok: bool) -> None:
        if not len(changed):
            return
        hit = np.isin(self.nb_slot, np.asarray(changed, np.int32)).any(1) & (self.ok == 1)
        self.lrd_ok[hit] = 0
        if clear_ok:
            self.ok[hit] = 0

    def insert(self, p: int, cs: np.ndarray, cd: np.ndarray) -> None:
        k = self.k
        self._set_list(p, cs[:k].astype(np.int32), cd[:k].astype(np.float32))
        changed = [p]
        for o, d in zip(cs.tolist(), cd.astype(np.float32).tolist()):
            if o < 0 or o == p or not self.ok[o]:
                continue
            row_s = self.nb_slot[o]
            keep = (row_s >= 0) & (row_s != p)
            had = bool(((row_s == p)).any())
            ts = row_s[keep].tolist()
            td = self.nb_dist[o][keep].tolist()
            if not had and len(ts) == k and not (d < td[-1] or (d == td[-1] and p < ts[-1])):
                continue
            at = len(ts)
            while at > 0 and (td[at - 1] > d or (td[at - 1] == d and ts[at - 1] > p)):
                at -= 1
            ts.insert(at, p)
            td.insert(at, d)
            self._set_list(o, np.asarray(ts[:k], np.int32), np.asarray(td[:k], np.float32))
            changed.append(o)
        self._mark(changed, False)

    def add(self, p: int, cs: np.ndarray, cd: np.ndarray, store: bool = True):
        """insert p with its candidates, then score it from the k nearest
        -> (score, []) or (None, missing)"""
        self.insert(p, cs, cd)
        return self.score(cs[:self.k], cd[:self.k], p if store else -1)

    def moved(self, slots) -> None:
        slots = [int(s) for s in slots]
        self.ensure(max(slots) + 1 if slots else 0)
        self._mark(slots, True)
        for s in slots:
            self.ok[s] = 0
            self.lrd_ok[s] = 0

    def set_lists(self, slots, lists) -> None:
        """lists[i]: (slots, dists) of row slots[i], ascending, may include itself"""
        for s, (ls, ld) in zip(slots, lists):
            ls = np.asarray(ls, np.int64)
            ld = np.asarray(ld, np.float32)
            keep = (ls >= 0) & (ls != s)
            self._set_list(int(s), ls[keep][:self.k].astype(np.int32), ld[keep][:self.k])
        self._mark(list(slots), False)

    def _lrd_of(self, sl: np.ndarray, dl: np.ndarray) -> float:
        m = sl >= 0
        if not m.any():
            return 0.0
        mean = float(np.maximum(self.kdist[sl[m]], dl[m]).astype(np.float32).mean(dtype=np.float32))
        return math.inf if mean <= 0 else float(np.float32(1.0) / np.float32(mean))

    def score(self, ts: np.ndarray, td: np.ndarray, store: int = -1):
        """-> (score, []) or (None, missing slots)"""
        missing = []
        for o in ts.tolist():
            if not self.ok[o]:
                missing.append(o)
                continue
            nb = self.nb_slot[o]
            bad = [x for x in nb[nb >= 0].tolist() if not self.ok[x]]
            if bad:
                missing.extend(bad)
                continue
            if self.lrd_ok[o]:
                continue
            self.lrd[o] = self._lrd_of(nb, self.nb_dist[o])
            self.lrd_ok[o] = 1
        if missing:
            return None, list(dict.fromkeys(missing))[:LOF_MAX_MISSING]
        if not ts.size:
            return 1.0, []
        lp = self._lrd_of(ts.astype(np.int32), td.astype(np.float32))
        lo = self.lrd[ts]
        mean_lo = math.inf if np.isinf(lo).any() else float(lo.astype(np.float32).sum(dtype=np.float32)
                                                          / np.float32(ts.size))
        if store >= 0:
            self.lrd[store] = lp
            self.lrd_ok[store] = 1
        return lof_score(lp, mean_lo), []


class DeviceLofState:
    """The same state in HBM; csrc/hip/lof.hip does the work."""

    def __init__(self, k: int, ignore_same: bool, device):
        if not 0 < k <= LOF_MAX_K:
            raise ValueError(f"nearest_neighbor_num must be in 1..{LOF_MAX_K}")
        import torch
        self.torch = torch
        self.k = k
        self.ignore_same = ignore_same
        self.device = torch.device(device)
        self._changed = torch.zeros(LOF_MAX_CHANGED, dtype=torch.int32, device=self.device)
        self._nchanged = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._up_host = torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True)
        self._up_dev = torch.empty(1 << 20, dtype=torch.uint8, device=self.device)
        from ..ops.hip import HostBuffer
        self._outbuf = HostBuffer(4 * (4 + LOF_MAX_MISSING))
        self._out = self._outbuf.view(np.int32, 4 + LOF_MAX_MISSING)
        self._pos = 0
        self.clear()

    def clear(self) -> None:
        torch = self.torch
        self.cap = 0
        d = self.device
        self.nb_slot = torch.zeros((0, self.k), dtype=torch.int32, device=d)
        self.nb_dist = torch.zeros((0, self.k), dtype=torch.float32, device=d)
        self.kdist = torch.zeros(0, dtype=torch.float32, device=d)
        self.lrd = torch.zeros(0, dtype=torch.float32, device=d)
        self.ok = torch.zeros(0, dtype=torch.uint8, device=d)
        self.lrd_ok = torch.zeros(0, dtype=torch.uint8, device=d)

    def ensure(self, n: int) -> None:
        if n <= self.cap:
            return
        torch = self.torch
        cap = max(n, 2 * self.cap, 1024)
        grow = cap - self.cap
        d = self.device
        self.nb_slot = torch.cat([self.nb_slot, torch.full((grow, self.k), -1, dtype=torch.int32,
                                                           device=d)])
        self.nb_dist = torch.cat([self.nb_dist, torch.full((grow, self.k), math.inf,
                                                           dtype=torch.float32, device=d)])
        self.kdist = torch.cat([self.kdist, torch.zeros(grow, dtype=torch.float32, device=d)])
        self.lrd = torch.cat([self.lrd, torch.zeros(grow, dtype=torch.float32, device=d)])
        self.ok = torch.cat([self.ok, torch.zeros(grow, dtype=torch.uint8, device=d)])
        self.lrd_ok = torch.cat([self.lrd_ok, torch.zeros(grow, dtype=torch.uint8, device=d)])
        self.cap = cap

    def _upload(self, *arrays: np.ndarray):
        """one H2D copy of several small host arrays -> device views. The
        pinned staging buffer is a ring: a region is reused only after a
        stream sync (``score`` syncs; a wrap-around syncs first)."""
        torch = self.torch
        sizes = [(a.nbytes + 15) // 16 * 16 for a in arrays]
        total = sum(sizes)
        if self._pos + total > self._up_host.numel():
            torch.cuda.current_stream(self.device).synchronize()
            self._pos = 0
            if total > self._up_host.numel():
                n = 1 << max(16, (total - 1).bit_length())
                self._up_host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
                self._up_dev = torch.empty(n, dtype=torch.uint8, device=self.device)
        hb = self._up_host.numpy()
        base = off = self._pos
        views = []
        for a, sz in zip(arrays, sizes):
            n = a.nbytes
            hb[off:off + n] = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
            views.append((off, n, a.dtype))
            off += sz
        self._up_dev[base:off].copy_(self._up_host[base:off], non_blocking=True)
        self._pos = off
        return [self._up_dev[o:o + n].view(torch.int32 if dt == np.int32 else torch.float32)
                for o, n, dt in views]

    def _result(self):
        o = self._out
        if o[0] == 2:
            nm = int(o[3])
            return None, list(dict.fromkeys(o[4:4 + nm].tolist()))
        if o[0] != 1:
            raise RuntimeError("lof: kernel did not complete")
        return float(o[1:2].view(np.float32)[0]), []

    def add(self, p: int, cs: np.ndarray, cd: np.ndarray, store: bool = True):
        """insert + mark + score of p in one host call (csrc/hip/lof.hip
        jb_lof_add; candidates in the kernel arguments)"""
        from ..ops import hip
        cs = np.ascontiguousarray(cs, np.int32)
        cd = np.ascontiguousarray(cd, np.float32)
        hip.lof_add(p, cs, cd, self, self._outbuf, LOF_MAX_MISSING)
        self._pos = 0
        return self._result()

    def moved(self, slots) -> None:
        slots = np.asarray(slots, np.int32)
        if not slots.size:
            return
        self.ensure(int(slots.max()) + 1)
        from ..ops import hip
        for i in range(0, slots.size, LOF_MAX_CHANGED):
            part = slots[i:i + LOF_MAX_CHANGED]
            (dv,) = self._upload(part)
            self._changed[:part.size].copy_(dv)
            self._nchanged.fill_(part.size)
            hip.lof_mark(self, True)
            idx = dv.long()
            self.ok.index_fill_(0, idx, 0)
            self.lrd_ok.index_fill_(0, idx, 0)

    def set_lists(self, slots, lists) -> None:
        from ..ops import hip
        kk = max((len(ls) for ls, _ in lists), default=0)
        if not kk:
            return
        n = len(slots)
        cs = np.full((n, kk), -1, np.int32)
        cd = np.full((n, kk), np.inf, np.float32)
        for i, (ls, ld) in enumerate(lists):
            cs[i, :len(ls)] = ls
            cd[i, :len(ld)] = ld
        for i in range(0, n, LOF_MAX_CHANGED):
            j = min(n, i + LOF_MAX_CHANGED)
            dsl, dcs, dcd = self._upload(np.asarray(slots[i:j], np.int32), cs[i:j], cd[i:j])
            hip.lof_set_lists(j - i, dsl, dcs, dcd, kk, self)
            hip.lof_mark(self, False)

    def score(self, ts: np.ndarray, td: np.ndarray, store: int = -1):
        from ..ops import hip
        if int(ts.size) == 0:
            return 1.0, []
        hip.lof_score(np.ascontiguousarray(ts, np.int32), np.ascontiguousarray(td, np.float32),
                      self, store, self._outbuf, LOF_MAX_MISSING)
        self._pos = 0
        return self._result()
