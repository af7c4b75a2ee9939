"""Row indexes for similarity search (nearest_neighbor, recommender, anomaly).

* ``LshIndex``       lsh / euclid_lsh / minhash signatures in a table
                     (HBM on a GPU: csrc/hip/lsh.hip), XOR-popcount scans
* ``InvertedIndex``  exact cosine (inverted_index) or euclidean
                     (inverted_index_euclid) over the sparse rows

Both map a row *slot* (int) to its representation; the id <-> slot mapping
lives in RowStore (models/rows.py). ``query(rows, k)`` returns, per query,
``[(slot, distance)]`` ascending; similarity views are derived by the
engines. The NumPy paths below are the oracles of the HIP kernels (same
splitmix64 hyperplane coefficients, same distance formulas).
"""
from __future__ import annotations

import math
import os
from typing import Any, Sequence

import numpy as np

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = (x + np.uint64(0x9E3779B97F4A7C15))
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def feat_hash(seed: int, idx: np.ndarray, j: np.ndarray) -> np.ndarray:
    idx = np.asarray(idx, dtype=np.uint64)
    j = np.asarray(j, dtype=np.uint64)
    return _splitmix(np.uint64(seed) ^ _splitmix((idx << np.uint64(20)) ^ j))


def gauss(h: np.ndarray) -> np.ndarray:
    u1 = ((h >> np.uint64(40)).astype(np.float64) + 1.0) / 16777217.0
    u2 = (h & np.uint64(0xFFFFFF)).astype(np.float64) / 16777216.0
    return (np.sqrt(-2.0 * np.log(u1)) * np.cos(6.2831853 * u2)).astype(np.float32)


def signature_host(idx: Sequence[int], val: Sequence[float], hash_num: int, seed: int,
                   mode: int) -> tuple[np.ndarray, float]:
    """(bits uint64[words], norm) of one sparse vector."""
    idx = np.asarray(idx, dtype=np.int64)
    val = np.asarray(val, dtype=np.float32)
    m = idx >= 0
    idx, val = idx[m], val[m]
    words = (hash_num + 63) // 64
    j = np.arange(words * 64, dtype=np.uint64)
    if len(idx) == 0:
        bits = np.zeros(words * 64, dtype=bool)
    else:
        h = feat_hash(seed, idx[:, None].astype(np.uint64), j[None, :])
        if mode == 0:
            acc = (val[:, None] * gauss(h)).sum(axis=0)
            bits = acc > 0
        else:
            keep = val != 0
            if not keep.any():
                bits = np.ones(words * 64, dtype=bool)  # min of nothing = all ones
            else:
                bits = (h[keep].min(axis=0) & np.uint64(1)) != 0
    bits[hash_num:] = False
    packed = np.zeros(words, dtype=np.uint64)
    for w in range(words):
        chunk = bits[w * 64:(w + 1) * 64]
        packed[w] = np.uint64(sum(1 << i for i, b in enumerate(chunk) if b))
    return packed, float(np.sqrt((val.astype(np.float64) ** 2).sum()))


def _popcount(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.uint64)
    c = np.zeros(x.shape, dtype=np.int64)
    while np.any(x):
        c += (x & np.uint64(1)).astype(np.int64)
        x >>= np.uint64(1)
    return c


METRIC = {"lsh": 0, "euclid_lsh": 1, "minhash": 2}


class LshIndex:
    def __init__(self, method: str, hash_num: int = 64, seed: int = 1091, device: Any = None):
        if method not in METRIC:
            raise ValueError(f"unknown lsh method {method}")
        if hash_num <= 0:
            raise ValueError("hash_num must be positive")
        self.method, self.hash_num, self.seed = method, int(hash_num), int(seed)
        self.metric = METRIC[method]
        self.mode = 1 if method == "minhash" else 0
        self.words = (self.hash_num + 63) // 64
        self.device = device
        self.gpu = device is not None
        self.cap = 0
        self._direct = None
        self._alloc(1024)

    def _alloc(self, cap: int) -> None:
        if self.gpu:
            import torch
            bits = torch.zeros((cap, self.words), dtype=torch.int64, device=self.device)
            norms = torch.zeros(cap, dtype=torch.float32, device=self.device)
            valid = torch.zeros(cap, dtype=torch.uint8, device=self.device)
            if self.cap:
                bits[:self.cap] = self.bits
                norms[:self.cap] = self.norms
                valid[:self.cap] = self.valid
        else:
            bits = np.zeros((cap, self.words), dtype=np.uint64)
            norms = np.zeros(cap, dtype=np.float32)
            valid = np.zeros(cap, dtype=np.uint8)
            if self.cap:
                bits[:self.cap] = self.bits
                norms[:self.cap] = self.norms
                valid[:self.cap] = self.valid
        self.bits, self.norms, self.valid, self.cap = bits, norms, valid, cap

    def clear(self) -> None:
        self.cap = 0
        self._alloc(1024)

    def _signatures(self, rows: list[tuple[Sequence[int], Sequence[float]]]):
        """-> (bits [n, words], norms [n]) on the index's device."""
        if self.gpu:
            import torch
            from ..ops import hip
            from ..ops.feature_pipeline import FeaturePipeline  # noqa: F401 (CSR helper below)
            row_ptr, fidx, fval = _csr_device(rows, self.device)
            n = len(rows)
            bits = torch.empty((max(n, 1), self.words), dtype=torch.int64, device=self.device)
            norms = torch.empty(max(n, 1), dtype=torch.float32, device=self.device)
            hip.signature(row_ptr, fidx, fval, n, self.hash_num, self.seed, self.mode, bits, norms)
            return bits[:n], norms[:n]
        out = [signature_host(i, v, self.hash_num, self.seed, self.mode) for i, v in rows]
        bits = np.stack([b for b, _ in out]) if out else np.zeros((0, self.words), np.uint64)
        norms = np.asarray([n for _, n in out], dtype=np.float32)
        return bits, norms

    def set_rows(self, slots: Sequence[int], rows: list[tuple[Sequence[int], Sequence[float]]]) -> None:
        if not slots:
            return
        need = max(slots) + 1
        if need > self.cap:
            c = self.cap
            while c < need:
                c *= 2
            self._alloc(c)
        bits, norms = self._signatures(rows)
        if self.gpu:
            import torch
            s = torch.as_tensor(list(slots), dtype=torch.int64, device=self.device)
            self.bits[s] = bits
            self.norms[s] = norms
            self.valid[s] = 1
        else:
            s = np.asarray(slots, dtype=np.int64)
            self.bits[s] = bits
            self.norms[s] = norms
            self.valid[s] = 1

    def set_rows_csr(self, slots: np.ndarray, row_ptr: np.ndarray, idx: np.ndarray,
                     val: np.ndarray) -> None:
        """bulk insert: host CSR of n rows -> one H2D copy + one signature
        launch + one scatter into the HBM table (MIX put_diff, load, bulk
        ingest)."""
        n = int(slots.size)
        if n == 0:
            return
        need = int(slots.max()) + 1
        if need > self.cap:
            c = self.cap
            while c < need:
                c *= 2
            self._alloc(c)
        if not self.gpu:
            rows = [(idx[row_ptr[i]:row_ptr[i + 1]], val[row_ptr[i]:row_ptr[i + 1]]) for i in range(n)]
            self.set_rows(slots.tolist(), rows)
            return
        import torch
        from ..ops import hip
        nnz = int(row_ptr[n])
        d = self.device
        rp = torch.from_numpy(np.ascontiguousarray(row_ptr[:n + 1], dtype=np.int64)).to(d)
        fi = torch.from_numpy(np.ascontiguousarray(idx[:max(nnz, 1)], dtype=np.int32)).to(d)
        fv = torch.from_numpy(np.ascontiguousarray(val[:max(nnz, 1)], dtype=np.float32)).to(d)
        bits = torch.empty((n, self.words), dtype=torch.int64, device=d)
        norms = torch.empty(n, dtype=torch.float32, device=d)
        hip.signature(rp, fi, fv, n, self.hash_num, self.seed, self.mode, bits, norms)
        st = torch.from_numpy(np.ascontiguousarray(slots, dtype=np.int64)).to(d)
        self.bits.index_copy_(0, st, bits)
        self.norms.index_copy_(0, st, norms)
        self.valid.index_fill_(0, st, 1)

    # MIX (parallel/row_mix.py): signatures travel as they are in the table
    def export_signatures(self, slots: np.ndarray):
        if self.gpu:
            import torch
            s = torch.as_tensor(np.asarray(slots, np.int64), device=self.device)
            return self.bits.index_select(0, s), self.norms.index_select(0, s)
        s = np.asarray(slots, np.int64)
        return self.bits[s].view(np.int64), self.norms[s]

    def import_signatures(self, slots: np.ndarray, bits, norms) -> None:
        n = int(np.asarray(slots).size)
        if n == 0:
            return
        need = int(np.max(slots)) + 1
        if need > self.cap:
            c = self.cap
            while c < need:
                c *= 2
            self._alloc(c)
        if self.gpu:
            import torch
            st = torch.as_tensor(np.asarray(slots, np.int64), device=self.device)
            self.bits.index_copy_(0, st, bits.to(self.device).view(torch.int64).reshape(n, self.words))
            self.norms.index_copy_(0, st, norms.to(self.device).view(torch.float32))
            self.valid.index_fill_(0, st, 1)
            return
        b = bits.cpu().numpy() if hasattr(bits, "cpu") else np.asarray(bits)
        nm = norms.cpu().numpy() if hasattr(norms, "cpu") else np.asarray(norms)
        s = np.asarray(slots, np.int64)
        self.bits[s] = b.reshape(n, self.words).view(np.uint64)
        self.norms[s] = nm
        self.valid[s] = 1

    def set_rows_direct(self, slots: np.ndarray, row_ptr: np.ndarray, idx: np.ndarray,
                        val: np.ndarray) -> bool:
        """latency path of set_row / update_row: one launch, the rows in the
        kernel arguments, signatures written straight into their slots"""
        if not self.gpu:
            return False
        need = int(slots.max()) + 1
        if need > self.cap:
            c = self.cap
            while c < need:
                c *= 2
            self._alloc(c)
        from ..ops import hip
        return hip.lsh_set_rows_direct(idx.ctypes.data, val.ctypes.data, row_ptr.ctypes.data,
                                       int(slots.size), slots.ctypes.data, self.hash_num,
                                       self.seed, self.mode, self.bits, self.norms, self.valid)

    def remove(self, slot: int) -> None:
        if slot < self.cap:
            self.valid[slot] = 0

    def distances(self, rows: list, nrows: int):
        """distance matrix [nq, nrows] (device tensor or ndarray)"""
        nq = len(rows)
        qb, qn = self._signatures(rows)
        if self.gpu:
            import torch
            from ..ops import hip
            out = torch.empty((nq, max(nrows, 1)), dtype=torch.float32, device=self.device)
            if nrows:
                hip.hamming_scan(qb.contiguous(), qn.contiguous(), nq, self.bits, self.norms,
                                 self.valid, nrows, self.hash_num, self.metric, out)
            return out[:, :nrows]
        tb = self.bits[:nrows]
        ham = np.zeros((nq, nrows), dtype=np.int64)
        for w in range(self.words):
            ham += _popcount(qb[:, w][:, None] ^ tb[:, w][None, :])
        frac = ham.astype(np.float32) / self.hash_num
        if self.metric == 1:
            a = qn[:, None].astype(np.float32)
            b = self.norms[:nrows][None, :]
            d = np.sqrt(np.maximum(0.0, a * a + b * b - 2 * a * b * np.cos(np.float32(math.pi) * frac)))
        else:
            d = frac
        d = d.astype(np.float32)
        d[:, self.valid[:nrows] == 0] = np.inf
        return d

    def similarity_of(self, d):
        """distance -> similarity as reported by similar_row_* (lsh / minhash:
        1 - d; euclid_lsh: -d)"""
        return -d if self.metric == 1 else 1.0 - d

    def query(self, rows: list, nrows: int, k: int, similar: bool) -> list[list[tuple[int, float]]]:
        if self.gpu and nrows > 0 and rows:
            from ..ops import hip
            if 0 < k <= hip.TOPK_MAX_K and self.words <= hip.TOPK_MAX_WORDS:
                # fused scan + exact top-k (csrc/hip/topk.hip): no nq x N matrix
                qb, qn = self._signatures(rows)
                d, i = hip.topk_hamming(qb.contiguous(), qn.contiguous(), len(rows), self.bits,
                                        self.norms, self.valid, nrows, self.hash_num,
                                        self.metric, k)
                return _pairs(d.cpu().numpy(), i.cpu().numpy(),
                              self.similarity_of if similar else None)
        return topk(self.distances(rows, nrows), k, self.similarity_of if similar else None)

    def query_direct(self, idx, val, row_ptr, nq: int, nrows: int, k: int,
                     similar: bool) -> list[list[tuple[int, float]]] | None:
        """latency path: host-hashed query CSR (numpy int32 / float32 / int64)
        -> one signature launch from kernel arguments + fused scan/top-k whose
        result lands in pinned host memory (csrc/hip/lsh.hip). None when not
        applicable (CPU index, large query / k)."""
        if not (self.gpu and nrows > 0):
            return None
        from ..ops import hip
        if self._direct is None:
            self._direct = hip.DirectQueryBuffers(self.device, self.words)
        import torch
        stream = torch.cuda.current_stream(self.device)
        r = hip.lsh_query_direct(idx.ctypes.data, val.ctypes.data, row_ptr.ctypes.data, nq,
                                 self.hash_num, self.seed, self.mode, self.metric, self.bits,
                                 self.norms, self.valid, nrows, k, self._direct,
                                 stream.cuda_stream)
        if r is None:
            return None
        return _pairs(r[0], r[1], self.similarity_of if similar else None)

    def query_slots(self, slots: Sequence[int], nrows: int, k: int,
                    similar: bool) -> list[list[tuple[int, float]]] | None:
        """queries by stored rows (their own signatures, no re-hashing); one
        fused scan + top-k launch for all of them. None: not supported here
        (the caller queries by feature vector)."""
        if not (self.gpu and nrows > 0 and slots):
            return None
        from ..ops import hip
        if not (0 < k <= hip.TOPK_MAX_K and self.words <= hip.TOPK_MAX_WORDS):
            return None
        import torch
        slots = list(slots)
        if len(slots) <= hip.QUERY_MAX:
            # latency path: rows gathered on the device, result in pinned host memory
            if self._direct is None:
                self._direct = hip.DirectQueryBuffers(self.device, self.words)
            if len(slots) == 1:
                s0 = int(slots[0])
                qb, qn = self.bits[s0:s0 + 1], self.norms[s0:s0 + 1]
            else:
                st = torch.as_tensor(slots, dtype=torch.int64).to(self.device, non_blocking=True)
                qb = self.bits.index_select(0, st)
                qn = self.norms.index_select(0, st)
            r = hip.topk_rows_direct(qb, qn, len(slots), self.bits, self.norms, self.valid, nrows,
                                     self.hash_num, self.metric, k, self._direct)
            return _pairs(r[0], r[1], self.similarity_of if similar else None)
        st = torch.as_tensor(slots, dtype=torch.int64).to(self.device)
        qb = self.bits.index_select(0, st).contiguous()
        qn = self.norms.index_select(0, st).contiguous()
        d, i = hip.topk_hamming(qb, qn, len(slots), self.bits, self.norms, self.valid, nrows,
                                self.hash_num, self.metric, k)
        return _pairs(d.cpu().numpy(), i.cpu().numpy(), self.similarity_of if similar else None)

    def state(self, nrows: int) -> dict:
        if self.gpu:
            bits = self.bits[:nrows].cpu().numpy().view(np.uint64)
            norms = self.norms[:nrows].cpu().numpy()
            valid = self.valid[:nrows].cpu().numpy()
        else:
            bits, norms, valid = self.bits[:nrows], self.norms[:nrows], self.valid[:nrows]
        return {"bits": np.ascontiguousarray(bits).tobytes(), "norms": norms.tobytes(),
                "valid": valid.tobytes(), "n": nrows}

    def load_state(self, st: dict) -> None:
        n = int(st["n"])
        self.clear()
        c = 1024
        while c < n:
            c *= 2
        self.cap = 0
        self._alloc(c)
        bits = np.frombuffer(st["bits"], dtype=np.uint64).reshape(n, self.words)
        norms = np.frombuffer(st["norms"], dtype=np.float32)
        valid = np.frombuffer(st["valid"], dtype=np.uint8)
        if self.gpu:
            import torch
            self.bits[:n] = torch.from_numpy(bits.view(np.int64).copy()).to(self.device)
            self.norms[:n] = torch.from_numpy(norms.copy()).to(self.device)
            self.valid[:n] = torch.from_numpy(valid.copy()).to(self.device)
        else:
            self.bits[:n], self.norms[:n], self.valid[:n] = bits, norms, valid


def topk(d, k: int, to_sim=None) -> list[list[tuple[int, float]]]:
    """smallest-k distances per query row (inf = absent), optionally mapped to
    similarities."""
    out = []
    if hasattr(d, "is_cuda"):
        import torch
        n = d.shape[1]
        kk = min(k, n)
        if kk <= 0:
            return [[] for _ in range(d.shape[0])]
        vals, idx = torch.topk(d, kk, dim=1, largest=False)
        vals, idx = vals.cpu().numpy(), idx.cpu().numpy()
    else:
        n = d.shape[1]
        kk = min(k, n)
        if kk <= 0:
            return [[] for _ in range(d.shape[0])]
        idx = np.argsort(d, axis=1, kind="stable")[:, :kk]
        vals = np.take_along_axis(d, idx, axis=1)
    for vr, ir in zip(vals, idx):
        row = []
        for v, i in zip(vr, ir):
            if not np.isfinite(v):
                continue
            row.append((int(i), float(to_sim(np.float32(v)) if to_sim else v)))
        out.append(row)
    return out


def _pairs(vals: np.ndarray, idx: np.ndarray, to_sim=None) -> list[list[tuple[int, float]]]:
    out = []
    for vr, ir in zip(vals, idx):
        row = []
        for v, i in zip(vr.tolist(), ir.tolist()):
            if not math.isfinite(v):
                break
            row.append((int(i), float(to_sim(np.float32(v)) if to_sim else v)))
        out.append(row)
    return out


def _csr_device(rows, device):
    import torch
    n = len(rows)
    lens = np.fromiter((len(r[0]) for r in rows), dtype=np.int64, count=n)
    rp = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(lens, out=rp[1:])
    nnz = int(rp[-1])
    idx = np.fromiter((i for r in rows for i in r[0]), dtype=np.int32, count=nnz)
    val = np.fromiter((v for r in rows for v in r[1]), dtype=np.float32, count=nnz)
    if nnz == 0:
        idx, val = np.zeros(1, np.int32), np.zeros(1, np.float32)
    return (torch.from_numpy(rp).to(device), torch.from_numpy(idx).to(device),
            torch.from_numpy(val).to(device))


def normalize_csr(row_ptr: np.ndarray, idx: np.ndarray, val: np.ndarray):
    """Per row: drop idx < 0, sort by feature, sum repeated features
    (vectorised over the whole batch). -> (lens int64[n], idx int32[nnz],
    val float32[nnz], squared norms float32[n])."""
    row_ptr = np.asarray(row_ptr, dtype=np.int64)
    n = row_ptr.size - 1
    idx = np.asarray(idx, dtype=np.int64)[:row_ptr[-1]]
    val = np.asarray(val, dtype=np.float64)[:row_ptr[-1]]
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(row_ptr))
    m = idx >= 0
    rows, idx, val = rows[m], idx[m], val[m]
    order = np.lexsort((idx, rows))
    rows, idx, val = rows[order], idx[order], val[order]
    if rows.size:
        new = np.ones(rows.size, dtype=bool)
        new[1:] = (rows[1:] != rows[:-1]) | (idx[1:] != idx[:-1])
        starts = np.flatnonzero(new)
        val = np.add.reduceat(val, starts)
        idx, rows = idx[starts], rows[starts]
    lens = np.bincount(rows, minlength=n).astype(np.int64)
    val32 = val.astype(np.float32)
    v = val32.astype(np.float64)           # the stored values, squared exactly
    n2 = np.bincount(rows, weights=v * v, minlength=n)
    return lens, idx.astype(np.int32), val32, n2


def _rows_to_csr(rows) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    lens = np.fromiter((len(r[0]) for r in rows), dtype=np.int64, count=len(rows))
    rp = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum(lens, out=rp[1:])
    nnz = int(rp[-1])
    idx = np.fromiter((i for r in rows for i in r[0]), dtype=np.int64, count=nnz)
    val = np.fromiter((v for r in rows for v in r[1]), dtype=np.float32, count=nnz)
    return rp, idx, val


class DevicePool:
    """HBM row pool of the device inverted index (csrc/hip/sparse_pool.hip):
    append-only runs of (feature, value) plus per-slot offset / length /
    squared norm / valid. The host keeps only the slots' offsets and lengths
    (no copy of the data) to size appends and compact the pool. Squared
    norms are float64 (the euclidean self-distance must cancel to ~0)."""

    def __init__(self, device):
        self.device = device
        self._stager = None
        self._scores = None
        self.nlive = 0                    # slots holding a row
        self.cap_rows = 0
        self.cap_entries = 0
        self.end = 0                      # next free pool entry
        self.live = 0                     # entries of the current runs
        self.off_h = np.zeros(0, dtype=np.int64)
        self.len_h = np.zeros(0, dtype=np.int64)
        self.has_h = np.zeros(0, dtype=bool)
        self._grow_rows(1024)
        self._grow_entries(1 << 16)

    def _grow_rows(self, need: int) -> None:
        import torch
        cap = max(1024, self.cap_rows)
        while cap < need:
            cap *= 2
        if cap == self.cap_rows:
            return
        d = self.device

        def grow(old, dtype, fill=0):
            t = torch.full((cap,), fill, dtype=dtype, device=d)
            if old is not None:
                t[:old.numel()].copy_(old)
            return t
        self.r_off = grow(getattr(self, "r_off", None), torch.int64)
        self.r_len = grow(getattr(self, "r_len", None), torch.int32)
        self.r_n2 = grow(getattr(self, "r_n2", None), torch.float64)
        self.valid = grow(getattr(self, "valid", None), torch.uint8)
        off_h = np.zeros(cap, dtype=np.int64)
        len_h = np.zeros(cap, dtype=np.int64)
        has_h = np.zeros(cap, dtype=bool)
        off_h[:self.off_h.size] = self.off_h
        len_h[:self.len_h.size] = self.len_h
        has_h[:self.has_h.size] = self.has_h
        self.off_h, self.len_h, self.has_h = off_h, len_h, has_h
        self.cap_rows = cap

    def _grow_entries(self, need: int) -> None:
        import torch
        cap = max(1 << 16, self.cap_entries)
        while cap < need:
            cap *= 2
        if cap == self.cap_entries:
            return
        pi = torch.empty(cap, dtype=torch.int32, device=self.device)
        pv = torch.empty(cap, dtype=torch.float32, device=self.device)
        if self.cap_entries:
            pi[:self.end].copy_(self.p_idx[:self.end])
            pv[:self.end].copy_(self.p_val[:self.end])
        self.p_idx, self.p_val = pi, pv
        self.cap_entries = cap

    def score_scratch(self, n: int):
        """device score matrix of the latency query path ([nq][nrows] fp32)"""
        import torch
        if self._scores is None or self._scores.numel() < n:
            self._scores = torch.empty(max(n, 1 << 16), dtype=torch.float32, device=self.device)
        return self._scores

    def lanes_per_row(self, nq: int = 1) -> int:
        """scan lanes per row from the mean run length (measured at 1M rows:
        4 lanes beat 1 from ~12 entries per row for one query, 148 -> 104 us
        at ~20; with 4+ queries per pass the per-entry work dominates and one
        lane per row stays ahead up to ~24)"""
        forced = os.environ.get("JUBATUS_POOL_LPR")
        if forced in ("1", "4", "16"):
            return int(forced)
        rows = max(1, self.nlive)
        mean = self.live / rows
        if nq >= 4 and mean <= 24:
            return 1
        return 1 if mean <= 8 else 4 if mean <= 64 else 16

    def compact(self) -> None:
        """rewrite the live runs contiguously (device gather), dropping the
        runs that updates and removals left behind"""
        import torch
        live = np.flatnonzero(self.len_h > 0)
        lens = self.len_h[live]
        new_off = np.zeros(live.size, dtype=np.int64)
        if live.size:
            np.cumsum(lens[:-1], out=new_off[1:])
        total = int(lens.sum())
        if total:
            d = self.device
            src = torch.from_numpy(np.repeat(self.off_h[live] - new_off, lens)).to(d) + \
                torch.arange(total, dtype=torch.int64, device=d)
            self.p_idx[:total] = self.p_idx[src].clone()
            self.p_val[:total] = self.p_val[src].clone()
            self.r_off[torch.from_numpy(live).to(d)] = torch.from_numpy(new_off).to(d)
        self.off_h[live] = new_off
        self.end = self.live = total

    def append(self, slots: np.ndarray, lens: np.ndarray, idx: np.ndarray, val: np.ndarray,
               n2: np.ndarray) -> None:
        import torch
        from ..ops import hip
        n, nnz = int(slots.size), int(idx.size)
        if n == 0:
            return
        self._grow_rows(int(slots.max()) + 1)
        if self.end + nnz > self.cap_entries and self.end - self.live > self.live:
            self.compact()
        self._grow_entries(self.end + nnz)
        run = np.zeros(n, dtype=np.int64)
        if n > 1:
            np.cumsum(lens[:-1], out=run[1:])
        meta = np.empty((n, 4), dtype=np.int64)
        meta[:, 0] = slots
        meta[:, 1] = lens
        meta[:, 2] = np.asarray(n2, dtype=np.float64).view(np.int64)
        meta[:, 3] = run
        pack = np.concatenate([meta.reshape(-1).view(np.uint8), idx.astype(np.int32).view(np.uint8),
                               val.astype(np.float32).view(np.uint8)])
        if pack.nbytes <= (256 << 10):
            (dev,) = self.stager().put(pack)      # latency path: pinned ring, async
        else:
            dev = torch.from_numpy(pack).to(self.device)
        hip.pool_append(dev, n, nnz, self.end, self)
        old = self.len_h[slots]
        self.live += nnz - int(old.sum())
        self.nlive += int((~self.has_h[slots]).sum())
        self.has_h[slots] = True
        self.off_h[slots] = self.end + run
        self.len_h[slots] = lens
        self.end += nnz

    def remove(self, slot: int) -> None:
        if 0 <= slot < self.cap_rows and self.len_h[slot] >= 0:
            ln = int(self.len_h[slot])
            self.live -= ln
            if self.has_h[slot]:
                self.nlive -= 1
                self.has_h[slot] = False
            self.len_h[slot] = 0
            self.valid[slot] = 0

    def stager(self):
        if self._stager is None:
            from ..ops.staging import Stager
            self._stager = Stager(self.device)
        return self._stager

    def query_slots_device(self, slots: Sequence[int]):
        """stored rows as queries, read by the scan kernel from the pool:
        -> ("slots", device int32 slots, total entries)"""
        slots = np.asarray(slots, dtype=np.int32)
        (ds,) = self.stager().put(slots)
        return ("slots", ds, int(self.len_h[slots].sum()))


class InvertedIndex:
    """Exact sparse similarity (inverted_index: cosine; inverted_index_euclid:
    euclidean distance). On a GPU the rows live in an HBM pool updated in
    place (DevicePool, csrc/hip/sparse_pool.hip) and up to 8 queries are
    scored per pass over it, then the fused top-k (csrc/hip/topk.hip) picks
    the k best; without a GPU the rows are sorted sparse vectors on the
    host (the oracle)."""

    def __init__(self, euclid: bool = False, device: Any = None):
        self.euclid = euclid
        self.device = device
        self.gpu = device is not None
        self.rows: dict[int, tuple[np.ndarray, np.ndarray]] = {}
        self.pool = DevicePool(device) if self.gpu else None
        self._direct = None

    def clear(self) -> None:
        self.rows.clear()
        if self.gpu:
            self.pool = DevicePool(self.device)

    @staticmethod
    def _norm_row(idx, val) -> tuple[np.ndarray, np.ndarray]:
        d: dict[int, float] = {}
        for i, v in zip(idx, val):
            if i >= 0:
                d[int(i)] = d.get(int(i), 0.0) + float(v)
        ks = np.asarray(sorted(d), dtype=np.int32)
        return ks, np.asarray([d[int(k)] for k in ks], dtype=np.float32)

    def set_rows(self, slots, rows) -> None:
        if self.gpu:
            rp, idx, val = _rows_to_csr(rows)
            self.set_rows_csr(np.asarray(slots, dtype=np.int64), rp, idx, val)
            return
        for s, (i, v) in zip(slots, rows):
            self.rows[int(s)] = self._norm_row(i, v)

    def set_rows_csr(self, slots: np.ndarray, row_ptr: np.ndarray, idx: np.ndarray,
                     val: np.ndarray) -> None:
        slots = np.asarray(slots, dtype=np.int64)
        if self.gpu:
            from .._native import native
            lens, ni, nv, n2 = native().csr_normalize(row_ptr[:slots.size + 1], idx, val)
            self.pool.append(slots, lens, ni, nv, n2)
            return
        rows = [(idx[row_ptr[i]:row_ptr[i + 1]], val[row_ptr[i]:row_ptr[i + 1]])
                for i in range(int(slots.size))]
        self.set_rows(slots.tolist(), rows)

    def remove(self, slot: int) -> None:
        if self.gpu:
            self.pool.remove(int(slot))
            return
        self.rows.pop(int(slot), None)

    # latency paths (models/row_engine.py): natively hashed host CSR
    def set_rows_direct(self, slots: np.ndarray, row_ptr: np.ndarray, idx: np.ndarray,
                        val: np.ndarray) -> bool:
        if not self.gpu:
            return False
        n = int(np.asarray(slots).size)
        self.set_rows_csr(np.asarray(slots, np.int64), row_ptr[:n + 1], idx[:int(row_ptr[n])],
                          val[:int(row_ptr[n])])
        return True

    def _direct_pairs(self, r, similar: bool):
        out = _pairs(r[0], r[1])
        if similar:
            out = [[(j, float(-dd if self.euclid else 1.0 - dd)) for j, dd in x] for x in out]
        return out

    def _bufs(self):
        if self._direct is None:
            from ..ops import hip
            self._direct = hip.DirectQueryBuffers(self.device, 1)
        return self._direct

    def query_direct(self, idx, val, row_ptr, nq: int, nrows: int, k: int,
                     similar: bool) -> list[list[tuple[int, float]]] | None:
        if not (self.gpu and nrows > 0 and k > 0):
            return None
        from ..ops import hip
        if nq <= hip.POOL_MAX_Q and k <= hip.TOPK_MAX_K:
            r = hip.pool_query_direct(self.pool, nrows, 1 if self.euclid else 0, k, self._bufs(),
                                      idx=np.ascontiguousarray(idx, np.int32),
                                      val=np.ascontiguousarray(val, np.float32),
                                      row_ptr=np.ascontiguousarray(row_ptr, np.int64), nq=nq)
            if r is not None:
                return self._direct_pairs(r, similar)
        rp = np.asarray(row_ptr[:nq + 1], np.int64)
        return self._query_batches(
            lambda a, b: self._queries_csr(rp[a:b + 1] - rp[a], idx[rp[a]:rp[b]], val[rp[a]:rp[b]]),
            nq, nrows, k, similar)

    # ------------------------------------------------------------ device
    def _queries_device(self, rows):
        return self._queries_csr(*_rows_to_csr(rows))

    def _queries_csr(self, rp, idx, val):
        """host query CSR (may hold idx < 0 / repeats) -> device queries,
        one async H2D through the pool's pinned stager"""
        from .._native import native
        lens, qi, qv, qn2 = native().csr_normalize(rp, idx, val)
        qptr = np.zeros(lens.size + 1, dtype=np.int64)
        np.cumsum(lens, out=qptr[1:])
        if qi.size == 0:
            qi, qv = np.zeros(1, np.int32), np.zeros(1, np.float32)
        dq = self.pool.stager().put(qptr, qi, qv, np.asarray(qn2, np.float64))
        return (*dq, int(qptr[-1]))

    def _scan(self, q, nq: int, nrows: int):
        import torch
        from ..ops import hip
        out = torch.empty(nq * nrows, dtype=torch.float32, device=self.device)
        metric = 1 if self.euclid else 0
        if q[0] == "slots":
            if q[2] > hip.POOL_MAX_Q_ENTRIES:
                raise ValueError("query batch has more than 4096 features")
            hip.pool_scan(None, None, None, None, nq, self.pool, nrows, metric, out,
                          qslots=q[1], qtotal=q[2])
            return out
        qptr, qi, qv, qn2, total = q
        if total > hip.POOL_MAX_Q_ENTRIES:
            raise ValueError("query batch has more than 4096 features")
        hip.pool_scan(qptr, qi, qv, qn2, nq, self.pool, nrows, metric, out, qtotal=total)
        return out

    def _query_batches(self, make, n: int, nrows: int, k: int, similar: bool):
        from ..ops import hip
        res = []
        for b0 in range(0, n, hip.POOL_MAX_Q):
            b1 = min(n, b0 + hip.POOL_MAX_Q)
            q = make(b0, b1)
            if q[-1] > hip.POOL_MAX_Q_ENTRIES and b1 - b0 > 1:     # one query at a time
                for j in range(b0, b1):
                    res += self._topk(self._scan(make(j, j + 1), 1, nrows), 1, nrows, k, similar)
                continue
            res += self._topk(self._scan(q, b1 - b0, nrows), b1 - b0, nrows, k, similar)
        return res

    def _topk(self, sc, nq: int, nrows: int, k: int, similar: bool):
        from ..ops import hip
        if k <= hip.TOPK_MAX_K and nq <= hip.QUERY_MAX:
            # latency path: result lands in pinned host memory
            d, i = hip.topk_scores_direct(sc, nq, nrows, k, not self.euclid, self._bufs())
            self.pool.stager().synced()
            out = _pairs(d, i)
            if similar:
                out = [[(j, float(-dd if self.euclid else 1.0 - dd)) for j, dd in r] for r in out]
            return out
        if k <= hip.TOPK_MAX_K:
            d, i = hip.topk_scores(sc, nq, nrows, k, flip=not self.euclid)
        else:       # wider than the fused top-k: torch.topk on the score matrix
            import torch
            m = sc.view(nq, nrows)
            dist = m if self.euclid else (1.0 - m).nan_to_num(posinf=math.inf)
            d, i = torch.topk(dist, min(k, nrows), dim=1, largest=False, sorted=True)
        d, i = self.pool.stager().fetch(d, i)
        out = _pairs(d, i)
        if similar:
            out = [[(j, float(-dd if self.euclid else 1.0 - dd)) for j, dd in r] for r in out]
        return out

    def scores_device(self, row, nrows: int):
        """device score vector (cosine similarity / euclidean distance)"""
        return self._scan(self._queries_device([row]), 1, nrows)

    def scores(self, row, nrows: int) -> np.ndarray:
        """similarity (cosine) or distance (euclid) of one query vs every slot"""
        if self.gpu:
            return self.scores_device(row, nrows).cpu().numpy() if nrows else \
                np.zeros(0, np.float32)
        qi, qv = self._norm_row(*row)
        q2 = float((qv.astype(np.float64) ** 2).sum())
        out = np.full(nrows, np.inf if self.euclid else -np.inf, dtype=np.float32)
        qd = dict(zip(qi.tolist(), qv.tolist()))
        for s, (i, v) in self.rows.items():
            if s >= nrows:
                continue
            dot = sum(float(x) * qd.get(int(k), 0.0) for k, x in zip(i, v))
            r2 = float((v.astype(np.float64) ** 2).sum())
            if self.euclid:
                out[s] = math.sqrt(max(0.0, q2 + r2 - 2 * dot))
            else:
                den = math.sqrt(q2) * math.sqrt(r2)
                out[s] = dot / den if den > 0 else 0.0
        return out

    def query(self, rows: list, nrows: int, k: int, similar: bool) -> list[list[tuple[int, float]]]:
        if self.gpu and nrows > 0 and k > 0:
            return self._query_batches(lambda a, b: self._queries_device(rows[a:b]), len(rows),
                                       nrows, k, similar)
        res = []
        for row in rows:
            s = self.scores(row, nrows)
            d = s if self.euclid else (1.0 - s)        # distance view
            d = np.where(np.isfinite(s), d, np.inf).astype(np.float32)
            (r,) = topk(d[None, :], k, None)
            if similar:
                r = [(i, float(-dd if self.euclid else 1.0 - dd)) for i, dd in r]
            res.append(r)
        return res

    def query_slots(self, slots, nrows: int, k: int, similar: bool) -> list[list[tuple[int, float]]]:
        """queries that are stored rows (similar_row_from_id, LOF neighbours
        of stored points): taken from the pool on the device"""
        slots = list(slots)
        if self.gpu:
            if nrows <= 0 or k <= 0:
                return [[] for _ in slots]
            from ..ops import hip
            if len(slots) <= hip.POOL_MAX_Q and k <= hip.TOPK_MAX_K:
                r = hip.pool_query_direct(self.pool, nrows, 1 if self.euclid else 0, k,
                                          self._bufs(), slots=np.asarray(slots, np.int32),
                                          nq=len(slots))
                if r is not None:
                    return self._direct_pairs(r, similar)
            return self._query_batches(lambda a, b: self.pool.query_slots_device(slots[a:b]),
                                       len(slots), nrows, k, similar)
        return self.query([self.rows.get(int(s), (np.zeros(0, np.int32), np.zeros(0, np.float32)))
                           for s in slots], nrows, k, similar)
