"""Linear online classifier driver (perceptron, PA, PA1, PA2, CW, AROW, NHERD).

Reference surface: jubatus/server/server/classifier_serv.cpp:91-225 (train,
classify, get_labels, set_label, delete_label, clear) on top of jubatus_core's
linear classifiers (EXTERNAL).

Model: hashed tables W[H][LC] (+ P[H][LC] = diagonal precision 1/S for
CW/AROW/NHERD, init 1.0; see linear_oracle.py) with
H = converter ``hash_max_size`` and LC = label capacity (power of two, grown
on demand). On a GPU the tables live in HBM and every update/score runs in
csrc/hip/linear.hip; without a GPU the NumPy oracle (linear_oracle.py) runs
the same semantics on the host.

Update semantics: a request's samples are applied in order (exact online
learning). Several requests submitted together (``train_requests``) run as
concurrent lock-free streams, like concurrent train RPCs on the reference's
giant-lock-free classifier (ChangeLog.rst:152).
"""
from __future__ import annotations

import collections
import os
import threading
import time
from typing import Any, Sequence

import msgpack
import numpy as np

from .._native import native
from ..fv_converter.converter import DatumToFvConverter
from ..fv_converter.datum import as_datum
from . import linear_oracle as lo

LINEAR_METHODS = ("perceptron", "PA", "PA1", "PA2", "CW", "AROW", "NHERD")
LABEL_CAPS = (8, 16, 32, 64, 128, 256, 512, 1024)


class ClassifierConfigError(ValueError):
    pass


def _pack_body(items: Sequence[Any]) -> bytes:
    return msgpack.packb(items, use_bin_type=False)


def dist_all_reduce(t, op: str, group):
    """async all-reduce helper for the MIX metadata (None when not distributed)"""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return None
    o = dist.ReduceOp.MAX if op == "max" else dist.ReduceOp.SUM
    return dist.all_reduce(t, op=o, group=group, async_op=True)


def _label_cap(n: int) -> int:
    for c in LABEL_CAPS:
        if c >= n:
            return c
    raise ClassifierConfigError(f"at most {LABEL_CAPS[-1]} labels are supported")


class LinearClassifier:
    def __init__(self, method: str, parameter: dict | None, converter: DatumToFvConverter,
                 device: Any = None, concurrent_update: str = "exact", weight_dtype: str = "fp32"):
        if method not in LINEAR_METHODS:
            raise ClassifierConfigError(f"unknown linear method: {method}")
        parameter = dict(parameter or {})
        self.method = method
        self.mid = lo.METHOD_IDS[method]
        if method != "perceptron" and method != "PA":
            if "regularization_weight" not in parameter:
                raise ClassifierConfigError("parameter.regularization_weight is required")
        self.C = float(parameter.get("regularization_weight", 1.0))
        if method not in ("perceptron", "PA") and not self.C > 0:
            raise ClassifierConfigError("regularization_weight must be positive")
        if concurrent_update not in ("exact", "atomic", "hogwild"):
            raise ClassifierConfigError("concurrent_update must be 'exact', 'atomic' or 'hogwild'")
        self.concurrent_update = concurrent_update
        if weight_dtype not in ("fp32", "bf16"):
            raise ClassifierConfigError("weight_dtype must be 'fp32' or 'bf16'")
        # storage of W on the GPU: fp32, or bf16 with stochastic rounding
        # (csrc/hip/jb_linear.hpp; P stays fp32, arithmetic is fp32). The host
        # path has no bf16 table and keeps fp32.
        self.weight_dtype = weight_dtype if device is not None else "fp32"
        self.conv = converter
        self.H = converter.hash_max_size
        self.use_s = self.mid in lo.USES_COVARIANCE
        self.labels = native().LabelTable()
        self._lock = threading.RLock()
        self.device = device
        self.gpu = device is not None
        self._devfv = False
        self.direct = True        # single-launch path for small classify requests
        # train batches scanned on the GPU (csrc/hip/scan.hip); their checks
        # complete asynchronously (_drain)
        self.gpu_scan = os.environ.get("JUBATUS_GPU_SCAN", "1") != "0"
        self._pending: collections.deque = collections.deque()
        self._served_prof = [0, 0] + [0.0] * 6   # train_arena_sync timing sums
        self._scan_stats = {"gpu": 0, "replayed": 0, "host": 0,  # train batches by scan path
                            "replay_failed": 0}
        self._replay_error = ""
        self._free_checks: list = []
        self._draining = False
        self._result_cols = None
        self.LC = 0
        self._label_version = -1
        self._host_stats = {"updated": 0, "trained": 0}
        # hot-row replica of the concurrent train kernel (csrc/hip/hot.hip,
        # linear.hip "Hot rows"; atomic / hogwild modes only): off unless
        # JUBATUS_HOT_ROWS=1 (it trades distance to the serial model for speed),
        # JUBATUS_HOT_MERGE sets the merge interval in samples
        self.hot_rows = os.environ.get("JUBATUS_HOT_ROWS", "0") == "1"
        self.hot_merge = max(1, int(os.environ.get("JUBATUS_HOT_MERGE", "1")))
        self.hot_min_streams = 16
        self.hot_min_count: int | None = None    # None: max(1024, samples / 128)
        if self.gpu:
            import torch
            from ..ops import hip
            from ..ops.feature_pipeline import FeaturePipeline
            self.torch = torch
            self.pipe = FeaturePipeline(converter, device)
            # datum -> features on the device: the fixed-slot fast path or the
            # wide rule-set kernels (ngram / idf / bm25 / combinations)
            self._devfv = self.pipe.fast or self.pipe.wide
            self._hots = [hip.HotRows(device), hip.HotRows(device)]
            self._serial = hip.SerialScratch(device)
            self._hot_turn = 0
            self._hot_count_buf = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self._hot_seen = None            # (pinned count, event) of a detection in flight
            self._hot_seen_ev = hip.DevEvent()
            self._hot_last = -1              # hot rows found by the last completed detection
            self._hot_batches = 0
            # [samples that updated, samples trained] (device counters)
            self._train_stats = torch.zeros(2, dtype=torch.int64, device=device)
            # rows written since the last MIX (sparse MIX, parallel/sparse_mix.py)
            self.touched = torch.zeros(self.H, dtype=torch.uint8, device=device)
        # False after a change the touched map does not describe (model load,
        # label re-layout): the next MIX is dense
        self._touched_valid = True
        self._last_mix: dict = {}
        self._mix_job = None      # TableMix of an overlapped MIX in flight
        self._alloc(LABEL_CAPS[0])

    # ------------------------------------------------------------ storage
    def _tables_replaced(self) -> None:
        """the W / P tensors (or their contents, on a load) change outside the
        train path: an overlapped MIX in flight must not fold its result into
        them (its snapshot describes the old tables), and the touched map no
        longer tells which rows differ across ranks, so the next MIX is dense"""
        job = self._mix_job
        if job is not None:
            job.abandon()
        self._touched_valid = False

    def _alloc(self, LC: int) -> None:
        H = self.H
        # a label re-layout copies every column over and zero-fills the new
        # ones on every rank alike: the touched map still names every row that
        # differs across ranks - unless an overlapped MIX was in flight (its
        # fold is abandoned, and the rows it had taken out of the map were not
        # reconciled), which makes the next MIX dense
        if self._mix_job is not None:
            self._tables_replaced()
        if self.gpu:
            t = self.torch
            W = t.zeros((H, LC), dtype=self._wdt(), device=self.device)
            P = t.ones((H, LC), dtype=t.float32, device=self.device) if self.use_s else None
            if self.LC:
                W[:, :self.LC].copy_(self.W)
                if P is not None:
                    P[:, :self.LC].copy_(self.P)
            self.W, self.P = W, P
            self.active = t.zeros(LC, dtype=t.int32, device=self.device)
        else:
            W = np.zeros((H, LC), dtype=np.float32)
            P = np.ones((H, LC), dtype=np.float32) if self.use_s else None
            if self.LC:
                W[:, :self.LC] = self.W
                if P is not None:
                    P[:, :self.LC] = self.P
            self.W, self.P = W, P
            self.active = np.zeros(LC, dtype=np.int32)
        self.LC = LC
        self._label_version = -1

    def _wdt(self):
        return self.torch.bfloat16 if self.weight_dtype == "bf16" else self.torch.float32

    def _sync_labels(self) -> None:
        """grow the tables and refresh the active-column mask after label changes"""
        v = self.labels.version()
        if v == self._label_version:
            return
        n = self.labels.size()
        if n > self.LC:
            self._alloc(_label_cap(n))
        alive = self.labels.alive()
        mask = np.zeros(self.LC, dtype=np.int32)
        mask[:len(alive)] = np.asarray(alive, dtype=np.int32)
        if self.gpu:
            self.active.copy_(self.torch.from_numpy(mask))
        else:
            self.active[:] = mask
        self._label_version = v

    # -------------------------------------------------------------- train
    def _mode(self, nstreams: int) -> int:
        """exact (default): several streams give the result of applying them
        one after the other (csrc/hip/serial.hip); atomic / hogwild: lock-free
        concurrent streams"""
        from ..ops import hip
        if nstreams <= 1:
            return hip.UPDATE_EXACT
        return hip.UPDATE_MODES[self.concurrent_update]

    def _train_batch(self, b) -> int:
        self._sync_labels()
        if b.n:
            self._launch_train(b)
        return b.n

    def _hot_wanted(self, nstreams: int) -> bool:
        """detect hot rows for a batch of ``nstreams`` streams? While the last
        detection found none, only every 8th batch looks (and trains with the
        plain 4-stream-block launch)."""
        from ..ops import hip
        if not (self.gpu and self.hot_rows and self.weight_dtype == "fp32"
                and self.LC <= 64 and nstreams >= self.hot_min_streams
                and self._mode(nstreams) in (hip.UPDATE_ATOMIC, hip.UPDATE_HOGWILD)):
            return False
        self._hot_batches += 1
        seen = self._hot_seen
        if seen is not None and seen[1].query():
            self._hot_last = int(seen[0][0])
            self._hot_seen = None
        return self._hot_last != 0 or self._hot_batches % 8 == 0

    def _detect_hot(self, b) -> None:
        """enqueue hot-row detection of batch ``b`` on the current stream into
        the next of two alternating sets (a set is reused once the train
        launch that read it has run: a device-side wait)"""
        from ..ops import hip
        hs = self._hots[self._hot_turn]
        self._hot_turn ^= 1
        if hs.free_used:
            hs.free.wait_on()
        min_count = self.hot_min_count or max(1024, b.n // 128)
        hip.hot_detect(b.row_ptr, b.n, b.fidx, b.nnz, hs, min_count,
                       max_rows=hip.hot_max_rows(self.LC))
        if self._hot_seen is None:       # learn the count without a host sync
            self._hot_count_buf.copy_(hs.n, non_blocking=True)
            self._hot_seen_ev.record()
            self._hot_seen = (self._hot_count_buf, self._hot_seen_ev)
        b.hot = hs

    def _launch_train(self, b) -> None:
        """one train launch over a device batch (after its preparation, if it
        was prepared on another stream); concurrent batches use the hot-row
        replica when hot rows were detected (csrc/hip/hot.hip)"""
        from ..ops import hip
        if b.ready is not None:
            hip.stream_wait(b.ready)
        mode = self._mode(b.nstreams)
        if b.hot is None and b.ready is None and self._hot_wanted(b.nstreams):
            self._detect_hot(b)
        hs = b.hot
        hip.linear_train(b.row_ptr, b.fidx, b.fval, b.labels, b.stream_ptr, b.nstreams,
                         self.W, self.P, self.active, self.mid, self.C, mode=mode, hot=hs,
                         merge_every=self.hot_merge, stats=self._train_stats,
                         touched=self.touched, n_max=b.n, scratch=self._serial)
        if hs is not None:
            hs.free.record()
            hs.free_used = True

    def _submit_scan(self, arena, offs, lens, chk, counts=None) -> int | None:
        """One GPU-scan train batch in a single native call
        (csrc/hip/train_batch.hip: H2D, scan, hashing, hot-row detection,
        train). -> samples queued, or None when the host scanner must take
        the batch (nothing was launched)."""
        from ..ops import hip
        self._sync_labels()
        r = self.pipe.scan_batch_args(arena, offs, lens, self.labels, chk, counts)
        if r is None:
            return None
        a, _ = r
        R, n = int(a.R), int(a.n)
        if self.LC not in hip.LABEL_CAPS or (self.mid >= hip.METHODS["CW"] and self.P is None):
            raise ValueError("label capacity / covariance table not supported by the train kernel")
        a.W = self.W.data_ptr()
        a.w_bf16 = int(self.weight_dtype == "bf16")
        a.S = self.P.data_ptr() if self.P is not None else None
        a.active = self.active.data_ptr()
        a.LC = self.LC
        a.method = self.mid
        a.C = float(self.C)
        a.mode = self._mode(R)
        # exact with several streams runs as serial-equivalent (linear.hip),
        # which needs the scratch as much as an explicit serial mode does
        if a.mode == hip.UPDATE_SERIAL or (a.mode == hip.UPDATE_EXACT and R > 1):
            a.serial_scratch = self._serial.ptr(max(1, n), self.LC)
            a.serial_bytes = self._serial.nbytes
        a.merge_every = self.hot_merge
        a.hot_waves = hip.HOT_WAVES
        a.stats = self._train_stats.data_ptr()
        a.touched = self.touched.data_ptr() if self.touched is not None else None
        if n > 0 and self._hot_wanted(R):
            hs = self._hots[self._hot_turn]
            self._hot_turn ^= 1
            a.hot_rows = hs.rows.data_ptr()
            a.hot_n = hs.n.data_ptr()
            a.hot_rep = hs.rep.data_ptr()
            a.gkey = hs.gkey.data_ptr()
            a.gcnt = hs.gcnt.data_ptr()
            a.gcap = hs.CAP
            a.block_min = 8
            a.min_count = self.hot_min_count or max(1024, n // 128)
            a.max_rows = min(hip.hot_max_rows(self.LC), hs.rows.numel())
            a.hot_free = hs.free.h
            a.hot_free_valid = int(hs.free_used)
            hs.free_used = True
            if self._hot_seen is None:       # learn the count without a host sync
                a.hot_count_host = self._hot_count_buf.data_ptr()
                a.hot_seen = self._hot_seen_ev.h
                self._hot_seen = (self._hot_count_buf, self._hot_seen_ev)
        hip.train_batch_submit(a)
        return n

    def train_stats(self) -> dict[str, int]:
        """samples trained / samples that changed the model since creation"""
        if not self.gpu:
            return dict(self._host_stats)
        v = self._train_stats.cpu().tolist()
        return {"updated": int(v[0]), "trained": int(v[1])}

    def train_arena(self, arena, offs, lens) -> int:
        """Train on request bodies that already sit in a pinned RequestArena
        (zero-copy receive path; one stream per span).

        With the GPU scan the call returns once the batch is queued: the
        arena spans must stay unchanged until the next call into this model
        (which checks the batch; a batch the device scan could not take -
        new labels, binary values, malformed bytes - is then re-run through
        the host scanner, which adds labels / raises as before)."""
        with self._lock:
            if not self._devfv:
                bodies = [bytes(arena.np[o:o + n]) for o, n in zip(offs, lens)]
                return self.train_requests(bodies)
            if self.gpu_scan and self.pipe.fast and self.labels.size() > 0:
                self._drain(block=True, keep=3)
                self._sync_labels()
                chk = self._check_record(self.labels.size())
                offs = np.ascontiguousarray(offs, dtype=np.int64)
                lens = np.ascontiguousarray(lens, dtype=np.int64)
                n = self._submit_scan(arena, offs, lens, chk)
                if n is not None:
                    self._scan_stats["gpu"] += 1
                    chk.replay = lambda: self._train_batch(
                        self.pipe.from_arena(arena, offs, lens, True, self.labels))
                    self._pending.append(chk)
                    return n
                self._free_checks.append(chk)
            self._drain(block=True)
            self._scan_stats["host"] += 1
            return self._train_batch(self.pipe.from_arena(arena, offs, lens, True, self.labels))

    def train_arena_sync(self, arena, offs, lens) -> tuple[np.ndarray, dict]:
        """Served train batch (the RPC transport copied the request bodies
        into a pinned arena slot, csrc/native/jb_rpc.cpp arena batching):
        GPU scan -> fv_hash -> train, then wait (lock released) until the
        batch's scan check is known, so each request gets its own reply.
        -> (samples per request, or -1 = ARGUMENT_ERROR; {} reserved for
        error messages). A batch the device scan rejected is re-run one
        request at a time through the host scanner (which validates before
        it changes the label table), so only the bad requests fail."""
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        lens = np.ascontiguousarray(lens, dtype=np.int64)
        R = int(offs.size)
        res = np.full(R, -1, dtype=np.int64)
        from ..ops.feature_pipeline import body_counts
        prof = self._served_prof
        t0 = time.perf_counter()
        with self._lock:
            t1 = time.perf_counter()
            counts = body_counts(arena.np, offs, lens)
            chk = b = None
            if (self.gpu and self.pipe.fast and self.gpu_scan and counts is not None
                    and self.labels.size() > 0):
                self._drain(block=True, keep=3)
                self._sync_labels()
                chk = self._check_record(self.labels.size())
                ta = time.perf_counter()
                if self._submit_scan(arena, offs, lens, chk, counts) is not None:
                    self._scan_stats["gpu"] += 1
                    prof[6] += ta - t1
                    prof[7] += time.perf_counter() - ta
                else:
                    self._free_checks.append(chk)
                    chk = None
        if chk is not None:
            t2 = time.perf_counter()
            chk.wait()                       # releases the GIL: other RPCs proceed
            t3 = time.perf_counter()
            with self._lock:
                if int(chk.err[0]) == 0:
                    h = chk.hist[:chk.nhist]
                    for lid in np.flatnonzero(h).tolist():
                        self.labels.add_count(lid, int(h[lid]))
                    self._free_checks.append(chk)
                    res[:] = counts
                    # batches, requests, lock wait, submit, scan wait, finish (seconds)
                    t4 = time.perf_counter()
                    prof[0] += 1
                    prof[1] += R
                    prof[2] += t1 - t0
                    prof[3] += t2 - t1
                    prof[4] += t3 - t2
                    prof[5] += t4 - t3
                    return res, {}
                self._free_checks.append(chk)
                self._scan_stats["replayed"] += 1
        # host path, one request at a time (bad requests fail alone)
        with self._lock:
            self._scan_stats["host"] += 1
            for k in range(R):
                body = bytes(arena.np[offs[k]:offs[k] + lens[k]])
                try:
                    res[k] = self.train_requests([body])
                except (TypeError, ValueError):
                    res[k] = -1
        return res, {}

    def _check_record(self, nhist: int):
        """a free completion record; allocated in a batch (fine-grained host
        memory is slow to allocate and synchronises the device)"""
        from ..ops.feature_pipeline import ScanCheck
        while True:
            while self._free_checks:
                c = self._free_checks.pop()
                if c.hist.size >= nhist:
                    return c
            self._free_checks = [ScanCheck(max(64, nhist * 2)) for _ in range(8)]

    def _drain(self, block: bool = True, keep: int = 0) -> None:
        """process GPU-scan checks in order: label counts of accepted batches,
        host re-run of rejected ones. block: wait until at most ``keep``
        batches are outstanding (completed ones are always processed)."""
        if self._draining:
            return
        self._draining = True
        try:
            while self._pending:
                c = self._pending[0]
                if not c.done() and not (block and len(self._pending) > keep):
                    break
                c.wait()
                self._pending.popleft()
                replay, c.replay = c.replay, None
                try:
                    if int(c.err[0]):
                        self._scan_stats["replayed"] += 1
                        try:
                            replay()
                        except (TypeError, ValueError, RuntimeError) as e:
                            # the batch was acknowledged when it was queued: its
                            # failure is recorded here (status train_scan.replay_failed
                            # / last_replay_error), not raised into whichever call
                            # happens to drain it
                            self._scan_stats["replay_failed"] += 1
                            self._replay_error = f"{type(e).__name__}: {e}"
                    else:
                        h = c.hist[:c.nhist]
                        for lid in np.flatnonzero(h).tolist():
                            self.labels.add_count(lid, int(h[lid]))
                finally:
                    self._free_checks.append(c)
        finally:
            self._draining = False

    def train_requests(self, bodies: Sequence[Any]) -> int:
        """Train on raw msgpack ``list<labeled_datum>`` bodies (one stream each)."""
        with self._lock:
            self._drain()
            if self._devfv:
                return self._train_batch(self.pipe.from_requests(list(bodies), True, self.labels))
            total = 0
            streams = [msgpack.unpackb(bytes(x), raw=False) for x in bodies]
            rows, labs, sizes = [], [], []
            for items in streams:
                for lab, d in items:
                    idx, val = self.conv.hashed(self.conv.convert_and_update_weight(as_datum(d)))
                    rows.append((idx, val))
                    labs.append(self.labels.get_or_add(_s(lab)))
                    self.labels.add_count(labs[-1], 1)
                sizes.append(len(items))
                total += len(items)
            self._train_rows(rows, labs, sizes)
            return total

    def train(self, data: Sequence[tuple[str, Any]]) -> int:
        data = list(data)
        if not data:
            return 0
        if self._devfv:
            body = _pack_body([[lab, as_datum(d).to_msgpack()] for lab, d in data])
            return self.train_requests([body])
        with self._lock:
            self._drain()
            rows, labs = [], []
            for lab, d in data:
                rows.append(self.conv.hashed(self.conv.convert_and_update_weight(as_datum(d))))
                labs.append(self.labels.get_or_add(_s(lab)))
                self.labels.add_count(labs[-1], 1)
            self._train_rows(rows, labs, [len(rows)])
        return len(data)

    def _train_rows(self, rows, labs, sizes) -> None:
        self._sync_labels()
        if self.gpu:
            self._launch_train(self.pipe.from_rows(rows, labs, sizes))
            return
        for (idx, val), y in zip(rows, labs):
            up = lo.train_one(self.W, self.P, np.asarray(idx, np.int64), np.asarray(val, np.float32),
                              y, self.active, self.mid, self.C)
            self._host_stats["trained"] += 1
            self._host_stats["updated"] += int(up)

    # ----------------------------------------------------------- classify
    def _results(self, scores: np.ndarray) -> list[list[tuple[str, float]]]:
        v = self.labels.version()
        cache = self._result_cols
        if cache is None or cache[0] != v:
            names = self.labels.names()
            alive = self.labels.alive()
            cols = [i for i, a in enumerate(alive) if a]
            cache = self._result_cols = (v, cols, [names[c] for c in cols])
        _, cols, names = cache
        sub = scores[:, cols].tolist()
        return [list(zip(names, row)) for row in sub]

    def classify_requests(self, bodies: Sequence[Any]) -> list[list[tuple[str, float]]]:
        with self._lock:
            self._drain()
            if self._devfv:
                from ..ops import hip
                self._sync_labels()
                scores = self.pipe.classify_direct(list(bodies), self.W) \
                    if self.direct and self.pipe.fast else None
                if scores is not None:
                    return self._results(scores)
                b = self.pipe.from_requests(list(bodies), False, None)
                self._sync_labels()
                if b.n == 0:
                    return []
                out = self.pipe._dev.get("scores", b.n * self.LC, self.torch.float32)
                hip.linear_classify(b.row_ptr, b.fidx, b.fval, b.n, self.W, out)
                scores = out[:b.n * self.LC].view(b.n, self.LC).cpu().numpy()
                return self._results(scores)
        ds = [d for x in bodies for d in msgpack.unpackb(bytes(x), raw=False)]
        return self.classify(ds)

    def classify(self, data: Sequence[Any]) -> list[list[tuple[str, float]]]:
        data = list(data)
        if not data:
            return []
        if self._devfv:
            return self.classify_requests([_pack_body([as_datum(d).to_msgpack() for d in data])])
        rows = [self.conv.hashed(self.conv.convert(as_datum(d))) for d in data]
        with self._lock:
            self._drain()
            self._sync_labels()
            if self.gpu:
                from ..ops import hip
                b = self.pipe.from_rows(rows, None)
                out = self.torch.empty(b.n * self.LC, dtype=self.torch.float32, device=self.device)
                hip.linear_classify(b.row_ptr, b.fidx, b.fval, b.n, self.W, out)
                scores = out.view(b.n, self.LC).cpu().numpy()
            else:
                scores = np.stack([lo.scores(self.W, np.asarray(i, np.int64),
                                             np.asarray(v, np.float32)) for i, v in rows])
        return self._results(scores)

    # ------------------------------------------------------------- labels
    def get_labels(self) -> dict[str, int]:
        with self._lock:
            self._drain()
        names = self.labels.names()
        alive = self.labels.alive()
        return {n: int(self.labels.count(i)) for i, n in enumerate(names) if alive[i]}

    def set_label(self, label: str) -> bool:
        with self._lock:
            self._drain()
            if self.labels.lookup(label) >= 0:
                return False
            self.labels.get_or_add(label)
            self._sync_labels()
            return True

    def delete_label(self, label: str) -> bool:
        with self._lock:
            self._drain()
            i = self.labels.lookup(label)
            if i < 0:
                return False
            self.labels.remove(label)
            self._tables_replaced()
            self.W[:, i] = 0.0
            if self.P is not None:
                self.P[:, i] = 1.0
            self._sync_labels()
            return True

    def clear(self) -> None:
        with self._lock:
            self._drain()
            self.labels.clear()
            self.LC = 0
            self._alloc(LABEL_CAPS[0])
            self.conv.weights.clear()

    # ------------------------------------------------------------ persist
    def synchronize(self) -> None:
        with self._lock:
            self._drain()
        if self.gpu:
            self.torch.cuda.synchronize(self.device)

    def _host_tables(self) -> tuple[np.ndarray, np.ndarray | None]:
        if self.gpu:
            W = self.W.float().cpu().numpy()
            S = self.P.cpu().numpy() if self.P is not None else None
            return W, S
        return self.W, self.P

    def pack(self) -> dict:
        """Model payload (user_data of the model file).

        Sparse: only feature rows that differ from the initial state are
        stored, as (row indices, W rows, P rows) over the live label columns
        (P = diagonal precision of CW/AROW/NHERD).
        """
        with self._lock:
            self._drain()
            self.synchronize()
            W, S = self._host_tables()
            names = self.labels.names()
            alive = self.labels.alive()
            cols = [i for i, a in enumerate(alive) if a]
            Wc = W[:, cols]
            touched = np.any(Wc != 0.0, axis=1)
            if S is not None:
                Sc = S[:, cols]
                touched |= np.any(Sc != 1.0, axis=1)
            rows = np.nonzero(touched)[0].astype(np.int64)
            out = {
                "method": self.method, "H": self.H,
                "labels": [names[c] for c in cols],
                "counts": [int(self.labels.count(c)) for c in cols],
                "rows": rows.tobytes(),
                "W": np.ascontiguousarray(Wc[rows]).astype(np.float32).tobytes(),
                "P": (np.ascontiguousarray(S[:, cols][rows]).astype(np.float32).tobytes()
                      if S is not None else b""),
                "weights": self.conv.weights.pack(),
            }
            return out

    def unpack(self, obj: dict) -> None:
        obj = {(k.decode() if isinstance(k, bytes) else k): v for k, v in obj.items()}
        with self._lock:
            self._drain()
            if int(obj["H"]) != self.H:
                raise ValueError("model hash_max_size differs from the configuration")
            labels = [(x.decode() if isinstance(x, bytes) else x) for x in obj["labels"]]
            self.labels.clear()
            self.LC = 0
            self._alloc(_label_cap(max(1, len(labels))))
            for i, (name, cnt) in enumerate(zip(labels, obj["counts"])):
                self.labels.get_or_add(name)
                self.labels.set_count(i, int(cnt))
            self._sync_labels()
            self._tables_replaced()
            rows = np.frombuffer(obj["rows"], dtype=np.int64)
            L = len(labels)
            Wr = np.frombuffer(obj["W"], dtype=np.float32).reshape(len(rows), L)
            W = np.zeros((self.H, self.LC), dtype=np.float32)
            W[rows, :L] = Wr
            P = None
            if self.use_s:
                P = np.ones((self.H, self.LC), dtype=np.float32)
                if len(obj["P"]):
                    P[rows, :L] = np.frombuffer(obj["P"], dtype=np.float32).reshape(len(rows), L)
            if self.gpu:
                self.W.copy_(self.torch.from_numpy(W))
                if P is not None:
                    self.P.copy_(self.torch.from_numpy(P))
            else:
                self.W, self.P = W, P
            if obj.get("weights"):
                self.conv.weights.unpack(obj["weights"])
            self._touched_valid = False

    # ----------------------------------------------------------------- MIX
    def _live_labels(self) -> list[str]:
        names, alive = self.labels.names(), self.labels.alive()
        return [n for n, a in zip(names, alive) if a]

    def _reorder_labels(self, order: list[str]) -> None:
        """Re-lay the label columns in ``order`` (labels missing locally get
        fresh columns)."""
        old = {n: i for i, n in enumerate(self.labels.names()) if self.labels.lookup(n) == i}
        counts = {n: int(self.labels.count(i)) for n, i in old.items()}
        LC = _label_cap(max(1, len(order)))
        if self.gpu:
            t = self.torch
            perm = t.tensor([old.get(n, -1) for n in order], dtype=t.int64, device=self.device)
            have = perm >= 0
            W = t.zeros((self.H, LC), dtype=self._wdt(), device=self.device)
            P = t.ones((self.H, LC), dtype=t.float32, device=self.device) if self.use_s else None
            src = perm.clamp(min=0)
            W[:, :len(order)] = t.where(have, self.W.index_select(1, src), W[:, :len(order)])
            if P is not None:
                P[:, :len(order)] = t.where(have, self.P.index_select(1, src), P[:, :len(order)])
        else:
            W = np.zeros((self.H, LC), dtype=np.float32)
            P = np.ones((self.H, LC), dtype=np.float32) if self.use_s else None
            for c, n in enumerate(order):
                if n in old:
                    W[:, c] = self.W[:, old[n]]
                    if P is not None:
                        P[:, c] = self.P[:, old[n]]
        self.labels.clear()
        for c, n in enumerate(order):
            self.labels.get_or_add(n)
            self.labels.set_count(c, counts.get(n, 0))
        self._tables_replaced()
        self.W, self.P, self.LC = W, P, LC
        self.active = (self.torch.zeros(LC, dtype=self.torch.int32, device=self.device)
                       if self.gpu else np.zeros(LC, dtype=np.int32))
        self._label_version = -1
        self._sync_labels()

    def mix(self, group=None) -> int:
        """Collective model averaging across the ranks of ``group`` (RCCL):
        label layout agreement, then a sparse (touched rows) or chunked
        dense all-reduce mean (parallel/table_mix.py). Returns the bytes
        all-reduced per rank."""
        from ..parallel import collective as coll
        with self._lock:
            self._drain()
            names = self.labels.names()
            alive = self.labels.alive()
            fp = coll.fingerprint([n + ("+" if a else "-") for n, a in zip(names, alive)])
            if not coll.all_equal(fp, self.device if self.gpu else None, group):
                lists = coll.all_gather_object(self._live_labels(), group)
                order: list[str] = []
                seen = set()
                for lst in lists:
                    for n in lst:
                        if n not in seen:
                            seen.add(n)
                            order.append(n)
                self._reorder_labels(order)
            job = self._table_mix(group)
            nbytes = job.end()
            self._last_mix = job.stats()
            self._mix_counts(group)
            nbytes += self._mix_weights(group)
            return nbytes

    def _mix_weights(self, group=None) -> int:
        """document-frequency diffs of idf / bm25 converters (the reference
        mixes the weight manager with the model, linear_mixer get_diff):
        sparse (index, count) records over the collective"""
        if not self.conv.uses_global_weight:
            return 0
        from ..fv_converter.converter import WeightManager
        from ..parallel import wire
        wm = self.conv.weights
        mine = wm.get_diff()
        diffs = wire.all_gather(mine, group)
        mixed = diffs[0]
        for d in diffs[1:]:
            mixed = WeightManager.mix(mixed, d)
        wm.put_diff(mixed)
        return len(wire.encode(mine))

    def _table_mix(self, group):
        from ..parallel.table_mix import TableMix
        touched = self.touched if (self.gpu and self._touched_valid) else None
        job = TableMix(self._tables(), touched, group).begin()
        if self.gpu:
            self._touched_valid = True        # the map is exact again from here on
        return job

    # ------------------------------------------------ overlapped MIX
    def mix_begin(self, group=None, meta_group=None, agreed_version: int | None = None) -> dict:
        """Start an overlapped MIX: snapshot the touched rows (or the first
        chunks of a dense MIX) and start their SUM all-reduce on the
        communicator stream, then return; training continues meanwhile.
        ``mix_ready`` advances it, ``mix_end`` folds the cluster mean in with
        T += mean(snapshot) - snapshot, so updates made during the collective
        are kept. Label agreement and count deltas ride on ``meta_group`` (a
        host/gloo group: no GPU synchronisation). If the label layouts
        disagree the synchronous ``mix`` runs instead (it re-lays the label
        columns first). ``agreed_version``: the caller knows every rank still
        has the label layout agreed at this label-table version; if the
        table is still at it, the host collective comparing layouts is
        skipped."""
        import torch
        from ..parallel import collective as coll
        with self._lock:
            self._drain(block=False)   # batches still in flight join the next MIX
            names = self.labels.names()
            alive = self.labels.alive()
            fp = coll.fingerprint([n + ("+" if a else "-") for n, a in zip(names, alive)])
            cur = np.array([self.labels.count(i) for i in range(len(names))], dtype=np.int64)
            base = getattr(self, "_count_base", {})
            b = np.array([base.get(n, 0) for n in names], dtype=np.int64)
            mg = meta_group if meta_group is not None else group
            on_dev = self.gpu and coll.is_dist() and coll.backend(mg) == "nccl"
            mdev = self.device if on_dev else "cpu"
            # the label-layout check is blocking (a host collective on the
            # meta group); everything after it is asynchronous
            agreed = agreed_version is not None and self.labels.version() == agreed_version
            if not agreed and not coll.all_equal(fp, mdev if on_dev else torch.device("cpu"), mg):
                return {"sync": self.mix(group)}
            meta_cnt = torch.from_numpy(cur - b).to(mdev)
            works = [dist_all_reduce(meta_cnt, "sum", mg)]
            job = self._table_mix(group)
            self._mix_job = job
            return {"group": group, "names": names, "cur": cur, "base": b,
                    "meta": works, "meta_cnt": meta_cnt, "job": job}

    @staticmethod
    def mix_ready(h: dict | None) -> bool:
        """True when an overlapped MIX's collectives have finished
        (non-blocking; advances a chunked dense MIX)"""
        if h is None or "sync" in h:
            return True
        return h["job"].ready() and all(w is None or w.is_completed() for w in h["meta"])

    def mix_end(self, h: dict) -> int:
        """Finish a ``mix_begin``; returns the bytes all-reduced per rank."""
        if "sync" in h:
            return h["sync"]
        for w in h["meta"]:
            if w is not None:
                w.wait()
        with self._lock:
            self._drain(block=False)   # batches still in flight join the next MIX
            job = h["job"]
            nbytes = job.end()         # (no fold if the tables were replaced meanwhile)
            if self._mix_job is job:
                self._mix_job = None
            self._last_mix = job.stats()
            names, cur, b = h["names"], h["cur"], h["base"]
            new_base = b + h["meta_cnt"].cpu().numpy()
            # keyed by label name: a clear / load / re-layout between begin and
            # end moves or removes columns; labels that are gone are skipped
            base = {}
            for i, nm in enumerate(names):
                j = self.labels.lookup(nm)
                if j < 0:
                    continue
                since = int(self.labels.count(j)) - int(cur[i])
                self.labels.set_count(j, int(max(0, new_base[i] + since)))
                base[nm] = int(max(0, new_base[i]))
            self._count_base = base
            return nbytes + self._mix_weights(h.get("group"))

    def _tables(self) -> list:
        """the mixable tensors (torch views of the host arrays on the CPU backend)"""
        tables = [self.W] + ([self.P] if self.P is not None else [])
        if self.gpu:
            return tables
        import torch
        return [torch.from_numpy(t) for t in tables]

    def _mix_counts(self, group=None) -> None:
        """label counts: base + cluster-wide sum of the per-rank deltas since
        the last MIX (the local_mixture semantics of get_labels)."""
        import torch
        from ..parallel import collective as coll
        names = self.labels.names()
        base = getattr(self, "_count_base", {})
        cur = np.array([self.labels.count(i) for i in range(len(names))], dtype=np.int64)
        b = np.array([base.get(n, 0) for n in names], dtype=np.int64)
        delta = torch.from_numpy(cur - b)
        if self.gpu and coll.is_dist() and coll.backend(group) == "nccl":
            d = delta.to(self.device)
            coll.allreduce_sum_([d], group)
            delta = d.cpu()
        else:
            coll.allreduce_sum_([delta], group)
        new = b + delta.numpy()
        for i, n in enumerate(names):
            self.labels.set_count(i, int(max(0, new[i])))
        self._count_base = {n: int(max(0, new[i])) for i, n in enumerate(names)}

    def broadcast_from(self, src: int, apply: bool = True) -> None:
        """hand the whole model to newly joined members (obsolete protocol);
        apply=False: an up-to-date member takes part in the collectives
        without replacing its model"""
        import torch
        import torch.distributed as dist
        with self._lock:
            self._drain()
            names = self.labels.names()
            meta = [[names, [int(self.labels.count(i)) for i in range(len(names))],
                     self.labels.alive()]]
            from ..parallel import wire
            names, counts, alive = wire.broadcast(meta[0], src)
            me = dist.get_rank()
            if me != src and apply:
                self.labels.clear()
                self.LC = 0
                self._alloc(_label_cap(max(1, len(names))))
                for i, (n, c) in enumerate(zip(names, counts)):
                    self.labels.get_or_add(n)
                    self.labels.set_count(i, int(c))
                for n, a in zip(names, alive):
                    if not a:
                        self.labels.remove(n)
                self._sync_labels()
            if me != src and not apply:
                LC = _label_cap(max(1, len(names)))
                dts = [self._wdt() if self.gpu else torch.float32] + ([torch.float32] if self.use_s else [])
                dev = self.device if self.gpu else "cpu"
                for dt in dts:
                    dist.broadcast(torch.empty((self.H, LC), dtype=dt, device=dev), src=src)
                return
            self._tables_replaced()
            for t in self._tables():
                dist.broadcast(t, src=src)
            self._count_base = {n: int(c) for n, c in zip(names, counts)}

    def pair_mix(self, peer: int) -> None:
        """push_mixer exchange with one peer: agree on the label layout, then
        swap the tables point-to-point and keep the pairwise mean."""
        import torch
        import torch.distributed as dist
        with self._lock:
            self._drain()
            from ..parallel import wire
            me = dist.get_rank()
            mine = self._live_labels()
            theirs = wire.exchange(mine, peer)
            lists = [mine, theirs] if me < peer else [theirs, mine]
            order: list[str] = []
            for lst in lists:
                for n in lst:
                    if n not in order:
                        order.append(n)
            if order != self.labels.names() or not all(self.labels.alive()):
                self._reorder_labels(order)
            self._tables_replaced()
            for t in self._tables():
                buf = torch.empty_like(t)
                ops = [dist.P2POp(dist.isend, t, peer), dist.P2POp(dist.irecv, buf, peer)]
                for r in dist.batch_isend_irecv(ops):
                    r.wait()
                if t.dtype == torch.float32:
                    t.add_(buf).mul_(0.5)
                else:                      # bf16 W: the mean in fp32, one rounding
                    t.copy_(t.float().add_(buf.float()).mul_(0.5))

    def get_status(self) -> dict[str, str]:
        st = {"num_classes": str(len(self.get_labels())), "num_features": str(self.H),
              "label_capacity": str(self.LC), "method": self.method,
              "storage": "hbm" if self.gpu else "host", "weight_dtype": self.weight_dtype,
              "fv_path": ("gpu" if self.pipe.fast else "gpu-wide") if self._devfv else "host"}
        if self.gpu:
            for k, v in self._scan_stats.items():
                st[f"train_scan.{k}"] = str(v)
            if self._replay_error:
                st["train_scan.last_replay_error"] = self._replay_error
        for k, v in self._last_mix.items():
            st[f"mix.last_{k}"] = str(v)
        for k, v in self.train_stats().items():
            st[f"train.samples_{k}"] = str(v)
        st["train.update_mode"] = self.concurrent_update
        return st


def _s(x: Any) -> str:
    return x.decode() if isinstance(x, (bytes, bytearray)) else str(x)
