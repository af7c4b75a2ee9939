"""Host -> HBM feature pipeline.

Turns train/classify request bodies into device CSR batches:

* fast path (config eligible, see fv_converter/gpu_path.py): the native
  scanner validates the msgpack bodies, resolves labels and copies the raw
  bytes into a pinned staging buffer (multi-threaded over requests); one
  async H2D copy moves bytes + descriptors; ``fv_hash`` parses and hashes on
  the GPU into CSR (row_ptr, idx, val).
* host path (any other config): the host converter produces feature names,
  which are hashed on the host and shipped as CSR.

Pinned staging sets and device input sets are double-buffered and the H2D
copies run on a dedicated copy stream: the host scan of batch k+1 and its
DMA overlap the kernels of batch k. Events order everything:
  copy(k)      waits for the compute work that last read device set k%2
               (the train of batch k-2), recorded when batch k-1 was launched
  fv_hash(k)   waits for copy(k)
  host reuse of pinned set k%2 waits for copy(k).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass

import numpy as np
import torch

from .._native import native
from ..fv_converter.gpu_path import GpuRuleTable, fast_eligible, wide_eligible
from ..utils import trace
from . import hip


def _grow(cap: int, need: int) -> int:
    c = max(cap, 1)
    while c < need:
        c *= 2
    return c


def scan_threads() -> int:
    """host scanner threads for this process: the CPUs it may run on, shared
    by the ranks of this node (one process per GPU), at most 16"""
    try:
        ncpu = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        ncpu = os.cpu_count() or 4
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    from ..utils.numa import binding
    b = binding()
    if b.get("before"):       # bound to the GPU's node: shared by that node's ranks only
        local = max(1, -(-local * b["cpus"] // b["before"]))
    return max(1, min(16, ncpu // local))


def fnv1a64(b: bytes) -> int:
    h = 0xCBF29CE484222325
    for x in b:
        h = ((h ^ x) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def label_table_arrays(names: list, alive: list) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """the device label table of csrc/hip/scan.hip: open addressing on
    FNV-1a 64 of the label bytes; meta = [blob offset, length, id] (id -1:
    empty). Only live labels are entered (a deleted one goes to the host
    path, which revives it)."""
    live = [(i, n.encode("utf-8", "surrogateescape")) for i, (n, a) in enumerate(zip(names, alive))
            if a]
    cap = 16
    while cap < 2 * len(live):
        cap *= 2
    th = np.zeros(cap, np.uint64)
    tm = np.full(3 * cap, -1, np.int32)
    blob = bytearray()
    mask = cap - 1
    for lid, b in live:
        h = fnv1a64(b)
        j = h & mask
        while tm[3 * j + 2] >= 0:
            j = (j + 1) & mask
        th[j] = h
        tm[3 * j:3 * j + 3] = (len(blob), len(b), lid)
        blob += b
    return th.view(np.int64), tm, np.frombuffer(bytes(blob) or b"\0", np.uint8).copy()


def body_counts(buf: np.ndarray, offs: np.ndarray, lens: np.ndarray) -> np.ndarray | None:
    """element count of each body's top-level array header, None if any
    body does not start with one (the host scanner reports those)"""
    if offs.size == 0:
        return np.zeros(0, np.int64)
    if (lens < 1).any():
        return None
    t = buf[offs].astype(np.int64)
    n = np.full(offs.size, -1, np.int64)
    fix = (t & 0xF0) == 0x90
    n[fix] = t[fix] & 0x0F
    m16 = (t == 0xDC) & (lens >= 3)
    if m16.any():
        o = offs[m16]
        n[m16] = (buf[o + 1].astype(np.int64) << 8) | buf[o + 2]
    m32 = (t == 0xDD) & (lens >= 5)
    if m32.any():
        o = offs[m32]
        n[m32] = ((buf[o + 1].astype(np.int64) << 24) | (buf[o + 2].astype(np.int64) << 16)
                  | (buf[o + 3].astype(np.int64) << 8) | buf[o + 4])
    return None if (n < 0).any() else n


SCAN_LDS_BYTES = 27 * 1024      # csrc/hip/scan.hip kScanBytes
SCAN_MAX_SAMPLES = 768          # csrc/hip/scan.hip kMaxSamples


def scan_too_big(offs: np.ndarray, lens: np.ndarray, counts: np.ndarray) -> bool:
    """any request the GPU scan would reject for size (its 16-B aligned
    window exceeds the LDS stage, or too many samples)"""
    if offs.size == 0:
        return False
    return bool(((lens + (offs & 15)) > SCAN_LDS_BYTES).any() or (counts > SCAN_MAX_SAMPLES).any())


class ScanCheck:
    """completion record of a GPU-scanned train batch: the batch's error
    bits and label counts land in pinned memory when ``event`` completes"""

    def __init__(self, nhist: int):
        nh = max(1, nhist)
        self.buf = hip.HostBuffer(4 * (1 + nh))   # written by the fixup kernel
        self.err = self.buf.view(np.int32, 1)
        self.hist = self.buf.view(np.int32, nh, 4)
        self.event: hip.DevEvent | None = None
        self.replay = None        # re-runs the batch through the host scanner
        self.nhist = 0
        self._ev: hip.DevEvent | None = None     # this record's scan-complete event

    def scan_event(self) -> "hip.DevEvent":
        if self._ev is None:
            self._ev = hip.DevEvent()
        return self._ev

    def done(self) -> bool:
        return self.event is None or self.event.query()

    def wait(self) -> None:
        if self.event is not None:
            self.event.synchronize()


@dataclass
class DeviceBatch:
    n: int
    nnz: int
    nstreams: int
    row_ptr: torch.Tensor     # int64 [n+1]
    fidx: torch.Tensor        # int32 [nnz]
    fval: torch.Tensor        # float32 [nnz]
    labels: torch.Tensor | None   # int32 [n]
    stream_ptr: torch.Tensor  # int64 [nstreams+1]
    ready: object | None = None    # torch.cuda.Event / hip.DevEvent: prepared on the prep stream
    hot: object | None = None               # hot rows detected for this batch (classifier)


class _Pinned:
    def __init__(self):
        self.cap_bytes = 0
        self.cap_samples = 0
        self.cap_streams = 0
        self.staging = self.datum_off = self.labels = self.row_ptr = self.stream_ptr = None
        self.event: torch.cuda.Event | None = None

    def ensure(self, nbytes: int, nsamples: int, nstreams: int) -> None:
        if nbytes > self.cap_bytes:
            self.cap_bytes = _grow(self.cap_bytes or (1 << 16), nbytes)
            self.staging = torch.empty(self.cap_bytes, dtype=torch.uint8, pin_memory=True)
        if nsamples > self.cap_samples:
            self.cap_samples = _grow(self.cap_samples or 1024, nsamples)
            self.datum_off = torch.empty(self.cap_samples, dtype=torch.int64, pin_memory=True)
            self.datum_len = torch.empty(self.cap_samples, dtype=torch.int32, pin_memory=True)
            self.labels = torch.empty(self.cap_samples, dtype=torch.int32, pin_memory=True)
            self.row_ptr = torch.empty(self.cap_samples + 1, dtype=torch.int64, pin_memory=True)
        if nstreams + 1 > self.cap_streams:
            self.cap_streams = _grow(self.cap_streams or 64, nstreams + 1)
            self.stream_ptr = torch.empty(self.cap_streams, dtype=torch.int64, pin_memory=True)

    def wait(self) -> None:
        if self.event is not None:
            self.event.synchronize()
            self.event = None


class RequestArena:
    """Pinned receive arena: request bodies are written here once (by the
    RPC reader, or by the benchmark's synthetic client) and DMA'd to HBM
    straight from it - no host-side copy on the train path."""

    def __init__(self, capacity: int):
        import torch
        self.buf = torch.empty(max(16, capacity), dtype=torch.uint8,
                               pin_memory=torch.cuda.is_available())
        self.np = self.buf.numpy()
        self.used = 0
        self.offs: list[int] = []
        self.lens: list[int] = []

    def append(self, body) -> tuple[int, int]:
        mv = memoryview(body).cast("B")
        n = mv.nbytes
        off = (self.used + 15) & ~15
        if off + n > self.np.size:
            raise MemoryError("request arena full")
        self.np[off:off + n] = np.frombuffer(mv, dtype=np.uint8)
        self.used = off + n
        self.offs.append(off)
        self.lens.append(n)
        return off, n

    @classmethod
    def over(cls, buf: torch.Tensor, offs, lens) -> "RequestArena":
        """an arena over an existing (pinned) uint8 tensor that already holds
        request bodies at ``offs`` / ``lens`` (e.g. a slice of a large
        pinned block filled by the native generator)"""
        a = cls.__new__(cls)
        a.buf = buf
        a.np = buf.numpy()
        a.offs = [int(x) for x in offs]
        a.lens = [int(x) for x in lens]
        a.used = (a.offs[-1] + a.lens[-1]) if a.offs else 0
        return a

    def reset(self) -> None:
        self.used = 0
        self.offs.clear()
        self.lens.clear()

    def spans(self) -> tuple[np.ndarray, np.ndarray]:
        return np.asarray(self.offs, dtype=np.int64), np.asarray(self.lens, dtype=np.int64)


class _DeviceBufs:
    def __init__(self, device):
        self.device = device
        self.cap = {}
        self.t = {}

    def get(self, name: str, n: int, dtype) -> torch.Tensor:
        if self.cap.get(name, -1) < n:
            c = _grow(self.cap.get(name, 0) or 1024, n)
            self.t[name] = torch.empty(c, dtype=dtype, device=self.device)
            self.cap[name] = c
        return self.t[name]


class _ScanSet:
    """device buffers + pinned request table + events of one GPU-scan batch
    slot (csrc/hip/train_batch.hip); the set is reused once ``free`` (the
    compute-stream work of its last batch) has completed"""

    def __init__(self, device):
        self.bufs = _DeviceBufs(device)
        self.meta: torch.Tensor | None = None      # pinned [off R | len R | base R+1]
        self.copy_done = hip.DevEvent()
        self.ready = hip.DevEvent()
        self.free = hip.DevEvent()
        self.used = False
        self.args = hip.TrainBatchArgs()


class FeaturePipeline:
    def __init__(self, converter, device, nthreads: int | None = None):
        self.conv = converter
        self.device = torch.device(device)
        self.H = converter.hash_max_size
        self.fast = fast_eligible(converter)
        # the wide rule set (ngram / idf / bm25 / combinations) converts on
        # the device too (csrc/hip/fv_wide.hip), after the host scanner
        self.wide = not self.fast and wide_eligible(converter)
        self.nthreads = nthreads or scan_threads()
        self._pinned = [_Pinned(), _Pinned()]
        self._turn = 0
        self._devsets = [_DeviceBufs(self.device), _DeviceBufs(self.device)]
        self._dev = self._devsets[0]      # scratch for single-shot users (classify)
        self._copy_stream = torch.cuda.Stream(device=self.device)
        # GPU-scan batches are prepared (scan, fv_hash, hot-row detection) on
        # their own stream, so batch k+1's preparation runs beside batch k's
        # train kernel (which occupies only part of the CUs)
        self._prep_stream = torch.cuda.Stream(device=self.device)
        self._last_mark: torch.cuda.Event | None = None
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        self._direct = None
        # GPU-scan batches rotate over their own device sets; a set is reused
        # once the host has seen its last batch's kernels complete (an event
        # the host synchronises on, not a cross-stream wait: a copy-engine
        # copy that waits on a compute-queue event can block the enqueuing
        # thread for milliseconds)
        self._gsets: list[_ScanSet] | None = None     # created on the first GPU-scan batch
        self._gnext = 0
        self._gprev = None
        self.set_wait_s = 0.0           # host time waiting for a device set to come free

        self._ltab = None                 # (label version, device hash, meta, blob)
        if self.fast:
            rt = GpuRuleTable(converter)
            self.rules = rt
            self.d_srules = torch.from_numpy(rt.srules).to(self.device)
            self.d_nrules = torch.from_numpy(rt.nrules).to(self.device)
            self.d_blob = torch.from_numpy(rt.blob).to(self.device)
        elif self.wide:
            from .fv_wide import WideDevice
            self.wdev = WideDevice(converter, self.device)
            # the host scanner's slot estimate is unused on this path
            self.rules = type("SlotCounts", (), {"n_srules": 1, "n_nrules": 1})()

    # ------------------------------------------------------------ fast path
    def from_requests(self, bodies: list, labeled: bool, table=None) -> DeviceBatch:
        """bodies: buffer-protocol objects, each a msgpack list<labeled_datum>
        (labeled) or list<datum>; every body is one update stream."""
        if not (self.fast or self.wide):
            raise RuntimeError("converter config is not eligible for the GPU path")
        nat = native()
        pin = self._pinned[self._turn]
        self._turn ^= 1
        t0 = time.perf_counter_ns()
        pin.wait()
        trace.record("pipe.wait_pinned", time.perf_counter_ns() - t0)
        R = len(bodies)
        need_bytes = sum(memoryview(b).nbytes for b in bodies) + 16 * R + 16
        pin.ensure(need_bytes, max(1024, pin.cap_samples), R)
        while True:
            n, nbytes, nslots, err, err_req = nat.pack_requests(
                bodies, labeled, self.rules.n_srules, self.rules.n_nrules, table,
                pin.staging.data_ptr(), pin.cap_bytes, pin.datum_off.data_ptr(),
                pin.datum_len.data_ptr(), pin.labels.data_ptr() if labeled else 0, pin.row_ptr.data_ptr(),
                pin.stream_ptr.data_ptr(), pin.cap_samples, self.nthreads)
            if err == 2:
                pin.ensure(nbytes, n, R)
                continue
            if err == 1:
                raise TypeError(f"malformed datum list in request {err_req}")
            if err == 3:
                raise RuntimeError("label table full")
            break
        return self._launch(pin, pin.staging, n, nbytes, nslots, R, labeled)

    def from_arena(self, arena: RequestArena, offs: np.ndarray, lens: np.ndarray, labeled: bool,
                   table=None) -> DeviceBatch:
        """Zero-copy variant of from_requests: bodies are spans of a pinned
        RequestArena; the scanner reads them in place and one H2D copy moves
        the arena prefix to HBM."""
        if not (self.fast or self.wide):
            raise RuntimeError("converter config is not eligible for the GPU path")
        nat = native()
        pin = self._pinned[self._turn]
        self._turn ^= 1
        pin.wait()
        R = int(offs.size)
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        lens = np.ascontiguousarray(lens, dtype=np.int64)
        pin.ensure(0, max(1024, pin.cap_samples), R)
        while True:
            n, nbytes, nslots, err, err_req = nat.pack_spans(
                arena.buf.data_ptr(), offs.ctypes.data, lens.ctypes.data, R, labeled,
                self.rules.n_srules, self.rules.n_nrules, table, pin.datum_off.data_ptr(),
                pin.datum_len.data_ptr(), pin.labels.data_ptr() if labeled else 0, pin.row_ptr.data_ptr(),
                pin.stream_ptr.data_ptr(), pin.cap_samples, self.nthreads)
            if err == 2:
                pin.ensure(0, n, R)
                continue
            if err == 1:
                raise TypeError(f"malformed datum list in request {err_req}")
            if err == 3:
                raise RuntimeError("label table full")
            break
        return self._launch(pin, arena.buf, n, nbytes, nslots, R, labeled)

    def label_table(self, table) -> tuple:
        v = table.version()
        if self._ltab is None or self._ltab[0] != v:
            th, tm, blob = label_table_arrays(table.names(), table.alive())
            self._ltab = (v, torch.from_numpy(th).to(self.device),
                          torch.from_numpy(tm).to(self.device), torch.from_numpy(blob).to(self.device))
        return self._ltab[1:]

    def scan_batch_args(self, arena: RequestArena, offs: np.ndarray, lens: np.ndarray, table,
                        check: ScanCheck, counts: np.ndarray | None = None):
        """Prepare one GPU-scan batch (csrc/hip/scan.hip -> fv_hash.hip) for
        ``hip.train_batch_submit``: the H2D of the raw arena prefix on the
        copy stream, scan + hashing on the prep stream, the ready event the
        compute stream waits on. -> (args, set) with the scan / hash fields
        filled (the caller adds the train and hot-row fields, or leaves W
        null), or None when a request must go to the host scanner (a body
        that does not start with an array header, or one larger than the
        device scan stages). ``check`` receives the batch's error bits and
        label counts (pinned, valid once ``check.event`` completes); a batch
        with error bits set trained nothing and must be re-run on the host."""
        if not self.fast:
            raise RuntimeError("converter config is not eligible for the GPU fast path")
        if counts is None:
            counts = body_counts(arena.np, offs, lens)
            if counts is None:
                return None
        # requests the device scan does not stage (larger than its LDS window
        # or with more samples than its slot table): the host scanner takes
        # the batch right away instead of after a rejected launch
        if scan_too_big(offs, lens, counts):
            return None
        R = int(offs.size)
        if R == 0:
            return None
        if self._gsets is None:
            self._gsets = [_ScanSet(self.device) for _ in range(4)]
        n = int(counts.sum())
        used = int((offs + lens).max())
        empty_off = ((used + 15) & ~15) + 16
        buf_need = empty_off + 16
        sps, spn = self.rules.n_srules, self.rules.n_nrules
        slot_cap = (used // 3 + 1) * max(1, sps, spn)
        turn = self._gnext
        self._gnext = (turn + 1) % len(self._gsets)
        self._gprev = turn
        st = self._gsets[turn]
        if st.used:
            t0 = time.perf_counter()
            st.free.synchronize()          # its last batch's train (and so its copies) finished
            self.set_wait_s += time.perf_counter() - t0
        st.used = True
        if st.meta is None or st.meta.numel() < 3 * R + 1:
            st.meta = torch.empty(_grow(1024, 3 * R + 1), dtype=torch.int64, pin_memory=True)
        mnp = st.meta.numpy()
        mnp[:R] = offs
        mnp[R:2 * R] = lens
        mnp[2 * R] = 0
        np.cumsum(counts, out=mnp[2 * R + 1:3 * R + 1])
        dev = st.bufs
        g = dev.get
        a = st.args
        d_buf = g("buf", buf_need, torch.uint8)
        a.d_buf = d_buf.data_ptr()
        a.buf_cap = d_buf.numel()
        a.d_meta = g("scan_meta", 3 * R + 1, torch.int64).data_ptr()
        a.d_off = g("datum_off", max(n, 1), torch.int64).data_ptr()
        a.d_len = g("datum_len", max(n, 1), torch.int32).data_ptr()
        a.d_row = g("row_ptr", n + 1, torch.int64).data_ptr()
        a.d_lab = g("labels", max(n, 1), torch.int32).data_ptr()
        a.d_slots = g("req_slots", R, torch.int64).data_ptr()
        a.d_idx = g("fidx", slot_cap, torch.int32).data_ptr()
        a.d_val = g("fval", slot_cap, torch.float32).data_ptr()
        a.d_hist = g("label_hist", check.hist.size, torch.int32).data_ptr()
        a.d_err = g("scan_err", 1, torch.int32).data_ptr()
        if not a.copy_stream:                # constant for the set
            a.copy_stream = self._copy_stream.cuda_stream
            a.prep_stream = self._prep_stream.cuda_stream
            a.copy_done = st.copy_done.h
            a.ready = st.ready.h
            a.set_free = st.free.h
            a.srules = self.d_srules.data_ptr()
            a.nrules = self.d_nrules.data_ptr()
            a.n_srules = sps
            a.n_nrules = spn
            a.blob = self.d_blob.data_ptr()
            a.blob_len = self.d_blob.numel()
            a.H = self.H
            a.hash_err = self.err.data_ptr()
        a.compute_stream = torch.cuda.current_stream(self.device).cuda_stream
        ev = check.scan_event()
        a.check_done = ev.h
        a.host_out = check.buf.ptr
        a.nhist = check.hist.size
        check.nhist = check.hist.size
        check.event = ev
        th, tm, tb = self.label_table(table)
        a.lt_hash = th.data_ptr()
        a.lt_meta = tm.data_ptr()
        a.lt_cap = th.numel()
        a.lt_blob = tb.data_ptr()
        a.lt_blob_len = tb.numel()
        a.sps = sps
        a.spn = spn
        a.arena = arena.buf.data_ptr()
        a.used = used
        a.meta_host = st.meta.data_ptr()
        a.R = R
        a.n = n
        a.empty_off = empty_off
        a.slot_cap = slot_cap
        a.hot_rows = None
        a.hot_count_host = None
        a.W = None
        return a, st

    def from_arena_gpu(self, arena: RequestArena, offs: np.ndarray, lens: np.ndarray, table,
                       check: ScanCheck) -> DeviceBatch | None:
        """A GPU-scan batch without training (tests, tools): the device CSR
        of the scanned and hashed requests; its ``ready`` event covers the
        work. None: a request the host scanner must take."""
        offs = np.ascontiguousarray(offs, dtype=np.int64)
        lens = np.ascontiguousarray(lens, dtype=np.int64)
        r = self.scan_batch_args(arena, offs, lens, table, check)
        if r is None:
            return None
        a, st = r
        hip.train_batch_submit(a)
        R, n, t = int(a.R), int(a.n), st.bufs.t
        return DeviceBatch(n, int(a.slot_cap), R, t["row_ptr"], t["fidx"], t["fval"], t["labels"],
                           t["scan_meta"][2 * R:3 * R + 1], ready=st.ready)

    def _launch(self, pin: "_Pinned", src: torch.Tensor, n: int, nbytes: int, nslots: int,
                R: int, labeled: bool) -> DeviceBatch:
        compute = torch.cuda.current_stream(self.device)
        dev = self._devsets[self._turn]   # the set not used by the previous batch
        prev_mark = self._last_mark
        mark = torch.cuda.Event()
        mark.record(compute)
        self._last_mark = mark
        d_buf = dev.get("buf", max(nbytes, 1), torch.uint8)
        d_off = dev.get("datum_off", max(n, 1), torch.int64)
        d_len = dev.get("datum_len", max(n, 1), torch.int32)
        d_row = dev.get("row_ptr", n + 1, torch.int64)
        d_sp = dev.get("stream_ptr", R + 1, torch.int64)
        d_idx = dev.get("fidx", max(nslots, 1), torch.int32)
        d_val = dev.get("fval", max(nslots, 1), torch.float32)
        d_lab = dev.get("labels", max(n, 1), torch.int32) if labeled else None
        cs = self._copy_stream
        if prev_mark is not None:
            cs.wait_event(prev_mark)
        else:
            cs.wait_stream(compute)
        with torch.cuda.stream(cs):
            d_buf[:nbytes].copy_(src[:nbytes], non_blocking=True)
            d_off[:n].copy_(pin.datum_off[:n], non_blocking=True)
            d_len[:n].copy_(pin.datum_len[:n], non_blocking=True)
            d_row[:n + 1].copy_(pin.row_ptr[:n + 1], non_blocking=True)
            d_sp[:R + 1].copy_(pin.stream_ptr[:R + 1], non_blocking=True)
            if labeled:
                d_lab[:n].copy_(pin.labels[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(cs)
        compute.wait_event(ev)
        pin.event = ev
        if self.wide:
            # train batches (labeled) advance the document statistics
            row, idx, val, total = self.wdev.convert(d_buf, nbytes, d_off, d_len, n, labeled)
            if int(self.wdev.err.item()):
                self.wdev.err.zero_()
                raise TypeError("malformed datum (device wide converter)")
            return DeviceBatch(n, max(total, 1), R, row, idx, val, d_lab, d_sp)
        if n > 0:
            hip.fv_hash(d_buf, nbytes, d_off, d_len, d_row, n, self.d_srules, self.rules.n_srules,
                        self.d_nrules, self.rules.n_nrules, self.d_blob, self.H, d_idx, d_val,
                        self.err)
        return DeviceBatch(n, nslots, R, d_row, d_idx, d_val, d_lab, d_sp)

    # ------------------------------------------------------ direct classify
    def classify_direct(self, bodies: list, W: torch.Tensor) -> np.ndarray | None:
        """Latency path for small classify requests: the native host hasher
        (csrc/native/jb_hostfv.hpp, bit-identical to fv_hash) turns the
        bodies into CSR, then ONE kernel (csrc/hip/classify_direct.hip)
        whose arguments carry the (idx, val) pairs scores them against the
        HBM-resident W and writes into pinned host memory. Returns [n, LC]
        scores, or None when the request is too large for the direct path."""
        if not self.fast:
            return None
        LC = W.shape[1]
        d = self._direct
        if d is None or d["LC"] < LC:
            cap, slots = hip.DIRECT_MAX_SAMPLES, hip.DIRECT_MAX_SLOTS
            r = self.rules
            d = self._direct = {
                "LC": LC,
                "hasher": native().HostFvHasher(r.srules, r.n_srules, r.nrules, r.n_nrules, r.blob,
                                                self.H),
                "idx": np.zeros(slots, np.int32),
                "val": np.zeros(slots, np.float32),
                "row_ptr": np.zeros(cap + 1, np.int64),
                "out": hip.HostBuffer(cap * LC * 4),
                "done": hip.HostBuffer(4 * cap),
                # high-priority stream: used when the compute stream is idle
                # (a launch on the busy compute stream keeps train -> classify order)
                "stream": torch.cuda.Stream(device=self.device, priority=-1),
            }
        n, _, err = d["hasher"].hash(bodies, d["idx"].ctypes.data, d["val"].ctypes.data,
                                     d["row_ptr"].ctypes.data, hip.DIRECT_MAX_SAMPLES,
                                     hip.DIRECT_MAX_SLOTS)
        if err == 2:
            return None
        if err == 1:
            raise TypeError("malformed datum list in classify request")
        if n == 0:
            return np.zeros((0, LC), dtype=np.float32)
        compute = torch.cuda.current_stream(self.device)
        st = d["stream"].cuda_stream if compute.query() else compute.cuda_stream
        if not hip.classify_direct(d["idx"].ctypes.data, d["val"].ctypes.data,
                                   d["row_ptr"].ctypes.data, n, W, d["out"], d["done"], stream=st):
            return None
        return d["out"].view(np.float32, n * LC).reshape(n, LC).copy()

    # ------------------------------------------------------------ host path
    def from_rows(self, rows: list[tuple[list[int], list[float]]], labels: list[int] | None,
                  stream_sizes: list[int] | None = None) -> DeviceBatch:
        n = len(rows)
        lens = np.fromiter((len(r[0]) for r in rows), dtype=np.int64, count=n)
        row_ptr = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=row_ptr[1:])
        nnz = int(row_ptr[-1])
        idx = np.fromiter((i for r in rows for i in r[0]), dtype=np.int32, count=nnz)
        val = np.fromiter((v for r in rows for v in r[1]), dtype=np.float32, count=nnz)
        sizes = stream_sizes if stream_sizes is not None else [n]
        sp = np.zeros(len(sizes) + 1, dtype=np.int64)
        np.cumsum(np.asarray(sizes, dtype=np.int64), out=sp[1:])
        dev = self.device
        d_row = torch.from_numpy(row_ptr).to(dev, non_blocking=False)
        d_idx = torch.from_numpy(idx if nnz else np.zeros(1, np.int32)).to(dev)
        d_val = torch.from_numpy(val if nnz else np.zeros(1, np.float32)).to(dev)
        d_lab = None
        if labels is not None:
            d_lab = torch.from_numpy(np.asarray(labels, dtype=np.int32).reshape(-1)).to(dev)
        d_sp = torch.from_numpy(sp).to(dev)
        return DeviceBatch(n, nnz, len(sizes), d_row, d_idx, d_val, d_lab, d_sp)

    def check_errors(self) -> None:
        e = int(self.err.item())
        if e:
            self.err.zero_()
            raise RuntimeError(f"GPU datum parser reported error mask {e}")
