"""Sparse, memory-bounded MIX of HBM-resident row tables (linear models).

Reference: ``linear_mixer`` ships only what changed since the last MIX -
``get_diff`` packs the diff accumulated by the local_mixture storage
(jubatus/server/framework/mixer/linear_mixer.cpp:547-564), the master folds
the diffs and ``put_diff`` applies the result (:613-662). Here a MIX is a
collective over the process group (RCCL over xGMI on GPUs, gloo on hosts):

* the train kernel marks every row it writes in ``touched`` (uint8[H],
  csrc/hip/linear.hip);
* ``begin`` starts an asynchronous MAX all-reduce of the touched bitmap (the
  union, the same on every rank) and returns - no host synchronisation;
* ``ready`` (polled between train batches) copies the union's row count to
  the host once the all-reduce finished (async D2H + event), then compacts
  the rows on the device (``nonzero_static`` with that size), snapshots them
  of every table into one contiguous buffer and starts the SUM all-reduce;
* ``end`` folds the cluster mean in: ``T[rows] += mean(snapshot) - snapshot``,
  so updates made while the collective ran are kept (and marked touched
  again for the next MIX).

Rows nobody touched since the last MIX are equal on every rank (the last MIX
made them so), so leaving them out is exact. The bytes moved scale with the
touched rows, and the extra memory is 2 x the union's rows.

``wire_dtype`` (``JUBATUS_MIX_DTYPE``): ``fp32`` (default) or
``bf16`` - the SUM all-reduce then moves bf16 values (half the bytes over
xGMI). The snapshot and the fold stay fp32, so updates made during the
collective are kept exactly, but the wire's rounding is not: the all-reduce
itself adds in bf16, so a ring rounds at every hop (relative error of the
sum ~ world x 2^-9, growing with the world size, not a fixed 2^-8), and the
fold writes ``mean_bf16 - snapshot`` into the tables, so that error becomes
part of the model (a later MIX does not undo it; it averages on from there).
The native mixer (csrc/server/jubaclassifier.cpp) keeps the precision
tables (S / P of CW, AROW, NHERD) in fp32 on the wire and sends only the
weights in bf16.

When the union exceeds ``dense_frac`` of the table (or no touched map
exists: host backend, after a model load or a label re-layout), the MIX is
dense but chunked: at most two chunks of ``chunk_bytes`` are snapshotted and
in flight at a time (``poll`` advances them between train batches), so the
extra memory stays <= 4 chunks (<= 1/4 of the tables for tables of 4 GiB
and more) instead of two full copies.
"""
from __future__ import annotations

import os
import time
from typing import Sequence

import torch
import torch.distributed as dist

DEFAULT_CHUNK_BYTES = int(os.environ.get("JUBATUS_MIX_CHUNK_BYTES", 256 << 20))
DEFAULT_DENSE_FRAC = float(os.environ.get("JUBATUS_MIX_DENSE_FRAC", "0.5"))
DEFAULT_WIRE_DTYPE = os.environ.get("JUBATUS_MIX_DTYPE", "fp32")


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


class TableMix:
    """One MIX of ``tables`` (each [H, C], same H, same device)."""

    def __init__(self, tables: Sequence[torch.Tensor], touched: torch.Tensor | None, group=None,
                 dense_frac: float = DEFAULT_DENSE_FRAC, chunk_bytes: int = DEFAULT_CHUNK_BYTES,
                 wire_dtype: str = DEFAULT_WIRE_DTYPE):
        if not tables:
            raise ValueError("nothing to mix")
        if wire_dtype not in ("fp32", "bf16"):
            raise ValueError(f"mix wire dtype must be fp32 or bf16, not {wire_dtype}")
        self.wire = torch.bfloat16 if wire_dtype == "bf16" else torch.float32
        self.tables = list(tables)
        self.H = self.tables[0].shape[0]
        if any(t.shape[0] != self.H or not t.is_contiguous() for t in self.tables):
            raise ValueError("mix tables must be contiguous with the same row count")
        self.touched = touched
        self.group = group
        self.n = _world(group)
        self.dense_frac = dense_frac
        self.row_bytes = sum(t[0].numel() * t.element_size() for t in self.tables)
        total = self.H * self.row_bytes
        # chunk: at most chunk_bytes, at most 1/16 of the tables (>= 4 MiB)
        cb = min(chunk_bytes, max(4 << 20, total // 16))
        self.chunk_rows = max(1, cb // max(1, self.row_bytes))
        self.mode = "none"
        self.rows = 0              # rows mixed (union size or H)
        self.nbytes = 0            # bytes all-reduced per rank
        self._sparse = None        # (rows idx, snap, red, work)
        self._next_row = 0         # dense: first row not launched yet
        self._inflight: list = []  # dense: (r0, r1, snap, red, work)
        self._done = False
        self._mark = None          # union bitmap (all-reduce MAX in flight)
        self._mark_work = None
        self._count = None         # (pinned count, event) of the union size copy
        self._aux = None           # the union all-reduce of a rank that went dense at once
        self.abandoned = False     # tables replaced meanwhile: run the collectives, fold nothing
        self._t0 = None            # host clock at begin()
        self.latency_ms = None     # begin() -> first observed completion (ready() or end())

    # ----------------------------------------------------------- begin
    def begin(self) -> "TableMix":
        """start the MIX (asynchronous: no host synchronisation here)"""
        self._t0 = time.perf_counter()
        if self.n <= 1:
            if self.touched is not None:
                self.touched.zero_()
            self.mode, self._done = "single", True
            return self
        # union of the ranks' touched rows = MAX all-reduce of the bitmaps; a
        # rank without a map (after a load / re-layout) contributes all rows,
        # so every rank then sees a dense union
        t = self.touched
        if t is not None:
            self._mark = t.clone()
            t.zero_()
        else:
            self._mark = torch.ones(self.H, dtype=torch.uint8, device=self.tables[0].device)
        self._mark_work = dist.all_reduce(self._mark, op=dist.ReduceOp.MAX, group=self.group,
                                          async_op=True)
        self.nbytes = self.H
        self.mode = "union"
        if t is None:
            # this rank's all-ones map makes the union dense on every rank:
            # the first chunks go out right away (the other ranks issue the
            # same collectives once they see the union)
            self._aux = self._mark_work       # waited for in end()
            self._mark = None
            self._mark_work = None
            self.mode = "dense"
            self.rows = self.H
            self._pump()
        return self

    def _advance_union(self, block: bool) -> bool:
        """union all-reduce -> size on the host -> the sparse or dense MIX
        proper; False while waiting (block=False)"""
        if self._count is None:
            if not block and not self._mark_work.is_completed():
                return False
            self._mark_work.wait()
            cnt = self._mark.sum(dtype=torch.int64).reshape(1)
            if cnt.is_cuda:
                host = torch.empty(1, dtype=torch.int64, pin_memory=True)
                host.copy_(cnt, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                self._count = (host, ev)
            else:
                self._count = (cnt, None)
        host, ev = self._count
        if ev is not None:
            if not block and not ev.query():
                return False
            ev.synchronize()
        rows_n = int(host[0])
        # a full union always goes dense: a rank without a touched map went
        # dense in begin() (its all-ones map makes the union full on every
        # rank), so whatever dense_frac is, every rank must pick the same path
        if rows_n >= self.H or rows_n > self.dense_frac * self.H:
            self._mark = None
            self.mode = "dense"
            self.rows = self.H
            self._pump()
            return True
        self.mode = "sparse"
        self.rows = rows_n
        if rows_n == 0:
            self._mark = None
            self._done = True
            return True
        rows = torch.nonzero_static(self._mark, size=rows_n).flatten()   # sorted, same on every rank
        self._mark = None
        # fp32 snapshot and sums whatever the tables store (bf16 W: the
        # collective adds fp32, the fold rounds once)
        snap = torch.cat([t.index_select(0, rows).reshape(self.rows, -1).float() for t in self.tables],
                         dim=1)
        red = snap.to(self.wire, copy=True)   # never an alias of snap
        self.nbytes += red.numel() * red.element_size()
        work = dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._sparse = (rows, snap, red, work)
        return True

    # ------------------------------------------------------------ dense
    def _launch(self, r0: int, r1: int) -> None:
        snap = torch.cat([t[r0:r1].reshape(r1 - r0, -1).float() for t in self.tables], dim=1)
        red = snap.to(self.wire, copy=True)   # never an alias of snap
        self.nbytes += red.numel() * red.element_size()
        work = dist.all_reduce(red, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self._inflight.append((r0, r1, snap, red, work))

    def abandon(self) -> None:
        """The owner replaced (or reloaded) its tables while this MIX was in
        flight: the remaining collectives still run (every rank must issue
        the same sequence), but no result is folded into the tables"""
        self.abandoned = True

    def _fold(self, r0: int, r1: int, snap: torch.Tensor, red: torch.Tensor) -> None:
        if self.abandoned:
            return
        upd = red.float().mul_(1.0 / self.n).sub_(snap)
        c0 = 0
        for t in self.tables:
            w = t[0].numel()
            tv = t[r0:r1].view(r1 - r0, -1)
            if t.dtype == torch.float32:
                tv.add_(upd[:, c0:c0 + w])
            else:
                tv.copy_(tv.float().add_(upd[:, c0:c0 + w]))
            c0 += w

    def _pump(self, block: bool = False) -> None:
        """fold finished chunks (in order), keep two chunks in flight"""
        while self._inflight:
            r0, r1, snap, red, work = self._inflight[0]
            if not block and not work.is_completed():
                break
            work.wait()
            self._fold(r0, r1, snap, red)
            self._inflight.pop(0)
        while len(self._inflight) < 2 and self._next_row < self.H:
            r0 = self._next_row
            r1 = min(self.H, r0 + self.chunk_rows)
            self._next_row = r1
            self._launch(r0, r1)
        if not self._inflight and self._next_row >= self.H:
            self._done = True

    # ------------------------------------------------------------ poll
    def ready(self) -> bool:
        """advance without blocking; True when ``end`` will not wait"""
        r = self._ready()
        if r:
            self._stamp()
        return r

    def _stamp(self) -> None:
        if self.latency_ms is None and self._t0 is not None:
            self.latency_ms = round((time.perf_counter() - self._t0) * 1e3, 3)

    def _ready(self) -> bool:
        if self._done:
            return True
        if self.mode == "union" and not self._advance_union(block=False):
            return False
        if self._done:
            return True
        if self.mode == "dense":
            self._pump()
            return self._done
        return self._sparse[3].is_completed()

    def end(self) -> int:
        """finish the MIX (blocking); returns the bytes all-reduced per rank"""
        if self.mode == "union":
            self._advance_union(block=True)
        if self._aux is not None:
            self._aux.wait()
            self._aux = None
        if self.mode == "dense":
            while not self._done:
                self._pump(block=True)
        elif self._sparse is not None:
            rows, snap, red, work = self._sparse
            work.wait()
            if not self.abandoned:
                upd = red.float().mul_(1.0 / self.n).sub_(snap)
                c0 = 0
                for t in self.tables:
                    w = t[0].numel()
                    tv = t.view(self.H, -1)
                    if t.dtype == torch.float32:
                        tv.index_add_(0, rows, upd[:, c0:c0 + w])
                    else:            # bf16: current rows + delta in fp32, one rounding
                        cur = tv.index_select(0, rows).float().add_(upd[:, c0:c0 + w])
                        tv.index_copy_(0, rows, cur.to(t.dtype))
                    c0 += w
            self._sparse = None
        self._done = True
        self._stamp()
        return self.nbytes

    def stats(self) -> dict:
        return {"mode": self.mode, "rows": self.rows, "bytes": self.nbytes,
                "abandoned": self.abandoned, "latency_ms": self.latency_ms, "world": self.n,
                "wire": "bf16" if self.wire == torch.bfloat16 else "fp32"}
