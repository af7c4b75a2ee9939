#!/usr/bin/env python3
"""Where does a bench.py step go? Times each stage of the AROW train step in
isolation on 1 GPU, with the bench's own config (1024 requests x 128 samples):

  host_scan_ms   native scan of the request spans (pack_spans, N threads)
  h2d_ms         the arena -> HBM copy (request bytes + descriptors)
  fv_hash_ms     GPU parse + feature hashing kernel
  train_ms       GPU AROW update kernel (1024 streams, atomic mode)
  step_ms        the pipelined step as bench.py runs it (stages overlap)

The step is bounded by max(host_scan, h2d, fv_hash + train) when the
pipeline overlaps perfectly.

Usage: python tools/bench_breakdown.py [--threads N]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch
    from jubatus_amd._native import native
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier
    from jubatus_amd.ops import hip
    from jubatus_amd.ops.feature_pipeline import RequestArena

    dev = torch.device("cuda", 0)
    cfg = json.loads(json.dumps(bench.AROW_CONFIG))
    cfg["converter"]["hash_max_size"] = 1 << 20
    clf = LinearClassifier("AROW", cfg["parameter"], DatumToFvConverter(cfg["converter"]), device=dev)
    for y in range(16):
        clf.set_label(f"label{y}")
    if a.threads:
        clf.pipe.nthreads = a.threads
    bodies = bench.make_requests(random.Random(5), 1024, 128, 16, 8, 8, 100000)
    arena = RequestArena(sum(len(b) for b in bodies) + 16 * len(bodies) + 64)
    for b in bodies:
        arena.append(b)
    offs, lens = arena.spans()
    nbytes = arena.used
    res = {"samples_per_step": 131072, "request_bytes_per_step": nbytes,
           "scan_threads": clf.pipe.nthreads}

    def med(xs):
        return round(statistics.median(xs), 3)

    # 1. host scan alone
    n = 131072
    d_off = np.zeros(n, np.int64)
    d_len = np.zeros(n, np.int32)
    labs = np.zeros(n, np.int32)
    row = np.zeros(n + 1, np.int64)
    sp = np.zeros(1025, np.int64)
    nat = native()
    t = []
    for _ in range(a.iters):
        t0 = time.perf_counter()
        r = nat.pack_spans(arena.buf.data_ptr(), offs.ctypes.data, lens.ctypes.data, 1024, True,
                           clf.pipe.rules.n_srules, clf.pipe.rules.n_nrules, clf.labels,
                           d_off.ctypes.data, d_len.ctypes.data, labs.ctypes.data, row.ctypes.data,
                           sp.ctypes.data, n, clf.pipe.nthreads)
        t.append((time.perf_counter() - t0) * 1e3)
        assert r[3] == 0, r
    res["host_scan_ms"] = med(t)
    # 2. H2D of the request bytes
    dbuf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t = []
    for _ in range(a.iters):
        e0.record()
        dbuf.copy_(arena.buf[:nbytes], non_blocking=True)
        e1.record()
        torch.cuda.synchronize()
        t.append(e0.elapsed_time(e1))
    res["h2d_ms"] = med(t)
    res["h2d_GBps"] = round(nbytes / (res["h2d_ms"] * 1e-3) / 1e9, 1)
    # 3/4. kernels on one prepared batch
    b = clf.pipe.from_arena(arena, offs, lens, True, clf.labels)
    torch.cuda.synchronize()
    t_fv, t_tr = [], []
    pipe = clf.pipe
    dev_set = pipe._devsets[pipe._turn]
    for _ in range(a.iters):
        e0.record()
        hip.fv_hash(dev_set.t["buf"], nbytes, dev_set.t["datum_off"], dev_set.t["datum_len"],
                    b.row_ptr, b.n, pipe.d_srules, pipe.rules.n_srules, pipe.d_nrules,
                    pipe.rules.n_nrules, pipe.d_blob, pipe.H, b.fidx, b.fval, pipe.err)
        e1.record()
        torch.cuda.synchronize()
        t_fv.append(e0.elapsed_time(e1))
        e0.record()
        clf._train_batch(b)
        e1.record()
        torch.cuda.synchronize()
        t_tr.append(e0.elapsed_time(e1))
    res["fv_hash_ms"] = med(t_fv)
    res["train_ms"] = med(t_tr)
    # 5. pipelined steps
    for _ in range(3):
        clf.train_arena(arena, offs, lens)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters * 2):
        clf.train_arena(arena, offs, lens)
    torch.cuda.synchronize()
    res["step_ms"] = round((time.perf_counter() - t0) * 1e3 / (a.iters * 2), 3)
    res["samples_per_s"] = round(131072 / (res["step_ms"] * 1e-3), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
