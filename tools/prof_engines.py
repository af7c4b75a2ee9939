"""Per-stage latency of the row-engine hot paths on the GPU (where the time
of one LOF add / similar_row query goes): host prep, H2D, scan kernel,
top-k, D2H. Prints one JSON line per stage group.

Usage: python tools/prof_engines.py [--rows N] [--method inverted_index_euclid]
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
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _p50(fn, n=50, sync=None):
    xs = []
    for _ in range(5):
        fn()
    for _ in range(n):
        if sync:
            sync()
        t = time.perf_counter()
        fn()
        if sync:
            sync()
        xs.append((time.perf_counter() - t) * 1e6)
    return round(statistics.median(xs), 1)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--method", default="inverted_index_euclid")
    args = ap.parse_args()
    import torch
    from bench_engines import _datum
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.fv_converter.datum import as_datum
    from jubatus_amd.models.anomaly import LOF
    from jubatus_amd.ops import hip
    dev = torch.device("cuda", 0)
    conv = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin",
                              "global_weight": "bin"}],
            "num_rules": [{"key": "*", "type": "num"}]}
    p = {"method": args.method, "nearest_neighbor_num": 10, "reverse_nearest_neighbor_num": 30,
         "parameter": {"hash_num": 64}}
    lof = LOF("lof", p, DatumToFvConverter(conv), dev)
    rng = random.Random(2)
    for b in range(0, args.rows, 65536):
        lof.set_rows([(str(i), _datum(rng)) for i in range(b, min(args.rows, b + 65536))])
    sync = torch.cuda.synchronize
    n = lof.rows.nslots
    idx = lof.index
    out = {"rows": n, "method": args.method}
    q = [lof.fv_of(as_datum(_datum(rng)))]
    if args.method.startswith("inverted_index"):
        qd = idx._queries_device(q)
        sc = idx._scan(qd, 1, n)
        out["host_prep_queries_device"] = _p50(lambda: idx._queries_device(q), sync=sync)
        out["pool_scan_kernel_nq1"] = _p50(lambda: idx._scan(qd, 1, n), sync=sync)
        q8 = idx._queries_device(q * 8)
        out["pool_scan_kernel_nq8"] = _p50(lambda: idx._scan(q8, 8, n), sync=sync)
        out["topk_scores_k31"] = _p50(lambda: hip.topk_scores(sc, 1, n, 31, flip=False), sync=sync)
        out["topk_scores_k10"] = _p50(lambda: hip.topk_scores(sc, 1, n, 10, flip=False), sync=sync)
        db = hip.DirectQueryBuffers(dev, 1)
        out["topk_scores_direct_k10"] = _p50(lambda: hip.topk_scores_direct(sc, 1, n, 10, False, db))
        out["topk_scores_direct_k31"] = _p50(lambda: hip.topk_scores_direct(sc, 1, n, 31, False, db))
        sc8 = idx._scan(q8, 8, n)
        out["topk_scores_q8_k10"] = _p50(lambda: hip.topk_scores(sc8, 8, n, 10, flip=False),
                                         sync=sync)
        out["query_slots_device"] = _p50(lambda: idx.pool.query_slots_device([5]), sync=sync)
        out["pool_bytes_per_scan"] = int(idx.pool.live * 8 + n * 21)
    # recommender default-config latency path, stage by stage
    import msgpack
    import numpy as np
    from jubatus_amd.models.recommender import Recommender
    with open(os.path.join(ROOT, "config", "recommender", "default.json")) as f:
        rcfg = json.load(f)
    rec = Recommender(rcfg["method"], rcfg.get("parameter", {}),
                      DatumToFvConverter(rcfg["converter"]), dev)
    for b in range(0, args.rows, 65536):
        rec.set_rows([(f"r{i}", _datum(rng)) for i in range(b, min(args.rows, b + 65536))])
    dq = as_datum(_datum(rng))
    h = rec._hasher()
    body = msgpack.packb([dq.to_msgpack()], use_bin_type=False)
    hi = np.empty(256, np.int32)
    hv = np.empty(256, np.float32)
    hr = np.zeros(2, np.int64)
    out["rec_hash_datum"] = _p50(lambda: h.hash([body], hi.ctypes.data, hv.ctypes.data,
                                                  hr.ctypes.data, 1, 256, False))
    h.hash([body], hi.ctypes.data, hv.ctypes.data, hr.ctypes.data, 1, 256, False)
    nr = rec.rows.nslots
    out["rec_index_query_direct_k10"] = _p50(lambda: rec.index.query_direct(hi, hv, hr, 1, nr, 10, True))
    out["rec_similar_row_from_datum_k10"] = _p50(lambda: rec.similar_row_from_datum(dq, 10))
    it2 = iter(range(10 ** 9))
    out["rec_update_row"] = _p50(lambda: rec.update_row(f"u{next(it2) % 5000}", _datum(rng)))
    out["rec_datum_gen"] = _p50(lambda: _datum(rng))
    out["query_slot_lists_k31"] = _p50(lambda: lof.query_slot_lists([5], 31, False))
    out["query_fv_slots_k10"] = _p50(lambda: lof.query_fv_slots(q[0], 10, False))
    lof.build_lists() if n <= 200_000 else None
    it = iter(range(n, 10 ** 9))
    out["lof_add"] = _p50(lambda: lof.add(str(next(it)), _datum(rng)))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
