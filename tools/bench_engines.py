#!/usr/bin/env python3
"""Secondary BASELINE.json configs on one device (MI355X, or --device cpu
for the in-house CPU baseline): one JSON line per engine.

  recommender  config/recommender/euclid_lsh.json: bulk ingest (rows/s),
               update_row per call, similar_row_from_datum / _from_id
               latency over N rows, batched query throughput
  anomaly      config/anomaly/lof.json (lof over euclid_lsh): add / calc_score
               latency and throughput over N stored points
  clustering   config/clustering/{kmeans,gmm}.json: push throughput
               (points/s incl. bucket compression + reclustering) and
               get_nearest_center latency

Data: synthetic datums (random-init models). The reference publishes no
numbers: vs_baseline is null; --device cpu gives our own CPU
reference-semantics numbers for comparison.

Usage: python tools/bench_engines.py [recommender|anomaly|clustering ...]
           [--rows N] [--device gpu|cpu]
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


def _log(msg: str) -> None:
    print(f"[bench_engines {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _lat(fn, iters: int, warm: int = 5) -> dict:
    for _ in range(warm):
        fn()
    xs = []
    for _ in range(iters):
        t = time.perf_counter()
        fn()
        xs.append((time.perf_counter() - t) * 1e6)
    xs.sort()
    return {"p50_us": round(statistics.median(xs), 1),
            "p99_us": round(xs[min(len(xs) - 1, int(0.99 * len(xs)))], 1)}


def _datum(rng: random.Random, nstr: int = 4, nnum: int = 8, vocab: int = 1000) -> dict:
    c = rng.randrange(16)  # cluster id: structure for the searches
    d = {f"s{j}": f"t{(c * 37 + rng.randrange(8)) % vocab}" for j in range(nstr)}
    for j in range(nnum):
        d[f"n{j}"] = c * 0.5 + rng.gauss(0.0, 0.3)
    return d


def _config(path: str) -> dict:
    with open(os.path.join(ROOT, "config", path)) as f:
        return json.load(f)


def _device(kind: str):
    if kind == "cpu":
        return None
    import torch
    return torch.device("cuda", 0)


def _sync(dev):
    if dev is not None:
        import torch
        torch.cuda.synchronize()


def bench_recommender(args, dev) -> dict:
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.recommender import Recommender
    cfg = _config(args.recommender_config)
    rec = Recommender(cfg["method"], cfg.get("parameter", {}), DatumToFvConverter(cfg["converter"]), dev)
    rng = random.Random(1)
    N = args.rows
    pool = [_datum(rng) for _ in range(4096)]
    t0 = time.perf_counter()
    B = 65536
    for b in range(0, N, B):
        rec.set_rows([(f"r{i}", pool[i % 4096]) for i in range(b, min(N, b + B))])
    _sync(dev)
    ingest = N / (time.perf_counter() - t0)
    it = iter(range(10 ** 9))
    upd = _lat(lambda: rec.update_row(f"u{next(it) % 5000}", pool[next(it) % 4096]), args.iters)
    q = pool[7]
    sim_d = _lat(lambda: rec.similar_row_from_datum(q, 10), args.iters)

    def upd_query():
        j = next(it)
        rec.update_row(f"u{j % 5000}", pool[j % 4096])
        rec.similar_row_from_datum(pool[(j * 7) % 4096], 10)
    inter = _lat(upd_query, args.iters)
    sim_i = _lat(lambda: rec.similar_row_from_id("r123", 10), args.iters)
    # batched queries: nq signatures scanned + top-k'd in one launch
    from jubatus_amd.fv_converter.datum import as_datum
    fvs = [rec.fv_of(as_datum(pool[i])) for i in range(256)]
    n = rec.rows.nslots
    rec.index.query(fvs, n, 10, True)
    _sync(dev)
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        rec.index.query(fvs, n, 10, True)
    _sync(dev)
    qps = 256 * reps / (time.perf_counter() - t0)
    return {"engine": f"jubarecommender {cfg['method']} (config/{args.recommender_config})",
            "rows": N, "bulk_ingest_rows_per_s": round(ingest, 1),
            "update_row_call": upd, "similar_row_from_datum_k10": sim_d,
            "similar_row_from_id_k10": sim_i, "batched_query_k10_per_s": round(qps, 1),
            "interleaved_update_then_query": inter}


def bench_anomaly(args, dev) -> dict:
    """1M distinct rows (16 clusters + noise) bulk-loaded, then every row's
    neighbour list built in batched kNN launches (the state a model fed by
    add() has); add = one rnn query + the device list insert / staleness
    mark / fused lrd+LOF score"""
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.anomaly import LOF
    cfg = _config(args.anomaly_config)
    lof = LOF(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]), dev)
    rng = random.Random(2)
    N = args.rows
    t0 = time.perf_counter()
    B = 65536
    for b in range(0, N, B):
        lof.set_rows([(str(i), _datum(rng)) for i in range(b, min(N, b + B))])
        _log(f"anomaly ingest {min(N, b + B)}/{N}")
    _sync(dev)
    ingest = N / (time.perf_counter() - t0)
    pool = [_datum(rng) for _ in range(4096)]
    it = iter(range(N, 10 ** 9))
    cold = _lat(lambda: lof.add(str(next(it)), pool[next(it) % 4096]), args.iters)
    _log("anomaly cold adds done; building neighbour lists")
    t0 = time.perf_counter()
    built = lof.build_lists(progress=lambda d, t: _log(f"lists {d}/{t}"))
    _sync(dev)
    build_s = time.perf_counter() - t0
    add = _lat(lambda: lof.add(str(next(it)), pool[next(it) % 4096]), args.iters)
    score = _lat(lambda: lof.calc_score(pool[11]), args.iters)
    score_new = _lat(lambda: lof.calc_score(_datum(rng)), args.iters)
    return {"engine": f"jubaanomaly {cfg['method']} over {cfg['parameter']['method']} "
                      f"(config/{args.anomaly_config})",
            "rows": N, "bulk_ingest_rows_per_s": round(ingest, 1),
            "add_call_cold_lists": cold, "list_build_s": round(build_s, 2), "lists_built": built,
            "add_call": add, "calc_score_call": score, "calc_score_new_point": score_new,
            "add_per_s": round(1e6 / add["p50_us"], 1)}


def bench_clustering(args, dev) -> list[dict]:
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.clustering import Clustering
    out = []
    for name in ("kmeans", "gmm"):
        cfg = _config(f"clustering/{name}.json")
        cl = Clustering(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]), dev)
        rng = random.Random(3)
        pts = [_datum(rng) for _ in range(args.points)]
        t0 = time.perf_counter()
        for b in range(0, len(pts), 500):
            cl.push(pts[b:b + 500])
        _sync(dev)
        rate = len(pts) / (time.perf_counter() - t0)
        near = _lat(lambda: cl.get_nearest_center(pts[5]), args.iters)
        out.append({"engine": f"jubaclustering {name} (config/clustering/{name}.json)",
                    "points": len(pts), "push_points_per_s": round(rate, 1),
                    "revision": cl.get_revision(), "get_nearest_center_call": near})
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("engines", nargs="*", default=["recommender", "anomaly", "clustering"])
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--points", type=int, default=20_000)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu")
    ap.add_argument("--recommender-config", default="recommender/euclid_lsh.json")
    ap.add_argument("--anomaly-config", default="anomaly/lof.json")
    args = ap.parse_args()
    dev = _device(args.device)
    for e in args.engines:
        t = time.perf_counter()
        r = {"recommender": bench_recommender, "anomaly": bench_anomaly,
             "clustering": bench_clustering}[e](args, dev)
        for x in (r if isinstance(r, list) else [r]):
            x.update({"device": "MI355X" if dev is not None else "cpu", "data": "synthetic",
                      "vs_baseline": None, "wall_s": round(time.perf_counter() - t, 1)})
            print(json.dumps(x), flush=True)


if __name__ == "__main__":
    main()
