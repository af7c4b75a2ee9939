"""Classify latency breakdown (1 GPU): full classify_requests vs its parts
(host scan, direct kernel round trip, result formatting) and the batch path.

Usage: python tools/bench_latency.py [iters]
"""
import json
import os
import random
import statistics
import sys
import time

import msgpack
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def pct(xs):
    xs = sorted(xs)
    return {"p50": round(statistics.median(xs), 1), "p99": round(xs[int(0.99 * (len(xs) - 1))], 1),
            "min": round(xs[0], 1)}


def timeit(fn, iters):
    for _ in range(20):
        fn()
    out = []
    for _ in range(iters):
        t = time.perf_counter()
        fn()
        out.append((time.perf_counter() - t) * 1e6)
    return pct(out)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    import torch
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier
    from jubatus_amd.ops import hip

    dev = torch.device("cuda", 0)
    cfg = json.loads(json.dumps(bench.AROW_CONFIG))
    cfg["converter"]["hash_max_size"] = 1 << 20
    clf = LinearClassifier("AROW", cfg["parameter"], DatumToFvConverter(cfg["converter"]), device=dev)
    bodies = bench.make_requests(random.Random(1), 64, 128, 16, 8, 8, 100000)
    clf.train_requests(bodies)
    torch.cuda.synchronize()
    items = msgpack.unpackb(bodies[0], raw=False)
    one = msgpack.packb([items[0][1]], use_bin_type=False)
    eight = msgpack.packb([d for _, d in items[:8]], use_bin_type=False)
    res = {"datum_bytes": len(one)}
    res["classify_1"] = timeit(lambda: clf.classify_requests([one]), iters)
    res["classify_8"] = timeit(lambda: clf.classify_requests([eight]), iters)
    pipe = clf.pipe
    res["direct_1"] = timeit(lambda: pipe.classify_direct([one], clf.W), iters)
    d = pipe._direct
    hasher = d["hasher"]
    res["host_hash_1"] = timeit(lambda: hasher.hash([one], d["idx"].ctypes.data, d["val"].ctypes.data,
                                                    d["row_ptr"].ctypes.data, 32, 320), iters)

    def kr(stream=None):
        return lambda: hip.classify_direct(d["idx"].ctypes.data, d["val"].ctypes.data,
                                           d["row_ptr"].ctypes.data, 1, clf.W, d["out"], d["done"],
                                           stream=stream)
    ns = torch.cuda.Stream(device=dev)
    hs = torch.cuda.Stream(device=dev, priority=-1)
    for name, st in (("cur", None), ("new", ns.cuda_stream), ("hiprio", hs.cuda_stream)):
        res[f"kernel_roundtrip_{name}"] = timeit(kr(st), iters)
        res[f"empty_{name}_spin"] = timeit(lambda: hip.diag_empty(d["done"], True, st), iters)
        res[f"empty_{name}_sync"] = timeit(lambda: hip.diag_empty(d["done"], False, st), iters)
    sc = np.zeros((1, clf.LC), np.float32)
    res["format_1"] = timeit(lambda: clf._results(sc), iters)
    s = torch.cuda.current_stream()
    res["empty_sync"] = timeit(lambda: s.synchronize(), iters)
    # one train request (one update stream, exact sequential semantics)
    for nsamp in (1, 16, 128):
        body = msgpack.packb([[lab, d] for lab, d in items[:nsamp]], use_bin_type=False)

        def tr():
            clf.train_requests([body])
            torch.cuda.synchronize()
        res[f"train_1x{nsamp}_sync"] = timeit(tr, max(50, iters // 5))
    for nreq in (16, 64):
        bodies64 = [msgpack.packb([[lab, d] for lab, d in items[:128]], use_bin_type=False)] * nreq

        def trn():
            clf.train_requests(bodies64)
            torch.cuda.synchronize()
        res[f"train_{nreq}x128_sync"] = timeit(trn, 50)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b = clf.pipe.from_requests([body], True, clf.labels)
    torch.cuda.synchronize()
    ks = []
    for _ in range(30):
        ev0.record()
        clf._train_batch(b)
        ev1.record()
        torch.cuda.synchronize()
        ks.append(ev0.elapsed_time(ev1) * 1e3)
    res["train_kernel_1x128_us"] = round(statistics.median(ks), 1)
    clf.direct = False
    res["classify_1_batch_path"] = timeit(lambda: clf.classify_requests([one]), iters)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
