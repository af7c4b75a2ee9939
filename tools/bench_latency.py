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
    from jubatus_amd._native import native
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
    nat = native()
    res["scan_1"] = timeit(lambda: nat.pack_requests(
        [one], False, pipe.rules.n_srules, pipe.rules.n_nrules, None, d["staging"].data_ptr(),
        d["staging"].numel(), d["datum_off"].data_ptr(), d["datum_len"].data_ptr(), 0,
        d["row_ptr"].data_ptr(), d["stream_ptr"].data_ptr(), hip.DIRECT_MAX_SAMPLES, 1), iters)
    n, nbytes = 1, len(one)
    res["kernel_roundtrip_1"] = timeit(lambda: hip.classify_direct(
        d["staging"].data_ptr(), nbytes, d["datum_off"].data_ptr(), d["datum_len"].data_ptr(),
        d["row_ptr"].data_ptr(), n, pipe.d_srules, pipe.rules.n_srules, pipe.d_nrules,
        pipe.rules.n_nrules, pipe.d_blob, pipe.H, clf.W, d["out"], d["err"], d["done"]), iters)
    sc = np.zeros((1, clf.LC), np.float32)
    res["format_1"] = timeit(lambda: clf._results(sc), iters)
    s = torch.cuda.current_stream()
    res["empty_sync"] = timeit(lambda: s.synchronize(), iters)
    clf.direct = False
    res["classify_1_batch_path"] = timeit(lambda: clf.classify_requests([one]), iters)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
