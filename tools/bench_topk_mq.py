"""Multi-query similarity scan (fused signature scan + exact top-k, topk.hip):
time per call and the table bytes it streams per second, for 1..16 queries.
Run once with JB_TOPK_MQ=0 (the previous kernels: topk_wq_kernel for 2..16
queries, topk_kernel for one) and once without (topk_mq_kernel) for an A/B.

Usage: python tools/bench_topk_mq.py [--rows 10000000] [--iters 30]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jubatus_amd.ops import hip  # noqa: E402


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--quick", action="store_true", help="64-bit tables, 1 and 8 queries, k 10")
    a = ap.parse_args()
    d = torch.device("cuda", 0)
    g = torch.Generator(device=d).manual_seed(0)
    n = a.rows
    mq = os.environ.get("JB_TOPK_MQ", "1") != "0"
    for bits in ((64,) if a.quick else (64, 128)):
        words = bits // 64
        tb = torch.randint(-2**62, 2**62, (n, words), device=d, dtype=torch.int64, generator=g)
        tn = torch.rand(n, device=d, generator=g) + 0.5
        valid = torch.ones(n, dtype=torch.uint8, device=d)
        for metric in (0, 1):
            for nq in ((1, 8) if a.quick else (1, 2, 4, 8, 16)):
                qb = torch.randint(-2**62, 2**62, (nq, words), device=d, dtype=torch.int64, generator=g)
                qn = torch.rand(nq, device=d, generator=g) + 0.5
                for k in ((10,) if a.quick else (10, 31)):
                    us = timeit(lambda: hip.topk_hamming(qb, qn, nq, tb, tn, valid, n, bits, metric, k),
                                a.iters)
                    table = n * (8 * words + 1 + (4 if metric == 1 else 0))
                    stats = {}
                    if os.environ.get("JB_TOPK_MQ_STATS") == "1":
                        hip.topk_mq_stats()
                        hip.topk_hamming(qb, qn, nq, tb, tn, valid, n, bits, metric, k)
                        sv = hip.topk_mq_stats()
                        stats = {"survivor_passes": sv[0], "chunks": sv[1], "first_cuts": sv[2], "pops": sv[3]}
                    print(json.dumps({"mq": mq, "rows": n, "bits": bits, "metric": metric, "nq": nq, "k": k,
                                      "us": round(us, 1), "table_GBps": round(table / us / 1e3, 1),
                                      "queries_per_s": round(nq / us * 1e6), **stats}), flush=True)
        del tb, tn, valid
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
