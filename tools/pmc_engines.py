"""Short driver for PMC passes over the similarity kernels (rocprofv3
--pmc reruns the whole program once per counter set, so this builds its
tables directly on the device instead of ingesting datums):

* LSH signature table of 10M rows (64-bit signatures), fused scan + top-k
  for 1 and 8 queries, k 10 (csrc/hip/topk.hip);
* inverted-index pool of 1M rows x ~12 entries, scan + radix top-k
  (csrc/hip/sparse_pool.hip, topk.hip).

Usage: python tools/pmc_engines.py [--lsh-rows N] [--pool-rows N] [--iters N]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--lsh-rows", type=int, default=10_000_000)
    ap.add_argument("--pool-rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    import torch
    from jubatus_amd.models.similarity import InvertedIndex, LshIndex
    from jubatus_amd.ops import hip
    dev = torch.device("cuda", 0)
    out = {}
    # ---- LSH table
    n = args.lsh_rows
    ix = LshIndex("euclid_lsh", 64, 1091, dev)
    ix._alloc(n)
    g = torch.Generator(device=dev).manual_seed(1)
    ix.bits.copy_(torch.randint(-2**62, 2**62, (n, 1), generator=g, device=dev, dtype=torch.int64))
    ix.norms.copy_(torch.rand(n, generator=g, device=dev) + 0.5)
    ix.valid.fill_(1)
    rng = np.random.default_rng(2)
    for nq in (1, 8):
        rows = [(rng.integers(0, 1 << 20, 12).tolist(), rng.standard_normal(12).tolist())
                for _ in range(nq)]
        ix.query(rows, n, 10, similar=False)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(args.iters):
            ix.query(rows, n, 10, similar=False)
        torch.cuda.synchronize()
        out[f"lsh_{n}_q{nq}_k10_us"] = round((time.perf_counter() - t) / args.iters * 1e6, 1)
    del ix
    torch.cuda.empty_cache()
    # ---- inverted-index pool
    m = args.pool_rows
    ii = InvertedIndex(True, dev)
    per = 12
    for b in range(0, m, 262144):
        e = min(m, b + 262144)
        k = e - b
        rp = np.arange(k + 1, dtype=np.int64) * per
        idx = rng.integers(0, 1 << 16, k * per).astype(np.int32)
        val = rng.standard_normal(k * per).astype(np.float32)
        ii.set_rows_csr(np.arange(b, e, dtype=np.int64), rp, idx, val)
    q = (rng.integers(0, 1 << 16, per).astype(np.int32), rng.standard_normal(per).astype(np.float32))
    qrp = np.asarray([0, per], np.int64)
    for k in (10, 31):
        ii.query_direct(q[0], q[1], qrp, 1, m, k, False)
        t = time.perf_counter()
        for _ in range(args.iters):
            ii.query_direct(q[0], q[1], qrp, 1, m, k, False)
        out[f"pool_{m}_q1_k{k}_us"] = round((time.perf_counter() - t) / args.iters * 1e6, 1)
    print(json.dumps(out), flush=True)
    assert hip.POOL_MAX_Q == 8


if __name__ == "__main__":
    main()
