"""Latency of the signature-table top-k of the LSH latency path
(csrc/hip/topk.hip jb_topk_direct_query_path) at 1M rows: tile path (scan +
per-block top-k, then a merge of blocks x k candidates) vs one launch
(topk_fused_kernel). Random 64-bit signatures, euclid_lsh (metric 1) and lsh
(metric 0). Both paths must return the same rows. One JSON line per case."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jubatus_amd.ops import hip  # noqa: E402


def run(t, nq, n, k, metric, path, bufs):
    qbd, qnd, tbd, tnd, vd = t
    sd, si = hip._topk_scratch(tbd.device, hip._direct_scratch(n, k, nq))
    rc = hip._fn("jb_topk_direct_query_path")(hip._p(qbd), hip._p(qnd), nq, hip._p(tbd), hip._p(tnd),
                                              hip._p(vd), n, 1, 64, metric, k, hip._p(sd), hip._p(si),
                                              bufs.out_d.ptr, bufs.out_i.ptr, bufs.done.ptr, path,
                                              hip._stream())
    hip._check(rc, "jb_topk_direct_query_path")
    return bufs.out_i.view(np.int32, nq * k).reshape(nq, k).copy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--cases", default="1:10,4:10,1:100", help="nq:k pairs")
    ap.add_argument("--paths", default="tile,fused,onepass,select,default")
    ap.add_argument("--metrics", default="1,0")
    a = ap.parse_args()
    cases = [tuple(int(x) for x in c.split(":")) for c in a.cases.split(",")]
    paths = [p for p in (("tile", 0), ("fused", 2), ("onepass", 3), ("select", 4), ("default", -1))
             if p[0] in a.paths.split(",")]
    d = torch.device("cuda", 0)
    n = a.rows
    g = torch.Generator().manual_seed(0)
    tb = torch.randint(-2**62, 2**62, (n, 1), generator=g, dtype=torch.int64)
    tn = torch.rand(n, generator=g)
    valid = torch.ones(n, dtype=torch.uint8)
    bufs = hip.DirectQueryBuffers(d, 1)
    for metric in (int(m) for m in a.metrics.split(",")):
        for nq, k in cases:
            qb = torch.randint(-2**62, 2**62, (nq, 1), generator=g, dtype=torch.int64)
            qn = torch.rand(nq, generator=g)
            t = tuple(x.to(d) for x in (qb, qn, tb, tn, valid))
            ref = None
            for name, path in paths:
                if path == 3 and k > 16:
                    continue
                lat = []
                for it in range(a.iters + 20):
                    t0 = time.perf_counter()
                    idx = run(t, nq, n, k, metric, path, bufs)
                    if it >= 20:
                        lat.append((time.perf_counter() - t0) * 1e6)
                if ref is None:
                    ref = idx
                print(json.dumps({"rows": n, "metric": metric, "nq": nq, "k": k, "path": name,
                                  "fuse_rows": os.environ.get("JB_FUSE_ROWS", ""),
                                  "p50_us": round(float(np.median(lat)), 1),
                                  "p90_us": round(float(np.percentile(lat, 90)), 1),
                                  "same_rows_as_tile": bool(np.array_equal(idx, ref)),
                                  "table_mb": round(n * 13 / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
