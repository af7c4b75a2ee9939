"""Latency of the score-vector top-k (csrc/hip/topk.hip
jb_topk_scores_direct_path, the inverted-index recommender / LOF query
tail) on synthetic score vectors: a fraction of rows with a nonzero cosine
score (the rest 0, distance 1 after the flip), continuous or quantized
(ties). Paths: tile (scan + merge), chain (radix hist / select x2, collect,
rank: 6 launches + a memset), fused (one launch). Exactness against a
stable (distance, row) sort. One JSON line per case."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jubatus_amd.ops import hip  # noqa: E402

PATHS = {"tile": 0, "chain": 1, "fused": 2, "onepass": 3, "select": 4, "default": -1}


def run(sc, nq, rows, k, path, bufs):
    sd, si = hip._topk_scratch(sc.device, hip._direct_scratch(rows, k, nq))
    rc = hip._fn("jb_topk_scores_direct_path")(hip._p(sc), 1, nq, rows, k, hip._p(sd), hip._p(si),
                                               bufs.out_d.ptr, bufs.out_i.ptr, bufs.done.ptr,
                                               PATHS[path], hip._stream())
    hip._check(rc, "jb_topk_scores_direct_path")
    d = bufs.out_d.view(np.float32, nq * k).reshape(nq, k).copy()
    i = bufs.out_i.view(np.int32, nq * k).reshape(nq, k).copy()
    return d, i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--paths", default="chain,fused,onepass,default")
    a = ap.parse_args()
    d = torch.device("cuda", 0)
    bufs = hip.DirectQueryBuffers(d, 8)
    g = torch.Generator(device=d).manual_seed(0)
    for nq, k in ((1, 10), (1, 100), (4, 10)):
        for frac in (0.01, 0.2):
            for levels in (0, 64):
                sc = torch.zeros(nq, a.rows, device=d)
                m = torch.rand(nq, a.rows, device=d, generator=g) < frac
                v = torch.rand(nq, a.rows, device=d, generator=g)
                if levels:
                    v = torch.ceil(v * levels) / levels
                sc[m] = v[m]
                dist_ref = (1.0 - sc).cpu().numpy()
                ref_i = [np.lexsort((np.arange(a.rows), dist_ref[q]))[:k] for q in range(nq)]
                for path in a.paths.split(","):
                    if path == "onepass" and k > 16:
                        continue
                    torch.cuda.synchronize()
                    lat = []
                    ok = True
                    for it in range(a.iters + 20):
                        t0 = time.perf_counter()
                        dist, idx = run(sc, nq, a.rows, k, path, bufs)
                        if it >= 20:
                            lat.append((time.perf_counter() - t0) * 1e6)
                        if it in (0, a.iters + 19):
                            ok &= all(np.array_equal(idx[q], ref_i[q]) for q in range(nq))
                    print(json.dumps({"rows": a.rows, "nq": nq, "k": k, "nonzero_frac": frac,
                                      "levels": levels, "path": path,
                                      "p50_us": round(float(np.median(lat)), 1),
                                      "p90_us": round(float(np.percentile(lat, 90)), 1),
                                      "exact": bool(ok)}), flush=True)


if __name__ == "__main__":
    main()
