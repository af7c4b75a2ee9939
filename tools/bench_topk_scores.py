"""Latency of the score-vector top-k (csrc/hip/topk.hip jb_topk_scores_direct,
the inverted-index recommender / LOF query tail) on synthetic score vectors
of 1M rows: a fraction of rows with a nonzero cosine score (the rest 0,
distance 1 after the flip), continuous or quantized (ties). Radix chain vs
the tile path (JB_TOPK_SCORES_TILE). One JSON line per case."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jubatus_amd.ops import hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--radix-only", action="store_true")
    a = ap.parse_args()
    d = torch.device("cuda", 0)
    bufs = hip.DirectQueryBuffers(d, 1)
    g = torch.Generator(device=d).manual_seed(0)
    for frac in (0.01, 0.2):
        for levels in (0, 64):
            sc = torch.zeros(a.rows, device=d)
            m = torch.rand(a.rows, device=d, generator=g) < frac
            v = torch.rand(a.rows, device=d, generator=g)
            if levels:
                v = torch.ceil(v * levels) / levels
            sc[m] = v[m]
            ref = torch.topk(1.0 - sc, a.k, largest=False)
            for path in (("radix",) if a.radix_only else ("radix", "tile")):
                if path == "tile":
                    os.environ["JB_TOPK_SCORES_TILE"] = "1"
                else:
                    os.environ.pop("JB_TOPK_SCORES_TILE", None)
                torch.cuda.synchronize()
                lat = []
                for it in range(a.iters + 20):
                    t0 = time.perf_counter()
                    dist, _ = hip.topk_scores_direct(sc, 1, a.rows, a.k, True, bufs)
                    if it >= 20:
                        lat.append((time.perf_counter() - t0) * 1e6)
                ok = bool(np.allclose(dist[0], ref.values.cpu().numpy(), atol=1e-6))
                print(json.dumps({"radix_blocks": os.environ.get("JB_RADIX_BLOCKS", "512"),
                                  "rows": a.rows, "k": a.k, "nonzero_frac": frac, "levels": levels,
                                  "path": path, "p50_us": round(float(np.median(lat)), 1),
                                  "p90_us": round(float(np.percentile(lat, 90)), 1),
                                  "exact": ok}), flush=True)
    os.environ.pop("JB_TOPK_SCORES_TILE", None)


if __name__ == "__main__":
    main()
