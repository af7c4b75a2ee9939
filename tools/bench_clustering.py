"""push throughput of the clustering engine (config/clustering/{kmeans,gmm}.json)
in process: msgpack list<datum> bodies of `--batch` points through
Clustering.push_body (the server's raw push path), on the GPU when present.

Usage: python tools/bench_clustering.py [--points 200000] [--batch 1000] [--method kmeans]
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=200_000)
    ap.add_argument("--batch", type=int, default=1000)
    ap.add_argument("--method", default="kmeans")
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    import msgpack
    import torch
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.clustering import Clustering
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = json.load(open(os.path.join(root, "config", "clustering", f"{a.method}.json")))
    dev = None if a.cpu or not torch.cuda.is_available() else torch.device("cuda", 0)
    c = Clustering(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]), dev)
    r = random.Random(0)
    centers = [(0.0, 0.0, 0.0), (10.0, 10.0, 0.0), (-10.0, 10.0, 5.0)]
    bodies = []
    for b in range(0, a.points, a.batch):
        pts = []
        for i in range(a.batch):
            cx = centers[(b + i) % 3]
            pts.append([[["tag", f"t{(b + i) % 7}"]],
                        [["a", cx[0] + r.gauss(0, 0.5)], ["b", cx[1] + r.gauss(0, 0.5)],
                         ["c", cx[2] + r.gauss(0, 0.5)]], []])
        bodies.append(msgpack.packb(pts, use_bin_type=True))
    c.push_body(bodies[0])
    if dev is not None:
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for b in bodies[1:]:
        c.push_body(b)
    if dev is not None:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = a.batch * (len(bodies) - 1)
    print(json.dumps({"method": a.method, "points": n, "seconds": round(dt, 3),
                      "points_per_s": round(n / dt, 1), "revision": c.get_revision(),
                      "device": str(dev) if dev is not None else "cpu",
                      "converter": c.get_status()["converter"]}))


if __name__ == "__main__":
    main()
