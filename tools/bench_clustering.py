"""push throughput of the clustering engine (config/clustering/{kmeans,gmm}.json)
in process: msgpack list<datum> bodies of `--batch` points through
Clustering.push_body (the server's raw push path), on the GPU when present.
With --native the same bodies go as pre-encoded push requests over one TCP
connection to the native server (native_bin/jubaclustering), one in flight.

Usage: python tools/bench_clustering.py [--points 200000] [--batch 1000] [--method kmeans] [--native]
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
    ap.add_argument("--native", action="store_true")
    a = ap.parse_args()
    import msgpack
    import torch
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.clustering import Clustering
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cfg = json.load(open(os.path.join(root, "config", "clustering", f"{a.method}.json")))
    dev = None if a.cpu or not torch.cuda.is_available() else torch.device("cuda", 0)
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
    if a.native:
        return native(a, cfg, bodies)
    c = Clustering(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]), dev)
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


def native(a, cfg, bodies):
    import socket
    import subprocess
    import tempfile

    import msgpack
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    tmp = tempfile.mkdtemp()
    path = os.path.join(tmp, "c.json")
    with open(path, "w") as f:
        json.dump(cfg, f)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = subprocess.Popen([os.path.join(root, "jubatus_amd", "native_bin", "jubaclustering"), "-p", str(port),
                          "-b", "127.0.0.1", "-d", tmp, "-f", path])
    try:
        for _ in range(600):
            try:
                conn = socket.create_connection(("127.0.0.1", port))
                break
            except OSError:
                time.sleep(0.1)
        conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        up = msgpack.Unpacker(raw=False)

        def call(msgid, frame):
            conn.sendall(frame)
            while True:
                for resp in up:
                    assert resp[1] == msgid and resp[2] is None, resp
                    return resp[3]
                up.feed(conn.recv(1 << 20))

        # [0, msgid, "push", ["", body]] with the body spliced in as is
        frames = [b"\x94\x00" + msgpack.packb(i) + msgpack.packb("push") + b"\x92\xa0" + b
                  for i, b in enumerate(bodies)]
        call(0, frames[0])
        t0 = time.perf_counter()
        for i in range(1, len(frames)):
            call(i, frames[i])
        dt = time.perf_counter() - t0
        rev = call(len(frames), b"\x94\x00" + msgpack.packb(len(frames)) + msgpack.packb("get_revision")
                   + b"\x91\xa0")
        conn.close()
    finally:
        p.terminate()
        p.wait(timeout=30)
    n = a.batch * (len(bodies) - 1)
    print(json.dumps({"method": a.method, "points": n, "seconds": round(dt, 3),
                      "points_per_s": round(n / dt, 1), "revision": rev, "server": "native"}))


if __name__ == "__main__":
    main()
