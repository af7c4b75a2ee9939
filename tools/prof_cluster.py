"""Phase profile of the native jubaclustering push path (one GPU): the
server runs with JB_CLUSTER_PROF=1 and logs, every 50 closed buckets, the
wall time per bucket of compress / merge-compress / k-means++ / Lloyd / EM;
the push stream is bench.py's clustering record (1000-point requests of
three blobs, pushed by jubaloadgen).

Usage: python tools/prof_cluster.py [--method gmm] [--points 200000] [--out LOG]
"""
import argparse
import json
import os
import shlex
import subprocess
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="gmm")
    ap.add_argument("--points", type=int, default=200_000)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import msgpack
    import numpy as np

    import bench
    from jubatus_amd.common.mprpc import RpcClient
    root = bench.ROOT
    exe = os.path.join(root, "jubatus_amd", "native_bin", "jubaloadgen")
    srv = os.path.join(root, "jubatus_amd", "native_bin", "jubaclustering")
    cfg = os.path.join(root, "config", "clustering", f"{a.method}.json")
    tmp = tempfile.mkdtemp()
    rng = np.random.default_rng(5)
    centers = np.array([[0.0, 0.0, 0.0], [10.0, 10.0, 0.0], [-10.0, 10.0, 5.0]])
    push = os.path.join(tmp, "push.bin")
    with open(push, "wb") as f:
        for b in range(0, a.points, 1000):
            pts = []
            for i in range(1000):
                c = centers[(b + i) % 3] + rng.normal(0, 0.5, 3)
                pts.append([[["tag", f"t{(b + i) % 7}"]], [["a", float(c[0])], ["b", float(c[1])],
                                                          ["c", float(c[2])]], []])
            f.write(msgpack.packb(["", pts], use_bin_type=False))
    port = bench._free_port()
    log = a.out or os.path.join(tmp, "server.log")
    env = dict(os.environ, JB_CLUSTER_PROF="1")
    with open(log, "w") as lf:
        # JB_SERVED_WRAP: a command prefix for the server (e.g. rocprofv3 ... --)
        wrap = shlex.split(os.environ.get("JB_SERVED_WRAP", ""))
        p = subprocess.Popen(wrap + [srv, "-p", str(port), "-b", "127.0.0.1", "-f", cfg, "-d", tmp, "-c", "4"],
                             stdout=lf, stderr=lf, env=env)
        try:
            deadline = time.time() + 60
            while True:
                try:
                    with RpcClient("127.0.0.1", port, 30.0) as c:
                        c.call("get_status", "")
                    break
                except Exception:  # noqa: BLE001 - not listening yet
                    if p.poll() is not None or time.time() > deadline:
                        raise
                    time.sleep(0.2)
            t0 = time.perf_counter()
            r = bench._loadgen(exe, port, "push", push, 1, 2, once=True)
            dt = time.perf_counter() - t0
            print(json.dumps({"method": a.method, "points": a.points, "push_points_per_s": round(a.points / dt),
                              "push_rpc_p50_us": r["p50_us"]}), flush=True)
        finally:
            p.terminate()
            p.wait(timeout=90)
    with open(log) as lf:
        lines = [ln.strip() for ln in lf if "cluster prof" in ln]
    if lines:
        print(lines[-1], flush=True)


if __name__ == "__main__":
    main()
