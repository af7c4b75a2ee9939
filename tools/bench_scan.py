"""Host scanner throughput (native pack_spans) vs worker-thread count."""
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from jubatus_amd._native import native  # noqa: E402


def main():
    nreq, per = int(sys.argv[1]) if len(sys.argv) > 1 else 1024, 128
    bodies = bench.make_requests(random.Random(1), nreq, per, 16, 8, 8, 100000)
    total = sum(len(b) for b in bodies)
    arena = np.zeros(total + 16 * nreq + 64, np.uint8)
    offs, lens, o = [], [], 0
    for b in bodies:
        o = (o + 15) & ~15
        arena[o:o + len(b)] = np.frombuffer(b, np.uint8)
        offs.append(o)
        lens.append(len(b))
        o += len(b)
    offs = np.asarray(offs, np.int64)
    lens = np.asarray(lens, np.int64)
    n = native()
    t = n.LabelTable()
    ns = nreq * per
    off = np.zeros(ns, np.int64)
    dl = np.zeros(ns, np.int32)
    lab = np.zeros(ns, np.int32)
    row = np.zeros(ns + 1, np.int64)
    sp = np.zeros(nreq + 1, np.int64)
    print(f"{ns} samples, {total / ns:.0f} B/sample, cpus={os.cpu_count()}")
    for th in (1, 2, 4, 8, 16, 32):
        best = 1e9
        for _ in range(5):
            t0 = time.perf_counter()
            r = n.pack_spans(arena.ctypes.data, offs.ctypes.data, lens.ctypes.data, nreq, True, 1, 1, t,
                             off.ctypes.data, dl.ctypes.data, lab.ctypes.data, row.ctypes.data, sp.ctypes.data, ns, th)
            best = min(best, time.perf_counter() - t0)
        assert r[3] == 0, r
        print(f"threads={th:2d}  {best * 1e3:7.2f} ms  {ns / best / 1e6:7.1f} M samples/s")


if __name__ == "__main__":
    main()
