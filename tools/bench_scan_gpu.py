"""GPU request scanner (csrc/hip/scan.hip) on the headline batch: kernel
time, and per-phase cycle counts (s_memtime at the phase boundaries of every
workgroup) from jb_scan_train_profile.

Usage: python tools/bench_scan_gpu.py [nreq] [per_request]
"""
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from jubatus_amd.fv_converter.converter import DatumToFvConverter  # noqa: E402
from jubatus_amd.models.classifier import LinearClassifier  # noqa: E402
from jubatus_amd.ops import hip  # noqa: E402
from jubatus_amd.ops.feature_pipeline import RequestArena, ScanCheck  # noqa: E402

PHASES = ["stage", "spec walk", "extend", "chain+mark", "depth+starts", "per-sample+row_ptr", "hist"]


def main():
    nreq = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 128
    dev = torch.device("cuda", 0)
    cfg = dict(bench.AROW_CONFIG)
    cfg["converter"] = dict(cfg["converter"], hash_max_size=1 << 20)
    clf = LinearClassifier("AROW", cfg["parameter"], DatumToFvConverter(cfg["converter"]), dev)
    for y in range(16):
        clf.set_label(f"label{y}")
    bodies = bench.make_requests(random.Random(1), nreq, per, 16, 8, 8, 100000)
    arena = RequestArena(sum(len(b) for b in bodies) + 16 * nreq + 64)
    for b in bodies:
        arena.append(b)
    offs, lens = arena.spans()
    pipe = clf.pipe
    chk = ScanCheck(64)
    for _ in range(3):
        pipe.from_arena_gpu(arena, offs, lens, clf.labels, chk)
    torch.cuda.synchronize()
    assert int(chk.err[0]) == 0
    # kernel-only timing through the profile entry point
    dset = pipe._gsets[pipe._gprev].bufs
    R = nreq
    n = nreq * per
    th, tm, tb = pipe.label_table(clf.labels)
    d_meta = dset.t["scan_meta"]
    prof = torch.zeros(8 * R, dtype=torch.int64, device=dev)
    args = lambda p: (hip._p(dset.t["buf"]), hip._p(d_meta), d_meta.data_ptr() + 8 * R,  # noqa: E731
                      d_meta.data_ptr() + 16 * R, R, hip._p(th), hip._p(tm), th.numel(), hip._p(tb),
                      tb.numel(), pipe.rules.n_srules, pipe.rules.n_nrules,
                      hip._p(dset.t["datum_off"]), hip._p(dset.t["datum_len"]),
                      hip._p(dset.t["labels"]), hip._p(dset.t["row_ptr"]),
                      hip._p(dset.t["req_slots"]), hip._p(dset.t["label_hist"]), 64,
                      hip._p(dset.t["scan_err"]), p, hip._stream())
    fn = hip._fn("jb_scan_train_profile")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(10):
        e0.record()
        fn(*args(None))
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3)
    fn(*args(prof.data_ptr()))
    torch.cuda.synchronize()
    P = prof.view(R, 8).cpu().numpy().astype(np.int64)
    order = [6, 0, 1, 2, 3, 4, 5, 7]
    d = np.diff(P[:, order], axis=1)
    print(f"{nreq} requests x {per} samples, {sum(lens) / nreq:.0f} B/request: "
          f"scan kernel {best:.1f} us (best of 10)")
    for name, col in zip(PHASES, d.T):
        print(f"  {name:20s} mean {col.mean():9.0f}  max {col.max():9.0f} cycles")
    print(f"  {'total':20s} mean {d.sum(1).mean():9.0f}  max {d.sum(1).max():9.0f} cycles")


if __name__ == "__main__":
    main()
