"""Batched LOF adds on the device without the server (csrc/hip/lof.hip
jb_lof_add_many -> lof_add_batch_kernel): a table of `rows` rows with valid
k-nearest lists, then batches of adds of fresh rows, each with `rnn`
candidates drawn from the table. Prints the wall time per add and the
kernel's phase stamps (shader cycles per add: candidates to LDS, list loads,
edits, write-back, score loads, score, host copy).

Usage: python tools/bench_lof_kernel.py [--rows 100000] [--batch 32] [--batches 200]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jubatus_amd.ops import hip  # noqa: E402

PHASES = ["cand_lds", "list_loads", "edits", "write_back", "unused", "score_loads", "score", "host_copy"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--rnn", type=int, default=30)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--batches", type=int, default=200)
    a = ap.parse_args()
    d = torch.device("cuda", 0)
    n, k, rnn, B = a.rows, a.k, a.rnn, a.batch
    cap = n + B * a.batches + 1024
    g = torch.Generator(device=d).manual_seed(0)
    # valid lists for the stored rows: k random neighbours at ascending distances
    nb_slot = torch.full((cap, k), -1, dtype=torch.int32, device=d)
    nb_dist = torch.full((cap, k), float("inf"), dtype=torch.float32, device=d)
    nb_slot[:n] = torch.randint(0, n, (n, k), generator=g, device=d, dtype=torch.int32)
    nb_dist[:n] = torch.sort(torch.rand(n, k, generator=g, device=d) + 0.1, dim=1).values
    kdist = torch.zeros(cap, dtype=torch.float32, device=d)
    kdist[:n] = nb_dist[:n, -1]
    lrd = torch.ones(cap, dtype=torch.float32, device=d)
    ok = torch.zeros(cap, dtype=torch.uint8, device=d)
    ok[:n] = 1
    lrd_ok = ok.clone()
    kstamp = torch.zeros(cap, dtype=torch.int32, device=d)
    lstamp = torch.zeros(cap, dtype=torch.int32, device=d)
    changed = torch.zeros(1024, dtype=torch.int32, device=d)
    nchanged = torch.zeros(1, dtype=torch.int32, device=d)
    cand = torch.zeros(2 * 64 * 128, dtype=torch.int32, device=d)
    stride_out = 4 + 1024
    res = torch.zeros(64 * stride_out, dtype=torch.int32, device=d)
    prof = torch.zeros(16, dtype=torch.int64, device=d)
    stage = hip.HostBuffer(4 * (2 * 64 + 2 * 64 * 128))
    out = hip.HostBuffer(4 * 64 * stride_out)
    lib = hip.hip_lib()
    f = lib.jb_lof_add_many
    P, I, U = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint32
    f.argtypes = [I, P, P, P, P, I, I, I, P, P, P, P, P, P, P, P, P, P, U, P, P, P, I, I, P, P, I, P]
    f.restype = I
    rng = np.random.default_rng(1)
    hps = stage.view(np.int32, 64)
    hnc = stage.view(np.int32, 64, 4 * 64)
    hcs = stage.view(np.int32, B * rnn, 4 * 128)
    hcd = stage.view(np.float32, B * rnn, 4 * 128 + 4 * B * rnn)
    status = out.view(np.uint32, 64 * stride_out)
    torch.cuda.synchronize()
    times = []
    epoch = 1
    for b in range(a.batches + 5):
        p0 = n + b * B
        hps[:B] = np.arange(p0, p0 + B, dtype=np.int32)
        hnc[:B] = rnn
        hcs[:] = np.concatenate([rng.choice(n, rnn, replace=False) for _ in range(B)]).astype(np.int32)
        hcd[:] = np.sort(rng.random((B, rnn), dtype=np.float32) + 0.05, axis=1).reshape(-1)
        if b == 5:
            prof.zero_()
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = f(B, stage.ptr, stage.ptr + 4 * 128, stage.ptr + 4 * 128 + 4 * B * rnn, stage.ptr + 4 * 64, rnn, k, 0,
               nb_slot.data_ptr(), nb_dist.data_ptr(), kdist.data_ptr(), ok.data_ptr(), lrd.data_ptr(),
               lrd_ok.data_ptr(), changed.data_ptr(), nchanged.data_ptr(), kstamp.data_ptr(), lstamp.data_ptr(),
               epoch, cand.data_ptr(), res.data_ptr(), out.ptr, stride_out, 1024,
               prof.data_ptr() if b >= 5 else None, hip._stream(), 1, None)
        times.append(time.perf_counter() - t0)
        epoch += B
        if rc != 0:
            raise SystemExit(f"jb_lof_add_many rc={rc}")
        st = status[::stride_out][:B]
        if b >= 5 and not np.all(st == 1):
            print(json.dumps({"batch": b, "statuses": np.unique(st).tolist()}))
    torch.cuda.synchronize()
    pr = prof.cpu().numpy()
    adds = max(1, int(pr[8]))
    # s_memtime runs at the shader clock; the wall time per add calibrates it
    us = float(np.median(times[5:])) * 1e6
    cyc = {PHASES[i]: round(float(pr[i]) / adds, 1) for i in range(8)}
    tot = sum(cyc.values())
    print(json.dumps({"rows": n, "k": k, "rnn": rnn, "batch": B, "wall_us_per_batch": round(us, 1),
                      "wall_us_per_add": round(us / B, 2), "cycles_per_add": cyc,
                      "cycles_per_add_total": round(tot, 1),
                      "share": {kk: round(v / tot, 3) for kk, v in cyc.items()} if tot else {}}))


if __name__ == "__main__":
    main()
