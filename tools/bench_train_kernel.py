"""Micro-benchmark of the linear train kernel alone (no host scan / H2D).

Builds one device batch per variant with the real pipeline, then times
``hip.linear_train`` with HIP events. Variants isolate what bounds the
kernel: update mode (atomic / hogwild / exact single stream), stream count,
numeric (always-present, hot) features vs string-only data.

Each variant also runs with the hot-row LDS replica off (``nohot``) and on:
the replica is what removes the hot-row atomic contention
(csrc/hip/hot.hip, linear.hip "Hot rows").

Usage: python tools/bench_train_kernel.py [--iters N] [--only SUBSTR]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys

import msgpack

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make(rng, nreq, per, nlab, n_str, n_num, vocab, hot=16):
    """hot = 0: noise strings (every sample updates; the worst case)"""
    bodies = []
    for _ in range(nreq):
        items = []
        for _ in range(per):
            y = rng.randrange(nlab)
            if hot == 0:
                sv = [[f"s{j}", f"z{rng.getrandbits(40)}"] for j in range(n_str)]
            else:
                sv = [[f"s{j}", f"t{(y * 131 + rng.randrange(hot)) if rng.random() < 0.6 else rng.randrange(vocab)}"]
                      for j in range(n_str)]
            nv = [[f"n{j}", (y - nlab / 2) * 0.05 + rng.gauss(0.0, 1.0)] for j in range(n_num)]
            items.append([f"label{y}", [sv, nv, []]])
        bodies.append(msgpack.packb(items, use_bin_type=False))
    return bodies


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="run the variants whose name contains this")
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch

    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier
    from jubatus_amd.ops import hip

    dev = torch.device("cuda", 0)
    conv = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
            "num_rules": [{"key": "*", "type": "num"}], "hash_max_size": 1 << 20}
    variants = [
        ("atomic 1024x128 8s+8n", "atomic", 1024, 128, 8, 8, 16),
        ("atomic 1024x128 8s+8n worst", "atomic", 1024, 128, 8, 8, 0),
        ("hogwild 1024x128 8s+8n", "hogwild", 1024, 128, 8, 8, 16),
        ("atomic 1024x128 16s cold", "atomic", 1024, 128, 16, 0, 100000),
        ("atomic 1024x128 8s+8n cold-str", "atomic", 1024, 128, 8, 8, 100000),
        ("hogwild 1024x128 8s+8n cold-str", "hogwild", 1024, 128, 8, 8, 100000),
        ("atomic 1024x128 8s+1n cold-str", "atomic", 1024, 128, 8, 1, 100000),
        ("atomic 64x128 8s+8n cold-str", "atomic", 64, 128, 8, 8, 100000),
        ("atomic 4096x32 8s+8n", "atomic", 4096, 32, 8, 8, 16),
        ("atomic 256x512 8s+8n", "atomic", 256, 512, 8, 8, 16),
        ("exact 1x2048 8s+8n", "exact", 1, 2048, 8, 8, 16),
    ]
    out = []
    for name, mode, nreq, per, ns, nn, hot in variants:
        if args.only and args.only not in name:
            continue
        bodies = make(random.Random(1), nreq, per, 16, ns, nn, 100000, hot)
        for use_hot in (False, True):
            if use_hot and mode == "exact":
                continue
            clf = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(conv),
                                   device=dev, concurrent_update=mode if mode != "exact" else "atomic")
            clf.hot_rows = use_hot
            for y in range(16):
                clf.set_label(f"label{y}")
            b = clf.pipe.from_requests(bodies, True, clf.labels)
            clf._sync_labels()
            if mode == "exact":
                clf._mode = lambda n: hip.UPDATE_EXACT
            # fresh model per timed launch would need a reset; every launch
            # re-trains the same batch, so report the first launch separately
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            st0 = clf.train_stats()
            e0.record()
            clf._launch_train(b)
            e1.record()
            torch.cuda.synchronize()
            first_us = e0.elapsed_time(e1) * 1e3
            st1 = clf.train_stats()
            e0.record()
            for _ in range(args.iters):
                clf._launch_train(b)
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / args.iters
            st2 = clf.train_stats()
            nsamp = nreq * per
            rec = {"variant": name + (" hot" if use_hot else " nohot"), "first_us": round(first_us, 1),
                   "first_update_fraction": round((st1["updated"] - st0["updated"]) / nsamp, 3),
                   "us_per_launch": round(us, 1), "samples": nsamp,
                   "update_fraction": round((st2["updated"] - st1["updated"]) / nsamp / args.iters, 3),
                   "Msamples_per_s": round(nsamp / us, 1)}
            out.append(rec)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
