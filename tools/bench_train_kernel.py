"""Micro-benchmark of the linear train kernel alone (no host scan / H2D).

Builds one device batch per variant with the real pipeline, then times
``hip.linear_train`` with HIP events. Variants isolate what bounds the
kernel: update mode (atomic / hogwild / exact single stream), stream count,
numeric (always-present, hot) features vs string-only data.

Usage: python tools/bench_train_kernel.py [--iters N]
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
    bodies = []
    for _ in range(nreq):
        items = []
        for _ in range(per):
            y = rng.randrange(nlab)
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
        clf = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(conv),
                               device=dev)
        for y in range(16):
            clf.set_label(f"label{y}")
        bodies = make(random.Random(1), nreq, per, 16, ns, nn, 100000, hot)
        b = clf.pipe.from_requests(bodies, True, clf.labels)
        clf._sync_labels()
        m = hip.UPDATE_MODES.get(mode, hip.UPDATE_EXACT)
        run = lambda: hip.linear_train(b.row_ptr, b.fidx, b.fval, b.labels, b.stream_ptr, b.nstreams,
                                       clf.W, clf.P, clf.active, clf.mid, clf.C, mode=m)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.iters
        nsamp = nreq * per
        rec = {"variant": name, "us_per_launch": round(us, 1), "samples": nsamp,
               "ns_per_sample_per_stream": round(us * 1e3 / per, 1),
               "Msamples_per_s": round(nsamp / us, 1)}
        out.append(rec)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
