#!/usr/bin/env python3
"""Headline benchmark: AROW classifier training throughput (samples/s) +
p50/p99 classify latency on MI355X, 1..N GPUs (one rank per GPU, RCCL MIX).

Metric/config: BASELINE.json - "samples/sec (train) + p50 classify latency,
AROW classifier at 1/2/4/8 MI355X", config/classifier/arow.json
(AROW, regularization_weight 1.0, converter str bin/bin + num).

One timed step on every rank =
  * R concurrent ``train`` request bodies (msgpack list<labeled_datum>, as
    the RPC reader leaves them in a pinned receive arena) of S samples each:
    header pass (host), one H2D copy of the raw bytes, GPU request scan
    (csrc/hip/scan.hip: sample boundaries, label ids, validation), GPU
    msgpack parse + feature hashing (fv_hash), GPU AROW update (R lock-free
    update streams, each exact-sequential) - the train path minus the socket.
    Batches the device scan rejects (new labels, ...) are re-run through the
    host scanner; the RPC server itself still feeds its (smaller, latency-
    bound) batches through the host scanner, see docs/PERFORMANCE.md;
  * the MIX: label-set agreement (host gloo group) + RCCL all-reduce mean
    of W and P (hash_max_size x labels x 2 tables, fp32) over xGMI (N > 1),
    overlapped: the all-reduce of a snapshot runs on the communicator stream
    during the following steps and is folded in as W += mean(snapshot) -
    snapshot, so no update is lost; a new MIX starts as soon as the previous
    one finished (the reference's trigger); ``--mix-mode sync`` blocks.
Per-GPU work is fixed as N grows (weak scaling). Data: synthetic datums
(8 string + 8 numeric features, 16 labels), random-init (zero) model.

Usage: python bench.py --gpus N --steps K --warmup W
       (N > 1: launched by torch.distributed.run, one process per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

import msgpack
import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

AROW_CONFIG = {
    "converter": {
        "string_filter_types": {}, "string_filter_rules": [],
        "num_filter_types": {}, "num_filter_rules": [],
        "string_types": {},
        "string_rules": [{"key": "*", "type": "str", "sample_weight": "bin",
                          "global_weight": "bin"}],
        "num_types": {},
        "num_rules": [{"key": "*", "type": "num"}],
    },
    "parameter": {"regularization_weight": 1.0},
    "method": "AROW",
}


def make_requests(rng: random.Random, nreq: int, per_req: int, nlabels: int, n_str: int,
                  n_num: int, vocab: int) -> list[bytes]:
    """Synthetic, label-correlated datums, msgpack-encoded per request."""
    bodies = []
    for _ in range(nreq):
        items = []
        for _ in range(per_req):
            y = rng.randrange(nlabels)
            sv = []
            for j in range(n_str):
                tok = (y * 131 + rng.randrange(16)) if rng.random() < 0.6 else rng.randrange(vocab)
                sv.append([f"s{j}", f"t{tok}"])
            nv = [[f"n{j}", (y - nlabels / 2) * 0.05 + rng.gauss(0.0, 1.0)] for j in range(n_num)]
            items.append([f"label{y}", [sv, nv, []]])
        bodies.append(msgpack.packb(items, use_bin_type=False))
    return bodies


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--requests", type=int, default=1024, help="concurrent train requests per step per GPU")
    ap.add_argument("--per-request", type=int, default=128, help="samples per train request")
    ap.add_argument("--labels", type=int, default=16)
    ap.add_argument("--str-features", type=int, default=8)
    ap.add_argument("--num-features", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=100000)
    ap.add_argument("--hash-bits", type=int, default=20)
    ap.add_argument("--pools", type=int, default=4, help="distinct synthetic batches cycled")
    ap.add_argument("--mix-every", type=int, default=0,
                    help="N > 0: MIX every N steps; 0 (default): the reference's trigger - a new MIX "
                         "starts as soon as the previous one has finished and updates arrived "
                         "(linear_mixer.cpp:337-344,358-390: interval_count 512 updates, the mixer "
                         "wakes on the threshold), agreed across ranks each step")
    ap.add_argument("--latency-iters", type=int, default=300)
    ap.add_argument("--update-mode", choices=("atomic", "hogwild"), default="atomic",
                    help="how concurrent request streams update shared rows")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="gloo: rehearse the multi-rank GPU path with several ranks on one GPU "
                         "(not a benchmark configuration)")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu: host engine + gloo, for rehearsing the multi-rank path without a GPU "
                         "(not a benchmark configuration)")
    ap.add_argument("--mix-mode", choices=("overlap", "sync"), default="overlap",
                    help="overlap: the RCCL all-reduce of step k runs during step k+1 and its "
                         "mean is folded in afterwards (updates made meanwhile are kept); "
                         "sync: blocking MIX at the end of every step")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if args.device == "gpu":
        if args.dist_backend == "gloo":
            local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
        from jubatus_amd.utils.numa import bind_to_device
        numa = bind_to_device(local)      # before pinned buffers and worker threads exist
        if world > 1:
            if args.dist_backend == "nccl":
                dist.init_process_group("nccl", device_id=device)
            else:
                dist.init_process_group("gloo")
    else:
        device = None
        numa = {}
        if world > 1:
            dist.init_process_group("gloo")

    def sync():
        if device is not None:
            torch.cuda.synchronize()

    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier

    cfg = json.loads(json.dumps(AROW_CONFIG))
    cfg["converter"]["hash_max_size"] = 1 << args.hash_bits
    conv = DatumToFvConverter(cfg["converter"])
    clf = LinearClassifier(cfg["method"], cfg["parameter"], conv, device=device,
                           concurrent_update=args.update_mode)
    for y in range(args.labels):  # same label order on every rank (set_label, as a client would)
        clf.set_label(f"label{y}")

    from jubatus_amd.ops.feature_pipeline import RequestArena

    rng = random.Random(1234 + rank)
    pools = []
    for _ in range(args.pools):
        bodies = make_requests(rng, args.requests, args.per_request, args.labels,
                               args.str_features, args.num_features, args.vocab)
        # the synthetic client "sends" the step's requests into a pinned
        # receive arena, as the RPC reader does for real connections
        arena = RequestArena(sum(len(b) for b in bodies) + 16 * len(bodies) + 64)
        for b in bodies:
            arena.append(b)
        offs, lens = arena.spans()
        pools.append((arena, offs, lens))
    samples_per_step = args.requests * args.per_request

    # host-side metadata (label agreement, count deltas) rides on a gloo group
    # so the MIX never forces a GPU synchronisation
    meta = dist.new_group(backend="gloo") if world > 1 else None
    pending = [None]

    def barrier():
        if world > 1:
            dist.barrier()

    def finish_mix():
        if pending[0] is not None:
            clf.mix_end(pending[0])
            pending[0] = None

    mixes = [0]

    agreed = {"version": None, "labels": False}

    inflight = {"work": None, "flags": None}

    def mix_due(i: int) -> bool:
        if args.mix_every > 0 or args.mix_mode == "sync":
            return (i + 1) % max(1, args.mix_every) == 0
        # adaptive: every rank must agree (the collectives have to match).
        # One tiny host all-reduce per step carries [not ready, labels
        # changed]; it is issued asynchronously and read one step later, so
        # the host never waits on it (all ranks act on the same lagged flags)
        due = False
        if inflight["work"] is not None:
            inflight["work"].wait()
            f = inflight["flags"]
            agreed["labels"] = f[1].item() == 0
            due = f[0].item() == 0
        v = clf.labels.version()
        # a MIX that starts this step is not finished by the next one
        flags = torch.tensor([0 if (not due and clf.mix_ready(pending[0])) else 1,
                              0 if v == agreed["version"] else 1], dtype=torch.int32)
        inflight["flags"] = flags
        inflight["work"] = dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=meta, async_op=True)
        return due

    def step(i: int) -> None:
        arena, offs, lens = pools[i % len(pools)]
        n = clf.train_arena(arena, offs, lens)
        assert n == samples_per_step
        if world > 1 and mix_due(i):
            mixes[0] += 1
            if args.mix_mode == "sync":
                clf.mix()
            else:
                finish_mix()
                v = clf.labels.version()
                pending[0] = clf.mix_begin(meta_group=meta,
                                           agreed_version=agreed["version"] if agreed["labels"] else None)
                if "sync" not in pending[0] and clf.labels.version() == v:
                    agreed["version"] = v

    # setup objects (synthetic bodies, torch modules) move to the permanent
    # generation, so a cyclic-GC pass in the timed loop does not traverse them
    import gc
    gc.collect()
    gc.freeze()
    for i in range(args.warmup):
        step(i)
    finish_mix()
    if device is not None:
        clf.pipe.check_errors()
    sync()
    barrier()
    sync()
    trace_steps = os.environ.get("JB_BENCH_TRACE") == "1"
    marks = []
    mixes[0] = 0
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i)
        if trace_steps:
            marks.append(time.perf_counter())
    finish_mix()          # the last MIX completes inside the timed region
    if inflight["work"] is not None:
        inflight["work"].wait()
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if trace_steps and rank == 0:
        d = np.diff([t0] + marks) * 1e3
        print("step host ms: " + " ".join(f"{x:.2f}" for x in d), file=sys.stderr)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if device is not None else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if device is not None:
        clf.pipe.check_errors()

    # accuracy on a held-out synthetic request (sanity: the model learns)
    test = make_requests(random.Random(99), 1, 2048, args.labels, args.str_features,
                         args.num_features, args.vocab)[0]
    items = msgpack.unpackb(test, raw=False)
    res = clf.classify_requests([msgpack.packb([d for _, d in items], use_bin_type=False)])
    acc = float(np.mean([max(r, key=lambda t: t[1])[0] == lab for r, (lab, _) in zip(res, items)]))

    # classify latency: one datum per request, full round trip incl. D2H
    one = msgpack.packb([items[0][1]], use_bin_type=False)
    lat = []
    for i in range(args.latency_iters + 20):
        t1 = time.perf_counter()
        clf.classify_requests([one])
        dt = time.perf_counter() - t1
        if i >= 20:
            lat.append(dt * 1e6)
    lat.sort()
    p50 = statistics.median(lat)
    p99 = lat[min(len(lat) - 1, int(0.99 * len(lat)))]

    total = samples_per_step * args.steps * world
    value = total / elapsed
    if rank == 0:
        out = {
            "metric": "train_samples_per_sec",
            "value": round(value, 1),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (label-correlated datums, 8 str + 8 num features), random-init model",
            "config": {
                "model": "jubaclassifier AROW (config/classifier/arow.json: regularization_weight 1.0, "
                         "str bin/bin + num)",
                "global_batch": samples_per_step * world,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "requests_per_step_per_gpu": args.requests,
                "samples_per_request": args.per_request,
                "hash_max_size": 1 << args.hash_bits,
                "labels": args.labels,
                "mix": (f"linear, RCCL all-reduce mean of W and P, {args.mix_mode}, "
                        + (f"every {args.mix_every} step(s)" if args.mix_every > 0 else
                           "back to back (a new MIX as soon as the previous one finished)")
                        + f"; {mixes[0]} MIXes in the timed steps") if world > 1 else "standalone",
                "concurrent_update": args.update_mode,
                "numa_node": numa.get("node"),
            },
            "classify_latency_us_p50": round(p50, 1),
            "classify_latency_us_p99": round(p99, 1),
            "heldout_accuracy": round(acc, 4),
            "baseline_note": "reference publishes no numbers (BASELINE.md)",
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
