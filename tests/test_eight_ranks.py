"""8-rank rehearsals on the CPU (gloo, 127.0.0.1 rendezvous) of the paths an
8-GPU node runs over RCCL: bench.py's self-launched data-parallel run with
the overlapped MIX, and the push_mixer skip schedule (recursive doubling,
skip_mixer.hpp:46-57) whose pairwise averages reach the exact cluster mean
for a power-of-two world."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 8

CONV = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
        "num_rules": [{"key": "*", "type": "num"}], "hash_max_size": 1 << 10}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _skip_worker(rank, port, q):
    import torch.distributed as dist
    os.environ["JUBATUS_FORCE_CPU"] = "1"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=WORLD)
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier
    from jubatus_amd.parallel.push_mixer import skip_peers
    clf = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV))
    for lab in ("a", "b", "c"):
        clf.set_label(lab)
    data = [("abc"[(i + rank) % 3], {"x": f"v{(i * 7 + rank) % 11}", "n": float(i % 5 - rank)})
            for i in range(30)]
    clf.train(data)
    W0, P0 = clf.W.copy(), clf.P.copy()
    for peer in skip_peers(rank, WORLD):          # strides 4, 2, 1
        clf.pair_mix(peer)
    out = [None] * WORLD
    dist.all_gather_object(out, (W0, P0, clf.W.copy(), clf.P.copy()))
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


def test_skip_mixer_eight_ranks_reaches_the_mean():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_skip_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    meanW = np.mean([r[0] for r in res], axis=0)
    meanP = np.mean([r[1] for r in res], axis=0)
    for W0, P0, W, P in res:
        np.testing.assert_allclose(W, meanW, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(P, meanP, rtol=1e-5, atol=1e-6)


def test_bench_eight_ranks_cpu():
    """bench.py --gpus 8 self-launches 8 ranks; the overlapped MIX runs on
    every rank and rank 0 prints the one JSON line. The fresh stream of a
    rank is bounded by --fresh-gb (here a few MB per rank)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(WORLD), "--steps", "2",
           "--warmup", "1", "--device", "cpu", "--requests", "4", "--per-request", "8",
           "--hash-bits", "10", "--latency-iters", "2", "--batches-per-step", "2", "--engines", "none",
           "--dist-engines", "lof,kmeans,arow", "--dist-engine-rows", "120", "--dist-engine-seconds", "0.5",
           "--dist-cluster-points", "3000", "--dist-train-seconds", "1.5"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert out["n_gpus"] == WORLD and out["config"]["world_size_observed"] == WORLD
    assert out["config"]["parallelism"] == f"dp{WORLD}"
    assert out["timed_samples_per_rank"] == 2 * 2 * 4 * 8
    assert out["config"]["global_batch"] == WORLD * 2 * 4 * 8
    assert out["mix_last"] and out["mix_last"]["mode"] in ("sparse", "dense")
    mt = out["mix_timed"]
    assert mt["count"] >= 1 and mt["world"] == WORLD and mt["bytes_per_rank_mean"] > 0
    assert mt["latency_ms_p50"] is not None and mt["latency_ms_p50"] >= 0
    assert out["config"]["world_size_observed"] == WORLD
    # BASELINE #4 / #5 on 8 ranks: one server per rank in one cluster filled
    # by the native load generator, a MIX every member took part in, queries
    # after it (CPU: the Python row / clustering servers), and the headline
    # engine served natively (host backend here) under a timed train load
    # with MIXes inside the window
    for name, qry, key in (("lof", "calc_score", "add_rows"), ("kmeans", "get_nearest_center", "push_points"),
                           ("arow", "classify", "train_samples")):
        rec = out["engines_dist"][name]
        assert "errors" not in rec, rec
        assert rec["world_size_observed"] == WORLD and rec["do_mix"] is True
        assert rec[f"{key}_per_s_total"] > 0 and len(rec[f"{key}_per_s_per_rank"]) == WORLD
        counts = [int(c) for c in rec["mix_count_per_rank"]]
        assert min(counts) >= 1 and min(rec["mix_bytes_per_rank"]) > 0
        assert all(l.startswith(f"mixed with {WORLD} servers in ") for l in rec["mix_line_per_rank"])
        assert rec["mix_latency_ms"] > 0 and rec[f"{qry}_per_s_total"] > 0
        if name == "arow":    # the averaged linear model (LOF / k-means re-derive lists / centers per member)
            assert rec["members_agree_after_mix"] is True, rec
    assert out["engines_dist"]["arow"]["server_runtime"] == "native"


def test_bench_pinned_budget_eight_ranks():
    """the fresh-stream sizing rule: 8 local ranks together pin at most
    0.6 x MemAvailable and each at most 56 GB"""
    sys.path.insert(0, ROOT)
    import bench
    avail = bench._mem_available()
    per_rank = bench.fresh_budget(0, WORLD)
    assert per_rank <= 56e9 and WORLD * per_rank <= 0.6 * avail * 1.01
    assert bench.fresh_budget(2.5, WORLD) == 2.5e9
