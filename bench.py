#!/usr/bin/env python3
"""Headline benchmark: AROW classifier training throughput (samples/s) +
p50/p99 classify latency on MI355X, 1..N GPUs (one rank per GPU, RCCL MIX).

Metric/config: BASELINE.json - "samples/sec (train) + p50 classify latency,
AROW classifier at 1/2/4/8 MI355X", config/classifier/arow.json
(AROW, regularization_weight 1.0, converter str bin/bin + num).

Data: a NON-REPEATING synthetic stream. Every timed batch is a distinct set
of train request bodies (msgpack list<labeled_datum>, 8 string + 8 numeric
values, 16 labels) generated before the timed region by the native
generator (csrc/native/jb_synth.cpp) into pinned host memory, as the RPC
reader would leave them; the warmup steps train on a separate data set, so
no timed sample has been seen before. ``--worst-case`` makes every string
value fresh noise (no label signal), so (almost) every sample updates the
model; the numeric keys n0..n7 are in every sample (hot rows).

One timed step on every rank = ``batches-per-step`` train batches of
R concurrent requests x S samples:
  * header pass (host), one H2D copy of the batch's raw bytes, GPU request
    scan (csrc/hip/scan.hip: sample boundaries, label ids, validation), GPU
    msgpack parse + feature hashing (fv_hash.hip), hot-row detection
    (hot.hip) and the AROW update (linear.hip: R lock-free update streams,
    each exact-sequential; hot rows in a block-shared LDS replica);
  * the MIX (N > 1): label-set agreement (host gloo group) + RCCL all-reduce
    mean of W and P over xGMI, overlapped with the following batches and
    folded in as W += mean(snapshot) - snapshot; a new MIX starts as soon as
    the previous one finished (the reference's trigger); ``--mix-mode sync``
    blocks.
Per-GPU work is fixed as N grows (weak scaling). The model starts from zero
(random-init equivalent for a linear model); the JSON reports the fraction
of timed samples that updated it.

Usage: python bench.py --gpus N --steps K --warmup W
       (N > 1: launched by torch.distributed.run, one process per GPU; without
       WORLD_SIZE in the environment this script launches the N ranks itself)
"""
from __future__ import annotations

import argparse
import io
import json
import shlex
import os
import random
import shutil
import socket
import statistics
import subprocess
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

BLOCK_BYTES = 1 << 30          # pinned host blocks (a power of two: no allocator rounding)


def make_requests(rng: random.Random, nreq: int, per_req: int, nlabels: int, n_str: int,
                  n_num: int, vocab: int) -> list[bytes]:
    """Python twin of the native generator (held-out accuracy set)."""
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


def _progress(msg: str) -> None:
    """a progress line on stderr (long runs keep writing; the JSON line on
    stdout stays the only stdout output)"""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _mem_available() -> int:
    try:
        with open("/proc/meminfo") as f:
            for line in f:
                if line.startswith("MemAvailable:"):
                    return int(line.split()[1]) * 1024
    except OSError:
        pass
    return 16 << 30


class FreshStream:
    """Distinct request batches in pinned host blocks (generated once,
    outside the timed region; consumed once)."""

    def __init__(self, nat, torch, pinned: bool, args, seed: int, count: int, nthreads: int,
                 p_corr: float, vocab: int):
        from jubatus_amd.ops.feature_pipeline import RequestArena
        self.batches = []
        self.nbytes = 0
        blk, blk_np, used_in_blk = None, None, 0
        offs = np.zeros(args.requests, np.int64)
        lens = np.zeros(args.requests, np.int64)
        for b in range(count):
            for attempt in range(2):
                if blk is not None:
                    start = (used_in_blk + 4095) & ~4095
                    cap = BLOCK_BYTES - start - 64
                    used = nat.synth_requests(blk_np.ctypes.data + start, cap, offs.ctypes.data,
                                              lens.ctypes.data, seed, b * args.requests,
                                              args.requests, args.per_request, args.labels,
                                              args.str_features, args.num_features, vocab, 16,
                                              p_corr, nthreads)
                    if used >= 0:
                        view = blk[start:start + used + 64]
                        self.batches.append(RequestArena.over(view, offs.copy(), lens.copy()))
                        used_in_blk = start + used + 64
                        self.nbytes += used
                        break
                if attempt == 1:
                    raise MemoryError("one batch does not fit a pinned block")
                blk = torch.empty(BLOCK_BYTES, dtype=torch.uint8, pin_memory=pinned)
                blk_np = blk.numpy()
                used_in_blk = 0


def _cpu(a, b) -> float:
    return (b.ru_utime - a.ru_utime) + (b.ru_stime - a.ru_stime)


def _thread_cpu() -> dict:
    """CPU seconds of this process's threads, summed by thread name"""
    out: dict = {}
    tck = os.sysconf("SC_CLK_TCK")
    for tid in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        fields = st[st.rindex(")") + 2:].split()
        out[name] = out.get(name, 0.0) + (int(fields[11]) + int(fields[12])) / tck
        out[name + ":sys"] = out.get(name + ":sys", 0.0) + int(fields[12]) / tck   # (kernel time: the TCP stack)
    return out


def _handler_profile(clf) -> dict:
    """mean time per served batch in the arena handler (models/classifier.py
    train_arena_sync): waiting for the model lock, submitting the GPU work,
    waiting for the scan check, finishing"""
    p = clf._served_prof
    if not p[0]:
        return {}
    return {"batches": p[0], "requests_per_batch": round(p[1] / p[0], 1),
            "lock_wait": round(p[2] / p[0] * 1e6, 1), "submit": round(p[3] / p[0] * 1e6, 1),
            "scan_wait": round(p[4] / p[0] * 1e6, 1), "finish": round(p[5] / p[0] * 1e6, 1),
            "submit_pre": round(p[6] / p[0] * 1e6, 1), "submit_call": round(p[7] / p[0] * 1e6, 1),
            "submit_set_wait": round(clf.pipe.set_wait_s / p[0] * 1e6, 1)}


def served_train(args, local: int, nat) -> dict:
    """The served train path: an in-process jubaclassifier (AROW, this GPU)
    behind the native msgpack-RPC transport, driven by the native load
    generator (csrc/tools/jubaloadgen.cpp) with train requests of
    ``per_request`` samples over loopback TCP. The transport copies each
    request body into a pinned arena slot; one Python call per slot runs
    the GPU scan -> fv_hash -> train pipeline and replies per request
    (classifier_impl.cpp:54-57 -> classifier_serv.cpp:128-147)."""
    import resource
    import tempfile
    exe = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaloadgen")
    if not os.access(exe, os.X_OK):
        return {"skipped": "jubaloadgen not built"}
    from jubatus_amd.framework.server_helper import ServerHelper
    from jubatus_amd.framework.server_util import ServerArgv
    from jubatus_amd.server import get_serv
    tmp = tempfile.mkdtemp(prefix="jb_served_")
    cfg = json.loads(json.dumps(AROW_CONFIG))
    cfg["converter"]["hash_max_size"] = 1 << args.hash_bits
    cfg_path = os.path.join(tmp, "arow.json")
    with open(cfg_path, "w") as f:
        json.dump(cfg, f)
    a = ServerArgv.parse(["-p", "9199", "-b", "127.0.0.1", "-f", cfg_path, "-d", tmp,
                          "-c", str(args.rpc_threads), "--gpu", str(local)], "classifier")
    a.port = 0
    old_mode = os.environ.get("JUBATUS_UPDATE_MODE")
    os.environ["JUBATUS_UPDATE_MODE"] = args.update_mode      # the headline's update mode
    try:
        h = ServerHelper(get_serv("classifier"), a, install_signals=False)
    finally:
        if old_mode is None:
            os.environ.pop("JUBATUS_UPDATE_MODE", None)
        else:
            os.environ["JUBATUS_UPDATE_MODE"] = old_mode
    h.start(block=False)
    try:
        # K distinct train requests: params [cluster name "", body]
        K = args.rpc_distinct
        cap = K * args.per_request * 400 + (1 << 20)
        buf = np.zeros(cap, np.uint8)
        offs = np.zeros(K, np.int64)
        lens = np.zeros(K, np.int64)
        used = nat.synth_requests(buf.ctypes.data, cap, offs.ctypes.data, lens.ctypes.data, 4242, 0,
                                  K, args.per_request, args.labels, args.str_features,
                                  args.num_features, args.vocab, 16, 0.6, 8)
        assert used > 0
        pfile = os.path.join(tmp, "train_params.bin")
        with open(pfile, "wb") as f:
            for o, n in zip(offs, lens):
                f.write(b"\x92\xa0" + buf[o:o + n].tobytes())
        base = [exe, "-p", str(a.port), "-m", "train", "-f", pfile, "-c", str(args.rpc_conns),
                "-d", str(args.rpc_depth)] + _fresh_flag(args)
        subprocess.run(base + ["-t", "1.5"], capture_output=True, text=True, timeout=120)  # warmup
        clf = h.server.clf
        clf.synchronize()
        st0 = clf.train_stats()
        ru_self0 = resource.getrusage(resource.RUSAGE_SELF)
        thr0 = _thread_cpu()
        ans0, nb0 = h.rpc.arena_ns(), h.rpc.batches()
        ru_kid0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        r = subprocess.run(base + ["-t", str(args.rpc_seconds)], capture_output=True, text=True,
                           timeout=args.rpc_seconds + 120)
        ru_self1 = resource.getrusage(resource.RUSAGE_SELF)
        thr1 = _thread_cpu()
        ans1, nb1 = h.rpc.arena_ns(), h.rpc.batches()
        nb = max(1, nb1 - nb0)
        ru_kid1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        if r.returncode != 0:
            return {"error": (r.stderr or r.stdout)[-400:]}
        lg = json.loads(r.stdout.strip().splitlines()[-1])
        clf.synchronize()
        st1 = clf.train_stats()
        tr = st1["trained"] - st0["trained"]
        return {"served_train_samples_per_sec": round(lg["requests_per_s"] * args.per_request, 1),
                "requests_per_s": lg["requests_per_s"], "samples_per_request": args.per_request,
                "connections": lg["connections"], "depth": lg["depth"],
                "distinct_requests": lg["distinct_requests"], "fresh_values": lg.get("fresh_values"),
                "noise_per_mille": lg.get("noise_per_mille", 0),
                "rpc_p50_us": lg["p50_us"],
                "rpc_p99_us": lg["p99_us"], "seconds": lg["seconds"],
                "samples_trained_in_window": tr,
                "update_fraction": round((st1["updated"] - st0["updated"]) / tr, 4) if tr else None,
                "server_threads": args.rpc_threads,
                # CPU seconds per second of the timed window: the server process
                # (transport + Python + GPU driver threads) and the load generator
                "server_cpus": round(_cpu(ru_self0, ru_self1) / lg["seconds"], 2),
                "loadgen_cpus": round(_cpu(ru_kid0, ru_kid1) / lg["seconds"], 2),
                "server_cpus_by_thread": {k: round((v - thr0.get(k, 0.0)) / lg["seconds"], 2)
                                          for k, v in sorted(thr1.items())
                                          if v - thr0.get(k, 0.0) > 0.01 * lg["seconds"]},
                "train_scan": dict(clf._scan_stats),
                "handler_us_per_batch": _handler_profile(clf),
                "batches_in_window": nb,
                "transport_us_per_batch": {"handler_call": round((ans1[0] - ans0[0]) / nb / 1e3, 1),
                                           "send_replies": round((ans1[1] - ans0[1]) / nb / 1e3, 1)},
                "concurrent_update": clf.concurrent_update,
                "path": "loopback TCP -> native epoll transport -> pinned arena slot -> GPU scan/"
                        "fv_hash/AROW train; reply per request after the batch's scan check"}
    finally:
        h.stop()


def _proc_cpu(pid: int) -> float:
    tck = os.sysconf("SC_CLK_TCK")
    with open(f"/proc/{pid}/stat") as f:
        st = f.read()
    fields = st[st.rindex(")") + 2:].split()
    return (int(fields[11]) + int(fields[12])) / tck


def _proc_thread_cpu(pid: int) -> dict:
    """CPU seconds of a process's threads, summed by thread name (and the
    kernel-mode part of them under "<name>:sys")"""
    tck = os.sysconf("SC_CLK_TCK")
    out: dict = {}
    try:
        tids = os.listdir(f"/proc/{pid}/task")
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"/proc/{pid}/task/{tid}/stat") as f:
                st = f.read()
        except OSError:
            continue
        name = st[st.index("(") + 1:st.rindex(")")]
        fields = st[st.rindex(")") + 2:].split()
        out[name] = out.get(name, 0.0) + (int(fields[11]) + int(fields[12])) / tck
    return out


def served_train_native(args, local: int, nat, mode: str | None = None, noise_pm: int = 0,
                        classify: bool = True) -> dict:
    """The served train path of the native server binary
    (csrc/server/jubaclassifier.cpp: no Python in the server process): the
    same load generator, request set and configuration as served_train.
    mode: the server's update mode (default: the headline's); noise_pm: per
    mille of the samples sent with every string token redrawn (jubaloadgen
    -u: unseen features, the model keeps updating - a learning stream)."""
    import socket
    import tempfile
    from jubatus_amd.common.mprpc import RpcClient
    exe = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaloadgen")
    srv = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaclassifier")
    if not (os.access(exe, os.X_OK) and os.access(srv, os.X_OK)):
        return {"skipped": "native server / jubaloadgen not built"}
    tmp = tempfile.mkdtemp(prefix="jb_served_native_")
    cfg = json.loads(json.dumps(AROW_CONFIG))
    cfg["converter"]["hash_max_size"] = 1 << args.hash_bits
    cfg_path = os.path.join(tmp, "arow.json")
    with open(cfg_path, "w") as f:
        json.dump(cfg, f)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # JB_SERVED_WRAP: a command prefix for the server process (profiling:
    # "rocprofv3 --marker-trace --kernel-trace -d DIR -o srv --" with
    # JUBATUS_ROCTX=1 records the server's roctx ranges)
    wrap = shlex.split(os.environ.get("JB_SERVED_WRAP", ""))
    p = subprocess.Popen(wrap + [srv, "-p", str(port), "-b", "127.0.0.1", "-f", cfg_path, "-d", tmp,
                                 "-c", str(args.rpc_threads), "--gpu", str(local)],
                         stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                         env=dict(os.environ, JUBATUS_UPDATE_MODE=mode or args.update_mode))

    def status():
        with RpcClient("127.0.0.1", port, 30.0) as c:
            (_, st), = c.call("get_status", "").items()
        return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
                for k, v in st.items()}
    try:
        deadline = time.time() + 60
        while True:
            try:
                st = status()
                break
            except Exception:  # noqa: BLE001 - not listening yet
                if p.poll() is not None or time.time() > deadline:
                    return {"error": (p.stderr.read() or b"").decode(errors="replace")[-400:]}
                time.sleep(0.2)
        if st.get("server_runtime") != "native":
            return {"error": "the binary handed the configuration to the Python server"}
        K = args.rpc_distinct
        cap = K * args.per_request * 400 + (1 << 20)
        buf = np.zeros(cap, np.uint8)
        offs = np.zeros(K, np.int64)
        lens = np.zeros(K, np.int64)
        used = nat.synth_requests(buf.ctypes.data, cap, offs.ctypes.data, lens.ctypes.data, 4242, 0,
                                  K, args.per_request, args.labels, args.str_features,
                                  args.num_features, args.vocab, 16, 0.6, 8)
        assert used > 0
        pfile = os.path.join(tmp, "train_params.bin")
        with open(pfile, "wb") as f:
            for o, n in zip(offs, lens):
                f.write(b"\x92\xa0" + buf[o:o + n].tobytes())
        base = [exe, "-p", str(port), "-m", "train", "-f", pfile, "-c", str(args.rpc_conns),
                "-d", str(args.rpc_depth)] + _fresh_flag(args)
        if noise_pm > 0 and args.rpc_fresh:
            base += ["-u", str(noise_pm)]
        subprocess.run(base + ["-t", "1.5"], capture_output=True, text=True, timeout=120)  # warmup
        st0 = status()
        cpu0 = _proc_cpu(p.pid)
        th0 = _proc_thread_cpu(p.pid)
        r = subprocess.run(base + ["-t", str(args.rpc_seconds)], capture_output=True, text=True,
                           timeout=args.rpc_seconds + 120)
        cpu1 = _proc_cpu(p.pid)
        th1 = _proc_thread_cpu(p.pid)
        if r.returncode != 0:
            return {"error": (r.stderr or r.stdout)[-400:]}
        lg = json.loads(r.stdout.strip().splitlines()[-1])
        st1 = status()
        tr = int(st1["train.samples_trained"]) - int(st0["train.samples_trained"])
        up = int(st1["train.samples_updated"]) - int(st0["train.samples_updated"])
        # classify over RPC: one datum per request, one connection, one in flight
        cl = {"p50_us": None, "p99_us": None}
        if classify:
            one = msgpack.unpackb(buf[offs[0]:offs[0] + lens[0]].tobytes(), raw=False)[0][1]
            cfile = os.path.join(tmp, "classify_params.bin")
            with open(cfile, "wb") as f:
                f.write(msgpack.packb(["", [one]], use_bin_type=False))
            cl = _loadgen(exe, port, "classify", cfile, 1, 1, secs=2.0, timeout=120)
        return {"served_train_samples_per_sec": round(lg["requests_per_s"] * args.per_request, 1),
                "requests_per_s": lg["requests_per_s"], "samples_per_request": args.per_request,
                "connections": lg["connections"], "depth": lg["depth"],
                "distinct_requests": lg["distinct_requests"], "fresh_values": lg.get("fresh_values"),
                "rpc_p50_us": lg["p50_us"], "rpc_p99_us": lg["p99_us"], "seconds": lg["seconds"],
                "samples_trained_in_window": tr,
                "update_fraction": round(up / tr, 4) if tr else None,
                "server_threads": args.rpc_threads,
                "server_cpus": round((cpu1 - cpu0) / lg["seconds"], 2),
                "server_cpus_by_thread": {k: round((v - th0.get(k, 0.0)) / lg["seconds"], 2)
                                          for k, v in sorted(th1.items()) if v - th0.get(k, 0.0) > 0.005},
                "classify_rpc_p50_us": cl["p50_us"], "classify_rpc_p99_us": cl["p99_us"],
                "classify_rpc": "one datum per request, 1 connection x 1 in flight, loopback TCP",
                "train_scan": {k[len("train_scan."):]: int(v) for k, v in st1.items()
                               if k.startswith("train_scan.") and v.isdigit()},
                "concurrent_update": st1.get("train.update_mode"),
                "path": "loopback TCP -> native jubaclassifier (no Python) -> pinned arena slot -> "
                        "GPU scan/fv_hash/AROW train; reply per request after the batch's scan check"}
    finally:
        p.terminate()
        try:
            p.wait(timeout=90 if wrap else 30)
        except subprocess.TimeoutExpired:
            p.kill()


def _fresh_flag(args) -> list:
    """jubaloadgen -r: every sample sent carries a freshly drawn numeric value
    (csrc/tools/jubaloadgen.cpp), so the served stream does not repeat"""
    return ["-r", "4243"] if args.rpc_fresh else []


# ------------------------------------------------------- engine records
# BASELINE.json secondary configs measured over RPC against the native
# servers (csrc/server/jb_row_server.hpp; no Python in the server process),
# driven by the native load generator (csrc/tools/jubaloadgen.cpp)
ENGINE_CASES = (
    # (record name, engine, config, fill method, query method)
    ("recommender_euclid_lsh", "recommender", "config/recommender/euclid_lsh.json", "update_row",
     "similar_row_from_datum"),
    ("recommender_default", "recommender", "config/recommender/default.json", "update_row",
     "similar_row_from_datum"),
    ("anomaly_lof", "anomaly", "config/anomaly/lof.json", "add", "calc_score"),
)


def _row_datums(n: int, seed: int) -> list[bytes]:
    """n distinct synthetic rows (msgpack datums): 4 string values from a
    Zipf-like vocabulary (words of 3-8 letters, so ngram converters see
    text) and 4 numeric values"""
    rng = np.random.default_rng(seed)
    letters = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8)
    vocab = ["".join(chr(c) for c in rng.choice(letters, size=int(rng.integers(3, 9))))
             for _ in range(4096)]
    widx = np.minimum((rng.pareto(1.2, size=(n, 4)) * 40).astype(np.int64), 4095)
    nums = np.round(rng.normal(0.0, 1.0, size=(n, 4)) + (widx[:, :1] % 7) * 0.5, 4)
    out = []
    for i in range(n):
        w = widx[i]
        x = nums[i]
        out.append(msgpack.packb([[["title", vocab[w[0]] + " " + vocab[w[1]]], ["genre", vocab[w[2]]],
                                   ["tag", vocab[w[3]]], ["src", "s%d" % (w[0] % 13)]],
                                  [["n0", float(x[0])], ["n1", float(x[1])], ["n2", float(x[2])],
                                   ["n3", float(x[3])]], []], use_bin_type=False))
    return out


def _loadgen(exe: str, port: int, method: str, pfile: str, conns: int, depth: int, secs: float = 0.0,
             once: bool = False, timeout: float = 900.0) -> dict:
    cmd = [exe, "-p", str(port), "-m", method, "-f", pfile, "-c", str(conns), "-d", str(depth)]
    cmd += ["-o", "1"] if once else ["-t", str(secs)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"jubaloadgen {method}: {(r.stderr or r.stdout)[-300:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


DIST_ENGINE_CASES = (
    # name, engine, config, update RPC, query RPC
    ("lof", "anomaly", "config/anomaly/lof.json", "add", "calc_score"),
    ("kmeans", "clustering", "config/clustering/kmeans.json", "push", "get_nearest_center"),
    ("gmm", "clustering", "config/clustering/gmm.json", "push", "get_nearest_center"),
    # the headline engine served natively on every rank: jubaclassifier with
    # the linear mixer (touched-row diff all-reduce on the RCCL plane) under a
    # timed train load, MIXes running inside the window
    ("arow", "classifier", "config/classifier/arow.json", "train", "classify"),
)


def _dist_files(args, nat, name: str, upd: str, qry: str, cname: str, rank: int, tmp: str):
    """per-rank jubaloadgen parameter files of a distributed engine case:
    (fill file, query file, units the fill carries). LOF: one distinct row per
    add; clustering: 1000-point pushes (three blobs); AROW: 128-sample train
    requests of the headline's label-correlated stream"""
    cn = msgpack.packb(cname)
    fill = os.path.join(tmp, f"{name}_{rank}_fill.bin")
    qf = os.path.join(tmp, f"{name}_{rank}_query.bin")
    if upd == "add":
        rows = _row_datums(args.dist_engine_rows + 512, 101 + rank)
        queries, rows = rows[-512:], rows[:-512]
        with open(fill, "wb") as f:
            for d in rows:
                f.write(b"\x92" + cn + d)
        with open(qf, "wb") as f:
            for d in queries:
                f.write(b"\x92" + cn + d)
        return fill, qf, len(rows)
    if upd == "push":
        rng = np.random.default_rng(7 + rank)
        centers = np.array([[0.0, 0.0, 0.0], [10.0, 10.0, 0.0], [-10.0, 10.0, 5.0]])
        npts, per = args.dist_cluster_points, 1000

        def point(i):
            c = centers[i % 3] + rng.normal(0, 0.5, 3)
            return [[["tag", f"t{i % 7}"]], [["a", float(c[0])], ["b", float(c[1])], ["c", float(c[2])]], []]
        with open(fill, "wb") as f:
            for b0 in range(0, npts, per):
                f.write(b"\x92" + cn + msgpack.packb([point(b0 + i) for i in range(per)], use_bin_type=False))
        with open(qf, "wb") as f:
            for i in range(512):
                f.write(b"\x92" + cn + msgpack.packb(point(i), use_bin_type=False))
        return fill, qf, (npts + per - 1) // per * per
    # train: the headline's request shape and stream (fresh values per send)
    K = max(16, min(args.rpc_distinct, 256))
    cap = K * args.per_request * 400 + (1 << 20)
    buf = np.zeros(cap, np.uint8)
    offs = np.zeros(K, np.int64)
    lens = np.zeros(K, np.int64)
    used = nat.synth_requests(buf.ctypes.data, cap, offs.ctypes.data, lens.ctypes.data, 4242 + rank, 0,
                              K, args.per_request, args.labels, args.str_features, args.num_features,
                              args.vocab, 16, 0.6, 8)
    assert used > 0
    with open(fill, "wb") as f:
        for o, n in zip(offs, lens):
            f.write(b"\x92" + cn + buf[o:o + n].tobytes())
    one = msgpack.unpackb(buf[offs[0]:offs[0] + lens[0]].tobytes(), raw=False)
    with open(qf, "wb") as f:
        for _, d in one[:64]:
            f.write(b"\x92" + cn + msgpack.packb([d], use_bin_type=False))
    return fill, qf, args.per_request


def dist_engine_records(args, rank: int, world: int, local: int, device, group) -> dict:
    """BASELINE #4 / #5 (and the headline engine) on N ranks through the
    native servers: one engine server per rank joins one cluster through a
    coordinator rank 0 starts; every rank fills its own server with the
    native load generator (csrc/tools/jubaloadgen.cpp) at BASELINE scale -
    LOF 100 K rows per rank (anomaly add: cluster-wide ids, CHT owners,
    server-to-server update; anomaly_serv.cpp:178-211), k-means / GMM 200 K
    points per rank (1000-point pushes), AROW train requests at full rate for
    a timed window with a MIX every second inside it. Then rank 0 forces a
    MIX and times it (do_mix: row diffs / coresets / touched W-P rows over the
    group's plane, RCCL between GPUs), every rank reports the reference's MIX
    line (linear_mixer.cpp:538-543: bytes and seconds of its last MIX) and
    queries its server (1 connection x 1 in flight for p50, 8 x 4 for the
    rate). Per engine: observed world size, fill rate (sum over ranks), MIX
    latency / bytes / plane per rank, query p50 and rate, and whether the
    members answer alike after the MIX. --device cpu rehearses the same calls
    (the row / clustering binaries hand over to the Python servers there; the
    classifier serves on its native host backend)."""
    import shutil
    import tempfile
    import torch.distributed as dist
    from jubatus_amd._native import native
    from jubatus_amd.common.mprpc import RpcClient
    exe = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaloadgen")
    nat = native()
    out: dict = {}
    coord = None
    ls = None
    if rank == 0:
        from jubatus_amd.common.coordinator import NativeCoordinator
        from jubatus_amd.common.lock_service import CoordinatorClient
        coord = NativeCoordinator(0, "127.0.0.1")
        ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=10.0)
    box = [coord.port if coord else 0]
    dist.broadcast_object_list(box, src=0, group=group)
    zk = f"127.0.0.1:{box[0]}"
    # the servers are not ranks of this job: no torch.distributed environment
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK", "ROLE_WORLD_SIZE", "ROLE_NAME")
           and not k.startswith("TORCHELASTIC_")}
    if device is None:
        env["JUBATUS_FORCE_CPU"] = "1"     # no GPU: host backends / Python servers
    tmp = tempfile.mkdtemp(prefix=f"jb_dist_{rank}_")

    def status_of(port, cname):
        with RpcClient("127.0.0.1", port, 60.0) as c:
            (_, raw), = c.call("get_status", cname).items()
        return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
                for k, v in raw.items()}

    def gather(x):
        xs = [None] * world
        dist.all_gather_object(xs, x, group=group)
        return xs

    try:
        for name, engine, cfg, upd, qry in DIST_ENGINE_CASES:
            if args.dist_engines != "all" and name not in args.dist_engines.split(","):
                continue
            _progress(f"dist engine {name}: start")
            # every rank makes the same collective calls in the same order;
            # a local failure only empties its contribution
            cname = f"bench_{name}"
            if rank == 0:
                from jubatus_amd.common import config as zkconfig
                zkconfig.config_tozk(ls, engine, cname, open(os.path.join(ROOT, cfg)).read())
            dist.barrier(group=group)
            fill, qf, units = _dist_files(args, nat, name, upd, qry, cname, rank, tmp)
            port = _free_port()
            # MIX trigger: forced only (-s 0 -i 0), except the served train
            # window, which MIXes every second as the reference's time trigger
            # does every 16 s (server_util.cpp:184-189)
            interval = "1" if upd == "train" else "0"
            srv = subprocess.Popen([os.path.join(ROOT, "jubatus_amd", "native_bin", f"juba{engine}"),
                                    "-z", zk, "-n", cname, "-p", str(port), "-b", "127.0.0.1", "-s", interval,
                                    "-i", "0", "-I", "60", "-Z", "10", "-c", "16", "--gpu", str(local)],
                                   stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, env=env)
            rec: dict = {"config": cfg, "world_size_observed": world}
            err = None
            st: dict = {}
            try:
                deadline = time.time() + 180
                while time.time() < deadline:
                    try:
                        st = status_of(port, cname)
                        if st.get("linear_mixer.group_size") == str(world):
                            break
                    except Exception:  # noqa: BLE001 - not up yet
                        if srv.poll() is not None:
                            raise RuntimeError(f"juba{engine} exited ({srv.returncode})")
                    time.sleep(0.3)
                else:
                    raise RuntimeError("the group did not form")
            except Exception as e:  # noqa: BLE001
                err = repr(e)[:300]
            up = gather(err is None)
            rec["server_runtime"] = st.get("server_runtime", "python")
            if st.get("storage"):
                rec["storage"] = st.get("storage")     # hbm (device tables) / host (host backend)
            rate = None
            fill_info = None
            if all(up):
                dist.barrier(group=group)      # the ranks' loads start together
                try:
                    t0 = time.perf_counter()
                    if upd == "train":
                        secs = args.dist_train_seconds
                        r = subprocess.run([exe, "-p", str(port), "-m", "train", "-f", fill, "-c", "16", "-d", "8",
                                            "-t", str(secs)] + _fresh_flag(args),
                                           capture_output=True, text=True, timeout=secs + 300)
                        if r.returncode != 0:
                            raise RuntimeError(f"jubaloadgen train: {(r.stderr or r.stdout)[-300:]}")
                        lg = json.loads(r.stdout.strip().splitlines()[-1])
                        rate = lg["requests_per_s"] * units
                        fill_info = {"rpc_p50_us": lg["p50_us"], "rpc_p99_us": lg["p99_us"], "seconds": lg["seconds"]}
                    else:
                        # a distributed add blocks its RPC worker on the CHT owners' updates
                        # (anomaly_serv.cpp:178-211): fewer adds in flight than workers, so
                        # the peers' update calls always find one free
                        conns, depth = (8, 1) if upd == "add" else (4, 2)
                        r = _loadgen(exe, port, upd, fill, conns, depth, once=True)
                        dt = time.perf_counter() - t0
                        rate = units / dt
                        fill_info = {"seconds": round(dt, 2), "rpc_p50_us": r["p50_us"]}
                except Exception as e:  # noqa: BLE001
                    err, rate = repr(e)[:300], None
            rates = gather(rate)
            infos = gather(fill_info)
            if all(r is not None for r in rates):
                rec["units_per_rank"] = units if upd != "train" else None
                key = {"add": "add_rows", "push": "push_points", "train": "train_samples"}[upd]
                rec[f"{key}_per_s_total"] = round(sum(rates), 1)
                rec[f"{key}_per_s_per_rank"] = [round(r, 1) for r in rates]
                rec["fill_per_rank"] = infos
                if upd == "train":
                    rec["load"] = (f"jubaloadgen per rank: 16 connections x 8 in flight, {args.per_request}-sample "
                                   f"requests, {args.dist_train_seconds} s, fresh values; MIX every 1 s")
                if rank == 0:
                    try:
                        with RpcClient("127.0.0.1", port, 600.0) as c:
                            t0 = time.perf_counter()
                            rec["do_mix"] = bool(c.call("do_mix", cname))
                            rec["mix_latency_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
                    except Exception as e:  # noqa: BLE001
                        err = repr(e)[:300]
            # the forced MIX's count on rank 0: every member waits until its own
            # count shows it (a member finishes its fold after rank 0's round returns)
            target = [0]
            if rank == 0 and rec.get("do_mix"):
                try:
                    target = [int(status_of(port, cname).get("linear_mixer.mix_count") or 0)]
                except Exception:  # noqa: BLE001
                    target = [0]
            dist.broadcast_object_list(target, src=0, group=group)
            mine = None
            if all(r is not None for r in rates):
                try:
                    st = status_of(port, cname)
                    t_w = time.time() + 30
                    while int(st.get("linear_mixer.mix_count") or 0) < max(1, target[0]) and time.time() < t_w:
                        time.sleep(0.1)
                        st = status_of(port, cname)
                    lat = _loadgen(exe, port, qry, qf, 1, 1, secs=args.dist_engine_seconds)
                    thr = _loadgen(exe, port, qry, qf, 8, 4, secs=args.dist_engine_seconds)
                    # the members' answer to the same query (rank 0's first query)
                    q0 = gather(open(qf, "rb").read(4096))[0]
                    qargs = next(msgpack.Unpacker(io.BytesIO(q0), raw=False))
                    with RpcClient("127.0.0.1", port, 60.0) as c:
                        first = c.call(qry, cname, *qargs[1:])
                    if qry == "classify":   # label columns are in each member's own order
                        first = [sorted(((l.decode() if isinstance(l, bytes) else l), round(float(v), 4))
                                        for l, v in r) for r in first]
                    elif isinstance(first, float):
                        first = round(first, 4)
                    mine = {"mix_count": st.get("linear_mixer.mix_count"),
                            "bytes": int(st.get("linear_mixer.last_mix_bytes") or 0),
                            "sec": float(st.get("linear_mixer.last_mix_sec") or 0),
                            "plane": st.get("linear_mixer.backend"), "p50": lat["p50_us"],
                            "qps": thr["requests_per_s"], "first": repr(first)}
                except Exception as e:  # noqa: BLE001
                    err = repr(e)[:300]
            stats = gather(mine)
            errors = gather(err)
            if all(x is not None for x in stats):
                rec["mix_count_per_rank"] = [x["mix_count"] for x in stats]
                # linear_mixer.cpp:538-543: "mixed with N servers in T secs, S bytes"
                rec["mix_line_per_rank"] = [f"mixed with {world} servers in {x['sec']:.6f} secs, {x['bytes']} bytes"
                                            for x in stats]
                rec["mix_bytes_per_rank"] = [x["bytes"] for x in stats]
                rec["mix_seconds_per_rank"] = [x["sec"] for x in stats]
                rec["mix_plane"] = stats[0]["plane"]
                rec[f"{qry}_p50_us_per_rank"] = [x["p50"] for x in stats]
                rec[f"{qry}_per_s_total"] = round(sum(x["qps"] for x in stats), 1)
                rec["members_agree_after_mix"] = len({x["first"] for x in stats}) == 1
            if any(errors):
                rec["errors"] = [e for e in errors if e][:2]
            srv.terminate()
            try:
                srv.wait(timeout=30)
            except subprocess.TimeoutExpired:
                srv.kill()
            dist.barrier(group=group)
            out[name] = rec
            _progress(f"dist engine {name}: done")
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
        if coord is not None:
            ls.close()
            coord.stop()
    return out


def engine_records(args, local: int) -> dict:
    """Per BASELINE secondary config: fill N distinct rows through the
    engine's update RPC (rate over the whole fill), then over-RPC latency of
    the query RPC (one connection, one request in flight: p50 / p99) and its
    throughput (8 connections x 4 in flight), and of the update RPC on the
    filled table. Queries are fresh datums (not stored rows)."""
    import tempfile
    from jubatus_amd.common.mprpc import RpcClient
    exe = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaloadgen")
    out: dict = {}
    t_gen = time.perf_counter()
    rows = _row_datums(max(args.engine_rows, args.lof_rows) + 4096, 11)
    queries, rows = rows[-4096:], rows[:-4096]
    t_gen = time.perf_counter() - t_gen
    tmp = tempfile.mkdtemp(prefix="jb_engines_")
    nil = b"\xa0"          # cluster name ""
    for name, engine, cfg, fill_m, query_m in ENGINE_CASES:
        if args.engines != "all" and name not in args.engines.split(","):
            continue
        srv = os.path.join(ROOT, "jubatus_amd", "native_bin", f"juba{engine}")
        nrows = args.lof_rows if engine == "anomaly" else args.engine_rows
        rec: dict = {"config": cfg, "rows": nrows, "server": f"native juba{engine} (no Python)"}
        _progress(f"engine {name}: fill {nrows} rows")
        port = _free_port()
        wrap = shlex.split(os.environ.get("JB_SERVED_WRAP", ""))   # (profiling prefix)
        p = subprocess.Popen(wrap + [srv, "-p", str(port), "-b", "127.0.0.1", "-f", os.path.join(ROOT, cfg),
                                     "-d", tmp, "-c", "4", "--gpu", str(local)],
                             stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
        try:
            deadline = time.time() + 60
            while True:
                try:
                    with RpcClient("127.0.0.1", port, 30.0) as c:
                        (_, st), = c.call("get_status", "").items()
                    break
                except Exception:  # noqa: BLE001 - not listening yet
                    if p.poll() is not None or time.time() > deadline:
                        raise RuntimeError((p.stderr.read() or b"").decode(errors="replace")[-300:])
                    time.sleep(0.2)
            st = {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
                  for k, v in st.items()}
            if st.get("server_runtime") != "native":
                raise RuntimeError("the binary handed the configuration to the Python server")
            fill = os.path.join(tmp, f"{name}_fill.bin")
            with open(fill, "wb") as f:
                for i in range(nrows):
                    if fill_m == "add":
                        f.write(b"\x92" + nil + rows[i])
                    else:
                        f.write(b"\x93" + nil + msgpack.packb(f"row{i}") + rows[i])
            q = os.path.join(tmp, f"{name}_query.bin")
            with open(q, "wb") as f:
                for d in queries:
                    f.write((b"\x93" + nil + d + b"\x0a") if query_m.startswith("similar") else
                            (b"\x92" + nil + d))
            t0 = time.perf_counter()
            th0 = _proc_thread_cpu(p.pid)
            r = _loadgen(exe, port, fill_m, fill, 16, 8, once=True)
            th1 = _proc_thread_cpu(p.pid)
            rec["fill_s"] = round(time.perf_counter() - t0, 2)
            rec[f"{fill_m}_per_s_fill"] = r["requests_per_s"]
            # where the fill's server time goes (CPUs per thread name)
            rec["fill_server_cpus_by_thread"] = {k: round((v - th0.get(k, 0.0)) / max(1e-9, rec["fill_s"]), 2)
                                                 for k, v in sorted(th1.items())
                                                 if v - th0.get(k, 0.0) > 0.01 * rec["fill_s"]}
            with RpcClient("127.0.0.1", port, 60.0) as c:
                (_, st), = c.call("get_status", "").items()
            st = {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
                  for k, v in st.items()}
            rec["rows_stored"] = int(st.get("num_rows", -1))
            if int(st.get("write_batches", 0) or 0):   # the fill's write batches: count, rows, phases
                rec["fill_write_batches"] = {k: st.get(k) for k in ("write_batches", "write_batch_rows",
                                                                    "write_batch_us")}
            if "add_batch_us" in st:   # batched anomaly adds: LOF chunks, phase times
                rec["fill_add_batches"] = st["add_batch_us"]
            _progress(f"engine {name}: filled in {rec['fill_s']} s; queries")
            lat = _loadgen(exe, port, query_m, q, 1, 1, secs=args.engine_seconds)
            rec[f"{query_m}_p50_us"] = lat["p50_us"]
            rec[f"{query_m}_p99_us"] = lat["p99_us"]
            thr = _loadgen(exe, port, query_m, q, 8, 4, secs=args.engine_seconds)
            rec[f"{query_m}_per_s"] = thr["requests_per_s"]
            # the update RPC on the filled table (fresh rows beyond the fill for
            # add; rewrites of stored rows for update_row)
            ulat = _loadgen(exe, port, fill_m, fill, 1, 1, secs=args.engine_seconds)
            rec[f"{fill_m}_p50_us"] = ulat["p50_us"]
            rec[f"{fill_m}_p99_us"] = ulat["p99_us"]
            rec["rpc"] = "loopback TCP, native jubaloadgen; latency: 1 connection x 1 in flight; " \
                         "throughput: 8 connections x 4 in flight; k = 10"
        except Exception as e:  # noqa: BLE001 - recorded, the headline still prints
            rec["error"] = f"{type(e).__name__}: {e}"[:400]
        finally:
            p.terminate()
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
        out[name] = rec
    for method in ("kmeans", "gmm"):
        name = f"clustering_{method}"
        if args.engines != "all" and name not in args.engines.split(","):
            continue
        _progress(f"engine {name}: push")
        out[name] = _clustering_record(args, local, method, exe, tmp)
    out["row_gen_s"] = round(t_gen, 1)
    shutil.rmtree(tmp, ignore_errors=True)
    return out


def _clustering_record(args, local: int, method: str, exe: str, tmp: str) -> dict:
    """BASELINE config #5 on one GPU: the native jubaclustering
    (config/clustering/<method>.json, coresets + k-means++ / Lloyd / GMM EM
    on the device) fed push requests of 1000 points each (3 numeric features
    + 1 string, three well-separated blobs) over RPC by the native load
    generator, then get_nearest_center over RPC (1 connection, 1 in flight)"""
    from jubatus_amd.common.mprpc import RpcClient
    cfg = f"config/clustering/{method}.json"
    rec: dict = {"config": cfg, "server": "native jubaclustering (no Python)"}
    rng = np.random.default_rng(5)
    centers = np.array([[0.0, 0.0, 0.0], [10.0, 10.0, 0.0], [-10.0, 10.0, 5.0]])
    npts, per = args.cluster_points, 1000
    push = os.path.join(tmp, f"{method}_push.bin")
    with open(push, "wb") as f:
        for b in range(0, npts, per):
            pts = []
            for i in range(per):
                c = centers[(b + i) % 3] + rng.normal(0, 0.5, 3)
                pts.append([[["tag", f"t{(b + i) % 7}"]], [["a", float(c[0])], ["b", float(c[1])],
                                                          ["c", float(c[2])]], []])
            f.write(msgpack.packb(["", pts], use_bin_type=False))
    q = os.path.join(tmp, f"{method}_query.bin")
    with open(q, "wb") as f:
        for i in range(512):
            c = centers[i % 3] + rng.normal(0, 0.5, 3)
            f.write(msgpack.packb(["", [[["tag", f"t{i % 7}"]], [["a", float(c[0])], ["b", float(c[1])],
                                                                 ["c", float(c[2])]], []]],
                                  use_bin_type=False))
    port = _free_port()
    srv = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaclustering")
    p = subprocess.Popen([srv, "-p", str(port), "-b", "127.0.0.1", "-f", os.path.join(ROOT, cfg), "-d", tmp,
                          "-c", "4", "--gpu", str(local)], stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)
    try:
        deadline = time.time() + 60
        while True:
            try:
                with RpcClient("127.0.0.1", port, 30.0) as c:
                    (_, st), = c.call("get_status", "").items()
                break
            except Exception:  # noqa: BLE001 - not listening yet
                if p.poll() is not None or time.time() > deadline:
                    raise RuntimeError((p.stderr.read() or b"").decode(errors="replace")[-300:])
                time.sleep(0.2)
        st = {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
              for k, v in st.items()}
        if st.get("server_runtime") != "native":
            raise RuntimeError("the binary handed the configuration to the Python server")
        t0 = time.perf_counter()
        r = _loadgen(exe, port, "push", push, 1, 2, once=True)
        dt = time.perf_counter() - t0
        rec["points"] = npts
        rec["push_points_per_s"] = round(npts / dt, 1)
        rec["push_rpc_p50_us"] = r["p50_us"]
        lat = _loadgen(exe, port, "get_nearest_center", q, 1, 1, secs=args.engine_seconds)
        rec["get_nearest_center_p50_us"] = lat["p50_us"]
        rec["get_nearest_center_p99_us"] = lat["p99_us"]
        with RpcClient("127.0.0.1", port, 30.0) as c:
            rec["revision"] = int(c.call("get_revision", ""))
        rec["rpc"] = ("loopback TCP, native jubaloadgen; push: 1000-point requests, 1 connection x 2 in "
                      "flight (order kept); get_nearest_center: 1 connection x 1 in flight")
    except Exception as e:  # noqa: BLE001 - recorded, the headline still prints
        rec["error"] = f"{type(e).__name__}: {e}"[:400]
    finally:
        p.terminate()
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
    return rec


PIN_FRACTION = 0.6       # of MemAvailable, shared by the node's local ranks
PIN_CAP = 56e9           # per rank


def fresh_budget(fresh_gb: float, local_ranks: int) -> float:
    """pinned bytes one rank may take for its fresh (timed) stream: the
    ranks of a node together stay within PIN_FRACTION of the host's
    available memory, each within PIN_CAP"""
    if fresh_gb > 0:
        return fresh_gb * 1e9
    return min(PIN_CAP, PIN_FRACTION * _mem_available() / max(1, local_ranks))


def exact_record(args, cfg, device, warm, fresh, bps: int, samples_per_batch: int, sync,
                 mode: str = "exact", weight_dtype: str = "fp32", steps: int | None = None,
                 hot_rows: bool = False, warmup: int | None = None) -> dict:
    """The headline protocol in another configuration: a fresh model, the
    same warmup (the exact mode: over fresh batches past the timed ones),
    then timed steps over the first fresh batches. Default: the
    serial-equivalent update mode (``--exact-steps`` steps), whose result
    equals applying the batch's requests one after the other
    (csrc/hip/serial.hip), the reference's semantics. With weight_dtype
    bf16: the headline update mode over a bf16 W table."""
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier
    clf = LinearClassifier(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]),
                           device=device, concurrent_update=mode, weight_dtype=weight_dtype)
    clf.hot_rows = hot_rows
    for y in range(args.labels):
        clf.set_label(f"label{y}")

    def run(arena):
        clf.train_arena(arena, np.asarray(arena.offs, np.int64), np.asarray(arena.lens, np.int64))

    steps = min(args.exact_steps if steps is None else steps, args.steps)
    # the serial-equivalent committer's cost follows how many rows a batch
    # brings that the model has not seen: it warms up on fresh batches it
    # will not time (the cycled warm pool would leave the model young to the
    # timed stream), the other modes on the warm pool
    spare = fresh.batches[steps * bps:] if mode == "exact" else []
    src = spare if len(spare) >= bps else warm.batches
    nwarm = args.warmup if warmup is None else warmup
    for i in range(nwarm):
        for j in range(bps):
            run(src[(i * bps + j) % len(src)])
        sync()
        _progress(f"{mode}/{weight_dtype}: warmup step {i + 1}/{nwarm} done")
    st0 = clf.train_stats()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        for j in range(bps):
            run(fresh.batches[i * bps + j])
        _progress(f"{mode}/{weight_dtype}: timed step {i + 1}/{steps} queued")
    sync()
    elapsed = time.perf_counter() - t0
    clf.synchronize()
    st1 = clf.train_stats()
    trained = st1["trained"] - st0["trained"]
    updated = st1["updated"] - st0["updated"]
    n = samples_per_batch * bps * steps
    out = {"value": round(n / elapsed, 1), "unit": "samples/s", "steps": steps,
           "ms_per_step": round(elapsed / steps * 1e3, 3), "update_fraction": round(updated / max(1, trained), 5),
           "concurrent_update": mode, "weight_dtype": weight_dtype, "hot_rows": hot_rows}
    if mode == "exact":
        out["semantics"] = "serial-equivalent (requests applied one after another)"
        out["last_batch"] = clf._serial.last_batch() if getattr(clf, "_serial", None) is not None else None
    else:
        out["w_bytes"] = int(clf.W.numel() * clf.W.element_size())
    return out


def exact_shape_records(args, cfg, device, nat, torch, pinned, gen_threads, sync) -> dict:
    """The serial-equivalent mode on other stream shapes: a text-like stream
    (120 string + 8 numeric features a sample: the committer takes samples of
    up to 32 features, wider candidates hand chunks to the stepper) and 64 /
    256 labels (above 64 the batch runs on the single-stream kernel). Label-
    correlated streams; 2 batches a step, one warmup step over batches the
    timed step does not see, one timed step."""
    out = {}
    shapes = (("wide_128_features", {"str_features": 120, "num_features": 8, "requests": 256}),
              ("labels_64", {"labels": 64}),
              ("labels_256", {"labels": 256}))
    for i, (name, over) in enumerate(shapes):
        a = argparse.Namespace(**dict(vars(args), **over))
        _progress(f"exact mode, {name}")
        fs = FreshStream(nat, torch, pinned, a, 9090 + i, 4, gen_threads, 0.6, args.vocab)
        rec = exact_record(a, cfg, device, None, fs, 2, a.requests * a.per_request, sync, mode="exact", steps=1,
                           warmup=1)
        rec["stream"] = {k: v for k, v in over.items() if k != "requests"}
        rec["samples_per_batch"] = a.requests * a.per_request
        out[name] = rec
        del fs
    return out


def cpu_baseline_record(args, cfg, nat, warm_batches, timed_batches, worst_batches) -> dict:
    """The in-house CPU baseline (the reference publishes no
    numbers; its semantics trained on this host are the bar): the servers'
    default serial semantics on the host in native C++
    (csrc/native/jb_cpu_serial.cpp: the same msgpack parse, hasher and update
    rules as the GPU path; one sample after another, as the reference's
    classifier_serv.cpp:138-144), over the same fresh request batches the
    exact-mode record times. ``threads_1``: parse + hash + train on one core;
    ``threads_all``: parse + hash on all cores, the train (sequential by
    definition) on one. The model warms up on ``warm_batches`` first."""
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.fv_converter.gpu_path import GpuRuleTable
    H = int(cfg["converter"]["hash_max_size"])
    rt = GpuRuleTable(DatumToFvConverter(cfg["converter"]))
    hasher = nat.HostFvHasher(rt.srules, rt.n_srules, rt.nrules, rt.n_nrules, rt.blob, H)
    LC = 1
    while LC < args.labels:
        LC *= 2
    LC = max(LC, 8)
    ncpu = max(1, min(16, os.cpu_count() or 1))

    def model():
        table = nat.LabelTable()
        for y in range(args.labels):
            table.get_or_add(f"label{y}")
        return table, np.zeros((H, LC), np.float32), np.ones((H, LC), np.float32)

    active = np.zeros(LC, np.uint8)
    active[:args.labels] = 1

    def run(batches, table, W, P, threads):
        n = u = 0
        sec = 0.0
        for a in batches:
            k, up, dt = nat.cpu_train_arena(hasher, a.np.ctypes.data, np.asarray(a.offs, np.int64),
                                            np.asarray(a.lens, np.int64), table, 5, 1.0, LC,
                                            W.ctypes.data, P.ctypes.data, active, threads)
            n, u, sec = n + k, u + up, sec + dt
        return n, u, sec

    out = {"semantics": "serial (one sample after another), AROW, fp32, native C++ on the host",
           "host_cpus_used_all": ncpu, "warm_batches": len(warm_batches)}
    table, W, P = model()
    run(warm_batches, table, W, P, ncpu)
    W0, P0 = W.copy(), P.copy()
    for name, threads in (("threads_1", 1), ("threads_all", ncpu)):
        W[:], P[:] = W0, P0
        n, u, sec = run(timed_batches, table, W, P, threads)
        out[name] = {"value": round(n / sec, 1), "unit": "samples/s", "batches": len(timed_batches),
                     "update_fraction": round(u / max(1, n), 5), "threads": threads}
    if worst_batches:
        # the worst case on one core and with the parse pool (the train itself
        # is sequential either way)
        for name, threads in (("worst_case_threads_1", 1), ("worst_case", ncpu)):
            table, W, P = model()
            n, u, sec = run(worst_batches, table, W, P, threads)
            out[name] = {"value": round(n / sec, 1), "unit": "samples/s", "batches": len(worst_batches),
                         "update_fraction": round(u / max(1, n), 5), "threads": threads,
                         "data": "worst case: noise string values (every sample updates), fresh model"}
    return out


def _summary(out: dict) -> dict:
    """the records a reader looks for first, flat (the end of the JSON line)"""
    def g(d, *ks):
        for k in ks:
            if not isinstance(d, dict):
                return None
            d = d.get(k)
        return d
    ex = out.get("exact_mode") or {}
    sm = {"headline_samples_per_s": out.get("value"), "headline_update_mode": out.get("headline_update_mode"),
          "exact_mode_samples_per_s": g(ex, "value"), "exact_mode_update_fraction": g(ex, "update_fraction"),
          "exact_worst_case_samples_per_s": g(ex, "worst_case", "value"),
          "exact_worst_case_stepper_samples": g(ex, "worst_case", "last_batch", "stepper_samples"),
          "exact_wide_samples_per_s": g(ex, "shapes", "wide_128_features", "value"),
          "exact_wide_update_fraction": g(ex, "shapes", "wide_128_features", "update_fraction"),
          "exact_labels_64_samples_per_s": g(ex, "shapes", "labels_64", "value"),
          "exact_labels_256_samples_per_s": g(ex, "shapes", "labels_256", "value"),
          "cpu_threads_1": g(ex, "cpu_baseline", "threads_1", "value"),
          "cpu_threads_all": g(ex, "cpu_baseline", "threads_all", "value"),
          "cpu_worst_threads_1": g(ex, "cpu_baseline", "worst_case_threads_1", "value"),
          "cpu_worst_threads_all": g(ex, "cpu_baseline", "worst_case", "value"),
          "gpu_exact_worst_vs_cpu_worst_threads_1": g(ex, "cpu_baseline", "gpu_exact_worst_vs_cpu_worst_threads_1"),
          "bf16_weights_samples_per_s": g(out, "bf16_weights", "value"),
          "atomic_worst_case_samples_per_s": g(out, "worst_case", "value"),
          "served_native_samples_per_s": g(out, "served_native", "served_train_samples_per_sec"),
          "served_native_cpus": g(out, "served_native", "server_cpus"),
          "served_native_exact_samples_per_s": g(out, "served_native", "exact_mode", "served_train_samples_per_sec"),
          "served_native_learning_exact_samples_per_s": g(out, "served_native", "learning_stream_exact",
                                                          "served_train_samples_per_sec"),
          "served_native_learning_exact_p99_us": g(out, "served_native", "learning_stream_exact", "rpc_p99_us"),
          "classify_rpc_p50_us": g(out, "served_native", "classify_rpc_p50_us"),
          "classify_latency_us_p50": out.get("classify_latency_us_p50")}
    eng = out.get("engines") or {}
    for name, rec in eng.items():
        if isinstance(rec, dict):
            for k, v in rec.items():
                if k.endswith(("_per_s_fill", "_p50_us", "_per_s", "_points_per_s")) and isinstance(v, (int, float)):
                    sm[f"{name}.{k}"] = v
    for name, rec in (out.get("engines_dist") or {}).items():
        if isinstance(rec, dict):
            for k, v in rec.items():
                if k.endswith("_per_s_total") or k in ("mix_latency_ms", "members_agree_after_mix", "server_runtime"):
                    sm[f"dist.{name}.{k}"] = v
            if rec.get("mix_line_per_rank"):
                sm[f"dist.{name}.mix_line_rank0"] = rec["mix_line_per_rank"][0]
    return {k: v for k, v in sm.items() if v is not None}


def _mix_summary(log: list) -> dict:
    """per-MIX bytes per rank and host-observed latency (begin -> done) of
    the MIXes completed in the timed steps"""
    if not log:
        return {"count": 0}
    lat = sorted(m["latency_ms"] for m in log if m.get("latency_ms") is not None)
    modes = {}
    for m in log:
        modes[m.get("mode")] = modes.get(m.get("mode"), 0) + 1
    return {"count": len(log), "world": log[-1].get("world"), "modes": modes,
            "bytes_per_rank_mean": int(np.mean([m.get("bytes", 0) for m in log])),
            "rows_mean": int(np.mean([m.get("rows", 0) for m in log])),
            "latency_ms_p50": lat[len(lat) // 2] if lat else None,
            "latency_ms_max": lat[-1] if lat else None}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--requests", type=int, default=1024, help="concurrent train requests per batch per GPU")
    ap.add_argument("--per-request", type=int, default=128, help="samples per train request")
    ap.add_argument("--batches-per-step", type=int, default=0,
                    help="train batches per timed step (0: as many as the fresh-data budget allows, "
                         "at most 96, so that the timed region lasts about a second)")
    ap.add_argument("--fresh-gb", type=float, default=0.0,
                    help="host memory for the non-repeating timed stream per rank "
                         "(0: min(56 GB, 60%% of MemAvailable / local ranks))")
    ap.add_argument("--labels", type=int, default=16)
    ap.add_argument("--str-features", type=int, default=8)
    ap.add_argument("--num-features", type=int, default=8)
    ap.add_argument("--vocab", type=int, default=100000)
    ap.add_argument("--hash-bits", type=int, default=20)
    ap.add_argument("--worst-case", action="store_true",
                    help="string values are fresh noise: (almost) every sample updates the model")
    ap.add_argument("--warmup-pools", type=int, default=4, help="distinct batches cycled by warmup")
    ap.add_argument("--mix-every", type=int, default=0,
                    help="N > 0: MIX every N batches; 0 (default): the reference's trigger - a new MIX "
                         "starts as soon as the previous one has finished and updates arrived "
                         "(linear_mixer.cpp:337-344,358-390: interval_count 512 updates, the mixer "
                         "wakes on the threshold), agreed across ranks each batch")
    ap.add_argument("--latency-iters", type=int, default=300)
    ap.add_argument("--engines", default="all",
                    help="engine records (N = 1): all, none, or a comma list of "
                         + ", ".join(c[0] for c in ENGINE_CASES) + ", clustering_kmeans, clustering_gmm")
    ap.add_argument("--engine-rows", type=int, default=1_000_000,
                    help="rows filled into the recommender servers before their queries")
    ap.add_argument("--lof-rows", type=int, default=100_000,
                    help="rows added to the LOF server before its queries")
    ap.add_argument("--engine-seconds", type=float, default=3.0)
    ap.add_argument("--dist-engines", default="lof,kmeans,gmm,arow",
                    help="N > 1: distributed engine records (lof,kmeans,gmm,arow / all / none): one server per "
                         "rank in one cluster, a forced MIX, queries on every member")
    ap.add_argument("--dist-engine-rows", type=int, default=0,
                    help="LOF rows each rank adds (0: 100000 on GPUs, 300 with --device cpu)")
    ap.add_argument("--dist-cluster-points", type=int, default=0,
                    help="points each rank pushes into its clustering server (0: 200000 on GPUs, 3000 on cpu)")
    ap.add_argument("--dist-train-seconds", type=float, default=3.0,
                    help="N > 1: length of the served AROW train window per rank (MIX every second)")
    ap.add_argument("--dist-engine-seconds", type=float, default=1.5)
    ap.add_argument("--cluster-points", type=int, default=200_000,
                    help="points pushed into each clustering server (kmeans.json, gmm.json)")
    ap.add_argument("--no-rpc", action="store_true",
                    help="skip the served-path measurement (jubaclassifier + jubaloadgen, N = 1)")
    ap.add_argument("--served-runtime", choices=("python", "native", "both"), default="both",
                    help="which server --served-only measures")
    ap.add_argument("--served-only", action="store_true",
                    help="measure only the served path (prints its record; not the headline)")
    ap.add_argument("--rpc-seconds", type=float, default=4.0)
    ap.add_argument("--rpc-conns", type=int, default=64)
    ap.add_argument("--rpc-depth", type=int, default=32)
    ap.add_argument("--rpc-threads", type=int, default=32,
                    help="server RPC threads (a quarter of them are epoll IO threads)")
    ap.add_argument("--rpc-distinct", type=int, default=512, help="distinct train requests cycled")
    ap.add_argument("--rpc-fresh", type=int, default=1,
                    help="1 (default): the load generator redraws a numeric value of every sample it "
                         "sends, so no served sample repeats; 0: the distinct requests are replayed as is")
    ap.add_argument("--update-mode", choices=("exact", "atomic", "hogwild"), default="atomic",
                    help="how the concurrent requests of a batch update the headline model: exact = "
                         "the result of applying them one after the other (csrc/hip/serial.hip); "
                         "atomic / hogwild = lock-free concurrent streams")
    ap.add_argument("--exact-steps", type=int, default=3,
                    help="1 GPU: also time this many steps of the serial-equivalent exact mode (same "
                         "warmup, same fresh batches, its own model) and report them under exact_mode")
    ap.add_argument("--worst-steps", type=int, default=5,
                    help="1 GPU: also time this many steps (16 batches each) of the headline's update "
                         "mode on the worst-case stream (noise string values: every sample updates) "
                         "and report them under worst_case")
    ap.add_argument("--exact-shapes", type=int, default=1,
                    help="1: exact-mode records on a text-like stream and on 64 / 256 labels")
    ap.add_argument("--cpu-baseline", type=int, default=1,
                    help="1: the in-house CPU baseline record (serial semantics on the host) beside exact_mode")
    ap.add_argument("--weight-dtype", choices=("fp32", "bf16"), default="fp32",
                    help="storage of the headline model's W table (P and arithmetic stay fp32)")
    ap.add_argument("--bf16-steps", type=int, default=5,
                    help="1 GPU, fp32 headline: also time this many steps with a bf16 W table (same "
                         "warmup, same fresh batches, its own model) and report them under bf16_weights")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="gloo: rehearse the multi-rank GPU path with several ranks on one GPU "
                         "(not a benchmark configuration)")
    ap.add_argument("--device", choices=("gpu", "cpu"), default="gpu",
                    help="cpu: host engine + gloo, for rehearsing the multi-rank path without a GPU "
                         "(not a benchmark configuration)")
    ap.add_argument("--mix-mode", choices=("overlap", "sync"), default="overlap",
                    help="overlap: the RCCL all-reduce of batch k runs during batch k+1 and its "
                         "mean is folded in afterwards (updates made meanwhile are kept); "
                         "sync: blocking MIX at the end of every batch")
    ap.add_argument("--mix-dtype", choices=("fp32", "bf16"), default="fp32",
                    help="bf16: the MIX all-reduce moves bf16 values (half the bytes; the snapshot and "
                         "the fold stay fp32, the mean is rounded once per MIX)")
    args = ap.parse_args()
    os.environ["JUBATUS_MIX_DTYPE"] = args.mix_dtype     # parallel/table_mix.py (read at import)

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one rank per GPU: launch them before this process touches the GPU
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
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

    from jubatus_amd._native import native
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier

    cfg = json.loads(json.dumps(AROW_CONFIG))
    cfg["converter"]["hash_max_size"] = 1 << args.hash_bits
    conv = DatumToFvConverter(cfg["converter"])
    clf = LinearClassifier(cfg["method"], cfg["parameter"], conv, device=device,
                           concurrent_update=args.update_mode, weight_dtype=args.weight_dtype)
    for y in range(args.labels):  # same label order on every rank (set_label, as a client would)
        clf.set_label(f"label{y}")

    nat = native()
    if args.served_only:
        out = {}
        if args.served_runtime in ("python", "both"):
            out["python"] = served_train(args, local, nat)
        if args.served_runtime in ("native", "both"):
            out["native"] = served_train_native(args, local, nat)
        out["arena_threads"] = os.environ.get("JUBATUS_ARENA_THREADS", "2")
        print(json.dumps(out), flush=True)
        return
    gen_threads = max(1, min(16, (os.cpu_count() or 8) // max(1, local_world)))
    p_corr, vocab = (0.0, (1 << 31) - 1) if args.worst_case else (0.6, args.vocab)
    pinned = device is not None
    # warmup data: its own seed, a few batches cycled (untimed)
    warm = FreshStream(nat, torch, pinned, args, 1_000_003 * (rank + 1) + 17,
                       max(1, args.warmup_pools), gen_threads, p_corr, vocab)
    batch_bytes = warm.nbytes / max(1, len(warm.batches))
    if args.batches_per_step > 0:
        bps = args.batches_per_step
    else:
        budget = fresh_budget(args.fresh_gb, local_world)
        bps = int(budget // max(1.0, batch_bytes * args.steps))
        bps = max(1, min(96, bps))
    t_gen = time.perf_counter()
    fresh = FreshStream(nat, torch, pinned, args, 7_919 * (rank + 1) + 3, bps * args.steps,
                        gen_threads, p_corr, vocab)
    t_gen = time.perf_counter() - t_gen
    samples_per_batch = args.requests * args.per_request
    samples_per_step = samples_per_batch * bps

    # host-side metadata (label agreement, count deltas) rides on a gloo group
    # so the MIX never forces a GPU synchronisation
    meta = dist.new_group(backend="gloo") if world > 1 else None
    pending = [None]

    def barrier():
        if world > 1:
            dist.barrier()

    mix_log = []          # per-MIX stats (bytes per rank, begin->done latency) of the timed steps

    def finish_mix():
        if pending[0] is not None:
            clf.mix_end(pending[0])
            pending[0] = None
            mix_log.append(dict(clf._last_mix))

    mixes = [0]
    agreed = {"version": None, "labels": False}
    inflight = {"work": None, "flags": None}
    nbatch = [0]

    def mix_due() -> bool:
        i = nbatch[0]
        if args.mix_every > 0 or args.mix_mode == "sync":
            return (i + 1) % max(1, args.mix_every) == 0
        # adaptive: every rank must agree (the collectives have to match).
        # One tiny host all-reduce per batch carries [not ready, labels
        # changed]; it is issued asynchronously and read one batch later, so
        # the host never waits on it (all ranks act on the same lagged flags)
        due = False
        if inflight["work"] is not None:
            inflight["work"].wait()
            f = inflight["flags"]
            agreed["labels"] = f[1].item() == 0
            due = f[0].item() == 0
        v = clf.labels.version()
        # a MIX that starts this batch is not finished by the next one
        flags = torch.tensor([0 if (not due and clf.mix_ready(pending[0])) else 1,
                              0 if v == agreed["version"] else 1], dtype=torch.int32)
        inflight["flags"] = flags
        inflight["work"] = dist.all_reduce(flags, op=dist.ReduceOp.MAX, group=meta, async_op=True)
        return due

    def train_batch(arena) -> None:
        offs = np.asarray(arena.offs, np.int64)
        lens = np.asarray(arena.lens, np.int64)
        n = clf.train_arena(arena, offs, lens)
        assert n == samples_per_batch
        if world > 1 and mix_due():
            mixes[0] += 1
            if args.mix_mode == "sync":
                t1 = time.perf_counter()
                clf.mix()
                mix_log.append(dict(clf._last_mix, latency_ms=round((time.perf_counter() - t1) * 1e3, 3)))
            else:
                finish_mix()
                v = clf.labels.version()
                pending[0] = clf.mix_begin(meta_group=meta,
                                           agreed_version=agreed["version"] if agreed["labels"] else None)
                if "sync" not in pending[0] and clf.labels.version() == v:
                    agreed["version"] = v
        nbatch[0] += 1

    # setup objects (synthetic bodies, torch modules) move to the permanent
    # generation, so a cyclic-GC pass in the timed loop does not traverse them
    import gc
    gc.collect()
    gc.freeze()
    _progress(f"data ready ({t_gen:.1f} s): {bps} batches x {args.steps} steps; warmup")
    for i in range(args.warmup):
        for j in range(bps):
            train_batch(warm.batches[(i * bps + j) % len(warm.batches)])
        sync()
        _progress(f"warmup step {i + 1}/{args.warmup} done")
    finish_mix()
    if device is not None:
        clf.pipe.check_errors()
    sync()
    st0 = clf.train_stats()
    barrier()
    sync()
    trace_steps = os.environ.get("JB_BENCH_TRACE") == "1"
    marks = []
    mixes[0] = 0
    mix_log.clear()
    t0 = time.perf_counter()
    for i in range(args.steps):
        for j in range(bps):
            train_batch(fresh.batches[i * bps + j])
        if trace_steps:
            marks.append(time.perf_counter())
        if rank == 0 and (i + 1) % 5 == 0:
            _progress(f"timed step {i + 1}/{args.steps} queued")
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
    clf.synchronize()     # label-count records of the last batches
    st1 = clf.train_stats()
    trained = st1["trained"] - st0["trained"]
    updated = st1["updated"] - st0["updated"]
    replayed = clf._scan_stats.get("replayed", 0)

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

    exact = None
    if world == 1 and device is not None and args.exact_steps > 0 and args.update_mode != "exact":
        exact = exact_record(args, cfg, device, warm, fresh, bps, samples_per_batch, sync)
    bf16 = None
    if world == 1 and device is not None and args.bf16_steps > 0 and args.weight_dtype == "fp32":
        bf16 = exact_record(args, cfg, device, warm, fresh, bps, samples_per_batch, sync,
                            mode=args.update_mode, weight_dtype="bf16", steps=args.bf16_steps)
    worst = None
    if world == 1 and device is not None and args.worst_steps > 0 and not args.worst_case:
        # the headline's update mode on the worst-case stream: string values
        # are fresh noise, so (almost) every sample updates the model
        wb = 16
        ws = FreshStream(nat, torch, pinned, args, 31_337 * (rank + 1) + 5, wb * args.worst_steps,
                         gen_threads, 0.0, (1 << 31) - 1)
        worst = exact_record(args, cfg, device, warm, ws, wb, samples_per_batch, sync,
                             mode=args.update_mode, steps=args.worst_steps)
        worst["data"] = "worst case: noise string values (every sample a new feature set), fresh stream"
        worst["batches_per_step"] = wb
        # the same with the hot-row LDS replica (opt-in, JUBATUS_HOT_ROWS=1:
        # rows every stream writes - here the 8 numeric keys - are merged in
        # LDS instead of contended with device-scope atomics)
        hot = exact_record(args, cfg, device, warm, ws, wb, samples_per_batch, sync,
                           mode=args.update_mode, steps=args.worst_steps, hot_rows=True)
        worst["hot_rows_replica"] = {k: hot[k] for k in ("value", "ms_per_step", "update_fraction")}
        if exact is not None:
            # the servers' default (serial-equivalent) mode on the same stream
            ew = exact_record(args, cfg, device, warm, ws, wb, samples_per_batch, sync,
                              mode="exact", steps=min(2, args.worst_steps))
            ew["data"] = worst["data"]
            ew["batches_per_step"] = wb
            exact["worst_case"] = ew
        if args.exact_shapes and exact is not None:
            exact["shapes"] = exact_shape_records(args, cfg, device, nat, torch, pinned, gen_threads, sync)
        if args.cpu_baseline and exact is not None:
            _progress("cpu baseline (host serial trainer)")
            spare = fresh.batches[min(args.exact_steps, args.steps) * bps:]
            tb = fresh.batches[:min(len(fresh.batches), 8)]
            exact["cpu_baseline"] = cpu_baseline_record(args, cfg, nat, spare[:96], tb, ws.batches[:4])
            for k in ("threads_1", "threads_all"):
                exact["cpu_baseline"][f"gpu_exact_vs_{k}"] = round(
                    exact["value"] / max(1.0, exact["cpu_baseline"][k]["value"]), 2)
            exact["cpu_baseline"]["gpu_exact_worst_vs_cpu_worst"] = round(
                exact["worst_case"]["value"] / max(1.0, exact["cpu_baseline"]["worst_case"]["value"]), 2)
            exact["cpu_baseline"]["gpu_exact_worst_vs_cpu_worst_threads_1"] = round(
                exact["worst_case"]["value"] / max(1.0, exact["cpu_baseline"]["worst_case_threads_1"]["value"]), 2)
        del ws
    served = served_native = None
    if world == 1 and device is not None and not args.no_rpc:
        served = served_train(args, local, nat)
        served_native = served_train_native(args, local, nat)
        if isinstance(served_native, dict) and "error" not in served_native:
            # the servers' default (serial-equivalent) mode over RPC, and a
            # stream that keeps learning (2 % of the samples all-new tokens)
            served_native["exact_mode"] = served_train_native(args, local, nat, mode="exact", classify=False)
            served_native["learning_stream"] = served_train_native(args, local, nat, noise_pm=20,
                                                                   classify=False)
            served_native["learning_stream_exact"] = served_train_native(args, local, nat, mode="exact",
                                                                         noise_pm=20, classify=False)
    engines = None
    if world == 1 and device is not None and args.engines != "none":
        engines = engine_records(args, local)
    engines_dist = None
    if world > 1 and args.dist_engines != "none":
        if args.dist_engine_rows <= 0:
            args.dist_engine_rows = 100_000 if device is not None else 300
        if args.dist_cluster_points <= 0:
            args.dist_cluster_points = 200_000 if device is not None else 3000
        try:
            engines_dist = dist_engine_records(args, rank, world, local, device, meta)
        except Exception as e:  # noqa: BLE001 - the headline stands without it
            engines_dist = {"error": repr(e)[:300]}

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
            "dtype": "fp32" if args.weight_dtype == "fp32" else "bf16 W, fp32 P and arithmetic",
            "data": ("synthetic, non-repeating: every timed sample is new (native generator, pinned "
                     "host memory, H2D inside the timed region); "
                     + ("worst case: noise string values, every sample updates; " if args.worst_case
                        else "label-correlated datums; ")
                     + "8 str + 8 num features, zero-init model"),
            "config": {
                "model": "jubaclassifier AROW (config/classifier/arow.json: regularization_weight 1.0, "
                         "str bin/bin + num)",
                "global_batch": samples_per_step * world,
                "seq_len": None,
                "parallelism": f"dp{world}",
                "batches_per_step": bps,
                "requests_per_batch_per_gpu": args.requests,
                "samples_per_request": args.per_request,
                "hash_max_size": 1 << args.hash_bits,
                "labels": args.labels,
                "mix": (f"linear, RCCL all-reduce mean of the touched rows of W and P (sparse; "
                        f"chunked dense past half the table), {args.mix_mode}, "
                        + (f"every {args.mix_every} batch(es)" if args.mix_every > 0 else
                           "back to back (a new MIX as soon as the previous one finished)")
                        + f"; {mixes[0]} MIXes in the timed steps; {args.mix_dtype} on the wire")
                       if world > 1 else "standalone",
                "concurrent_update": args.update_mode,
                "hot_rows": clf.hot_rows,
                "numa_node": numa.get("node"),
                "world_size_observed": world,
            },
            "timed_region_s": round(elapsed, 3),
            "timed_samples_per_rank": samples_per_step * args.steps,
            "timed_bytes_per_rank": int(fresh.nbytes),
            "update_fraction": round(updated / trained, 4) if trained else None,
            "mix_last": getattr(clf, "_last_mix", {}),
            "mix_timed": _mix_summary(mix_log),
            "pinned_bytes_per_rank": int(fresh.nbytes + warm.nbytes) if pinned else 0,
            "pinned_budget": ({"fresh_gb_flag": args.fresh_gb,
                               "rule": f"min({PIN_CAP / 1e9:.0f} GB, {PIN_FRACTION} x MemAvailable / local ranks)",
                               "host_mem_available_bytes": int(_mem_available()), "local_ranks": local_world}
                              if args.batches_per_step <= 0 else {"batches_per_step_flag": bps}),
            "samples_replayed_batches": replayed,
            "data_gen_s": round(t_gen, 1),
            "headline_update_mode": args.update_mode,
            "servers_default_update_mode": "exact",
            "exact_mode_value": exact["value"] if exact else (round(value, 1) if args.update_mode == "exact" else None),
            "exact_mode": exact,
            "bf16_weights": bf16,
            "worst_case": worst,
            "served": served,
            "served_native": served_native,
            "engines": engines,
            "engines_dist": engines_dist,
            "classify_latency_us_p50": round(p50, 1),
            "classify_latency_us_p99": round(p99, 1),
            "heldout_accuracy": round(acc, 4),
            "baseline_note": "reference publishes no numbers (BASELINE.md)",
        }
        # the key records again, last: the driver keeps the tail of the line
        out["summary"] = _summary(out)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
