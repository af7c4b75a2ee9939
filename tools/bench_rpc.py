#!/usr/bin/env python3
"""End-to-end RPC latency of the flagship server (1 GPU): msgpack-RPC client
-> jubaclassifier (AROW, GPU) directly, and through the native coordinator
+ native proxy (distributed mode, one server) - the reference's
client -> proxy -> server path.

Prints one JSON line: classify / train p50/p99 per path, and
get_proxy_status of the native proxy.

Usage: python tools/bench_rpc.py [iters]   (needs the native binaries:
python -m jubatus_amd.build_ext)
"""
from __future__ import annotations

import json
import os
import random
import socket
import statistics
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def lat(fn, iters):
    for _ in range(20):
        fn()
    xs = []
    for _ in range(iters):
        t = time.perf_counter()
        fn()
        xs.append((time.perf_counter() - t) * 1e6)
    xs.sort()
    return {"p50_us": round(statistics.median(xs), 1), "p99_us": round(xs[int(0.99 * (len(xs) - 1))], 1)}


def wait_port(port, timeout=120):
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            socket.create_connection(("127.0.0.1", port), 0.5).close()
            return True
        except OSError:
            time.sleep(0.2)
    return False


def _client_proc(args):
    """one load-generating client process: pre-encoded train RPCs for `secs`"""
    port, name, body, secs, per = args
    sys.path.insert(0, ROOT)
    from jubatus_amd.common.mprpc import RpcClient
    c = RpcClient("127.0.0.1", port, 60)
    n = 0
    t_end = time.time() + secs
    while time.time() < t_end:
        assert c.call_raw("train", body) == per
        n += per
    c.close()
    return n


def concurrent_train(port, name, enc_train, nproc=16, secs=4.0):
    """samples/s of the server under nproc concurrent clients (the server's
    micro-batcher merges their train RPCs into shared launches)"""
    import multiprocessing as mp
    from jubatus_amd.common.mprpc import packb
    body = packb([name, enc_train])
    with mp.get_context("spawn").Pool(nproc) as pool:
        t0 = time.time()
        counts = pool.map(_client_proc, [(port, name, body, secs, len(enc_train))] * nproc)
        dt = time.time() - t0
    return round(sum(counts) / dt, 1)


def loadgen(port, method, params, per, conns=16, depth=4, secs=4.0):
    """native load generator (csrc/tools/jubaloadgen.cpp): `conns` connections
    x `depth` requests in flight; the server batches them per launch"""
    from jubatus_amd import build_ext
    f = tempfile.NamedTemporaryFile(delete=False, suffix=".bin")
    f.write(params)
    f.close()
    r = subprocess.run([os.path.join(build_ext.NATIVE_BIN, "jubaloadgen"), "-p", str(port), "-m", method,
                        "-f", f.name, "-c", str(conns), "-d", str(depth), "-t", str(secs)],
                       capture_output=True, text=True, timeout=secs + 60)
    os.unlink(f.name)
    if r.returncode != 0:
        return {"error": r.stderr.strip()}
    d = json.loads(r.stdout)
    d["samples_per_s"] = round(d["requests_per_s"] * per, 1)
    return d


class _SkipPython(Exception):
    pass


def main():
    native_only = "--native-only" in sys.argv
    argv = [a for a in sys.argv[1:] if a != "--native-only"]
    iters = int(argv[0]) if argv else 500
    from jubatus_amd import build_ext
    from jubatus_amd.client import Classifier, Datum
    from jubatus_amd.common import config as zkconfig
    from jubatus_amd.common import membership as mb
    from jubatus_amd.common.coordinator import NativeCoordinator
    from jubatus_amd.common.lock_service import CoordinatorClient

    build_ext.build_tools()
    build_ext.build_servers()
    env = dict(os.environ, PYTHONPATH=ROOT)
    cfg = os.path.join(ROOT, "config", "classifier", "arow.json")
    tmp = tempfile.mkdtemp()
    rng = random.Random(0)

    def datum(y):
        return Datum({**{f"s{j}": f"t{y * 7 + rng.randrange(4)}" for j in range(8)},
                      **{f"n{j}": y + rng.gauss(0, 1) for j in range(8)}})

    train = [(f"l{y}", datum(y)) for y in [rng.randrange(16) for _ in range(128)]]
    one = [datum(3)]
    out = {"model": "jubaclassifier AROW (config/classifier/arow.json)", "device": "MI355X",
           "note": "latency at the client; *_client_api includes Python client encoding"}
    from jubatus_amd.common.mprpc import RpcClient, packb
    enc_train = [[lab, d.to_msgpack()] for lab, d in train]
    enc_one = [d.to_msgpack() for d in one]
    cache = {}

    def p_train(name):
        return cache.setdefault(("t", name), packb([name, enc_train]))

    def p_one(name):
        return cache.setdefault(("c", name), packb([name, enc_one]))
    procs = []
    coord = None
    try:
        # standalone server, client -> server
        sp = free_port()
        if native_only:
            raise _SkipPython()
        procs.append(subprocess.Popen([sys.executable, "-m", "jubatus_amd.cmd.server", "classifier",
                                       "-p", str(sp), "-b", "127.0.0.1", "-f", cfg, "-d", tmp, "-c", "16"],
                                      env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        assert wait_port(sp), "server did not start"
        c = Classifier("127.0.0.1", sp, "", timeout=30)
        for _ in range(20):
            c.train(train)
        out["direct_train_128_client_api"] = lat(lambda: c.train(train), iters // 5)
        out["direct_classify_1_client_api"] = lat(lambda: c.classify(one), iters)
        c.close()
        # pre-encoded params (the server-side cost, without Python client encoding)
        rc = RpcClient("127.0.0.1", sp, 30)
        out["direct_train_128"] = lat(lambda: rc.call_raw("train", p_train("")), iters // 5)
        out["direct_classify_1"] = lat(lambda: rc.call_raw("classify", p_one("")), iters)
        rc.close()
        out["direct_concurrent_train_samples_per_s_py_clients"] = concurrent_train(sp, "", enc_train)
        out["direct_loadgen_train"] = loadgen(sp, "train", p_train(""), len(enc_train))
        # 1024 requests in flight (the in-process bench's concurrency)
        out["direct_loadgen_train_1024_inflight"] = loadgen(sp, "train", p_train(""), len(enc_train),
                                                            conns=64, depth=16)
        out["direct_loadgen_classify_1"] = loadgen(sp, "classify", p_one(""), 1, conns=8, depth=1)
        out["direct_loadgen_classify_1_single_conn"] = loadgen(sp, "classify", p_one(""), 1, conns=1,
                                                               depth=1)
        rc = RpcClient("127.0.0.1", sp, 30)
        (_, st), = rc.call("get_status", "").items()
        out["server_spans"] = {k: v for k, v in st.items()
                               if k.startswith(("trace.rpc.train", "trace.rpc.classify", "trace.hip.", "trace.batch.",
                                                "trace.pipe.",
                                                "batching."))}
        rc.close()
    except _SkipPython:
        pass
    try:
        # the native server binary (csrc/server/jubaclassifier.cpp), same calls
        nbin = os.path.join(build_ext.NATIVE_BIN, "jubaclassifier")
        if os.access(nbin, os.X_OK):
            npt = free_port()
            procs.append(subprocess.Popen([nbin, "-p", str(npt), "-b", "127.0.0.1", "-f", cfg, "-d", tmp,
                                           "-c", "16"], stdout=subprocess.DEVNULL,
                                          stderr=subprocess.DEVNULL))
            assert wait_port(npt), "native server did not start"
            rc = RpcClient("127.0.0.1", npt, 30)
            for _ in range(20):
                rc.call_raw("train", p_train(""))
            (_, st), = rc.call("get_status", "").items()
            out["native_server_runtime"] = st.get("server_runtime", "python")
            out["native_direct_train_128"] = lat(lambda: rc.call_raw("train", p_train("")), iters // 5)
            out["native_direct_classify_1"] = lat(lambda: rc.call_raw("classify", p_one("")), iters)
            rc.close()
            out["native_loadgen_classify_1"] = loadgen(npt, "classify", p_one(""), 1, conns=8, depth=1)
            out["native_loadgen_classify_1_single_conn"] = loadgen(npt, "classify", p_one(""), 1,
                                                                   conns=1, depth=1)
            rc = RpcClient("127.0.0.1", npt, 30)
            (_, st), = rc.call("get_status", "").items()
            out["native_status"] = {k: v for k, v in st.items() if k.startswith(("served.", "train_scan."))}
            rc.close()
        if native_only:
            raise _SkipPython()
        # distributed: native coordinator + server + native proxy
        coord = NativeCoordinator(0, "127.0.0.1")
        ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=10.0)
        zkconfig.config_tozk(ls, "classifier", "bench", open(cfg).read())
        dp = free_port()
        procs.append(subprocess.Popen([sys.executable, "-m", "jubatus_amd.cmd.server", "classifier",
                                       "-p", str(dp), "-b", "127.0.0.1", "-z", f"127.0.0.1:{coord.port}",
                                       "-n", "bench", "-d", tmp], env=env,
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        deadline = time.time() + 120
        while time.time() < deadline and not mb.get_all_actives(ls, "classifier", "bench"):
            time.sleep(0.2)
        pp = free_port()
        px = subprocess.Popen([os.path.join(build_ext.NATIVE_BIN, "jubaproxy"), "classifier",
                               "-p", str(pp), "-b", "127.0.0.1", "-z", f"127.0.0.1:{coord.port}"],
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True)
        procs.append(px)
        assert px.stdout.readline().startswith("jubaproxy ready")
        c = Classifier("127.0.0.1", pp, "bench", timeout=30)
        for _ in range(20):
            c.train(train)
        rc = RpcClient("127.0.0.1", pp, 30)
        out["proxy_train_128"] = lat(lambda: rc.call_raw("train", p_train("bench")), iters // 5)
        out["proxy_classify_1"] = lat(lambda: rc.call_raw("classify", p_one("bench")), iters)
        rc.close()
        (_, st), = c.get_proxy_status().items()
        out["proxy_status"] = {k: st[k] for k in ("request_count", "forward_count", "implementation")}
        c.close()
        ls.close()
    except _SkipPython:
        pass
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(15)
            except subprocess.TimeoutExpired:
                p.kill()
        if coord is not None:
            coord.stop()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
