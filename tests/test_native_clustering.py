"""Native jubaclustering (csrc/server/jubaclustering.cpp: no Python; coresets,
k-means++ / Lloyd / GMM EM on the GPU) against the Python driver
(models/clustering.py) on the GPU fed the same pushes: revisions, k centers,
core members, nearest center / members, model files read by the Python
driver and by a second native server, clear. The configuration check alone
runs on the CPU. Reference: clustering_serv.cpp:71-151."""
import json
import math
import os
import random
import socket
import subprocess
import time

import pytest

from helpers import ROOT
from jubatus_amd.common.mprpc import RpcClient, RpcIOError, RpcTimeoutError

NATIVE = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaclustering")

pytestmark = pytest.mark.skipif(not os.path.exists(NATIVE), reason="native jubaclustering not built")


def _check(path):
    r = subprocess.run([NATIVE, "--native-check", "-f", str(path)], capture_output=True, text=True, timeout=30)
    return r.stdout.strip()


def test_native_clustering_config_check(tmp_path):
    d = os.path.join(ROOT, "config", "clustering")
    for f in sorted(os.listdir(d)):    # default.json too: tf-idf bigrams (DocStats)
        assert _check(os.path.join(d, f)) == "native", f
    base = json.load(open(os.path.join(d, "kmeans.json")))
    for conv, why in (({"string_rules": [{"key": "/re/", "type": "str"}]}, "regex"),):
        p = tmp_path / "c.json"
        p.write_text(json.dumps(dict(base, converter=conv)))
        out = _check(p)
        assert out.startswith("python:"), out
    p = tmp_path / "c.json"
    p.write_text(json.dumps(dict(base, method="dbscan")))
    assert _check(p).startswith("python:")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _start(tmp_path, cfg_path=None, model=None):
    port = _free_port()
    cmd = [NATIVE, "-p", str(port), "-b", "127.0.0.1", "-d", str(tmp_path)]
    cmd += ["-m", model] if model else ["-f", str(cfg_path)]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    deadline = time.time() + 60
    while True:
        try:
            with RpcClient("127.0.0.1", port, 5.0) as c:
                c.call("get_config", "")
            return p, port
        except (OSError, RpcIOError, RpcTimeoutError):
            assert p.poll() is None and time.time() < deadline, p.stdout.read()
            time.sleep(0.1)


def _s(x):
    return x.decode() if isinstance(x, bytes) else x


def _datum(rng, c):
    cx, cy = ((0, 0), (6, 1), (2, 7))[c]
    return [[["tag", "abc"[c]]], [["x", round(cx + rng.gauss(0, 1), 4)], ["y", round(cy + rng.gauss(0, 1), 4)]],
            []]


def _num(d):
    return {_s(k): float(v) for k, v in d[1]}


def _same_centers(got, want):
    assert len(got) == len(want)
    for g, w in zip(got, want):
        g, w = _num(g), _num(w)
        assert sorted(g) == sorted(w), (g, w)
        for k in g:
            assert math.isclose(g[k], w[k], rel_tol=1e-3, abs_tol=1e-3), (k, g, w)


def _norm_datum(d):
    return [[[_s(k), _s(v)] for k, v in d[0]], [[_s(k), float(v)] for k, v in d[1]], list(d[2])]


def _same_members(got, want):
    assert len(got) == len(want)
    for (gw, gd), (ww, wd) in zip(got, want):
        assert math.isclose(gw, ww, rel_tol=1e-4), (gw, ww)
        assert _norm_datum(gd) == _norm_datum(wd)


@pytest.mark.gpu
@pytest.mark.parametrize("method,compressor,gw", [("kmeans", "compressive_kmeans", "bin"), ("kmeans", "simple", "bin"),
                                                  ("gmm", "compressive_gmm", "bin"),
                                                  ("kmeans", "compressive_kmeans", "idf")])
def test_native_clustering_matches_python_driver(method, compressor, gw, tmp_path):
    import torch
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.fv_converter.datum import Datum
    from jubatus_amd.framework.save_load import read_model_file
    from jubatus_amd.models.clustering import Clustering
    conv = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "tf" if gw == "idf" else "bin",
                              "global_weight": gw}],
            "num_rules": [{"key": "*", "type": "num"}]}
    par = {"k": 3, "compressor_method": compressor, "bucket_size": 60, "compressed_bucket_size": 12,
           "bicriteria_base_size": 4, "bucket_length": 2, "forgetting_factor": 0.0, "forgetting_threshold": 0.5,
           "seed": 7}
    cfg = {"method": method, "parameter": par, "converter": conv}
    path = tmp_path / "c.json"
    path.write_text(json.dumps(cfg))
    dev = torch.device("cuda:0")
    ref = Clustering(method, par, DatumToFvConverter(conv), device=dev)
    p, port = _start(tmp_path, path)
    p2 = None
    try:
        rng = random.Random(11)
        with RpcClient("127.0.0.1", port, 30.0) as c:
            with pytest.raises(Exception):
                c.call("get_k_center", "")
            for _ in range(9):
                batch = [_datum(rng, rng.randrange(3)) for _ in range(rng.randrange(20, 45))]
                assert c.call("push", "", batch) is True
                ref.push([Datum.from_msgpack(d) for d in batch])
                assert c.call("get_revision", "") == ref.get_revision()
            assert ref.get_revision() >= 3
            _same_centers(c.call("get_k_center", ""), [d.to_msgpack() for d in ref.get_k_center()])
            got = c.call("get_core_members", "")
            want = ref.get_core_members()
            assert len(got) == len(want)
            for g, w in zip(got, want):
                _same_members(g, [(ww, wd.to_msgpack()) for ww, wd in w])
            for _ in range(6):
                q = _datum(rng, rng.randrange(3))
                _same_centers([c.call("get_nearest_center", "", q)],
                              [ref.get_nearest_center(Datum.from_msgpack(q)).to_msgpack()])
                _same_members(c.call("get_nearest_members", "", q),
                              [(w, d.to_msgpack()) for w, d in ref.get_nearest_members(Datum.from_msgpack(q))])
            st = {_s(k): _s(v) for k, v in next(iter(c.call("get_status", "").values())).items()}
            assert st["server_runtime"] == "native"
            assert st["revision"] == str(ref.get_revision()) and st["converter"] == "native"
            # the native model file: read by the Python driver and by a second native server
            (_, mpath), = c.call("save", "", "m").items()
            mpath = _s(mpath)
            with open(mpath, "rb") as f:
                _, user = read_model_file(f)
            ref2 = Clustering(method, par, DatumToFvConverter(conv), device=dev)
            ref2.unpack(user[1])
            assert ref2.get_revision() == ref.get_revision()
            p2, port2 = _start(tmp_path, model=mpath)
            with RpcClient("127.0.0.1", port2, 30.0) as c2:   # both recluster the loaded coresets alike
                assert c2.call("get_revision", "") == ref.get_revision()
                _same_centers(c2.call("get_k_center", ""), [d.to_msgpack() for d in ref2.get_k_center()])
            assert c.call("clear", "") is True
            assert c.call("get_revision", "") == 0
            with pytest.raises(Exception):
                c.call("get_k_center", "")
    finally:
        for q in (p, p2):
            if q is not None:
                q.terminate()
                q.wait(timeout=30)


@pytest.mark.gpu
def test_native_clustering_concurrent_pushes(tmp_path):
    """pushes from several connections at once: each is hashed before the
    model lock (jubaclustering.cpp push_raw, a pooled converter per push in
    flight) and appended under it - every point lands once (pending + closed
    buckets account for all of them) and the feature names stay whole"""
    cfg = json.load(open(os.path.join(ROOT, "config", "clustering", "kmeans.json")))
    cfg["parameter"]["bucket_size"] = 500
    path = tmp_path / "kmeans.json"
    path.write_text(json.dumps(cfg))
    p, port = _start(tmp_path, path)
    try:
        import threading
        errs = []

        def worker(seed):
            rng = random.Random(seed)
            try:
                with RpcClient("127.0.0.1", port, 60.0) as c:
                    for _ in range(15):
                        assert c.call("push", "", [_datum(rng, rng.randrange(3)) for _ in range(70)]) is True
            except Exception as e:  # noqa: BLE001 - reported below
                errs.append(e)

        ts = [threading.Thread(target=worker, args=(s,)) for s in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errs, errs
        total = 6 * 15 * 70
        with RpcClient("127.0.0.1", port, 60.0) as c:
            (_, st), = c.call("get_status", "").items()
            st = {_s(k): _s(v) for k, v in st.items()}
            assert int(st["pending"]) == total % 500
            assert int(st["revision"]) >= 1
            centers = c.call("get_k_center", "")
            assert len(centers) == 3
            for cen in centers:   # whole feature names, finite values
                names = {_s(k) for k, _ in cen[1]}
                assert {"x@num", "y@num"} <= names, names
                assert names <= {"x@num", "y@num"} | {f"tag${t}@str#bin/bin" for t in "abc"}, names
                assert all(math.isfinite(float(v)) for _, v in cen[1])
    finally:
        p.terminate()
        p.wait(timeout=30)
