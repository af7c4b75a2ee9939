"""Native row-engine servers (csrc/server/jb_row_server.hpp: jubarecommender,
jubanearest_neighbor; no Python in the process) against the Python servers
(server/recommender_serv.py, server/nearest_neighbor_serv.py, in-process on
the same GPU) fed the same call sequence: every answer and error is
compared, and model files move both ways. Reference RPC surface:
recommender_serv.cpp:126-224, nearest_neighbor_serv.cpp:121-178."""
import json
import math
import os
import random
import shutil
import socket
import subprocess
import time
import zlib

import pytest

from helpers import ROOT, config_path
from jubatus_amd.common.mprpc import RpcClient, RpcIOError, RpcTimeoutError, RpcTypeError

pytestmark = pytest.mark.gpu

NATIVE_BIN = os.path.join(ROOT, "jubatus_amd", "native_bin")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _wait(port, proc=None):
    deadline = time.time() + 60
    while True:
        try:
            with RpcClient("127.0.0.1", port, 5.0) as c:
                c.call("get_config", "")
            return
        except (OSError, RpcIOError, RpcTimeoutError):
            if proc is not None:
                assert proc.poll() is None, proc.stdout.read()
            assert time.time() < deadline
            time.sleep(0.1)


class Pair:
    """a native server (subprocess) and a Python server (in-process) with
    the same configuration and data directory"""

    def __init__(self, engine, cfg_text, tmp_path):
        from jubatus_amd.framework.server_helper import ServerHelper
        from jubatus_amd.framework.server_util import ServerArgv
        from jubatus_amd.server import get_serv
        self.engine = engine
        self.dir = tmp_path
        cfg = tmp_path / f"{engine}.json"
        cfg.write_text(cfg_text)
        self.cfg = str(cfg)
        self.nport = _free_port()
        self.proc = subprocess.Popen([os.path.join(NATIVE_BIN, f"juba{engine}"), "-p", str(self.nport),
                                      "-b", "127.0.0.1", "-f", self.cfg, "-d", str(tmp_path)],
                                     stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
        a = ServerArgv.parse(["-p", "9199", "-b", "127.0.0.1", "-f", self.cfg, "-d", str(tmp_path),
                              "--gpu", "0"], engine)
        a.port = 0
        self.py = ServerHelper(get_serv(engine), a, install_signals=False)
        self.py.start(block=False)
        self.pport = self.py.argv.port
        _wait(self.nport, self.proc)
        self.n = RpcClient("127.0.0.1", self.nport, 60.0)
        self.p = RpcClient("127.0.0.1", self.pport, 60.0)

    def close(self):
        self.n.close()
        self.p.close()
        self.py.stop()
        self.proc.terminate()
        self.proc.wait(timeout=30)


def _call(c, m, *a):
    try:
        return ("ok", c.call(m, "", *a))
    except RpcTypeError:
        return ("arg", None)
    except Exception as e:  # noqa: BLE001 - application error text
        return ("err", str(e))


def _norm(x):
    """bytes -> str recursively (the two servers' raw / str encodings)"""
    if isinstance(x, bytes):
        return x.decode("utf-8", "surrogateescape")
    if isinstance(x, (list, tuple)):
        return [_norm(y) for y in x]
    if isinstance(x, dict):
        return {_norm(k): _norm(v) for k, v in x.items()}
    return x


def _same(a, b, path=""):
    if isinstance(a, float) or isinstance(b, float):
        assert isinstance(a, (int, float)) and isinstance(b, (int, float)), (path, a, b)
        assert math.isclose(a, b, rel_tol=1e-5, abs_tol=1e-5), (path, a, b)
        return
    if isinstance(a, list):
        assert isinstance(b, list) and len(a) == len(b), (path, a, b)
        for i, (x, y) in enumerate(zip(a, b)):
            _same(x, y, f"{path}[{i}]")
        return
    assert a == b, (path, a, b)


def _datum(rng, with_bin=True):
    sv = [[f"s{j}", f"t{rng.randrange(6)}{'x' * rng.randrange(3)}"] for j in range(rng.randrange(1, 4))]
    nv = [[f"n{j}", round(rng.gauss(0, 3), 3)] for j in range(rng.randrange(0, 4))]
    if rng.random() < 0.2:
        nv.append(["int", rng.randrange(-5, 50)])         # integer encodings
    bv = [["b", bytes([rng.randrange(256)])]] if with_bin and rng.random() < 0.2 else []
    return [sv, nv, bv]


def _drive(pair, rng, steps, kind):
    ids = [f"r{i}" for i in range(40)]
    upd = {"recommender": "update_row", "nearest_neighbor": "set_row", "anomaly": "update"}[kind]
    for i in range(steps):
        if kind == "anomaly":
            op = rng.choice(["add"] * 4 + ["update", "overwrite"] * 2 + ["clear_row", "calc_score"] * 2
                            + ["get_all_rows"])
        elif kind == "recommender":
            op = rng.choice([upd] * 6 + ["clear_row", "similar_row_from_id", "similar_row_from_datum",
                                         "complete_row_from_id", "complete_row_from_datum", "decode_row",
                                         "get_all_rows", "calc_similarity", "calc_l2norm"])
        else:
            op = rng.choice([upd] * 6 + ["neighbor_row_from_id", "neighbor_row_from_datum",
                                         "similar_row_from_id", "similar_row_from_datum", "get_all_rows"])
        rid = rng.choice(ids + ["missing"])
        k = rng.choice([1, 3, 10, 200])
        if op == "add":
            args = (_datum(rng, False),)
        elif op in (upd, "overwrite"):
            args = (rid, _datum(rng))
        elif op == "calc_score":
            args = (_datum(rng, False),)
        elif op in ("clear_row", "decode_row", "complete_row_from_id"):
            args = (rid,)
        elif op.endswith("_from_id"):
            args = (rid, k)
        elif op.endswith("_from_datum") and op.startswith(("similar", "neighbor")):
            args = (_datum(rng, False), k)
        elif op == "complete_row_from_datum":
            args = (_datum(rng, False),)
        elif op == "calc_similarity":
            args = (_datum(rng, False), _datum(rng, False))
        elif op == "calc_l2norm":
            args = (_datum(rng, False),)
        else:
            args = ()
        got = _call(pair.n, op, *args)
        want = _call(pair.p, op, *args)
        assert got[0] == want[0], (i, op, args, got, want)
        if got[0] == "ok":
            g, w = _norm(got[1]), _norm(want[1])
            if op.startswith(("similar_row", "neighbor_row")):
                _same_ranked(g, w, f"{i}:{op}")
            else:
                _same(g, w, f"{i}:{op}")
        elif got[0] == "err":
            assert got[1] == want[1], (i, op, got, want)


def _same_ranked(a, b, path):
    """[(id, score)] rankings: the same scores in the same order; ids equal
    up to the order inside a group of equal scores (the last group may be
    cut at a different member by k)"""
    assert len(a) == len(b), (path, a, b)
    for x, y in zip(a, b):
        assert math.isclose(x[1], y[1], rel_tol=1e-5, abs_tol=1e-5), (path, a, b)
    groups = {}
    for (ia, sa), (ib, _) in zip(a, b):
        key = round(sa, 5)
        ga, gb = groups.setdefault(key, (set(), set()))
        ga.add(ia)
        gb.add(ib)
    last = round(a[-1][1], 5) if a else None
    for key, (ga, gb) in groups.items():
        if key != last:
            assert ga == gb, (path, a, b)


CASES = [
    ("recommender", "recommender/euclid_lsh.json"),
    ("recommender", "recommender/lsh_unlearn_lru.json"),
    ("recommender", "recommender/minhash.json"),
    ("recommender", "recommender/default.json"),                 # inverted_index, bigram tf-idf
    ("recommender", "recommender/inverted_index_euclid_unlearn_lru.json"),
    ("recommender", "recommender/nearest_neighbor_recommender_euclid_lsh.json"),
    ("nearest_neighbor", "nearest_neighbor/euclid_lsh.json"),
    ("nearest_neighbor", "nearest_neighbor/default.json"),       # lsh, bigram tf-idf
    ("anomaly", "anomaly/lof.json"),                             # lof over euclid_lsh
    ("anomaly", "anomaly/lof_inverted_index_euclid.json"),
    ("anomaly", "anomaly/light_lof_unlearn_lru.json"),
    ("anomaly", "anomaly/default.json"),
]


@pytest.mark.parametrize("engine,cfg", CASES)
def test_native_row_server_matches_python(engine, cfg, tmp_path):
    pair = Pair(engine, open(config_path(cfg)).read(), tmp_path)
    try:
        rng = random.Random(zlib.crc32(cfg.encode()))
        _drive(pair, rng, 300, engine)
        (_, st), = pair.n.call("get_status", "").items()
        st = _norm(st)
        assert st["server_runtime"] == "native"
        (_, pst), = pair.p.call("get_status", "").items()
        pst = _norm(pst)
        for k in ("num_rows", "method", "unlearner", "update_count"):
            assert st[k] == pst[k], (k, st[k], pst[k])
        from test_status_keys import COMMON
        assert not [k for k in COMMON if k not in st]
        # arity / type errors, unknown methods
        assert _call(pair.n, "get_all_rows", "x")[0] == "arg"
        if engine != "anomaly":
            assert _call(pair.n, "similar_row_from_id", "r1", "five")[0] == "arg"
            assert _call(pair.n, "similar_row_from_datum", [[["k", 1]], []], 3)[0] == "arg"
        else:
            assert _call(pair.n, "calc_score", [[["k", 1]], []])[0] == "arg"
    finally:
        pair.close()


@pytest.mark.parametrize("engine,cfg", [("recommender", "recommender/default.json"),
                                        ("recommender", "recommender/euclid_lsh_unlearn_lru.json"),
                                        ("nearest_neighbor", "nearest_neighbor/minhash.json"),
                                        ("anomaly", "anomaly/lof.json")])
def test_native_row_model_files_both_ways(engine, cfg, tmp_path):
    pair = Pair(engine, open(config_path(cfg)).read(), tmp_path)
    try:
        rng = random.Random(7)
        upd = {"recommender": "update_row", "nearest_neighbor": "set_row", "anomaly": "overwrite"}[engine]
        for i in range(60):
            d = _datum(rng)
            a, b = pair.n.call(upd, "", f"{i % 45}", d), pair.p.call(upd, "", f"{i % 45}", d)
            _same(_norm(a), _norm(b), f"fill {i}")
        # native -> Python
        # native -> Python: both load the native file (a load re-hashes the
        # stored rows with the loaded document frequencies, re-lays the slots
        # and resets the anomaly id counter - on both sides alike)
        (_, npath), = pair.n.call("save", "", "m1").items()
        npath = _norm(npath)
        ppath = os.path.join(str(tmp_path), f"127.0.0.1_{pair.pport}_{engine}_m1.jubatus")
        shutil.copy(npath, ppath)
        assert pair.p.call("clear", "") is True
        assert pair.p.call("load", "", "m1") is True
        assert pair.n.call("load", "", "m1") is True
        assert _norm(pair.n.call("get_all_rows", "")) == _norm(pair.p.call("get_all_rows", ""))
        _drive(pair, random.Random(8), 80, engine)
        # Python -> native
        (_, ppath2), = pair.p.call("save", "", "m2").items()
        npath2 = os.path.join(str(tmp_path), f"127.0.0.1_{pair.nport}_{engine}_m2.jubatus")
        shutil.copy(_norm(ppath2), npath2)
        assert pair.n.call("clear", "") is True
        assert pair.n.call("load", "", "m2") is True
        assert pair.p.call("load", "", "m2") is True
        _drive(pair, random.Random(9), 80, engine)
        assert sorted(_norm(pair.n.call("get_all_rows", ""))) == sorted(_norm(pair.p.call("get_all_rows", "")))
    finally:
        pair.close()
