"""Batched writes of the native jubarecommender (csrc/server/jb_row_server.hpp
Model::write_many): update_row / clear_row pipelined on one connection are
served in batches - datums parsed and (fixed-slot converter) hashed on
several threads outside the model lock, one staged device launch per batch
for the LSH signatures (LshIndex::flush) and for the inverted index's runs
(PoolIndex::flush) - and must leave the store of the same writes sent one by
one: the same rows, the same merged datums, the same rankings. The
reference's writes are sequential (recommender_serv.cpp update_row). Both
servers are native, on one GPU."""
import json
import math
import os
import random
import socket
import subprocess
import time

import msgpack
import pytest

from helpers import ROOT, config_path
from jubatus_amd.common.mprpc import RpcClient, RpcIOError, RpcTimeoutError

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubarecommender")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start(cfg, tmp_path):
    port = _free_port()
    p = subprocess.Popen([BIN, "-p", str(port), "-b", "127.0.0.1", "-f", cfg, "-d", str(tmp_path)],
                         stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    deadline = time.time() + 60
    while True:
        try:
            with RpcClient("127.0.0.1", port, 5.0) as c:
                c.call("get_config", "")
            return p, port
        except (OSError, RpcIOError, RpcTimeoutError):
            assert p.poll() is None and time.time() < deadline
            time.sleep(0.1)


def _pipelined(port, calls):
    """every call written before any answer is read: the batch thread takes
    the queued writes several per batch"""
    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(b"".join(msgpack.packb([0, i, m, ["", *a]], use_bin_type=False) for i, (m, a) in enumerate(calls)))
    up = msgpack.Unpacker(raw=False)
    got = {}
    while len(got) < len(calls):
        chunk = s.recv(1 << 16)
        assert chunk
        up.feed(chunk)
        for msg in up:
            assert msg[2] is None, msg
            got[msg[1]] = msg[3]
    s.close()
    return [got[i] for i in range(len(calls))]


def _norm(x):
    if isinstance(x, bytes):
        return x.decode()
    if isinstance(x, (list, tuple)):
        return [_norm(y) for y in x]
    if isinstance(x, dict):
        return {_norm(k): _norm(v) for k, v in x.items()}
    return x


def _calls(rng, n):
    out = []
    for i in range(n):
        rid = f"r{rng.randrange(400)}"   # repeated ids: merges inside a batch
        if rng.random() < 0.04:
            out.append(("clear_row", [rid]))
            continue
        sv = [[f"s{j}", f"w{rng.randrange(30)}"] for j in range(rng.randrange(1, 4))]
        nv = [[f"n{j}", round(rng.gauss(0, 2), 3)] for j in range(rng.randrange(1, 5))]
        out.append(("update_row", [rid, [sv, nv, []]]))
    return out


@pytest.mark.parametrize("name", ["euclid_lsh.json", "lsh_unlearn_lru.json", "default.json",
                                  "inverted_index_euclid.json"])
def test_batched_writes_equal_sequential_writes(name, tmp_path):
    path = config_path(f"recommender/{name}")
    cfg = json.load(open(path))
    for sub in ("a", "b"):
        (tmp_path / sub).mkdir()
    rng = random.Random(11)
    calls = _calls(rng, 3000)
    (pa, porta), (pb, portb) = _start(path, tmp_path / "a"), _start(path, tmp_path / "b")
    try:
        with RpcClient("127.0.0.1", porta, 60.0) as c:
            seq = [c.call(m, "", *a) for m, a in calls]
        bat = _pipelined(portb, calls)
        assert seq == bat
        with RpcClient("127.0.0.1", porta, 60.0) as a, RpcClient("127.0.0.1", portb, 60.0) as b:
            ids_a, ids_b = sorted(_norm(a.call("get_all_rows", ""))), sorted(_norm(b.call("get_all_rows", "")))
            assert ids_a == ids_b and len(ids_a) > 100
            (_, st), = b.call("get_status", "").items()
            st = _norm(st)
            assert int(st["update_row_cnt"]) == sum(m == "update_row" for m, _ in calls)
            for rid in ids_a[::7]:
                assert _norm(a.call("decode_row", "", rid)) == _norm(b.call("decode_row", "", rid))
                ra = _norm(a.call("similar_row_from_id", "", rid, 8))
                rb = _norm(b.call("similar_row_from_id", "", rid, 8))
                assert len(ra) == len(rb), (rid, ra, rb)
                for (_, x), (_, y) in zip(ra, rb):
                    assert math.isclose(x, y, rel_tol=1e-5, abs_tol=1e-5), (rid, ra, rb)
                # the ids match wherever the score is not tied with the next one
                for q in range(len(ra) - 1):
                    if abs(ra[q][1] - ra[q + 1][1]) > 1e-5 and (q == 0 or abs(ra[q][1] - ra[q - 1][1]) > 1e-5):
                        assert ra[q][0] == rb[q][0], (rid, ra, rb)
        assert cfg["method"] in ("euclid_lsh", "lsh", "inverted_index", "inverted_index_euclid")
    finally:
        for p in (pa, pb):
            p.terminate()
            p.wait(timeout=30)
