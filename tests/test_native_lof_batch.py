"""Batched anomaly adds of the native jubaanomaly (csrc/server/jb_row_server.hpp
Model::add_many, csrc/hip/lof.hip jb_lof_add_many): adds pipelined on one
connection are served in batches (one staged signature launch, multi-query
neighbour passes, one LOF enqueue per batch) and must give the ids and scores
of the same adds sent one by one, in the same order - the reference's add is
sequential (anomaly_serv.cpp:157-176). Both servers are native, on one GPU."""
import json
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

BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaanomaly")


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


def _pipelined_adds(port, datums):
    """every add written before any answer is read: the server's batch
    thread takes them in arrival order, several per batch"""
    s = socket.create_connection(("127.0.0.1", port))
    s.sendall(b"".join(msgpack.packb([0, i, "add", ["", d]], use_bin_type=False) for i, d in enumerate(datums)))
    up = msgpack.Unpacker(raw=False)
    got = {}
    while len(got) < len(datums):
        chunk = s.recv(1 << 16)
        assert chunk
        up.feed(chunk)
        for msg in up:
            assert msg[2] is None, msg
            got[msg[1]] = msg[3]
    s.close()
    return [got[i] for i in range(len(datums))]


@pytest.mark.parametrize("name,k,rnn", [("lof.json", 5, 12), ("light_lof.json", 5, 12),
                                        # k > 16 (the LDS list edits), more than 64 candidates
                                        ("lof.json", 20, 70)])
def test_batched_adds_equal_sequential_adds(name, k, rnn, tmp_path):
    """(the batch thread stages each chunk of 8 adds while the previous
    chunk's kernel runs: Model::add_many's pipeline keeps the arrival order)"""
    cfg = json.load(open(config_path(f"anomaly/{name}")))
    if "nearest_neighbor_num" in cfg.get("parameter", {}):
        cfg["parameter"]["nearest_neighbor_num"] = k
        cfg["parameter"]["reverse_nearest_neighbor_num"] = rnn
    path = tmp_path / name
    path.write_text(json.dumps(cfg))
    for sub in ("a", "b"):
        (tmp_path / sub).mkdir()
    rng = random.Random(7)
    datums = [[[["tag", f"t{rng.randrange(5)}"]],
               [["x", round(rng.gauss(0, 1), 4)], ["y", round(rng.gauss(0, 1), 4)]], []]
              for _ in range(600)]
    (pa, porta), (pb, portb) = _start(str(path), tmp_path / "a"), _start(str(path), tmp_path / "b")
    try:
        with RpcClient("127.0.0.1", porta, 60.0) as c:
            seq = [c.call("add", "", d) for d in datums]
        bat = _pipelined_adds(portb, datums)
        for (ia, sa), (ib, sb) in zip(seq, bat):
            ia = ia.decode() if isinstance(ia, bytes) else ia
            ib = ib.decode() if isinstance(ib, bytes) else ib
            assert ia == ib
            assert sa == pytest.approx(sb, rel=1e-5, abs=1e-5) or (sa == sb)
        # and the stores agree afterwards
        probe = [[[["tag", "t1"]], [["x", 0.3], ["y", -0.2]], []], [[], [["x", 5.0], ["y", 5.0]], []]]
        with RpcClient("127.0.0.1", porta, 60.0) as a, RpcClient("127.0.0.1", portb, 60.0) as b:
            for d in probe:
                assert a.call("calc_score", "", d) == pytest.approx(b.call("calc_score", "", d), rel=1e-5)
    finally:
        for p in (pa, pb):
            p.terminate()
            p.wait(timeout=30)


def test_batched_adds_after_removals_equal_sequential_adds(tmp_path):
    """rows removed between two add streams leave rows without a valid list
    behind: batched adds then stop on them (status 2) - the chunk queued
    behind a stopped one does not run and is rerun after the lists are
    installed (LofState::finish_many, Model::add_many) - and the ids and
    scores must still be those of the adds one by one"""
    cfg = json.load(open(config_path("anomaly/lof.json")))
    cfg["parameter"]["nearest_neighbor_num"] = 5
    cfg["parameter"]["reverse_nearest_neighbor_num"] = 12
    path = tmp_path / "lof.json"
    path.write_text(json.dumps(cfg))
    for sub in ("a", "b"):
        (tmp_path / sub).mkdir()
    rng = random.Random(13)

    def datums(n):
        return [[[["tag", f"t{rng.randrange(5)}"]],
                 [["x", round(rng.gauss(0, 1), 4)], ["y", round(rng.gauss(0, 1), 4)]], []] for _ in range(n)]

    first, second = datums(400), datums(400)
    drop = [str(i) for i in rng.sample(range(400), 60)]
    (pa, porta), (pb, portb) = _start(str(path), tmp_path / "a"), _start(str(path), tmp_path / "b")
    try:
        with RpcClient("127.0.0.1", porta, 60.0) as a, RpcClient("127.0.0.1", portb, 60.0) as b:
            seq = [a.call("add", "", d) for d in first]
            bat = _pipelined_adds(portb, first)
            for rid in drop:
                assert a.call("clear_row", "", rid) == b.call("clear_row", "", rid)
            seq += [a.call("add", "", d) for d in second]
        bat += _pipelined_adds(portb, second)
        assert len(seq) == len(bat)
        for (ia, sa), (ib, sb) in zip(seq, bat):
            ia = ia.decode() if isinstance(ia, bytes) else ia
            ib = ib.decode() if isinstance(ib, bytes) else ib
            assert ia == ib
            assert sa == pytest.approx(sb, rel=1e-5, abs=1e-5) or (sa == sb)
    finally:
        for p in (pa, pb):
            p.terminate()
            p.wait(timeout=30)
