"""The row engines' MIX (csrc/server/jb_row_mix.hpp - the code the native
jubarecommender / jubanearest_neighbor / jubaanomaly servers run) on the CPU:
jb_mix_rehearsal -R processes hold versioned row stores, join a cluster
through the native coordinator and mix over the native group plane. After a
MIX every rank holds the union: the newest version of every row wins, a
removal wins over older writes, and later MIXes ship only what changed
(reference: linear_mixer.cpp:422-544 get_diff / mix / put_diff over row
stores; anomaly_serv.cpp:178-211). 4 and 8 ranks."""
import os
import random
import socket
import subprocess
import tempfile
import time

import pytest

from jubatus_amd.common.coordinator import NativeCoordinator, native_available
from jubatus_amd.common.mprpc import RpcClient, wait_server

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jb_mix_rehearsal")

pytestmark = pytest.mark.skipif(not (native_available() and os.path.exists(BIN)),
                                reason="native binaries not built")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture
def coord():
    srv = NativeCoordinator(0, "127.0.0.1")
    yield srv
    srv.stop()


class RowRank:
    def __init__(self, zport, name, ic=5, mixer="linear_mixer"):
        self.port = free_port()
        self.mixer = mixer
        log = open(os.path.join(tempfile.gettempdir(), f"rowmix_{name}_{self.port}.log"), "wb")
        self.proc = subprocess.Popen([BIN, "-R", "-x", mixer, "-z", f"127.0.0.1:{zport}", "-n", name, "-p",
                                      str(self.port), "-I", str(ic), "-i", "0", "-s", "0", "-Z", "3"],
                                     stdout=subprocess.DEVNULL, stderr=log)
        assert wait_server("127.0.0.1", self.port, 30)
        self.c = RpcClient("127.0.0.1", self.port, 60.0)

    def call(self, m, *a):
        return self.c.call(m, "n", *a)

    def rows(self):
        return {(k.decode() if isinstance(k, bytes) else k): (int(v), x.decode() if isinstance(x, bytes) else x)
                for k, (v, x) in self.call("rows").items()}

    def status(self):
        (_, st), = self.call("get_status").items()
        return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
                for k, v in st.items()}

    def stop(self):
        self.c.close()
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=15)
            except subprocess.TimeoutExpired:
                self.proc.kill()


def wait_group(ranks, n, timeout=60):
    deadline = time.time() + timeout
    k = ranks[0].mixer
    while time.time() < deadline:
        sts = [r.status() for r in ranks]
        if all(s.get(f"{k}.group_size") == str(n) and s.get(f"{k}.is_obsolete") == "0" for s in sts):
            return True
        time.sleep(0.2)
    return False


def expected_union(before, removed):
    """the protocol's fold: newest version wins (the later rank on ties),
    a removal with a version >= the winner's removes the row"""
    win = {}
    for rank, rows in enumerate(before):
        for rid, (v, x) in rows.items():
            if rid not in win or v >= win[rid][0]:
                win[rid] = (v, x, rank)
    gone = {}
    for rid, v in removed:
        gone[rid] = max(v, gone.get(rid, -1))
    out = {}
    for rid, (v, x, _) in win.items():
        if gone.get(rid, -1) >= v:
            continue
        out[rid] = (v, x)
    return out


def _run(coord, n):
    ranks = [RowRank(coord.port, f"rows{n}") for _ in range(n)]
    try:
        assert wait_group(ranks, n)
        rng = random.Random(n)
        removed = []
        for i, r in enumerate(ranks):
            r.call("put", 1000 + i, 40 + 7 * i, 120)         # overlapping key spaces
        for i, r in enumerate(ranks):
            mine = sorted(r.rows())
            for rid in rng.sample(mine, 3):
                v = r.rows()[rid][0]
                assert r.call("remove", rid) is True
                removed.append((rid, v + 1))
        before = [r.rows() for r in ranks]
        want = expected_union(before, removed)
        assert ranks[n // 2].call("do_mix") is True
        after = [r.rows() for r in ranks]
        # ties of version between ranks may keep a rank's own copy: compare
        # ids and versions everywhere, values where the newest version is unique
        tied = {rid for rid in want
                if sum(1 for b in before if rid in b and b[rid][0] == want[rid][0]) > 1}
        for a in after:
            assert sorted(a) == sorted(want)
            for rid, (v, x) in want.items():
                assert a[rid][0] == v, rid
                if rid not in tied:
                    assert a[rid][1] == x, rid
        # a second MIX ships only what changed since the first
        ranks[0].call("put", 77, 5, 10_000)
        assert ranks[-1].call("do_mix") is True
        new = {rid for rid in ranks[0].rows() if rid not in after[0]}
        assert new
        for r in ranks[1:]:
            assert new <= set(r.rows())
            assert r.status()["mix.last_rows_applied"] == str(len(new))
    finally:
        for r in ranks:
            r.stop()


def test_row_mix_four_ranks_reach_the_union(coord):
    _run(coord, 4)


def test_row_mix_eight_ranks_reach_the_union(coord):
    _run(coord, 8)


def test_late_row_rank_receives_the_store(coord):
    """obsolete protocol: a rank joining an existing group gets the whole
    store from an up-to-date member before it mixes"""
    ranks = [RowRank(coord.port, "late") for _ in range(2)]
    try:
        assert wait_group(ranks, 2)
        ranks[0].call("put", 5, 30, 100)
        assert ranks[0].call("do_mix") is True
        ranks.append(RowRank(coord.port, "late"))
        assert wait_group(ranks, 3)
        assert ranks[2].rows() == ranks[0].rows()
    finally:
        for r in ranks:
            r.stop()


@pytest.mark.parametrize("mixer", ["skip_mixer", "broadcast_mixer"])
def test_push_mixers_reach_the_union(coord, mixer):
    """push mixers (push_mixer.cpp:335-408): skip_mixer's butterfly rounds
    (strides N/2, N/4, ..., 1) and broadcast_mixer's tournament both bring
    every rank the union within one MIX - a round forwards what earlier
    rounds delivered"""
    ranks = [RowRank(coord.port, f"push_{mixer}", mixer=mixer) for _ in range(4)]
    try:
        assert wait_group(ranks, 4)
        for i, r in enumerate(ranks):
            r.call("put", 500 + i, 20, 1000)
        want = set()
        for r in ranks:
            want |= set(r.rows())
        assert ranks[0].call("do_mix") is True
        deadline = time.time() + 20
        # (a rank applies the rows before its MIX round ends and counts it)
        while time.time() < deadline and (any(set(r.rows()) != want for r in ranks) or
                                           any(int(r.status()[f"{mixer}.mix_count"]) < 1 for r in ranks)):
            time.sleep(0.1)
        for r in ranks:
            assert set(r.rows()) == want
            assert int(r.status()[f"{mixer}.mix_count"]) >= 1
    finally:
        for r in ranks:
            r.stop()


def test_random_mixer_pairs_up(coord):
    """random_mixer: one random perfect matching per MIX; each rank ends with
    its own rows and its partner's"""
    ranks = [RowRank(coord.port, "push_random", mixer="random_mixer") for _ in range(4)]
    try:
        assert wait_group(ranks, 4)
        for i, r in enumerate(ranks):
            r.call("put", 900 + i, 10, 1000)
        before = [set(r.rows()) for r in ranks]
        assert ranks[0].call("do_mix") is True
        time.sleep(1.0)
        after = [set(r.rows()) for r in ranks]
        for i in range(4):
            got = after[i] - before[i]
            partners = [j for j in range(4) if j != i and before[j] <= after[i]]
            assert len(partners) == 1 and got == before[partners[0]] - before[i], (i, partners)
    finally:
        for r in ranks:
            r.stop()


@pytest.mark.parametrize("n", [2 ** 62, 2 ** 61 + 1, -1, 1.5, float("nan"), 3])
def test_malformed_row_diff_is_rejected(coord, n):
    """a peer's row count must not pass the size checks by
    wrapping (n = 2^62 with 4-byte offsets) nor be negative / fractional /
    NaN; a diff whose arrays do not hold n rows is rejected whole and the
    store is untouched"""
    import msgpack
    import struct
    r = RowRank(coord.port, f"bad{abs(hash(str(n))) % 1000}")
    try:
        r.call("put", 3, 5, 100)
        before = r.rows()
        diff = {"n": n, "ids": b"abcd", "ido": struct.pack("<I", 0), "ver": b"",
                "dat": b"", "dato": struct.pack("<I", 0), "rp": struct.pack("<q", 0),
                "idx": b"", "val": b"", "removed": [], "w": [0, 0, b"", b""]}
        raw = msgpack.packb(diff, use_bin_type=True)
        with pytest.raises(Exception, match="malformed row diff"):
            r.call("apply_raw", raw)
        assert r.rows() == before
        # the same arrays with the count they do hold (0 rows) apply cleanly
        diff["n"] = 0
        assert r.call("apply_raw", msgpack.packb(diff, use_bin_type=True)) == 0
    finally:
        r.stop()
