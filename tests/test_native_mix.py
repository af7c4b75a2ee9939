"""The native distributed model plane (csrc/native/jb_mix_group.hpp) on the
CPU: jb_mix_rehearsal processes - the native linear mixer, group epochs,
control-plane star and the classifier's MIX protocol over a host model -
join a cluster through the native coordinator. Four ranks mix to the exact
mean (dense first MIX, sparse later ones), a killed rank is dropped by the
next epoch, a late joiner receives the model (obsolete protocol), and a rank
that stalls a MIX past the interconnect timeout is aborted by the watchdog
and re-joined (reference: linear_mixer.cpp:358-544, 394-410, 455-489;
server_util.cpp:184-194)."""
import os
import socket
import subprocess
import tempfile
import time

import numpy as np
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


class Rank:
    def __init__(self, zport, name, ic=3, env=None, H=512, mixer="linear_mixer"):
        self.port = free_port()
        log = open(os.path.join(tempfile.gettempdir(), f"mixreh_{name}_{self.port}.log"), "wb")
        self.proc = subprocess.Popen([BIN, "-x", mixer, "-z", f"127.0.0.1:{zport}", "-n", name, "-p", str(self.port),
                                      "-H", str(H), "-I", str(ic), "-i", "0", "-s", "0", "-Z", "3"],
                                     stdout=subprocess.DEVNULL, stderr=log,
                                     env=dict(os.environ, **(env or {})))
        assert wait_server("127.0.0.1", self.port, 30)
        self.c = RpcClient("127.0.0.1", self.port, 60.0)

    def call(self, m, *a):
        return self.c.call(m, "n", *a)

    def status(self):
        (_, st), = self.call("get_status").items()
        return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
                for k, v in st.items()}

    def model(self):
        out = {}
        for k, (cnt, w, s) in self.call("model").items():
            out[k.decode() if isinstance(k, bytes) else k] = (int(cnt), np.array(w, np.float32),
                                                               np.array(s, np.float32))
        return out

    def stop(self):
        self.c.close()
        if self.proc.poll() is None:
            self.proc.terminate()
            try:
                self.proc.wait(timeout=15)
            except subprocess.TimeoutExpired:
                self.proc.kill()


def wait_group(ranks, n, timeout=60, mixer="linear_mixer"):
    deadline = time.time() + timeout
    while time.time() < deadline:
        sts = [r.status() for r in ranks]
        if all(s.get(f"{mixer}.group_size") == str(n) and s.get(f"{mixer}.is_obsolete") == "0"
               for s in sts):
            return True
        time.sleep(0.2)
    return False


def mean_models(models):
    labels = sorted(set().union(*[m.keys() for m in models]))
    out = {}
    for lab in labels:
        ws = [m[lab][1] if lab in m else np.zeros_like(next(iter(models[0].values()))[1]) for m in models]
        ss = [m[lab][2] if lab in m else np.ones_like(next(iter(models[0].values()))[2]) for m in models]
        out[lab] = (np.mean(ws, axis=0), np.mean(ss, axis=0))
    return out


def check_mixed(ranks, before):
    want = mean_models(before)
    total = {lab: sum(m[lab][0] for m in before if lab in m) for lab in want}
    after = [r.model() for r in ranks]
    for m in after:
        assert sorted(m) == sorted(want)
        for lab, (w, s) in want.items():
            np.testing.assert_allclose(m[lab][1], w, rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(m[lab][2], s, rtol=1e-5, atol=1e-6)
            assert m[lab][0] == total[lab], (lab, m[lab][0], total[lab])


def test_four_ranks_mix_to_the_mean(coord):
    ranks = [Rank(coord.port, "four") for _ in range(4)]
    try:
        assert wait_group(ranks, 4)
        for i, r in enumerate(ranks):
            r.call("train", 100 + i, 300, 3 + i)        # different label sets per rank
        before = [r.model() for r in ranks]
        assert ranks[1].call("do_mix") is True
        check_mixed(ranks, before)
        assert ranks[0].status()["mix.last_mode"] == "dense"    # the first MIX: every row
        # a second round touching few rows: a sparse MIX of the union only
        base = {lab: v[0] for lab, v in ranks[0].model().items()}    # the mixed counts
        for i, r in enumerate(ranks):
            r.call("train", 200 + i, 20, 2)
        before = [r.model() for r in ranks]
        assert ranks[2].call("do_mix") is True
        after = [r.model() for r in ranks]
        want = mean_models(before)
        for m in after:
            for lab, (w, s) in want.items():
                np.testing.assert_allclose(m[lab][1], w, rtol=1e-5, atol=1e-6)
                np.testing.assert_allclose(m[lab][2], s, rtol=1e-5, atol=1e-6)
        st = ranks[3].status()
        assert st["mix.last_mode"] == "sparse" and 0 < int(st["mix.last_rows"]) <= 80
        assert st["linear_mixer.runtime"] == "native" and st["linear_mixer.backend"] == "host"
        # counts: every rank agrees, and they grew by the 80 updates of this round
        cnts = [{lab: v[0] for lab, v in m.items()} for m in after]
        assert all(c == cnts[0] for c in cnts)
        assert sum(cnts[0].values()) == sum(base.values()) + 4 * 20
    finally:
        for r in ranks:
            r.stop()


def _models_equal(a, b):
    assert sorted(a) == sorted(b)
    for lab in a:
        np.testing.assert_allclose(a[lab][1], b[lab][1], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(a[lab][2], b[lab][2], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mixer,n", [("skip_mixer", 4), ("random_mixer", 2)])
def test_push_mixers_reach_the_mean(coord, mixer, n):
    """the classifier's native pair MIX (label agreement with the peer, the
    pair's row union, pairwise mean): the skip mixer's butterfly over 4 ranks
    and the random mixer's one pair both end at the cluster mean"""
    ranks = [Rank(coord.port, f"push{n}", mixer=mixer) for _ in range(n)]
    try:
        assert wait_group(ranks, n, mixer=mixer)
        for i, r in enumerate(ranks):
            r.call("train", 300 + i, 200, 2 + i)
        before = [r.model() for r in ranks]
        assert ranks[0].call("do_mix") is True
        want = mean_models(before)
        for r in ranks:
            m = r.model()
            assert sorted(m) == sorted(want)
            for lab, (w, s) in want.items():
                np.testing.assert_allclose(m[lab][1], w, rtol=1e-5, atol=1e-6)
                np.testing.assert_allclose(m[lab][2], s, rtol=1e-5, atol=1e-6)
        st = ranks[-1].status()
        assert st[f"{mixer}.runtime"] == "native" and int(st[f"{mixer}.mix_count"]) >= 1
        # a second MIX moves only the rows trained since (sparse union)
        ranks[0].call("train", 999, 10, 2)
        assert ranks[1].call("do_mix") is True
        assert 0 < int(ranks[1].status()["mix.last_rows"]) <= 10 * (2 if mixer == "random_mixer" else 4)
        ms = [r.model() for r in ranks]
        if mixer == "random_mixer":
            _models_equal(ms[0], ms[1])
    finally:
        for r in ranks:
            r.stop()


def test_broadcast_mixer_spreads_labels(coord):
    """broadcast (round-robin tournament) over 3 ranks: every rank ends with
    every label, and models move toward each other"""
    ranks = [Rank(coord.port, "bcast3", mixer="broadcast_mixer") for _ in range(3)]
    try:
        assert wait_group(ranks, 3, mixer="broadcast_mixer")
        for i, r in enumerate(ranks):
            r.call("train", 500 + i, 150, 1 + 2 * i)
        before = [r.model() for r in ranks]
        assert ranks[2].call("do_mix") is True
        after = [r.model() for r in ranks]
        labels = sorted(set().union(*[m.keys() for m in before]))
        want = mean_models(before)
        for b, a in zip(before, after):
            assert sorted(a) == labels
            for lab in labels:   # closer to the mean than before
                if lab in b:
                    assert (np.abs(a[lab][1] - want[lab][0]).sum()
                            <= np.abs(b[lab][1] - want[lab][0]).sum() + 1e-4)
    finally:
        for r in ranks:
            r.stop()


def test_killed_rank_dropped_and_late_joiner_fetches_model(coord):
    ranks = [Rank(coord.port, "churn") for _ in range(3)]
    late = None
    try:
        assert wait_group(ranks, 3)
        for i, r in enumerate(ranks):
            r.call("train", 7 + i, 200, 4)
        ranks[2].proc.kill()                       # a rank dies (session expires after -Z 3 s)
        ranks[2].proc.wait()
        live = ranks[:2]
        assert wait_group(live, 2, timeout=60)
        before = [r.model() for r in live]
        assert live[0].call("do_mix") is True
        check_mixed(live, before)
        late = Rank(coord.port, "churn")           # joins obsolete: receives the model
        assert wait_group(live + [late], 3, timeout=60)
        ref = live[0].model()
        got = late.model()
        assert sorted(got) == sorted(ref)
        for lab in ref:
            np.testing.assert_allclose(got[lab][1], ref[lab][1], rtol=1e-6, atol=1e-7)
    finally:
        for r in ranks[:2] + ([late] if late else []):
            r.stop()
        if ranks[2].proc.poll() is None:
            ranks[2].proc.kill()


def test_stalled_rank_watchdog_aborts_and_regroups(coord):
    good = Rank(coord.port, "stall", ic=2)
    slow = Rank(coord.port, "stall", ic=2, env={"JUBATUS_FAULT": "mix_hang:phase=allreduce,at=1,ms=6000"})
    try:
        assert wait_group([good, slow], 2)
        good.call("train", 1, 100, 2)
        slow.call("train", 2, 100, 2)
        t0 = time.time()
        try:
            good.call("do_mix")                     # the slow rank stalls inside this MIX
        except Exception:  # noqa: BLE001
            pass
        deadline = time.time() + 90
        ok = False
        while time.time() < deadline:
            try:
                if good.call("do_mix") and good.status().get("linear_mixer.group_size") == "2":
                    ok = True
                    break
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.5)
        assert ok, "no MIX with both members after the stall"
        assert int(good.status()["linear_mixer.watchdog_aborts"]) >= 1
        assert time.time() - t0 < 90
        a, b = good.model(), slow.model()
        for lab in a:
            np.testing.assert_allclose(a[lab][1], b[lab][1], rtol=1e-6, atol=1e-7)
    finally:
        good.stop()
        slow.stop()
