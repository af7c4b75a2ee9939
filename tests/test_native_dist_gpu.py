"""Distributed mode of the native jubaclassifier (no Python in the server
process): coordinator membership, the native linear mixer over the group's
control plane and the device MIX (touched-row union, sparse all-reduce,
fold) - two servers sharing this box's GPU mix over the staged host plane;
the RCCL plane is checked on its own as a one-rank communicator
(jb_rccl_check). Reference: linear_mixer.cpp:358-544; the Python twins are
tests/test_distributed.py."""
import json
import os
import socket
import subprocess
import tempfile
import time

import pytest

from jubatus_amd.client import Classifier, Datum
from jubatus_amd.common import config as zkconfig
from jubatus_amd.common import membership as mb
from jubatus_amd.common.coordinator import NativeCoordinator
from jubatus_amd.common.lock_service import CoordinatorClient
from jubatus_amd.common.mprpc import wait_server

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NB = os.path.join(ROOT, "jubatus_amd", "native_bin")


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


def spawn(zport, name, port, extra=(), env=None, exe="jubaclassifier"):
    log = open(os.path.join(tempfile.gettempdir(), f"native_dist_{name}_{port}.log"), "wb")
    cmd = [os.path.join(NB, exe), "-z", f"127.0.0.1:{zport}", "-n", name, "-p", str(port),
           "-b", "127.0.0.1", "-s", "0", "-i", "0", "-I", "5", "-Z", "5", *extra]
    return subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=log, env=dict(os.environ, **(env or {})))


def _logs(name, ports):
    """the servers' stderr (spawn), for assertion messages"""
    out = {}
    for p in ports:
        try:
            with open(os.path.join(tempfile.gettempdir(), f"native_dist_{name}_{p}.log"), "rb") as f:
                out[p] = f.read().decode(errors="replace")[-3000:]
        except OSError:
            out[p] = ""
    return out


def stop(procs):
    for p in procs:
        if p.poll() is None:
            p.terminate()
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()


def wait_actives(ls, name, n, timeout=90, engine="classifier"):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if len(mb.get_all_actives(ls, engine, name)) >= n:
            return True
        time.sleep(0.2)
    return False


def status(c):
    (_, st), = c.get_status().items()
    return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
            for k, v in st.items()}


def wait_group(a, b, n, timeout=60):
    """both servers in one n-member group, neither obsolete"""
    deadline = time.time() + timeout
    while time.time() < deadline:
        sa, sb = status(a), status(b)
        if all(st.get("linear_mixer.group_size") == str(n) and st.get("linear_mixer.is_obsolete") == "0"
               for st in (sa, sb)):
            return True
        time.sleep(0.2)
    return False


def top(c, d):
    return max(c.classify([d])[0], key=lambda e: e.score).label


def test_rccl_plane_one_rank():
    r = subprocess.run([os.path.join(NB, "jb_rccl_check")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"] is True and out["plane"] == "rccl"


def test_native_classifier_distributed_mix(coord):
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    name = "ndist"
    zkconfig.config_tozk(ls, "classifier", name, open(os.path.join(ROOT, "config/classifier/arow.json")).read())
    ports = [free_port(), free_port()]
    procs = [spawn(coord.port, name, p) for p in ports]
    try:
        for p in ports:
            assert wait_server("127.0.0.1", p, 90)
        assert wait_actives(ls, name, 2)
        a = Classifier("127.0.0.1", ports[0], name, timeout=60.0)
        b = Classifier("127.0.0.1", ports[1], name, timeout=60.0)
        # the two-member group has formed and its hand-over is done: a member
        # still obsolete then would take the other's model (the obsolete
        # protocol), replacing what it trained in between
        assert wait_group(a, b, 2)
        # each server learns a different pair of labels
        a.train([("pos", Datum({"w": "good"})), ("neg", Datum({"w": "bad"}))] * 8)
        b.train([("spam", Datum({"w": "offer"})), ("ham", Datum({"w": "meeting"}))] * 8)
        assert a.do_mix() is True
        sa, sb = status(a), status(b)
        for st in (sa, sb):
            assert st["server_runtime"] == "native" and st["linear_mixer.runtime"] == "native"
            assert st["linear_mixer.group_size"] == "2" and st["is_standalone"] == "0"
            assert st["linear_mixer.backend"] == "host"      # both on one GPU: the staged plane
        assert int(sa["linear_mixer.mix_count"]) >= 1
        # both learnt all four labels through the MIX (the peer's fold may
        # still be running when do_mix returns here)
        deadline = time.time() + 30
        while time.time() < deadline and int(status(b).get("linear_mixer.mix_count", "0")) < 1:
            time.sleep(0.1)
        for c in (a, b):
            got = (top(c, Datum({"w": "good"})), top(c, Datum({"w": "offer"})))
            assert got == ("pos", "spam"), (got, sa, sb, _logs(name, ports))
            assert sorted(c.get_labels()) == ["ham", "neg", "pos", "spam"]
        # label counts are the cluster totals on both
        la, lb = a.get_labels(), b.get_labels()
        assert la == lb and la["pos"] == 8 and la["spam"] == 8
        # a second MIX after a little training is sparse (touched rows only)
        a.train([("pos", Datum({"w": "great"}))] * 2)
        assert a.do_mix() is True
        assert status(b)["mix.last_mode"] == "sparse"
        assert top(b, Datum({"w": "great"})) == "pos"
        a.close()
        b.close()
    finally:
        stop(procs)
        ls.close()


def test_native_stalled_rank_watchdog_aborts_and_regroups(coord):
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    name = "nstall"
    zkconfig.config_tozk(ls, "classifier", name, open(os.path.join(ROOT, "config/classifier/arow.json")).read())
    ports = [free_port(), free_port()]
    good = spawn(coord.port, name, ports[0], extra=("-I", "2"))
    slow = spawn(coord.port, name, ports[1], extra=("-I", "2"),
                 env={"JUBATUS_FAULT": "mix_hang:phase=allreduce,at=1,ms=7000"})
    try:
        for p in ports:
            assert wait_server("127.0.0.1", p, 90)
        assert wait_actives(ls, name, 2)
        a = Classifier("127.0.0.1", ports[0], name, timeout=90.0)
        a.train([("pos", Datum({"w": "good"})), ("neg", Datum({"w": "bad"}))] * 3)
        t0 = time.time()
        try:
            a.do_mix()
        except Exception:  # noqa: BLE001
            pass
        assert top(a, Datum({"w": "good"})) == "pos"     # serves while the group is aborted
        deadline = time.time() + 100
        ok = False
        while time.time() < deadline:
            try:
                if a.do_mix() and status(a).get("linear_mixer.group_size") == "2":
                    ok = True
                    break
            except Exception:  # noqa: BLE001
                pass
            time.sleep(0.5)
        assert ok, "no MIX with both members after the stall"
        assert int(status(a)["linear_mixer.watchdog_aborts"]) >= 1
        assert time.time() - t0 < 110
        b = Classifier("127.0.0.1", ports[1], name, timeout=30.0)
        assert top(b, Datum({"w": "good"})) == "pos"
        a.close()
        b.close()
    finally:
        stop([good, slow])
        ls.close()


def test_native_regression_distributed_mix(coord):
    """native jubaregression in distributed mode (csrc/server/jubaregression.cpp
    Mixable over the same linear mixer): two servers train different
    features, one MIX averages w and the target statistics, so both then
    estimate alike and know both features (models/regression.py mix: the
    mean of w and stats)"""
    from jubatus_amd.client import Regression
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    name = "nreg"
    zkconfig.config_tozk(ls, "regression", name, open(os.path.join(ROOT, "config/regression/pa.json")).read())
    ports = [free_port(), free_port()]
    procs = [spawn(coord.port, name, p, exe="jubaregression") for p in ports]
    try:
        for p in ports:
            assert wait_server("127.0.0.1", p, 90)
        assert wait_actives(ls, name, 2, engine="regression")
        a = Regression("127.0.0.1", ports[0], name, timeout=60.0)
        b = Regression("127.0.0.1", ports[1], name, timeout=60.0)
        assert wait_group(a, b, 2)
        assert a.train([(4.0, Datum({"x": 1.0}))] * 8) == 8
        assert b.train([(-2.0, Datum({"z": 1.0}))] * 8) == 8
        before = (a.estimate([Datum({"z": 1.0})])[0], b.estimate([Datum({"x": 1.0})])[0])
        assert before == (0.0, 0.0)          # neither knows the other's feature yet
        assert a.do_mix() is True
        # do_mix returns when this server's MIX is done; the peer folds on its
        # own mixer thread
        deadline = time.time() + 30
        while time.time() < deadline and status(b).get("mix.applied_count") in (None, "0"):
            time.sleep(0.1)
        for st in (status(a), status(b)):
            assert st["server_runtime"] == "native" and st["linear_mixer.runtime"] == "native", st
            assert st["linear_mixer.group_size"] == "2" and st["mix.last_applied"] == "1", st
        probe = [Datum({"x": 1.0}), Datum({"z": 1.0})]
        ea, eb = a.estimate(probe), b.estimate(probe)
        assert ea == pytest.approx(eb, abs=1e-5), (ea, eb)
        assert ea[0] > 0.5 and ea[1] < -0.2, ea     # both features, each at about half its weight
        a.close()
        b.close()
    finally:
        stop(procs)
        ls.close()
