"""Native executables under AddressSanitizer / ThreadSanitizer (the
reference's --fsanitize build option, wscript:55-57,143-146, and its
concurrency notes in SURVEY §5.2): the coordinator and the proxy are built
instrumented (build_ext --sanitize) and driven by concurrent clients; any
sanitizer report fails the test. Host code only (no GPU)."""
import os
import random
import subprocess
import threading

import pytest

from jubatus_amd import build_ext
from jubatus_amd.common.coordinator import NativeCoordinator
from jubatus_amd.common.lock_service import CoordinatorClient
from jubatus_amd.common.mprpc import RpcClient, RpcServer

SAN_ENV = {"ASAN_OPTIONS": "halt_on_error=1:detect_leaks=0:exitcode=66",
           "TSAN_OPTIONS": "halt_on_error=1:exitcode=66:report_signal_unsafe=0"}


def _reports(text: str) -> list[str]:
    return [ln for ln in text.splitlines()
            if "ERROR: AddressSanitizer" in ln or "WARNING: ThreadSanitizer" in ln]


@pytest.fixture(scope="module", params=["address", "thread"])
def san(request):
    return request.param, build_ext.build_tools(sanitize=request.param)


def _start_coord(bindir, tmp_path):
    err = open(tmp_path / "coord.err", "w")
    c = NativeCoordinator(0, "127.0.0.1", exe=os.path.join(bindir, "jubacoordinator"),
                          env=dict(os.environ, **SAN_ENV), stderr=err)
    return c, err


def test_coordinator_concurrent_sessions(san, tmp_path):
    kind, bindir = san
    coord, err = _start_coord(bindir, tmp_path)
    try:
        errors = []

        def worker(i):
            try:
                ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=2.0)
                ls.create("/s")
                ls.create(f"/s/w{i}")
                for j in range(30):
                    ls.create(f"/s/w{i}/e{j}", "x", j % 2 == 0)
                    ls.create_seq(f"/s/w{i}/q_")
                    ls.list("/s")
                    ls.read(f"/s/w{i}")
                    ls.set(f"/s/w{i}", str(j))
                ls.close()          # ephemerals of this session go away
            except Exception as e:  # noqa: BLE001
                errors.append(e)
        ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors
    finally:
        rc = coord.stop()
        err.close()
    text = (tmp_path / "coord.err").read_text()
    assert not _reports(text), text[-4000:]
    assert rc in (0, -15), (rc, text[-2000:])


def _fake_server(ls, name, i):
    """an engine-server stand-in behind the proxy (classifier surface)"""
    srv = RpcServer(nthreads=4)
    srv.add("train", lambda n, data: len(data), 2)
    srv.add("get_config", lambda n: "{}", 1)
    srv.add("set_label", lambda n, l: True, 2)
    srv.add("get_status", lambda n: {f"127.0.0.1_{i}": {"k": str(i)}}, 1)
    port = srv.listen(0, "127.0.0.1")
    srv.start()
    base = f"/jubatus/actors/classifier/{name}"
    for p in ("/jubatus", "/jubatus/actors", "/jubatus/actors/classifier", base, base + "/nodes",
              base + "/actives"):
        ls.create(p)
    ls.create(f"{base}/actives/127.0.0.1_{port}", "", True)
    return srv, port


def test_proxy_concurrent_fanout(san, tmp_path):
    kind, bindir = san
    coord, cerr = _start_coord(bindir, tmp_path)
    ls = CoordinatorClient(f"127.0.0.1:{coord.port}", timeout=5.0)
    servers = [_fake_server(ls, "san", i) for i in range(3)]
    perr = open(tmp_path / "proxy.err", "w")
    proxy = None
    try:
        import socket
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        pport = s.getsockname()[1]
        s.close()
        proxy = subprocess.Popen([os.path.join(bindir, "jubaproxy"), "classifier", "-p", str(pport),
                                  "-b", "127.0.0.1", "-z", f"127.0.0.1:{coord.port}", "-c", "8"],
                                 stdout=subprocess.PIPE, stderr=perr, text=True,
                                 env=dict(os.environ, **SAN_ENV))
        assert proxy.stdout.readline().startswith("jubaproxy ready")
        errors = []

        def client(seed):
            try:
                rng = random.Random(seed)
                c = RpcClient("127.0.0.1", pport, 20)
                for _ in range(40):
                    m = rng.randrange(3)
                    if m == 0:
                        assert c.call("train", "san", [["a", [[], [], []]]] * 3) == 3
                    elif m == 1:
                        assert c.call("set_label", "san", "x") is True
                    else:
                        assert len(c.call("get_status", "san")) == 3
                c.close()
            except Exception as e:  # noqa: BLE001
                errors.append(e)
        ts = [threading.Thread(target=client, args=(i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors
    finally:
        if proxy is not None:
            proxy.terminate()
            prc = proxy.wait(30)
        perr.close()
        ls.close()
        for srv, _ in servers:
            srv.stop()
        coord.stop()
        cerr.close()
    text = (tmp_path / "proxy.err").read_text()
    assert not _reports(text), text[-4000:]
    assert prc in (0, -15), (prc, text[-2000:])


def test_jubavisor_spawn_stop_reap(san, tmp_path):
    """supervisor start / stop / reap paths with concurrent RPCs; the children
    are a stand-in program (JUBAVISOR_SERVER_DIR) so no engine server runs"""
    kind, bindir = san
    coord, cerr = _start_coord(bindir, tmp_path)
    sdir = tmp_path / "servers"
    sdir.mkdir()
    fake = sdir / "jubafake"
    fake.write_text("#!/bin/sh\nexec sleep 30\n")
    fake.chmod(0o755)
    quick = sdir / "jubaquick"
    quick.write_text("#!/bin/sh\nexit 0\n")
    quick.chmod(0o755)
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    vport = s.getsockname()[1]
    s.close()
    verr = open(tmp_path / "visor.err", "w")
    visor = subprocess.Popen([os.path.join(bindir, "jubavisor"), "-p", str(vport), "-b", "127.0.0.1",
                              "-z", f"127.0.0.1:{coord.port}", "-m", "8"],
                             stdout=subprocess.PIPE, stderr=verr, text=True,
                             env=dict(os.environ, JUBAVISOR_SERVER_DIR=str(sdir), **SAN_ENV))
    vrc = None
    try:
        assert visor.stdout.readline().startswith("jubavisor ready")
        errors = []

        def client(i):
            try:
                c = RpcClient("127.0.0.1", vport, 20)
                for j in range(5):
                    assert c.call("start", f"jubafake/n{i}", 1, [0] * 19) == 0
                    assert c.call("start", f"jubaquick/q{i}", 1, [0] * 19) == 0
                    assert c.call("start", "bad", 1, [0] * 19) == -1
                    assert c.call("stop", f"jubafake/n{i}", 1) == 0
                c.close()
            except Exception as e:  # noqa: BLE001
                errors.append(e)
        ts = [threading.Thread(target=client, args=(i,)) for i in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert not errors, errors
        c = RpcClient("127.0.0.1", vport, 20)
        # quick children exited and were reaped: their ports are back, so a
        # full pool of 8 long-running children fits
        import time
        time.sleep(0.5)
        assert c.call("start", "jubafake/full", 8, [0] * 19) == 0
        c.close()
    finally:
        visor.terminate()       # stops the 8 children too
        vrc = visor.wait(60)
        verr.close()
        coord.stop()
        cerr.close()
    text = (tmp_path / "visor.err").read_text()
    assert not _reports(text), text[-4000:]
    assert vrc in (0, -15), (vrc, text[-2000:])
    assert text.count("stopped jubafake/full") == 8, text[-2000:]
