"""Operations tools: jubaconv, jubaconfig, jubavisor + jubactl (cluster
start / status / save / load / stop through the supervisor), jubadump
(reference C31-C34; the reference's own jubavisor test is empty, so this is
our coverage)."""
import io
import json
import os
import socket
import subprocess
import time

import pytest

from jubatus_amd.cmd import jubaconfig, jubaconv, jubactl, jubadump
from jubatus_amd.cmd.jubavisor import Jubavisor, argv_from_wire, argv_to_wire, split_server_name
from jubatus_amd.common import membership as mb
from jubatus_amd.common.coordinator import CoordinatorServer
from jubatus_amd.common.lock_service import CoordinatorClient
from jubatus_amd.common.mprpc import RpcClient, RpcMethodNotFound, RpcServer

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE_BIN_DIR = os.path.join(ROOT, "jubatus_amd", "native_bin")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def free_port_block(n: int = 4) -> int:
    """a free port whose next n ports are free too (jubavisor hands its
    children the ports after its own)"""
    for _ in range(200):
        base = free_port()
        socks = []
        try:
            for q in range(base, base + n + 1):
                s = socket.socket()
                socks.append(s)
                s.bind(("127.0.0.1", q))
            return base
        except OSError:
            continue
        finally:
            for s in socks:
                s.close()
    raise RuntimeError("no free port block")


@pytest.fixture
def coord():
    srv = CoordinatorServer(0, "127.0.0.1").start()
    yield srv
    srv.stop()


def test_jubaconv_json_datum_fv(tmp_path):
    js = '{"user": {"name": "taro", "age": 31, "tags": ["a", "b"], "vip": true, "x": null}}'
    out = io.StringIO()
    assert jubaconv.main(["-i", "json", "-o", "datum"], stdin=io.StringIO(js), out=out) == 0
    d = json.loads(out.getvalue())
    assert ["/user/name", "taro"] in d["string_values"] and ["/user/tags[1]", "b"] in d["string_values"]
    assert ["/user/age", 31.0] in d["num_values"] and ["/user/vip", 1.0] in d["num_values"]
    cfg = tmp_path / "c.json"
    cfg.write_text(json.dumps({"converter": {"string_rules": [{"key": "*", "type": "str",
                                                                "sample_weight": "bin", "global_weight": "bin"}],
                                              "num_rules": [{"key": "*", "type": "num"}]}}))
    out = io.StringIO()
    assert jubaconv.main(["-o", "fv", "-c", str(cfg)], stdin=io.StringIO(js), out=out) == 0
    lines = out.getvalue().splitlines()
    assert "/user/name$taro@str#bin/bin: 1" in lines and "/user/age@num: 31" in lines
    out = io.StringIO()
    assert jubaconv.main(["-i", "datum", "-o", "fv", "-c", str(cfg)],
                         stdin=io.StringIO(json.dumps(d)), out=out) == 0
    assert "/user/age@num: 31" in out.getvalue().splitlines()
    assert jubaconv.main(["-i", "datum", "-o", "json"], stdin=io.StringIO(json.dumps(d)), out=io.StringIO()) == -1


JUBACONV_INPUTS = [
    '{"user": {"name": "taro", "age": 31, "tags": ["a", "b"], "vip": true, "x": null}}',
    r'{"t": "caf\u00e9 \ud83d\ude00 \"q\" \t", "n": [1.5, -0.0, 1e-05, 1e16, 123456789.125, 3e30], '
    '"e": {}, "l": [], "deep": {"a": [{"b": false}]}}',
    '{"text": "the quick brown fox jumps over the lazy dog the end", "w": 2.0}',
]


@pytest.mark.parametrize("conf", [
    None,
    {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
     "num_rules": [{"key": "*", "type": "num"}]},
    {"string_types": {"bi": {"method": "ngram", "char_num": "2"}},
     "string_rules": [{"key": "/text", "type": "bi", "sample_weight": "tf", "global_weight": "bin"},
                      {"key": "*", "type": "space", "sample_weight": "log_tf", "global_weight": "bin"}],
     "num_rules": [{"key": "*", "type": "log"}],
     "combination_rules": [{"key_left": "*", "key_right": "*", "type": "add"}]},
    # plug-ins ("dynamic": splitter, string / num filters, num feature,
    # combination) and the built-in num filters / types: loaded natively (dlopen)
    {"string_filter_types": {"up": {"method": "dynamic", "path": "libjubatus_sample_plugins.so",
                                    "function": "create_upper_filter"}},
     "string_filter_rules": [{"key": "/t*", "type": "up", "suffix": "-up"}],
     "num_filter_types": {"aff": {"method": "dynamic", "path": "libjubatus_sample_plugins.so",
                                  "function": "create_affine_filter", "scale": "2", "shift": "1"},
                          "lin": {"method": "linear_normalization", "min": "0", "max": "100"},
                          "gs": {"method": "gaussian_normalization", "average": 1, "standard_deviation": 2.5},
                          "sg": {"method": "sigmoid_normalization", "gain": 0.5, "bias": 1.0},
                          "ad": {"method": "add", "value": 3}},
     "num_filter_rules": [{"key": "/n*", "type": "aff", "suffix": "-aff"},
                          {"key": "*", "type": "lin", "suffix": "-lin"},
                          {"key": "/w", "type": "gs", "suffix": "-gs"},
                          {"key": "/w", "type": "sg", "suffix": "-sg"},
                          {"key": "/user/age", "type": "ad", "suffix": "-ad"}],
     "string_types": {"sp": {"method": "dynamic", "path": "libjubatus_sample_plugins.so",
                             "function": "create_splitter", "delimiter": " ", "min_length": "2"}},
     "string_rules": [{"key": "*", "type": "sp", "sample_weight": "tf", "global_weight": "bin"},
                      {"key": "/user/name", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
     "num_types": {"bk": {"method": "dynamic", "path": "libjubatus_sample_plugins.so",
                          "function": "create_bucket_feature", "width": "10"},
                   "plus": {"method": "add", "value": "0.5"}, "s": {"method": "str"}},
     "num_rules": [{"key": "*", "type": "bk"}, {"key": "/w*", "type": "plus"}, {"key": "/user/age", "type": "s"},
                   {"key": "*", "type": "num"}],
     "combination_types": {"mx": {"method": "dynamic", "path": "libjubatus_sample_plugins.so",
                                  "function": "create_max_combination"}},
     "combination_rules": [{"key_left": "/w@num", "key_right": "*", "type": "mx"}]},
    # outside the native set (a regexp filter): the native tool hands it to the Python twin
    {"string_filter_types": {"dl": {"method": "regexp", "pattern": "o", "replace": ""}},
     "string_filter_rules": [{"key": "/text", "type": "dl", "suffix": "-x"}],
     "string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}]},
])
def test_native_jubaconv_matches_python(tmp_path, conf):
    """csrc/cmd/jubaconv.cpp against jubatus_amd/cmd/jubaconv.py: json / datum
    outputs byte for byte (json.dumps indent=2), fv lines of the same config"""
    exe = _native_tool("jubaconv")
    cfg = tmp_path / "c.json"
    cfg.write_text(json.dumps({"converter": conf or {}}))
    modes = [("json", "json"), ("json", "datum")] if conf is None else [("json", "fv")]
    for js in JUBACONV_INPUTS:
        for i, o in modes:
            args = ["-i", i, "-o", o] + (["-c", str(cfg)] if o == "fv" else [])
            py = io.StringIO()
            prc = jubaconv.main(args, stdin=io.StringIO(js), out=py)
            env = dict(os.environ, PYTHONPATH=ROOT)
            if '"dynamic"' in json.dumps(conf):
                env["PATH"] = "/nonexistent"     # plug-in configs: no Python fallback to hide behind
            r = subprocess.run([exe, *args], input=js, capture_output=True, text=True, timeout=60, env=env)
            assert (r.returncode, r.stdout) == (prc & 0xff, py.getvalue()), (i, o, js, r.stderr)
            if o == "datum":    # the datum output read back as input
                d = r.stdout
                py2 = io.StringIO()
                jubaconv.main(["-i", "datum", "-o", "datum"], stdin=io.StringIO(d), out=py2)
                r2 = subprocess.run([exe, "-i", "datum", "-o", "datum"], input=d, capture_output=True,
                                    text=True, timeout=60)
                assert r2.stdout == py2.getvalue() == d


def test_jubaconfig(coord):
    zk = f"127.0.0.1:{coord.port}"
    out = []
    cfg = os.path.join(ROOT, "config/classifier/pa.json")
    assert jubaconfig.main(["-c", "write", "-f", cfg, "-t", "classifier", "-n", "c1", "-z", zk], out=out.append) == 0
    assert jubaconfig.main(["-c", "read", "-t", "classifier", "-n", "c1", "-z", zk], out=out.append) == 0
    assert json.loads(out[-1])["method"] == "PA"
    out.clear()
    assert jubaconfig.main(["-c", "list", "-z", zk], out=out.append) == 0
    assert out[0] == "config of classifier/c1:"
    assert jubaconfig.main(["-c", "delete", "-t", "classifier", "-n", "c1", "-z", zk], out=out.append) == 0
    assert jubaconfig.main(["-c", "read", "-t", "classifier", "-n", "c1", "-z", zk], out=out.append) == 1


def _native_tool(name):
    exe = os.path.join(NATIVE_BIN_DIR, name)
    if not os.access(exe, os.X_OK):
        pytest.skip(f"native {name} not built (python -m jubatus_amd.build_ext)")
    return exe


def _run_native(name, args):
    r = subprocess.run([_native_tool(name), *args], capture_output=True, text=True, timeout=60)
    return r.returncode, r.stdout.splitlines(), r.stderr


def test_native_jubaconfig_matches_python(coord):
    """csrc/cmd/jubaconfig.cpp: same nodes, same output lines and exit codes
    as the Python twin; each reads what the other wrote"""
    zk = f"127.0.0.1:{coord.port}"
    pa = os.path.join(ROOT, "config/classifier/pa.json")
    arow = os.path.join(ROOT, "config/classifier/arow.json")
    assert _run_native("jubaconfig", ["-c", "write", "-f", pa, "-t", "classifier", "-n", "c1", "-z", zk])[0] == 0
    assert jubaconfig.main(["-c", "write", "-f", arow, "-t", "classifier", "-n", "c2", "-z", zk],
                           out=lambda *a: None) == 0
    rc, lines, _ = _run_native("jubaconfig", ["-c", "read", "-t", "classifier", "-n", "c2", "-z", zk])
    assert rc == 0 and json.loads("\n".join(lines))["method"] == "AROW"
    py = []
    assert jubaconfig.main(["-c", "read", "-t", "classifier", "-n", "c1", "-z", zk], out=py.append) == 0
    assert json.loads(py[0]) == json.load(open(pa))
    py = []
    assert jubaconfig.main(["-c", "list", "-z", zk], out=py.append) == 0
    rc, lines, _ = _run_native("jubaconfig", ["-c", "list", "-z", zk])
    assert rc == 0 and lines == "".join(x + "\n" for x in py).splitlines()   # print() lines
    assert lines[0] == "config of classifier/c1:"
    # bad JSON, missing config, delete, and a config refused while a server is registered
    bad = os.path.join(os.path.dirname(pa), "..", "..", "README.md")
    rc, lines, _ = _run_native("jubaconfig", ["-c", "write", "-f", bad, "-t", "classifier", "-n", "c3", "-z", zk])
    assert rc == 1 and lines[0].startswith("error: invalid config json")
    assert _run_native("jubaconfig", ["-c", "delete", "-t", "classifier", "-n", "c1", "-z", zk])[0] == 0
    rc, lines, _ = _run_native("jubaconfig", ["-c", "read", "-t", "classifier", "-n", "c1", "-z", zk])
    assert rc == 1 and lines == ["error: config is not found: /jubatus/config/classifier/c1"]
    ls = CoordinatorClient(zk, timeout=5.0)
    try:
        assert ls.create(mb.build_actor_path("classifier", "c2") + "/nodes/127.0.0.1_1", "", ephemeral=True)
        rc, lines, _ = _run_native("jubaconfig", ["-c", "write", "-f", pa, "-t", "classifier", "-n", "c2",
                                                  "-z", zk])
        assert rc == 1 and lines == ["error: any server is running"]
    finally:
        ls.close()
    rc, lines, _ = _run_native("jubaconfig", ["-c", "read", "-t", "classifier", "-z", zk])
    assert rc == 1 and lines == ["type (-t) and name (-n) are required"]
    assert _run_native("jubaconfig", ["--help"])[0] == 0


def test_native_jubactl_without_supervisors(coord):
    zk = f"127.0.0.1:{coord.port}"
    common = ["-s", "jubaclassifier", "-n", "none", "-t", "classifier", "-z", zk]
    rc, lines, _ = _run_native("jubactl", ["-c", "start", *common])
    assert rc == 1 and lines == ["no server to start jubaclassifier/none"]
    rc, lines, _ = _run_native("jubactl", ["-c", "save", *common])
    assert rc == 0 and lines == ["no server to save none"]
    rc, lines, _ = _run_native("jubactl", ["-c", "bogus", *common])
    assert rc == 1
    env = {k: v for k, v in os.environ.items() if k != "ZK"}
    r = subprocess.run([_native_tool("jubactl"), "-c", "status", "-s", "x", "-n", "y", "-t", "z"],
                       capture_output=True, text=True, timeout=30, env=env)
    assert r.returncode == 1 and "can't get ZK location" in r.stdout


@pytest.mark.parametrize("tool", ["jubactl", "jubaconfig", "jubaconv"])
def test_native_tool_flags_match_python(tool):
    """the native tool takes every flag of the Python twin's --help (the man
    page is rendered from the latter, tools/gen_man.py)"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from gen_man import flags_of
    rc, lines, _ = _run_native(tool, ["--help"])
    assert rc == 0
    py = subprocess.run([sys.executable, "-m", f"jubatus_amd.cmd.{tool}", "--help"], cwd=ROOT,
                        capture_output=True, text=True, timeout=60).stdout
    assert flags_of(py) <= flags_of("\n".join(lines)), flags_of(py) - flags_of("\n".join(lines))


def test_jubavisor_wire_helpers():
    assert split_server_name("jubaclassifier/foo") == ("jubaclassifier", "foo")
    with pytest.raises(ValueError):
        split_server_name("classifier")
    d = {"port": 1, "name": "x", "mixer": "linear_mixer", "daemon": False}
    assert argv_from_wire(argv_to_wire(d))["mixer"] == "linear_mixer"
    assert jubactl.split_counts(5, 2) == [3, 2] and jubactl.split_counts(0, 3) == [1, 1, 1]


def _cluster_roundtrip(zk, ls, tmp_path, gpus=0, native_ctl=False):
    """jubactl start 2 / status / save / load / stop against the registered supervisor(s);
    gpus > 0: the supervisor hands out one device per child (--gpu), visible in get_status;
    native_ctl: the native jubactl (csrc/cmd/jubactl.cpp) drives it"""
    out = []
    if native_ctl:
        class _Native:
            @staticmethod
            def main(args):
                rc, lines, err = _run_native("jubactl", args)
                assert all(ln.endswith("ok.") for ln in lines if ln.startswith("sending")), lines
                return rc
        jubactl = _Native
    else:
        from jubatus_amd.cmd import jubactl
    assert jubaconfig.main(["-c", "write", "-f", os.path.join(ROOT, "config/classifier/arow.json"),
                            "-t", "classifier", "-n", "cl", "-z", zk], out=out.append) == 0
    common = ["-s", "jubaclassifier", "-n", "cl", "-t", "classifier", "-z", zk]
    assert jubactl.main(["-c", "start", "-N", "2", "-D", str(tmp_path), "-S", "0", "-I", "0", *common]) == 0
    nodes_path = mb.build_actor_path("classifier", "cl") + "/nodes"
    deadline = time.time() + 90
    while len(ls.list(nodes_path)) < 2 and time.time() < deadline:
        time.sleep(0.3)
    nodes = ls.list(nodes_path)
    assert len(nodes) == 2, nodes
    assert jubactl.main(["-c", "status", *common]) == 0
    if gpus:
        seen = []
        for n in nodes:
            host, port = n.rsplit("_", 1)
            with RpcClient(host, int(port), 10.0) as c:
                st = c.call("get_status", "cl")
            st = {k.decode() if isinstance(k, bytes) else k: v for k, v in st.items()}
            v = list(st.values())[0]
            v = {(k.decode() if isinstance(k, bytes) else k): (x.decode() if isinstance(x, bytes) else x)
                 for k, x in v.items()}
            seen.append(v["gpu"])
        assert sorted(seen) == ["0", "1"], seen
    assert jubactl.main(["-c", "save", "-i", "m1", *common]) == 0
    saved = [f for f in os.listdir(tmp_path) if f.endswith("m1.jubatus")]
    assert len(saved) == 2, os.listdir(tmp_path)
    assert jubactl.main(["-c", "load", "-i", "m1", *common]) == 0
    # jubadump reads one of the saved models
    dumped = jubadump.dump(os.path.join(tmp_path, saved[0]))
    assert dumped["system"]["type"] == "classifier" and dumped["model"]["method"] == "AROW"
    assert jubactl.main(["-c", "stop", *common]) == 0
    deadline = time.time() + 30
    while ls.list(nodes_path) and time.time() < deadline:
        time.sleep(0.3)
    assert ls.list(nodes_path) == []


def test_jubavisor_jubactl_cluster(coord, tmp_path, monkeypatch):
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    zk = f"127.0.0.1:{coord.port}"
    vport = free_port_block()
    visor = Jubavisor(zk, vport, max_children=4, listen_addr="127.0.0.1", gpus=2)
    rpc = RpcServer(2)
    rpc.add("start", visor.start, arity=3)
    rpc.add("stop", visor.stop, arity=2)
    rpc.listen(vport, "127.0.0.1")
    rpc.start()
    ls = CoordinatorClient(zk, timeout=5.0)
    try:
        _cluster_roundtrip(zk, ls, tmp_path, gpus=2)
    finally:
        rpc.stop()
        visor.close()
        ls.close()


def _native_visor(zk, vport, tmp_path, maxc=4, gpus=None):
    exe = os.path.join(NATIVE_BIN_DIR, "jubavisor")
    if not os.access(exe, os.X_OK):
        pytest.skip("native jubavisor not built (python -m jubatus_amd.build_ext)")
    err = open(tmp_path / "visor.err", "w")
    extra = ["-G", str(gpus)] if gpus is not None else []
    p = subprocess.Popen([exe, "-p", str(vport), "-z", zk, "-m", str(maxc), "-b", "127.0.0.1", *extra],
                         stdout=subprocess.PIPE, stderr=err, text=True)
    line = p.stdout.readline()
    assert line.startswith("jubavisor ready"), (line, (tmp_path / "visor.err").read_text())
    return p, err


def test_native_jubavisor_jubactl_cluster(coord, tmp_path, monkeypatch):
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    zk = f"127.0.0.1:{coord.port}"
    vport = free_port_block()
    proc, err = _native_visor(zk, vport, tmp_path, gpus=2)
    ls = CoordinatorClient(zk, timeout=5.0)
    try:
        assert ls.list(mb.JUBAVISOR_BASE_PATH) == [f"127.0.0.1_{vport}"]
        _cluster_roundtrip(zk, ls, tmp_path, gpus=2, native_ctl=True)
    finally:
        proc.terminate()
        rc = proc.wait(30)
        err.close()
        ls.close()
    assert rc == 0, (tmp_path / "visor.err").read_text()[-2000:]


@pytest.mark.parametrize("impl", ["native", "python"])
def test_jubavisor_twins_rpc_errors_and_shutdown(coord, tmp_path, monkeypatch, impl):
    """the native supervisor and its Python twin (cmd/jubavisor.py) answer
    the same: bad names / arity, pool exhaustion, a start that registers the
    child, and shutdown (SIGTERM / close) stopping the children"""
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    zk = f"127.0.0.1:{coord.port}"
    vport = free_port_block(1)
    if impl == "native":
        proc, err = _native_visor(zk, vport, tmp_path, maxc=1)
    else:
        visor = Jubavisor(zk, vport, max_children=1, listen_addr="127.0.0.1")
        rpc = RpcServer(2)
        rpc.add("start", visor.start, arity=3)
        rpc.add("stop", visor.stop, arity=2)
        rpc.listen(vport, "127.0.0.1")
        rpc.start()
    ls = CoordinatorClient(zk, timeout=5.0)
    argv = argv_to_wire({"threadnum": 2, "timeout": 10, "interval_sec": 0, "interval_count": 0,
                         "datadir": str(tmp_path), "mixer": "linear_mixer"})
    assert jubaconfig.main(["-c", "write", "-f", os.path.join(ROOT, "config/classifier/pa.json"),
                            "-t", "classifier", "-n", "cx", "-z", zk], out=lambda *a, **k: None) == 0
    try:
        with RpcClient("127.0.0.1", vport, 10.0) as c:
            assert c.call("start", "classifier", 1, argv) == -1          # not juba<engine>/<name>
            assert c.call("start", "jubaclassifier/", 1, argv) == -1
            assert c.call("stop", "nothing", 1) == -1
            assert c.call("stop", "jubaclassifier/none", 1) == 0
            with pytest.raises(RpcMethodNotFound):
                c.call("restart", "jubaclassifier/x", 1)
            with pytest.raises(Exception):
                c.call("start", "jubaclassifier/x")                       # arity
            assert c.call("start", "jubaclassifier/cx", 2, argv) == -1    # pool of 1 port
            assert c.call("start", "jubaclassifier/cx", 1, argv) == 0
        nodes_path = mb.build_actor_path("classifier", "cx") + "/nodes"
        deadline = time.time() + 90
        while not ls.list(nodes_path) and time.time() < deadline:
            time.sleep(0.3)
        assert ls.list(nodes_path) == [f"127.0.0.1_{vport + 1}"]
    finally:
        if impl == "native":
            proc.terminate()          # the supervisor takes its children down with it
            rc = proc.wait(30)
            err.close()
        else:
            rpc.stop()
            visor.close()
            rc = 0
    deadline = time.time() + 30
    while ls.list(nodes_path) and time.time() < deadline:
        time.sleep(0.3)
    assert ls.list(nodes_path) == []
    assert ls.list(mb.JUBAVISOR_BASE_PATH) == []
    ls.close()
    assert rc == 0


def test_codestyle_clean():
    """tools/codestyle.py (include guards, whitespace, line length, unused
    imports) finds nothing in the tree"""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "codestyle.py")],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]


def test_man_pages_current():
    """man/*.{1,8} are rendered from the tools' own --help (tools/gen_man.py)"""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_man.py"), "--check"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
