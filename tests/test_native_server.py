"""Native jubaclassifier (csrc/server/jubaclassifier.cpp): the configuration
check that decides native vs Python service, and the hand-over to the Python
server (exec before any GPU call) on hosts without a GPU. The GPU behaviour
is in tests/test_native_server_gpu.py."""
import os
import socket
import subprocess
import time

import pytest

from helpers import ROOT, config_path
from jubatus_amd.common.mprpc import RpcClient, RpcIOError, RpcTimeoutError

BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaclassifier")
REG_BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaregression")

# every reference classifier config: linear methods on the fixed-slot GPU
# hasher or the host wide rule set (bigram, combinations, idf), the
# nearest-neighbor methods on the native row server
NATIVE = ["arow.json", "cw.json", "nherd.json", "pa.json", "pa1.json", "pa2.json", "perceptron.json",
          "arow_combinational_feature.json", "default.json", "cosine.json", "nn.json", "euclidean.json"]


def _check(cfg_file, binary=BIN):
    r = subprocess.run([binary, "--native-check", "-f", cfg_file], capture_output=True, text=True,
                       timeout=30)
    assert r.returncode == 0, r.stderr
    return r.stdout.strip()


@pytest.mark.parametrize("name", NATIVE)
def test_linear_configs_are_native(name):
    assert _check(config_path(f"classifier/{name}")) == "native"


def test_unknown_methods_go_to_python(tmp_path):
    import json
    p = tmp_path / "c.json"
    p.write_text(json.dumps({"method": "SVM", "converter": {}, "parameter": {}}))
    out = _check(str(p))
    assert out.startswith("python: "), out
    p.write_text(json.dumps({"method": "NN", "converter": {},
                             "parameter": {"method": "bogus", "nearest_neighbor_num": 4}}))
    assert "unknown nearest neighbor method" in _check(str(p))


@pytest.mark.parametrize("cfg,why", [
    ({"method": "AROW", "converter": {"num_rules": [{"key": "/x.*/", "type": "num"}]},
      "parameter": {"regularization_weight": 1.0}}, "regex"),
    ({"method": "CW", "converter": {}, "parameter": {}}, "regularization_weight"),
    # (a user num type shadowing a builtin name converts natively now, as in Python)
    ({"method": "PA", "converter": {"string_rules": [{"key": "*", "type": "str"}],
                                    "string_filter_types": {"x": {"method": "regexp", "pattern": "a"}},
                                    "string_filter_rules": [{"key": "*", "type": "x", "suffix": "_f"}]}},
     "regexp"),
])
def test_config_details(tmp_path, cfg, why):
    import json
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    out = _check(str(p))
    assert why in out, out


@pytest.mark.parametrize("name,want", [("pa.json", "native"), ("default.json", "native"),
                                       ("pa_combinational_feature.json", "native")])
def test_regression_configs(name, want):
    assert _check(config_path(f"regression/{name}"), REG_BIN).startswith(want)


def test_regression_parameter_checks(tmp_path):
    import json
    p = tmp_path / "r.json"
    p.write_text(json.dumps({"method": "PA", "parameter": {"sensitivity": -1},
                             "converter": {"num_rules": [{"key": "*", "type": "num"}]}}))
    assert "sensitivity" in _check(str(p), REG_BIN)
    p.write_text(json.dumps({"method": "NN", "converter": {}}))
    assert "not PA" in _check(str(p), REG_BIN)


def test_version():
    r = subprocess.run([BIN, "-v"], capture_output=True, text=True, timeout=30)
    assert r.returncode == 0 and "native" in r.stdout


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start(args, env_extra=None, timeout=60):
    port = _free_port()
    env = dict(os.environ, PATH="/nonexistent", JUBATUS_FORCE_CPU="1", **(env_extra or {}))
    p = subprocess.Popen([BIN, "-p", str(port), "-b", "127.0.0.1", *args], stdout=subprocess.PIPE,
                         stderr=subprocess.STDOUT, env=env)
    deadline = time.time() + timeout
    while time.time() < deadline:
        try:
            c = RpcClient("127.0.0.1", port, 30.0)
            c.call("get_config", "")
            return p, c
        except (OSError, RpcIOError, RpcTimeoutError):
            if p.poll() is not None:
                break
            time.sleep(0.2)
    out = p.stdout.read().decode(errors="replace") if p.poll() is not None else ""
    p.kill()
    raise AssertionError(f"server did not start: {out}")


def _status(c):
    (_, s), = c.call("get_status", "").items()
    return {(k.decode() if isinstance(k, bytes) else k): (v.decode() if isinstance(v, bytes) else v)
            for k, v in s.items()}


def _stream(n, seed, nlabels=4):
    import random
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        y = rng.randrange(nlabels)
        sv = [[f"s{j}", f"v{y * 7 + rng.randrange(3) if rng.random() < 0.7 else rng.randrange(200)}"]
              for j in range(4)]
        nv = [[f"n{j}", (y - 1.5) * 0.5 + rng.gauss(0, 1)] for j in range(3)]
        out.append([f"L{y}", [sv, nv, []]])
    return out


@pytest.mark.parametrize("cfg_name", ["pa.json", "arow.json", "pa1.json"])
def test_host_backend_serves_natively_without_python(tmp_path, cfg_name):
    """BASELINE config #1 (pa.json standalone on the CPU) with no Python
    reachable (PATH=/nonexistent) and no GPU (JUBATUS_FORCE_CPU): the native
    host backend trains one sample after another (classifier_serv.cpp:138-144)
    and agrees with the Python host classifier (models/linear_oracle.py);
    save / load round-trip through the shared model file format"""
    import json
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier

    cfg = json.load(open(config_path(f"classifier/{cfg_name}")))
    p, c = _start(["-f", config_path(f"classifier/{cfg_name}"), "-d", str(tmp_path)])
    try:
        st = _status(c)
        assert st["server_runtime"] == "native" and st["backend"] == "host", st
        data = _stream(600, seed=len(cfg_name))
        for i in range(0, len(data), 50):
            assert c.call("train", "", data[i:i + 50]) == 50
        ref = LinearClassifier(cfg["method"], cfg.get("parameter") or {}, DatumToFvConverter(cfg["converter"]))
        for i in range(0, len(data), 50):      # the host oracle (device=None), request after request
            ref.train([(l, d) for l, d in data[i:i + 50]])
        q = [d for _, d in data[:40]]
        got = c.call("classify", "", q)
        want = ref.classify(q)
        for g, w in zip(got, want):
            gd = {(k.decode() if isinstance(k, bytes) else k): v for k, v in g}
            wd = dict(w)
            assert sorted(gd) == sorted(wd)
            for k in wd:
                assert abs(gd[k] - wd[k]) <= 1e-3 * max(1.0, abs(wd[k])), (k, gd[k], wd[k])
        st = _status(c)
        assert int(st["train.samples_trained"]) == len(data)
        assert int(st["train.samples_updated"]) == ref.train_stats()["updated"]
        saved = c.call("save", "", "m1")
        (_, path), = saved.items()
        path = path.decode() if isinstance(path, bytes) else path
        assert c.call("clear", "") is True
        assert c.call("get_labels", "") == {}
        assert c.call("load", "", "m1") is True
        again = c.call("classify", "", q)
        assert again == got
        labels = {(k.decode() if isinstance(k, bytes) else k): v for k, v in c.call("get_labels", "").items()}
        assert sum(labels.values()) == len(data)
        assert c.call("delete_label", "", "L0") is True
        assert "L0" not in {(k.decode() if isinstance(k, bytes) else k) for k in c.call("get_labels", "")}
    finally:
        c.close()
        p.terminate()
        p.wait(timeout=30)
    # a server started from that model file (-m) serves the same model
    p, c = _start(["-m", path, "-d", str(tmp_path)])
    try:
        assert c.call("classify", "", q) == got
    finally:
        c.close()
        p.terminate()
        p.wait(timeout=30)


def test_unreadable_config_or_model_fails_cleanly(tmp_path):
    """the reference exits with an error (config.cpp:39-48 "can't read",
    server_helper.hpp:81-113 load_file) - no Python fallback"""
    env = dict(os.environ, PATH="/nonexistent")
    r = subprocess.run([BIN, "-f", str(tmp_path / "missing.json"), "-p", str(_free_port())],
                       capture_output=True, text=True, timeout=30, env=env)
    assert r.returncode == 1 and "can't read" in r.stderr, (r.returncode, r.stderr)
    bad = tmp_path / "bad.jubatus"
    bad.write_bytes(b"not a model file at all" * 10)
    r = subprocess.run([BIN, "-m", str(bad), "-p", str(_free_port())], capture_output=True, text=True,
                       timeout=30, env=env)
    assert r.returncode == 1 and str(bad) in r.stderr, (r.returncode, r.stderr)
    r = subprocess.run([BIN, "-m", str(tmp_path / "none.jubatus"), "-p", str(_free_port())],
                       capture_output=True, text=True, timeout=30, env=env)
    assert r.returncode == 1 and "cannot open input file" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU host serves natively")
def test_nn_classifier_hands_over_to_python_without_gpu(tmp_path):
    """the nearest-neighbor methods need the device: without a GPU the binary
    execs the Python server with the same flags"""
    port = _free_port()
    env = dict(os.environ, JUBATUS_FORCE_CPU="1")
    p = subprocess.Popen([BIN, "-p", str(port), "-b", "127.0.0.1", "-f",
                          config_path("classifier/nn.json"), "-d", str(tmp_path)],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
    try:
        deadline = time.time() + 120
        st = None
        while time.time() < deadline:
            try:
                with RpcClient("127.0.0.1", port, 5.0) as c:
                    st = c.call("get_status", "")
                break
            except (OSError, RpcIOError, RpcTimeoutError):
                if p.poll() is not None:
                    break
                time.sleep(0.5)
        assert st is not None, p.stdout.read().decode(errors="replace") if p.poll() is not None else ""
        (_, s), = st.items()
        s = {(k.decode() if isinstance(k, bytes) else k): v for k, v in s.items()}
        assert "server_runtime" not in s       # the Python server answered
    finally:
        p.terminate()
        p.wait(timeout=30)
