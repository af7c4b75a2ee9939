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


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU host serves natively")
def test_hands_over_to_python_without_gpu(tmp_path):
    """no /dev/kfd: the binary execs the Python server with the same flags"""
    port = _free_port()
    env = dict(os.environ, JUBATUS_FORCE_CPU="1")
    p = subprocess.Popen([BIN, "-p", str(port), "-b", "127.0.0.1", "-f",
                          config_path("classifier/arow.json"), "-d", str(tmp_path)],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env)
    try:
        deadline = time.time() + 120
        st = None
        while time.time() < deadline:
            try:
                with RpcClient("127.0.0.1", port, 5.0) as c:
                    st = c.call("get_status", "")
                    assert c.call("train", "", [["a", [[["w", "x"]], [], []]]]) == 1
                break
            except (OSError, RpcIOError, RpcTimeoutError):
                if p.poll() is not None:
                    break
                time.sleep(0.5)
        assert st is not None, p.stdout.read().decode(errors="replace") if p.poll() is not None else ""
        (_, s), = st.items()
        s = {(k.decode() if isinstance(k, bytes) else k): v for k, v in s.items()}
        assert "server_runtime" not in s       # the Python server answered
        assert s["storage"] == "host"
    finally:
        p.terminate()
        p.wait(timeout=30)
