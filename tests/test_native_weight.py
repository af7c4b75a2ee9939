"""Native jubaweight (csrc/server/jubaweight.cpp: no Python, no GPU) against
the Python driver (models/weight.py) fed the same calls: update /
calc_weight results (feature order, names and values; idf / bm25 against the
document statistics), clear, status, and model files both ways. Reference:
weight_serv.cpp:30-110."""
import json
import math
import os
import random
import shutil
import socket
import subprocess
import time

import pytest

from helpers import ROOT
from jubatus_amd.common.mprpc import RpcClient, RpcIOError, RpcTimeoutError

NATIVE = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaweight")

PLUG = "libjubatus_sample_plugins.so"
CONFIGS = {
    # plug-ins loaded by the native server (dlopen, jb_plugin_host.hpp): splitter,
    # string / num filters, num feature, combination; idf over the plug-in tokens
    "plugin": {"string_filter_types": {"up": {"method": "dynamic", "path": PLUG, "function": "create_upper_filter"}},
               "string_filter_rules": [{"key": "s", "type": "up", "suffix": "-up"}],
               "num_filter_types": {"aff": {"method": "dynamic", "path": PLUG, "function": "create_affine_filter",
                                            "scale": "2", "shift": "1"}},
               "num_filter_rules": [{"key": "*", "type": "aff", "suffix": "-aff"}],
               "string_types": {"sp": {"method": "dynamic", "path": PLUG, "function": "create_splitter",
                                       "delimiter": " ", "min_length": "2"}},
               "string_rules": [{"key": "*", "type": "sp", "sample_weight": "tf", "global_weight": "idf"}],
               "num_types": {"bk": {"method": "dynamic", "path": PLUG, "function": "create_bucket_feature",
                                    "width": "10"}},
               "num_rules": [{"key": "*", "type": "bk"}, {"key": "*", "type": "num"}],
               "combination_types": {"mx": {"method": "dynamic", "path": PLUG, "function": "create_max_combination"}},
               "combination_rules": [{"key_left": "*@num", "key_right": "*-aff@num", "type": "mx"}]},
    "bin": {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
            "num_rules": [{"key": "*", "type": "num"}]},
    "idf": {"string_types": {"bigram": {"method": "ngram", "char_num": "2"}},
            "string_rules": [{"key": "*", "type": "bigram", "sample_weight": "tf", "global_weight": "idf"},
                             {"key": "t*", "type": "space", "sample_weight": "log_tf", "global_weight": "bm25"}],
            "num_rules": [{"key": "*", "type": "num"}, {"key": "l*", "type": "log"}]},
}

pytestmark = pytest.mark.skipif(not os.path.exists(NATIVE), reason="native jubaweight not built")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start(cfg_path, tmp_path, model=None):
    port = _free_port()
    cmd = [NATIVE, "-p", str(port), "-b", "127.0.0.1", "-d", str(tmp_path)]
    cmd += ["-m", model] if model else ["-f", cfg_path]
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    deadline = time.time() + 30
    while True:
        try:
            with RpcClient("127.0.0.1", port, 5.0) as c:
                c.call("get_config", "")
            return p, port
        except (OSError, RpcIOError, RpcTimeoutError):
            assert p.poll() is None and time.time() < deadline, p.stdout.read()
            time.sleep(0.1)


def _datum(rng):
    words = ["alpha", "beta", "gamma", "delta", "eps"]
    sv = [["s", " ".join(rng.choice(words) for _ in range(rng.randrange(1, 4)))],
          ["title", rng.choice(words) + " " + rng.choice(words)]]
    nv = [["n", round(rng.uniform(-3, 3), 3)], ["len", round(rng.uniform(1, 50), 2)]]
    return [sv, nv, []]


def _same(got, want):
    assert len(got) == len(want), (got, want)
    for (gk, gv), (wk, wv) in zip(got, want):
        gk = gk.decode() if isinstance(gk, bytes) else gk
        assert gk == wk, (got, want)
        assert math.isclose(gv, wv, rel_tol=2e-6, abs_tol=1e-6), (gk, gv, wv)


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_native_weight_matches_python_driver(name, tmp_path):
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.fv_converter.datum import Datum
    from jubatus_amd.models.weight import Weight
    cfg = {"converter": CONFIGS[name], "method": "weight", "parameter": {}}
    path = tmp_path / "w.json"
    path.write_text(json.dumps(cfg))
    ref = Weight(DatumToFvConverter(cfg["converter"]))
    p, port = _start(str(path), tmp_path)
    try:
        rng = random.Random(3)
        with RpcClient("127.0.0.1", port, 10.0) as c:
            for i in range(120):
                d = _datum(rng)
                if rng.random() < 0.7:
                    _same(c.call("update", "", d), ref.update(Datum.from_msgpack(d)))
                else:
                    _same(c.call("calc_weight", "", d), ref.calc_weight(Datum.from_msgpack(d)))
            (_, st), = c.call("get_status", "").items()
            st = {k.decode() if isinstance(k, bytes) else k: v.decode() if isinstance(v, bytes) else v
                  for k, v in st.items()}
            assert st["server_runtime"] == "native" and st["weight_manager"] == "df"
            # model file: the native file loads into the Python driver and back
            (_, mpath), = c.call("save", "", "m").items()
            mpath = mpath.decode() if isinstance(mpath, bytes) else mpath
            from jubatus_amd.framework.save_load import read_model_file
            with open(mpath, "rb") as f:
                _, user = read_model_file(f)
            ref2 = Weight(DatumToFvConverter(cfg["converter"]))
            ref2.unpack(user[1])
            d = _datum(rng)
            _same(c.call("calc_weight", "", d), ref2.calc_weight(Datum.from_msgpack(d)))
            assert c.call("clear", "") is True
            d = _datum(rng)
            ref3 = Weight(DatumToFvConverter(cfg["converter"]))
            _same(c.call("update", "", d), ref3.update(Datum.from_msgpack(d)))
    finally:
        p.terminate()
        p.wait(timeout=30)


def test_native_weight_hands_unsupported_configs_to_python(tmp_path):
    cfg = {"converter": {"string_filter_types": {"rm": {"method": "regexp", "pattern": "a", "replace": ""}},
                         "string_filter_rules": [{"key": "*", "type": "rm", "suffix": "-x"}],
                         "string_rules": [{"key": "*", "type": "str", "sample_weight": "bin",
                                           "global_weight": "bin"}]}}
    path = tmp_path / "w.json"
    path.write_text(json.dumps(cfg))
    r = subprocess.run([NATIVE, "--native-check", "-f", str(path)], capture_output=True, text=True, timeout=30)
    assert r.stdout.startswith("python"), r.stdout
