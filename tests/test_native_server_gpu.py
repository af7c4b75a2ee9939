"""Native jubaclassifier on the GPU (csrc/server/jubaclassifier.cpp, no
Python in the server process): RPC behaviour of the reference client tests,
numerics against the host oracle (models/linear_oracle.py through
LinearClassifier on the host), concurrent train RPCs through the arena /
GPU-scan path, and model files interchangeable with the Python server's."""
import json
import os
import random
import socket
import subprocess
import threading
import time

import numpy as np
import pytest

from helpers import ROOT, config_path
from jubatus_amd.client import Classifier, Datum
from jubatus_amd.common.mprpc import RpcClient, RpcIOError, RpcTimeoutError, RpcTypeError

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaclassifier")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _start(cfg, tmp_path):
    port = _free_port()
    p = subprocess.Popen([BIN, "-p", str(port), "-b", "127.0.0.1", "-f", cfg, "-d", str(tmp_path),
                          "-c", "16"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    deadline = time.time() + 60
    while time.time() < deadline:
        try:
            with RpcClient("127.0.0.1", port, 5.0) as c:
                c.call("get_config", "")
            return port, p
        except (OSError, RpcIOError, RpcTimeoutError):
            if p.poll() is not None:
                break
            time.sleep(0.2)
    p.kill()
    raise RuntimeError("native server did not start: " + p.stdout.read().decode(errors="replace"))


@pytest.fixture
def native(tmp_path):
    port, p = _start(config_path("classifier/arow.json"), tmp_path)
    yield port
    p.terminate()
    try:
        p.wait(timeout=30)
    except subprocess.TimeoutExpired:
        p.kill()


def _data(rng, n):
    out = []
    for _ in range(n):
        y = rng.randrange(4)
        out.append((f"L{y}", Datum({"w": f"t{y * 10 + rng.randrange(3)}", "u": f"n{rng.randrange(50)}",
                                    "x": float(y) + rng.random()})))
    return out


def _status(c):
    (ident, st), = c.get_status().items()
    return ident, st


def _oracle(cfg_file):
    """the host model of a configuration, at the feature-table height the GPU
    servers resolve for it (device_hash_max_size when the converter names
    none), so model files of either load into it"""
    from jubatus_amd.fv_converter.converter import DatumToFvConverter, device_hash_max_size
    from jubatus_amd.models.classifier import LinearClassifier
    cfg = json.load(open(cfg_file))
    conv = DatumToFvConverter(cfg["converter"], default_hash_max_size=device_hash_max_size())
    return LinearClassifier(cfg["method"], cfg.get("parameter"), conv, device=None)


def _scores(rows):
    return [{e.label: e.score for e in r} for r in rows]


def test_native_server_matches_host_oracle(native):
    """sequential train requests (host path for new labels, then the GPU
    scan, exact single-stream updates) give the oracle's AROW model"""
    cfg = config_path("classifier/arow.json")
    c = Classifier("127.0.0.1", native, "", timeout=60)
    ora = _oracle(cfg)
    rng = random.Random(3)
    for _ in range(6):
        chunk = _data(rng, 50)
        assert c.train(chunk) == 50
        ora.train([(l, d) for l, d in chunk])
    test = [d for _, d in _data(random.Random(9), 40)]
    got = _scores(c.classify(test))
    want = [dict(r) for r in ora.classify(test)]
    for g, w in zip(got, want):
        assert set(g) == set(w)
        for k in w:
            assert abs(g[k] - w[k]) <= 1e-4 * max(1.0, abs(w[k])), (k, g[k], w[k])
    ident, st = _status(c)
    assert st["server_runtime"] == "native" and st["storage"] == "hbm"
    assert int(st["train_scan.gpu"]) >= 1 and int(st["train_scan.host"]) >= 1
    for k in ("PROGNAME", "RSS", "VERSION", "clock_time", "configpath", "datadir", "is_standalone",
              "last_loaded", "last_saved", "pid", "threadnum", "timeout", "update_count", "uptime",
              "user"):
        assert k in st, k
    assert st["is_standalone"] == "1"
    assert sum(c.get_labels().values()) == 300
    c.close()


def test_native_concurrent_train_and_bad_requests(native):
    c = Classifier("127.0.0.1", native, "", timeout=60)
    assert c.train(_data(random.Random(1), 32)) == 32
    errors, bad_seen = [], []

    def good(seed):
        try:
            cc = Classifier("127.0.0.1", native, "", timeout=60)
            r = random.Random(seed)
            for _ in range(20):
                assert cc.train(_data(r, 64)) == 64
            cc.close()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def bad():
        with RpcClient("127.0.0.1", native, 60.0) as rc:
            for _ in range(5):
                try:
                    rc.call("train", "", [["L1", [[["only-a-key"]], [], []]]])
                except RpcTypeError:
                    bad_seen.append(1)
    ts = [threading.Thread(target=good, args=(s,)) for s in range(16)] + [threading.Thread(target=bad)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    assert len(bad_seen) == 5
    assert sum(c.get_labels().values()) == 32 + 16 * 20 * 64
    test = _data(random.Random(77), 200)
    res = c.classify([d for _, d in test])
    acc = np.mean([max(r, key=lambda e: e.score).label == l for r, (l, _) in zip(res, test)])
    assert acc > 0.9, acc
    assert c.classify([]) == []
    big = c.classify([d for _, d in _data(random.Random(5), 300)])     # batch (non-direct) path
    assert len(big) == 300 and all(len(r) == 4 for r in big)
    c.close()


def test_native_labels_and_clear(native):
    c = Classifier("127.0.0.1", native, "", timeout=60)
    assert c.set_label("new") is True
    assert c.set_label("new") is False
    assert c.train(_data(random.Random(2), 20)) == 20
    labels = c.get_labels()
    assert labels["new"] == 0 and len(labels) == 5
    assert c.delete_label("L0") is True
    assert c.delete_label("L0") is False
    assert "L0" not in c.get_labels()
    r = c.classify([Datum({"w": "t1"})])
    assert {e.label for e in r[0]} == set(c.get_labels())
    assert c.clear() is True
    assert c.get_labels() == {}
    assert json.loads(c.get_config()) == json.load(open(config_path("classifier/arow.json")))
    with RpcClient("127.0.0.1", native, 10.0) as rc:
        with pytest.raises(Exception):
            rc.call("no_such_method", "")
    c.close()


def test_native_model_files_interoperate_with_python(native, tmp_path):
    from jubatus_amd.framework import save_load
    cfg_file = config_path("classifier/arow.json")
    cfg_text = open(cfg_file).read()
    c = Classifier("127.0.0.1", native, "", timeout=60)
    rng = random.Random(11)
    data = _data(rng, 300)
    for k in range(0, 300, 100):
        assert c.train(data[k:k + 100]) == 100
    test = [d for _, d in _data(random.Random(12), 30)]
    before = _scores(c.classify(test))
    ident, _ = _status(c)
    (_, path), = c.save("m1").items()
    assert os.path.exists(path)
    # native file -> Python driver
    with open(path, "rb") as f:
        _, pack = save_load.load_server(f, "classifier", cfg_text, 1, False)
    ora = _oracle(cfg_file)
    ora.unpack(pack)
    py = [dict(r) for r in ora.classify(test)]
    for g, w in zip(before, py):
        for k in w:
            assert abs(g[k] - w[k]) <= 1e-5 * max(1.0, abs(w[k]))
    assert ora.get_labels() == c.get_labels()
    # native load of its own file after clear
    assert c.clear() is True
    assert c.load("m1") is True
    again = _scores(c.classify(test))
    for g, w in zip(again, before):
        for k in w:
            assert abs(g[k] - w[k]) <= 1e-6 * max(1.0, abs(w[k]))
    # Python file -> native server
    ora2 = _oracle(cfg_file)
    ora2.train([(l, d) for l, d in _data(random.Random(13), 120)])
    p2 = os.path.join(os.path.dirname(path), f"{ident}_classifier_py.jubatus")
    with open(p2, "wb") as f:
        save_load.save_server(f, "classifier", "py", cfg_text, 1, ora2.pack())
    assert c.load("py") is True
    got = _scores(c.classify(test))
    want = [dict(r) for r in ora2.classify(test)]
    for g, w in zip(got, want):
        for k in w:
            assert abs(g[k] - w[k]) <= 1e-5 * max(1.0, abs(w[k]))
    assert c.get_labels() == ora2.get_labels()
    c.close()


# ------------------------------------------------------------------ regression
REG_BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaregression")


def _reg_data(rng, n):
    out = []
    for _ in range(n):
        x = rng.random() * 4
        out.append((3.0 * x + 1.0 + rng.gauss(0, 0.1), Datum({"x": x, "c": f"k{rng.randrange(5)}"})))
    return out


def test_native_regression_matches_oracle_and_files(tmp_path):
    """native jubaregression: sequential requests equal the host oracle
    (models/regression.py train_one), model files shared with the Python
    driver, status and clear"""
    from jubatus_amd.client import Regression
    from jubatus_amd.framework import save_load
    from jubatus_amd.fv_converter.converter import DatumToFvConverter, device_hash_max_size
    from jubatus_amd.models.regression import PARegression
    cfg_file = config_path("regression/pa.json")
    cfg = json.load(open(cfg_file))
    port = _free_port()
    p = subprocess.Popen([REG_BIN, "-p", str(port), "-b", "127.0.0.1", "-f", cfg_file, "-d", str(tmp_path)],
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        deadline = time.time() + 60
        while True:
            try:
                with RpcClient("127.0.0.1", port, 5.0) as c:
                    c.call("get_config", "")
                break
            except (OSError, RpcIOError, RpcTimeoutError):
                assert p.poll() is None and time.time() < deadline, p.stdout.read()
                time.sleep(0.2)
        c = Regression("127.0.0.1", port, "", timeout=60)
        ora = PARegression("PA", cfg.get("parameter"),
                           DatumToFvConverter(cfg["converter"], default_hash_max_size=device_hash_max_size()),
                           device=None)
        rng = random.Random(4)
        for _ in range(5):
            chunk = _reg_data(rng, 40)
            assert c.train(chunk) == 40
            ora.train([(s, d) for s, d in chunk])
        test = [d for _, d in _reg_data(random.Random(8), 30)]
        got = c.estimate(test)
        want = ora.estimate(test)
        np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-4)
        (ident, st), = c.get_status().items()
        assert st["server_runtime"] == "native" and st["is_standalone"] == "1"
        assert int(st["train.samples_trained"]) == 200
        with RpcClient("127.0.0.1", port, 10.0) as rc:
            with pytest.raises(RpcTypeError):
                rc.call("train", "", [[True, [[], [["x", 1.0]], []]]])
        (_, path), = c.save("r1").items()
        with open(path, "rb") as f:
            _, pack = save_load.load_server(f, "regression", open(cfg_file).read(), 1, False)
        ora2 = PARegression("PA", cfg.get("parameter"),
                            DatumToFvConverter(cfg["converter"], default_hash_max_size=device_hash_max_size()),
                            device=None)
        ora2.unpack(pack)
        np.testing.assert_allclose(ora2.estimate(test), got, rtol=1e-6, atol=1e-6)
        assert c.clear() is True
        assert all(v == 0.0 for v in c.estimate(test))
        assert c.load("r1") is True
        np.testing.assert_allclose(c.estimate(test), got, rtol=1e-6, atol=1e-6)
        # Python-written file -> native
        p2 = os.path.join(str(tmp_path), f"{ident}_regression_py.jubatus")
        with open(p2, "wb") as f:
            save_load.save_server(f, "regression", "py", open(cfg_file).read(), 1, ora.pack())
        assert c.load("py") is True
        np.testing.assert_allclose(c.estimate(test), want, rtol=1e-4, atol=1e-4)
        c.close()
    finally:
        p.terminate()
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()


@pytest.mark.parametrize("cfg_name", ["classifier/default.json", "classifier/arow_combinational_feature.json"])
def test_native_wide_converter_configs_match_oracle(cfg_name, tmp_path):
    """the reference's default classifier config (bigram tokens, tf / idf
    weights) and the mul-combination config run natively: host wide
    converter (jb_hostfv_wide.hpp) with the document statistics, exact
    single-stream updates; the model equals the host oracle's, the weights
    travel in the model file"""
    from jubatus_amd.framework import save_load
    cfg_file = config_path(cfg_name)
    port, p = _start(cfg_file, tmp_path)
    try:
        c = Classifier("127.0.0.1", port, "", timeout=60)
        ora = _oracle(cfg_file)
        rng = random.Random(13)
        words = ["alpha beta", "gamma", "beta gamma delta", "epsilon", "zeta eta"]
        for _ in range(4):
            chunk = []
            for _ in range(30):
                y = rng.randrange(3)
                chunk.append((f"L{y}", Datum({"text": words[(y + rng.randrange(2)) % 5] + f" w{y}",
                                              "x": float(y) + rng.random()})))
            assert c.train(chunk) == 30
            ora.train([(l, d) for l, d in chunk])
        test = [Datum({"text": words[i % 5] + f" w{i % 3}", "x": float(i % 3)}) for i in range(15)]
        got = _scores(c.classify(test))
        want = [dict(r) for r in ora.classify(test)]
        for g, w in zip(got, want):
            assert set(g) == set(w)
            for k in w:
                assert abs(g[k] - w[k]) <= 1e-3 * max(1.0, abs(w[k])), (k, g[k], w[k])
        _, st = _status(c)
        assert st["server_runtime"] == "native"
        (_, path), = c.save("wide").items()
        with open(path, "rb") as f:
            _, pack = save_load.load_server(f, "classifier", open(cfg_file).read(), 1, False)
        ora2 = _oracle(cfg_file)
        ora2.unpack(pack)
        want2 = [dict(r) for r in ora2.classify(test)]
        for g, w in zip(got, want2):
            for k in w:
                assert abs(g[k] - w[k]) <= 1e-3 * max(1.0, abs(w[k])), (k, g[k], w[k])
        c.close()
    finally:
        p.terminate()
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()


@pytest.mark.parametrize("cfg_name", ["classifier/cosine.json", "classifier/euclidean.json", "classifier/nn.json"])
def test_native_nn_classifier_matches_python_driver(cfg_name, tmp_path):
    """the nearest-neighbor classifier methods run natively on the row
    server (jb_row_server.hpp Kind::kClassifier: rows in HBM, batched k-NN
    scans): labels, scores and model files agree with the Python driver
    (models/nn_classifier.py over the same GPU row kernels)"""
    import torch
    from jubatus_amd.framework import save_load
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.nn_classifier import NNClassifier
    cfg_file = config_path(cfg_name)
    cfg = json.load(open(cfg_file))
    port, p = _start(cfg_file, tmp_path)
    try:
        c = Classifier("127.0.0.1", port, "", timeout=60)
        ora = NNClassifier(cfg["method"], cfg.get("parameter"), DatumToFvConverter(cfg["converter"]),
                           device=torch.device("cuda", 0))
        rng = random.Random(21)
        for _ in range(3):
            chunk = _data(rng, 40)
            assert c.train(chunk) == 40
            ora.train([(l, d) for l, d in chunk])
        assert c.set_label("spare") is True and ora.set_label("spare") is True
        test = [d for _, d in _data(random.Random(5), 12)]
        got = _scores(c.classify(test))
        want = [dict(r) for r in ora.classify(test)]
        for g, w in zip(got, want):
            assert set(g) == set(w), (g, w)
            for k in w:
                assert abs(g[k] - w[k]) <= 1e-4 * max(1.0, abs(w[k])), (k, g[k], w[k])
        labels = {(k.decode() if isinstance(k, bytes) else k): v for k, v in c.get_labels().items()}
        assert labels == ora.get_labels()
        _, st = _status(c)
        assert st["server_runtime"] == "native" and st["method"] == cfg["method"]
        # the model file loads into the Python driver and answers the same
        (_, path), = c.save("nn").items()
        with open(path, "rb") as f:
            _, pack = save_load.load_server(f, "classifier", open(cfg_file).read(), 1, False)
        ora2 = NNClassifier(cfg["method"], cfg.get("parameter"), DatumToFvConverter(cfg["converter"]),
                            device=torch.device("cuda", 0))
        ora2.unpack(pack)
        for g, w in zip(got, [dict(r) for r in ora2.classify(test)]):
            for k in w:
                assert abs(g[k] - w[k]) <= 1e-4 * max(1.0, abs(w[k])), (k, g[k], w[k])
        assert c.delete_label("L0") is True
        assert "L0" not in {(k.decode() if isinstance(k, bytes) else k) for k in c.get_labels()}
        c.close()
    finally:
        p.terminate()
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
