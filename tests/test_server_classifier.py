"""End-to-end standalone jubaclassifier over msgpack-RPC (reference
client_test/classifier_test.cpp:40-85 and the status key set
client_test/status_test.hpp:23-57)."""
import os
import threading

import pytest

from jubatus_amd.client import Classifier, Datum, EstimateResult
from jubatus_amd.framework.server_helper import ServerHelper
from jubatus_amd.framework.server_util import ServerArgv
from jubatus_amd.server import get_serv

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STATUS_KEYS = {"clock_time", "start_time", "uptime", "VIRT", "RSS", "SHR", "timeout", "threadnum",
               "datadir", "is_standalone", "VERSION", "PROGNAME", "type", "logdir", "log_config",
               "configpath", "pid", "user", "update_count", "last_saved", "last_saved_path",
               "last_loaded", "last_loaded_path"}


def start_standalone(engine, config, tmp_path, extra=()):
    cfg = tmp_path / f"{engine}.json"
    cfg.write_text(open(config).read() if os.path.exists(config) else config)
    a = ServerArgv.parse(["-p", "9199", "-b", "127.0.0.1", "-f", str(cfg), "-d", str(tmp_path),
                          "--cpu", *extra], engine)
    a.port = 0
    h = ServerHelper(get_serv(engine), a, install_signals=False)
    h.start(block=False)
    return h


@pytest.fixture
def server(tmp_path):
    h = start_standalone("classifier", os.path.join(ROOT, "config/classifier/arow.json"), tmp_path)
    yield h
    h.stop()


def test_classifier_e2e(server):
    port = server.argv.port
    with Classifier("127.0.0.1", port, "") as c:
        assert '"AROW"' in c.get_config()
        assert c.classify([]) == []
        data = [("pos", Datum({"w": "good", "x": 1.0})), ("neg", Datum({"w": "bad", "x": -1.0}))] * 5
        assert c.train(data) == 10
        res = c.classify([Datum({"w": "good", "x": 1.0})])
        assert isinstance(res[0][0], EstimateResult)
        top = max(res[0], key=lambda e: e.score)
        assert top.label == "pos"
        assert c.get_labels() == {"pos": 5, "neg": 5}
        assert c.set_label("new") is True
        assert c.delete_label("new") is True
        assert c.delete_label("missing") is False
        st = c.get_status()
        assert len(st) == 1
        (key, s), = st.items()
        assert key.endswith(f"_{port}")
        assert STATUS_KEYS <= set(s)
        assert s["type"] == "classifier" and s["update_count"] == "4"  # train, set_label, delete_label x2
        saved = c.save("m1")
        assert len(saved) == 1 and list(saved.values())[0].endswith("_classifier_m1.jubatus")
        assert c.clear() is True
        assert c.get_labels() == {}
        assert c.load("m1") is True
        assert c.get_labels() == {"pos": 5, "neg": 5}
        top2 = max(c.classify([Datum({"w": "good", "x": 1.0})])[0], key=lambda e: e.score)
        assert top2.label == "pos" and abs(top2.score - top.score) < 1e-5
        s2 = list(c.get_status().values())[0]
        assert s2["last_loaded_path"] == list(saved.values())[0]


def test_classifier_errors(server):
    from jubatus_amd.common.mprpc import RpcCallError, RpcMethodNotFound, RpcTypeError
    with Classifier("127.0.0.1", server.argv.port, "") as c:
        with pytest.raises(RpcMethodNotFound):
            c.call("no_such_method")
        with pytest.raises(RpcTypeError):
            c.get_client().call("train", "")            # missing data arg
        with pytest.raises(RpcTypeError):
            c.get_client().call("train", "", [["x", 5]])  # bad datum
        with pytest.raises(RpcCallError):
            c.load("does_not_exist")
        with pytest.raises(RpcCallError):
            c.save("")


def test_model_file_startup(tmp_path):
    h = start_standalone("classifier", os.path.join(ROOT, "config/classifier/pa.json"), tmp_path)
    try:
        with Classifier("127.0.0.1", h.argv.port, "") as c:
            c.train([("a", Datum({"k": "v"})), ("b", Datum({"k": "w"}))])
            path = list(c.save("snap").values())[0]
    finally:
        h.stop()
    # -m adopts the file's config (server_helper.hpp:81-89)
    a = ServerArgv.parse(["-p", "9199", "-b", "127.0.0.1", "-m", path, "-d", str(tmp_path), "--cpu"],
                         "classifier")
    a.port = 0
    h2 = ServerHelper(get_serv("classifier"), a, install_signals=False)
    h2.start(block=False)
    try:
        with Classifier("127.0.0.1", h2.argv.port, "") as c:
            assert c.get_labels() == {"a": 1, "b": 1}
            assert '"PA"' in c.get_config()
    finally:
        h2.stop()


def test_concurrent_train_and_classify(server):
    port = server.argv.port
    errs = []

    def worker(k):
        try:
            with Classifier("127.0.0.1", port, "") as c:
                for i in range(20):
                    c.train([(f"l{k}", Datum({"w": f"t{k}", "x": float(k)}))])
                    c.classify([Datum({"w": f"t{k}"})])
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs
    with Classifier("127.0.0.1", port, "") as c:
        assert sum(c.get_labels().values()) == 80


@pytest.mark.parametrize("cfg", ["nn.json", "cosine.json", "euclidean.json"])
def test_nn_classifiers(tmp_path, cfg):
    """NN / cosine / euclidean classifiers (models/nn_classifier.py)"""
    from helpers import config_path, start_standalone
    from jubatus_amd.client import Classifier, Datum, EstimateResult
    h = start_standalone("classifier", config_path(f"classifier/{cfg}"), tmp_path)
    try:
        with Classifier("127.0.0.1", h.argv.port, "") as c:
            data = []
            for i in range(30):
                lab = "pos" if i % 2 else "neg"
                x = 3.0 if lab == "pos" else -3.0
                data.append([lab, Datum({"x": x + 0.1 * (i % 5), "y": 1.0, "t": lab + "w"})])
            assert c.train(data) == 30
            assert c.get_labels() == {"pos": 15, "neg": 15}
            res = c.classify([Datum({"x": 3.2, "y": 1.0, "t": "posw"}), Datum({"x": -2.9, "y": 1.0, "t": "negw"})])
            assert all(isinstance(r, EstimateResult) for row in res for r in row)
            best = [max(row, key=lambda r: r.score).label for row in res]
            assert best == ["pos", "neg"]
            assert c.set_label("other") is True and c.set_label("other") is False
            assert c.get_labels()["other"] == 0
            c.save("nn")
            assert c.delete_label("pos") is True
            assert set(c.get_labels()) == {"neg", "other"}
            assert all(r.label != "pos" for r in c.classify([Datum({"x": 3.0})])[0])
            assert c.load("nn") is True and c.get_labels()["pos"] == 15
            assert c.clear() is True and c.get_labels() == {}
    finally:
        h.stop()
