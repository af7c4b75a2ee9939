"""regression / nearest_neighbor / recommender / anomaly engines end to end
(reference client_test/{regression,nearest_neighbor,recommender,anomaly}_test.cpp
API smoke + numeric checks of our own)."""
import math

import pytest

from helpers import config_path, start_standalone
from jubatus_amd.client import Anomaly, Datum, IdWithScore, NearestNeighbor, Recommender, Regression


@pytest.fixture
def srv(request, tmp_path):
    engine, cfg = request.param
    h = start_standalone(engine, config_path(cfg), tmp_path)
    yield h
    h.stop()


@pytest.mark.parametrize("srv", [("regression", "regression/pa.json")], indirect=True)
def test_regression(srv):
    with Regression("127.0.0.1", srv.argv.port, "") as c:
        data = [(2.0 * x, Datum({"x": float(x)})) for x in range(1, 30)] * 3
        assert c.train([[s, d] for s, d in data]) == len(data)
        est = c.estimate([Datum({"x": 10.0}), Datum({"x": 3.0})])
        assert abs(est[0] - 20.0) < 2.0 and abs(est[1] - 6.0) < 1.5
        assert c.estimate([]) == []
        path = list(c.save("r").values())[0]
        assert c.clear() is True
        assert c.estimate([Datum({"x": 10.0})]) == [0.0]
        assert c.load("r") is True
        assert abs(c.estimate([Datum({"x": 10.0})])[0] - est[0]) < 1e-5


NN_CFGS = [("nearest_neighbor", f"nearest_neighbor/{m}.json") for m in ("lsh", "euclid_lsh", "minhash")]


@pytest.mark.parametrize("srv", NN_CFGS, indirect=True)
def test_nearest_neighbor(srv):
    with NearestNeighbor("127.0.0.1", srv.argv.port, "") as c:
        assert c.get_all_rows() == []
        for i in range(20):
            assert c.set_row(f"r{i}", Datum({"x": float(i), "y": float(i % 3), "t": f"w{i % 4}"}))
        assert sorted(c.get_all_rows()) == sorted(f"r{i}" for i in range(20))
        nb = c.neighbor_row_from_id("r5", 4)
        assert len(nb) == 4 and all(isinstance(x, IdWithScore) for x in nb)
        assert [x.score for x in nb] == sorted(x.score for x in nb)        # ascending distance
        # the row itself is at distance 0 (minhash sees feature *sets*: ties are expected)
        assert nb[0].score == pytest.approx(0.0, abs=1e-6)
        assert "r5" in [x.id for x in nb if x.score == nb[0].score]
        sim = c.similar_row_from_datum(Datum({"x": 5.0, "y": 2.0, "t": "w1"}), 3)
        assert [x.score for x in sim] == sorted((x.score for x in sim), reverse=True)
        assert c.neighbor_row_from_datum(Datum({"x": 1.0}), 0) == []
        st = list(c.get_status().values())[0]
        assert st["num_rows"] == "20"
        assert c.clear() is True and c.get_all_rows() == []


REC_CFGS = [("recommender", f"recommender/{m}.json") for m in
            ("inverted_index", "inverted_index_euclid", "lsh", "minhash", "euclid_lsh",
             "nearest_neighbor_recommender_euclid_lsh", "lsh_unlearn_lru")]


@pytest.mark.parametrize("srv", REC_CFGS, indirect=True)
def test_recommender(srv):
    with Recommender("127.0.0.1", srv.argv.port, "") as c:
        for i in range(12):
            assert c.update_row(f"u{i}", Datum({"a": float(i % 4), "b": float(i % 4) * 2, "c": f"x{i % 4}"}))
        assert c.update_row("u0", Datum({"z": 5.0}))           # merge into the row
        dec = c.decode_row("u0")
        assert dict(dec.num_values)["z"] == 5.0 and dict(dec.num_values)["a"] == 0.0
        sim = c.similar_row_from_id("u1", 3)
        assert len(sim) == 3 and sim[0].id in ("u1", "u5", "u9")
        assert c.similar_row_from_datum(Datum({"a": 2.0, "b": 4.0, "c": "x2"}), 2)[0].id in ("u2", "u6", "u10")
        comp = c.complete_row_from_datum(Datum({"a": 3.0, "c": "x3"}))
        nv = dict(comp.num_values)
        assert "b" in nv and nv["a"] == 3.0
        assert dict(c.complete_row_from_id("u1").num_values)["a"] == 1.0
        s_same = c.calc_similarity(Datum({"a": 1.0, "b": 2.0}), Datum({"a": 1.0, "b": 2.0}))
        s_diff = c.calc_similarity(Datum({"a": 1.0, "b": 2.0}), Datum({"a": -3.0, "q": 7.0}))
        assert s_same > s_diff
        assert c.calc_l2norm(Datum({"a": 3.0, "b": 4.0})) == pytest.approx(5.0, rel=1e-5)
        assert c.clear_row("u3") is True
        assert "u3" not in c.get_all_rows()
        st = list(c.get_status().values())[0]
        assert st["update_row_cnt"] == "13" and st["clear_row_cnt"] == "1"
        c.save("m")
        assert c.clear() is True and c.get_all_rows() == []
        assert c.load("m") is True and len(c.get_all_rows()) == 11


def test_recommender_lru_unlearner(tmp_path):
    cfg = ('{"method": "inverted_index", "parameter": {"unlearner": "lru", '
           '"unlearner_parameter": {"max_size": 3}}, '
           '"converter": {"num_rules": [{"key": "*", "type": "num"}]}}')
    h = start_standalone("recommender", cfg, tmp_path)
    try:
        with Recommender("127.0.0.1", h.argv.port, "") as c:
            for i in range(5):
                c.update_row(f"r{i}", Datum({"v": float(i)}))
            assert sorted(c.get_all_rows()) == ["r2", "r3", "r4"]
            c.update_row("r2", Datum({"w": 1.0}))             # touch r2
            c.update_row("r5", Datum({"v": 5.0}))
            assert sorted(c.get_all_rows()) == ["r2", "r4", "r5"]
    finally:
        h.stop()


ANOM_CFGS = [("anomaly", f"anomaly/{m}.json") for m in
             ("lof", "light_lof", "lof_inverted_index_euclid", "default")]


@pytest.mark.parametrize("srv", ANOM_CFGS, indirect=True)
def test_anomaly(srv):
    with Anomaly("127.0.0.1", srv.argv.port, "") as c:
        ids = []
        for i in range(40):
            r = c.add(Datum({"x": float(i % 10) * 0.1, "y": float(i % 7) * 0.1}))
            assert isinstance(r, IdWithScore)
            ids.append(r.id)
        assert ids == [str(i) for i in range(40)]
        normal = c.calc_score(Datum({"x": 0.5, "y": 0.3}))
        outlier = c.calc_score(Datum({"x": 50.0, "y": -40.0}))
        assert outlier > normal or math.isinf(outlier)
        assert isinstance(c.update("3", Datum({"x": 0.3, "y": 0.3})), float)
        assert isinstance(c.overwrite("4", Datum({"x": 0.4})), float)
        assert c.clear_row("5") is True
        assert len(c.get_all_rows()) == 39
        c.save("a")
        assert c.clear() is True and c.get_all_rows() == []
        assert c.load("a") is True
        assert c.add(Datum({"x": 0.1})).id == "40"           # id counter restored (anomaly_serv.cpp:299-320)
