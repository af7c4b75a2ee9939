"""The reference's client smoke assertions (client_test/*_test.cpp, SURVEY
§4), per engine over msgpack-RPC: non-empty get_config, save returns one
{host_port: path} entry and load accepts it, clear returns true, empty
inputs give empty results, a fresh row store lists no rows."""
import pytest

from helpers import config_path, start_standalone
from jubatus_amd.common.mprpc import RpcClient

ENGINES = [("classifier", "classifier/pa.json"), ("regression", "regression/pa.json"),
           ("recommender", "recommender/lsh.json"), ("nearest_neighbor", "nearest_neighbor/lsh.json"),
           ("anomaly", "anomaly/lof.json"), ("clustering", "clustering/kmeans.json"),
           ("graph", "graph/default.json"), ("stat", "stat/default.json"),
           ("bandit", "bandit/ucb1.json"), ("burst", "burst/default.json"),
           ("weight", "weight/default.json")]

# engine -> [(method, args, expected result)] (classifier_test.cpp:40-85,
# recommender_test.cpp:55-133, nearest_neighbor_test.cpp:29-97, ...)
EMPTY_CALLS = {
    "classifier": [("classify", [[]], []), ("get_labels", [], {})],
    "regression": [("estimate", [[]], [])],
    "recommender": [("get_all_rows", [], [])],
    "nearest_neighbor": [("get_all_rows", [], [])],
    "anomaly": [("get_all_rows", [], [])],
}


def _s(x):
    return x.decode() if isinstance(x, bytes) else x


@pytest.mark.parametrize("engine,cfg", ENGINES)
def test_client_smoke(engine, cfg, tmp_path, monkeypatch):
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    h = start_standalone(engine, config_path(cfg), tmp_path)
    try:
        with RpcClient("127.0.0.1", h.argv.port, 10.0) as c:
            assert len(_s(c.call("get_config", ""))) > 2
            for method, args, want in EMPTY_CALLS.get(engine, []):
                assert c.call(method, "", *args) == want, method
            saved = c.call("save", "", "m0")
            assert len(saved) == 1
            path = _s(list(saved.values())[0])
            assert path.endswith("m0.jubatus")
            assert c.call("load", "", "m0") is True
            assert c.call("clear", "") is True
    finally:
        h.stop()
