"""get_status key set of every engine server (reference
client_test/status_test.hpp:23-57, assert_common_status): the common keys in
standalone mode, and none of the distributed-only keys."""
import pytest

from helpers import config_path, start_standalone
from jubatus_amd.common.mprpc import RpcClient

COMMON = ["PROGNAME", "RSS", "SHR", "VIRT", "VERSION", "clock_time", "configpath", "datadir",
          "is_standalone", "last_loaded", "last_loaded_path", "last_saved", "last_saved_path",
          "logdir", "pid", "start_time", "threadnum", "timeout", "update_count", "uptime", "user"]
DISTRIBUTED = ["connected_zookeeper", "interconnect_timeout", "interval_count", "interval_sec",
               "mixer", "name", "use_cht", "zk", "zookeeper_timeout"]

ENGINES = [("classifier", "classifier/pa.json"), ("regression", "regression/pa.json"),
           ("recommender", "recommender/lsh.json"), ("nearest_neighbor", "nearest_neighbor/lsh.json"),
           ("anomaly", "anomaly/lof.json"), ("clustering", "clustering/kmeans.json"),
           ("graph", "graph/default.json"), ("stat", "stat/default.json"),
           ("bandit", "bandit/ucb1.json"), ("burst", "burst/default.json"),
           ("weight", "weight/default.json")]


@pytest.mark.parametrize("engine,cfg", ENGINES)
def test_status_common_keys(engine, cfg, tmp_path, monkeypatch):
    monkeypatch.setenv("JUBATUS_FORCE_CPU", "1")
    h = start_standalone(engine, config_path(cfg), tmp_path)
    try:
        with RpcClient("127.0.0.1", h.argv.port, 10.0) as c:
            st = c.call("get_status", "")
    finally:
        h.stop()
    assert len(st) == 1
    status = {(k.decode() if isinstance(k, bytes) else k): v for k, v in list(st.values())[0].items()}
    missing = [k for k in COMMON if k not in status]
    assert not missing, (engine, missing)
    assert str(status["is_standalone"]) not in ("0", "false", "False")
    present = [k for k in DISTRIBUTED if k in status]
    assert not present, (engine, present)
