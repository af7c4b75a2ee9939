"""Observability and fault injection: span counters exported by get_status,
roctx-less operation, deterministic RPC delay / drop / error rules and the
MIX-phase kill rule."""
import time

import pytest

from helpers import config_path, start_standalone
from jubatus_amd.client import Datum, Stat
from jubatus_amd.common.mprpc import RpcClient, RpcTimeoutError
from jubatus_amd.utils import fault, trace


def test_span_counters():
    trace.reset()
    with trace.span("unit.x"):
        time.sleep(0.002)
    with trace.span("unit.x"):
        pass
    st = trace.stats()
    assert st["trace.unit.x.count"] == "2" and float(st["trace.unit.x.total_ms"]) >= 2.0


def test_fault_rule_parsing():
    rs = fault.parse("rpc_delay:method=train,ms=5; rpc_drop:method=*,every=2;mix_kill:phase=allreduce,at=3")
    assert [r.kind for r in rs] == ["rpc_delay", "rpc_drop", "mix_kill"]
    k = rs[2]
    assert [k.matches(phase="allreduce") for _ in range(4)] == [False, False, True, False]
    assert not k.matches(phase="handover")
    with pytest.raises(ValueError):
        fault.parse("explode:now=1")


def test_rpc_faults_and_status_counters(tmp_path):
    h = start_standalone("stat", config_path("stat/stat.json"), tmp_path)
    try:
        with Stat("127.0.0.1", h.argv.port, "") as c:
            c.push("k", 1.0)
            st = list(c.get_status().values())[0]
            assert int(st["trace.rpc.push.count"]) >= 1
            fault.configure("rpc_error:method=sum,after=1;rpc_delay:method=max,ms=60")
            assert c.sum("k") == 1.0            # first call passes
            with pytest.raises(Exception, match="injected fault"):
                c.sum("k")
            t0 = time.time()
            assert c.max("k") == 1.0
            assert time.time() - t0 >= 0.05
            fault.configure("rpc_drop:method=min")
            rc = RpcClient("127.0.0.1", h.argv.port, 0.5)
            with pytest.raises(RpcTimeoutError):
                rc.call("min", "", "k")
            rc.close()
    finally:
        fault.configure("")
        h.stop()
