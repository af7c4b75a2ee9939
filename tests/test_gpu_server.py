"""jubaclassifier on the GPU behind the real RPC transport: concurrent train
RPCs are micro-batched into shared launches (one update stream each), small
classify RPCs take the single-launch path, results match the host oracle
semantics (every sample trained, labels learned)."""
import os
import random
import threading

import pytest

from helpers import ROOT
from jubatus_amd.client import Classifier, Datum
from jubatus_amd.framework.server_helper import ServerHelper
from jubatus_amd.framework.server_util import ServerArgv
from jubatus_amd.server import get_serv

pytestmark = pytest.mark.gpu


@pytest.fixture
def gpu_server(tmp_path):
    cfg = os.path.join(ROOT, "config", "classifier", "arow.json")
    a = ServerArgv.parse(["-p", "9199", "-b", "127.0.0.1", "-f", cfg, "-d", str(tmp_path),
                          "-c", "16", "--gpu", "0"], "classifier")
    a.port = 0
    h = ServerHelper(get_serv("classifier"), a, install_signals=False)
    h.start(block=False)
    yield h
    h.stop()


def _data(rng, n):
    out = []
    for _ in range(n):
        y = rng.randrange(4)
        out.append((f"L{y}", Datum({"w": f"t{y * 10 + rng.randrange(3)}", "x": float(y)})))
    return out


def test_concurrent_train_rpcs_are_batched(gpu_server):
    port = gpu_server.argv.port
    errors = []

    def worker(seed):
        try:
            c = Classifier("127.0.0.1", port, "", timeout=60)
            rng = random.Random(seed)
            for _ in range(20):
                assert c.train(_data(rng, 32)) == 32
            c.close()
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    ts = [threading.Thread(target=worker, args=(s,)) for s in range(16)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    c = Classifier("127.0.0.1", port, "", timeout=60)
    labels = c.get_labels()
    assert sum(labels.values()) == 16 * 20 * 32
    (_, st), = c.get_status().items()
    assert int(st["batching.train.calls"]) == 320
    assert int(st["batching.train.launches"]) <= 320
    rng = random.Random(99)
    test = _data(rng, 64)
    res = c.classify([d for _, d in test])
    acc = sum(max(r, key=lambda e: e.score).label == l for r, (l, _) in zip(res, test)) / len(test)
    assert acc > 0.9, acc
    assert c.classify([]) == []
    c.close()


def test_train_rpcs_take_the_arena_gpu_path_and_fail_alone(gpu_server):
    """train bodies are copied by the transport into a pinned arena slot and
    scanned on the GPU (train_scan.gpu); a malformed request in the same
    batch gets ARGUMENT_ERROR alone while the good ones are trained"""
    import msgpack
    from jubatus_amd.common.mprpc import RpcClient, RpcTypeError
    port = gpu_server.argv.port
    c = Classifier("127.0.0.1", port, "", timeout=60)
    rng = random.Random(5)
    assert c.train(_data(rng, 32)) == 32          # labels become known
    errors, bad_seen = [], []

    def good(seed):
        try:
            cc = Classifier("127.0.0.1", port, "", timeout=60)
            r = random.Random(seed)
            for _ in range(10):
                assert cc.train(_data(r, 64)) == 64
            cc.close()
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def bad():
        with RpcClient("127.0.0.1", port, 60.0) as rc:
            for _ in range(5):
                try:
                    rc.call("train", "", [["L1", [[["only-a-key"]], [], []]]])
                except RpcTypeError:
                    bad_seen.append(1)
    ts = [threading.Thread(target=good, args=(s,)) for s in range(8)] + [threading.Thread(target=bad)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errors, errors
    assert len(bad_seen) == 5
    (_, st), = c.get_status().items()
    assert int(st["train_scan.gpu"]) >= 1
    labels = c.get_labels()
    assert sum(labels.values()) == 32 + 8 * 10 * 64      # the bad requests counted nothing
    c.close()
