"""The host serial trainer (csrc/native/jb_cpu_serial.cpp over
jb_host_linear.hpp): the in-house CPU baseline of bench.py and the native
jubaclassifier's host backend. One thread and the parse pool (nthreads > 1)
must train the same model, equal to the fp32 oracle
(models/linear_oracle.py) sample after sample."""
import random

import msgpack
import numpy as np
import pytest

from jubatus_amd._native import native
from jubatus_amd.fv_converter.converter import DatumToFvConverter
from jubatus_amd.fv_converter.datum import Datum
from jubatus_amd.fv_converter.gpu_path import GpuRuleTable
from jubatus_amd.models import linear_oracle as lo

CONV = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
        "num_rules": [{"key": "*", "type": "num"}], "hash_max_size": 1 << 14}
METHODS = {"perceptron": 0, "PA": 1, "PA1": 2, "PA2": 3, "CW": 4, "AROW": 5, "NHERD": 6}


def _arena(nreq=40, per=25, seed=0, nlabels=5):
    rng = random.Random(seed)
    bodies, samples = [], []
    for _ in range(nreq):
        items = []
        for _ in range(per):
            y = rng.randrange(nlabels)
            d = {f"s{j}": f"v{y * 5 + rng.randrange(4) if rng.random() < 0.6 else rng.randrange(300)}"
                 for j in range(4)}
            d["n"] = (y - 2) * 0.3 + rng.gauss(0, 1)
            items.append((f"L{y}", d))
        samples += items
        bodies.append(msgpack.packb([[l, Datum(d).to_msgpack()] for l, d in items], use_bin_type=False))
    buf = np.frombuffer(b"".join(bodies), np.uint8).copy()
    offs = np.cumsum([0] + [len(b) for b in bodies[:-1]]).astype(np.int64)
    lens = np.asarray([len(b) for b in bodies], np.int64)
    return buf, offs, lens, samples


@pytest.mark.parametrize("method", ["PA1", "AROW", "CW"])
def test_cpu_train_arena_threads_agree_with_oracle(method):
    nat = native()
    conv = DatumToFvConverter(CONV)
    rt = GpuRuleTable(conv)
    H, LC = CONV["hash_max_size"], 8
    hasher = nat.HostFvHasher(rt.srules, rt.n_srules, rt.nrules, rt.n_nrules, rt.blob, H)
    buf, offs, lens, samples = _arena(seed=len(method))
    active = np.zeros(LC, np.uint8)
    active[:5] = 1
    models = []
    for threads in (1, 4):
        table = nat.LabelTable()
        for y in range(5):
            table.get_or_add(f"L{y}")
        W, P = np.zeros((H, LC), np.float32), np.ones((H, LC), np.float32)
        n, upd, _ = nat.cpu_train_arena(hasher, buf.ctypes.data, offs, lens, table, METHODS[method], 0.5, LC,
                                        W.ctypes.data, P.ctypes.data, active, threads)
        assert n == len(samples)
        models.append((W, P, upd))
    assert models[0][2] == models[1][2]
    np.testing.assert_array_equal(models[0][0], models[1][0])
    np.testing.assert_array_equal(models[0][1], models[1][1])
    # the oracle, sample after sample
    Wo, Po = np.zeros((H, LC), np.float32), np.ones((H, LC), np.float32)
    upd = 0
    for lab, d in samples:
        idx, val = conv.hashed(conv.convert(d))
        upd += lo.train_one(Wo, Po if METHODS[method] >= 4 else None, np.asarray(idx, np.int64),
                            np.asarray(val, np.float32), int(lab[1:]), active, METHODS[method], 0.5)
    assert upd == models[0][2]
    scale = float(np.abs(Wo).max())
    np.testing.assert_allclose(models[0][0], Wo, rtol=2e-3, atol=2e-3 * scale)


def test_cpu_train_arena_rejects_malformed():
    nat = native()
    rt = GpuRuleTable(DatumToFvConverter(CONV))
    hasher = nat.HostFvHasher(rt.srules, rt.n_srules, rt.nrules, rt.n_nrules, rt.blob, 1 << 14)
    buf, offs, lens, _ = _arena(nreq=8)
    buf[offs[5]] = 0xc1       # never-used msgpack byte in request 5
    W, P = np.zeros((1 << 14, 8), np.float32), np.ones((1 << 14, 8), np.float32)
    active = np.ones(8, np.uint8)
    for threads in (1, 3):
        with pytest.raises(ValueError):
            nat.cpu_train_arena(hasher, buf.ctypes.data, offs, lens, nat.LabelTable(), 5, 1.0, 8,
                                W.ctypes.data, P.ctypes.data, active, threads)
