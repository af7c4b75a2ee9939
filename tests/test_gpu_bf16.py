"""bf16 W storage of the linear classifier (csrc/hip/jb_linear.hpp ldw / stw /
addw: bf16 table, fp32 arithmetic, stochastic rounding on store) against the
fp32 host oracle (models/linear_oracle.py), plus an HBM-sized table
(2^26 rows x 64 labels: 8 GiB bf16 W + 16 GiB fp32 P per rank) that trains
and mixes with two ranks on one GPU."""
import json
import os
import random
import socket
import subprocess
import sys

import msgpack
import numpy as np
import pytest

from jubatus_amd.fv_converter.converter import DatumToFvConverter

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONV = {
    "string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
    "num_rules": [{"key": "*", "type": "num"}],
    "hash_max_size": 1 << 16,
}


def _data(n, nlabels=5, seed=0):
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        y = rng.randrange(nlabels)
        d = {f"s{j}": f"v{(y * 7 + rng.randrange(4)) if rng.random() < 0.7 else rng.randrange(500)}"
             for j in range(4)}
        for j in range(3):
            d[f"n{j}"] = (y - 2) * 0.5 + rng.gauss(0, 1)
        out.append((f"L{y}", d))
    return out


def _device():
    import torch
    return torch.device("cuda", 0)


def _top(clf, data):
    return [max(r, key=lambda t: t[1])[0] for r in clf.classify([d for _, d in data])]


@pytest.mark.parametrize("method", ["PA1", "CW", "AROW", "NHERD"])
@pytest.mark.parametrize("mode", ["exact", "atomic"])
def test_bf16_weights_track_fp32_oracle(method, mode, capsys):
    """Requests applied one after another on the fp32 host oracle vs the
    same requests as concurrent streams over a bf16 W table (exact: one
    sequential stream; atomic: lock-free CAS adds). Measured on MI355X
    (exact): PA1 rel W diff 0.047, CW 0.155, decisions agree on >= 99.9 % of
    held-out datums and accuracy matches the fp32 model."""
    from jubatus_amd.fv_converter.datum import Datum
    from jubatus_amd.models.classifier import LinearClassifier

    param = {"regularization_weight": 1.0}
    g = LinearClassifier(method, param, DatumToFvConverter(CONV), device=_device(),
                         concurrent_update=mode, weight_dtype="bf16")
    c = LinearClassifier(method, param, DatumToFvConverter(CONV))
    assert g.W.dtype.itemsize == 2 and g.get_status()["weight_dtype"] == "bf16"
    data = _data(256 * 16, seed=5)
    reqs = [data[i:i + 16] for i in range(0, len(data), 16)]
    for r in reqs[:4]:
        g.train(r)
        c.train(r)
    bodies = [msgpack.packb([[l, Datum(d).to_msgpack()] for l, d in r], use_bin_type=False)
              for r in reqs[4:]]
    assert g.train_requests(bodies) == 16 * (len(reqs) - 4)
    for r in reqs[4:]:
        c.train(r)
    g.synchronize()
    Wg = g.W.float().cpu().numpy()[:, :c.LC]
    rel = float(np.linalg.norm(Wg - c.W) / np.linalg.norm(c.W))
    rel_f = 0.0
    if mode == "atomic":
        # the lock-free streams race in any storage: the fp32 table under the
        # same concurrency is the yardstick of the trajectory divergence
        f = LinearClassifier(method, param, DatumToFvConverter(CONV), device=_device(),
                             concurrent_update=mode)
        for r in reqs[:4]:
            f.train(r)
        f.train_requests(bodies)
        f.synchronize()
        rel_f = float(np.linalg.norm(f.W.float().cpu().numpy()[:, :c.LC] - c.W) / np.linalg.norm(c.W))
    test = _data(2000, seed=6)
    pg, pc = _top(g, test), _top(c, test)
    agree = float(np.mean([a == b for a, b in zip(pg, pc)]))
    acc_g = float(np.mean([p == l for p, (l, _) in zip(pg, test)]))
    acc_c = float(np.mean([p == l for p, (l, _) in zip(pc, test)]))
    with capsys.disabled():
        print(f"\nbf16 {method} {mode}: rel W diff {rel:.4f} (fp32 {mode}: {rel_f:.4f}), "
              f"agreement {agree:.3f}, acc {acc_g:.3f} vs fp32 {acc_c:.3f}")
    # the atomic mode's update order changes run to run (measured: PA1 atomic
    # 0.9715 and 0.959 vs 0.996); the exact mode is deterministic
    assert acc_g >= acc_c - (0.02 if mode == "exact" else 0.05), (acc_g, acc_c)
    assert agree >= (0.97 if mode == "exact" else 0.95), agree
    # the weight distance mixes rounding noise (a bf16 ulp is 2^-8 of the
    # weight, stochastically rounded on every store) with the divergence of
    # the online trajectory it causes (margins differ, so which samples update
    # differs); decisions stay the fp32 model's
    assert rel <= (0.3 if mode == "exact" else max(2.0, 2.0 * rel_f)), (rel, rel_f)
    assert g.train_stats()["trained"] == len(data)


def test_bf16_classify_equals_upcast_table():
    """scores over the bf16 table (batch kernel and the one-launch direct
    path) equal the fp32 dot products with the upcast weights"""
    from jubatus_amd.models.classifier import LinearClassifier

    g = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV),
                         device=_device(), weight_dtype="bf16")
    g.train(_data(600, seed=7))
    g.synchronize()
    W = g.W.float().cpu().numpy()
    test = [d for _, d in _data(300, seed=8)]
    names = g.labels.names()
    for direct in (True, False):
        g.direct = direct
        res = g.classify(test)
        for d, r in zip(test, res):
            idx, val = g.conv.hashed(g.conv.convert(d))
            ref = np.asarray(val, np.float32) @ W[np.asarray(idx, np.int64)]
            got = dict(r)
            for i, n in enumerate(names):
                assert abs(got[n] - ref[i]) <= 1e-4 * (1 + abs(ref[i])), (direct, n, got[n], ref[i])


def test_bf16_model_file_loads_into_fp32_model():
    """pack() writes fp32 rows whatever the storage: a bf16 model loads into
    an fp32 one (and back) with the same decisions"""
    from jubatus_amd.models.classifier import LinearClassifier

    g = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV),
                         device=_device(), weight_dtype="bf16")
    g.train(_data(800, seed=9))
    blob = msgpack.packb(g.pack(), use_bin_type=True)
    f = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV),
                         device=_device())
    f.unpack(msgpack.unpackb(blob, raw=False))
    test = _data(500, seed=10)
    assert _top(f, test) == _top(g, test)
    h = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV),
                         device=_device(), weight_dtype="bf16")
    h.unpack(msgpack.unpackb(msgpack.packb(f.pack(), use_bin_type=True), raw=False))
    assert np.array_equal(h.W.float().cpu().numpy(), g.W.float().cpu().numpy())


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_hbm_sized_bf16_table_trains_and_mixes_two_ranks():
    """2^26 rows x 64 labels AROW (bf16 W 8 GiB + fp32 P 16 GiB per rank),
    two ranks sharing the GPU over gloo: both train their own requests, one
    sparse MIX, then the tables agree on every mixed row"""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "tests", "bf16_mix_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(out) == 2, r.stdout[-2000:]
    for o in out:
        assert o["LC"] == 64 and o["H"] == 1 << 26 and o["w_bytes"] == (1 << 26) * 64 * 2
        assert o["mix"]["mode"] == "sparse" and o["mix"]["world"] == 2 and o["mix"]["rows"] > 0
        assert o["rows_equal"] and o["acc"] > 0.9
    assert out[0]["digest"] == out[1]["digest"]
