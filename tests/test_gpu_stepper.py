"""The sequential stepper (csrc/hip/stepper.hip): update-dense exact
training from an LDS row cache. Every case compares the GPU model with the
host oracle (models/linear_oracle.py, fp32 NumPy) trained request after
request - the reference's semantics (classifier_serv.cpp:138-144) - and checks
that no stepper wait timed out."""
import random

import msgpack
import numpy as np
import pytest

from jubatus_amd.fv_converter.converter import DatumToFvConverter

pytestmark = pytest.mark.gpu

CONV = {
    "string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
    "num_rules": [{"key": "*", "type": "num"}],
    "hash_max_size": 1 << 18,
}


def _device():
    import torch
    return torch.device("cuda", 0)


def _noise(n, nlabels, seed, nstr=8, nnum=8, vocab=1 << 30, wide_every=0, wide=0):
    """the bench's worst case: noise string values (every sample brings new
    rows) and shared numeric keys (hot rows), random labels: nearly every
    sample updates. wide_every: every k-th sample gets `wide` more features"""
    rng = random.Random(seed)
    out = []
    for i in range(n):
        y = rng.randrange(nlabels)
        sv = [[f"s{j}", f"t{rng.randrange(vocab)}"] for j in range(nstr)]
        if wide_every and i % wide_every == 0:
            sv += [[f"w{j}", f"x{rng.randrange(vocab)}"] for j in range(wide)]
        nv = [[f"n{j}", rng.gauss(0.0, 1.0)] for j in range(nnum)]
        out.append((f"L{y}", [sv, nv, []]))
    return out


def _train_both(method, data, per_req, nlabels, param=None):
    from jubatus_amd.models.classifier import LinearClassifier
    from jubatus_amd.ops import hip

    param = param or {"regularization_weight": 1.0}
    reqs = [data[i:i + per_req] for i in range(0, len(data), per_req)]
    g = LinearClassifier(method, param, DatumToFvConverter(CONV), device=_device())
    c = LinearClassifier(method, param, DatumToFvConverter(CONV))
    for y in range(nlabels):
        g.set_label(f"L{y}")
        c.set_label(f"L{y}")
    hip.stepper_error()
    g.train_requests([msgpack.packb([[l, d] for l, d in r], use_bin_type=False) for r in reqs])
    for r in reqs:
        c.train(r)
    g.synchronize()
    g.pipe.check_errors()
    assert hip.stepper_error() == 0
    return g, c


def _close(g, c):
    st, sc = g.train_stats(), c.train_stats()
    assert st["trained"] == sc["trained"]
    assert st["updated"] == sc["updated"], (st, sc)
    scale = float(np.abs(c.W).max()) or 1.0
    np.testing.assert_allclose(g.W.cpu().numpy()[:, :c.LC], c.W, rtol=2e-3, atol=2e-3 * scale)
    if c.P is not None:
        np.testing.assert_allclose(g.P.cpu().numpy()[:, :c.LC], c.P, rtol=2e-3, atol=2e-3 * float(c.P.max()))


@pytest.mark.parametrize("method", ["AROW", "PA1", "CW", "NHERD", "perceptron"])
def test_stepper_worst_case_matches_oracle(method):
    """every sample updates: the verified committer hands chunks of the batch
    to the stepper after its dense windows; the row cache streams the fresh
    rows through (evictions with write-back) and keeps the hot numeric rows"""
    data = _noise(24 * 1024, 6, seed=len(method))
    g, c = _train_both(method, data, 128, 6)
    d = g._serial.last_batch()
    assert d["stepper_samples"] > 0.5 * d["end"] and d["stepper_chunks"] >= 1, d
    assert g.train_stats()["updated"] > 0.5 * len(data) or method == "perceptron"
    _close(g, c)


@pytest.mark.parametrize("nlabels", [20, 40])
def test_stepper_label_capacities(nlabels):
    """label capacities 32 and 64 (fewer cache slots, more lanes per row)"""
    data = _noise(6 * 1024, nlabels, seed=nlabels, nstr=6, nnum=4)
    g, c = _train_both("AROW", data, 64, nlabels)
    _close(g, c)


def test_stepper_wide_and_direct_samples():
    """samples of 70 features (several lookup chunks, the wide update path)
    and of 300 features (past kFMax: applied on HBM by the stepper after the
    loader dropped their cached rows) inside an update-dense stream"""
    data = _noise(3 * 1024, 6, seed=5, wide_every=7, wide=62)
    rng = random.Random(9)
    for i in range(0, len(data), 29):
        l, (sv, nv, bv) = data[i]
        data[i] = (l, [sv + [[f"z{j}", f"q{rng.randrange(1 << 30)}"] for j in range(300)], nv, bv])
    g, c = _train_both("AROW", data, 64, 6)
    _close(g, c)


def test_stepper_single_request_and_repeated_rows():
    """one request (a single exact stream goes straight to the stepper), with
    rows repeated inside samples (hash collisions of a tiny table count twice)"""
    from jubatus_amd.models.classifier import LinearClassifier
    from jubatus_amd.ops import hip

    conv = dict(CONV, hash_max_size=64)
    rng = random.Random(3)
    data = [(f"L{rng.randrange(5)}", [[[f"s{j}", f"t{rng.randrange(200)}"] for j in range(10)],
                                      [["n", rng.gauss(0, 1)]], []]) for _ in range(3000)]
    for method in ("AROW", "PA2"):
        g = LinearClassifier(method, {"regularization_weight": 0.5}, DatumToFvConverter(conv), device=_device())
        c = LinearClassifier(method, {"regularization_weight": 0.5}, DatumToFvConverter(conv))
        hip.stepper_error()
        g.train(data)
        c.train(data)
        g.synchronize()
        assert hip.stepper_error() == 0
        _close(g, c)


def _easy(n, nlabels, seed):
    """a learnable stream: the label's own token in every sample (few updates
    once the model has seen each label)"""
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        y = rng.randrange(nlabels)
        sv = [["k", f"label{y}"], ["s", f"t{rng.randrange(50)}"]]
        nv = [["n", 1.0 + rng.random()]]
        out.append((f"L{y}", [sv, nv, []]))
    return out


def test_stepper_chunks_between_sparse_windows():
    """sparse, then update-dense, then sparse again in one batch: the
    committer hands the dense stretch to the stepper chunk by chunk and takes
    the batch back after it - no sequential tail at the end"""
    data = _easy(8192, 6, 1) + _noise(12 * 1024, 6, seed=2) + _easy(24 * 1024, 6, 3)
    g, c = _train_both("AROW", data, 128, 6)
    d = g._serial.last_batch()
    assert d["tail_start"] == d["end"], d
    assert d["stepper_chunks"] >= 1 and d["stepper_samples"] < 0.8 * d["end"], d
    _close(g, c)


def test_stepper_candidate_windows_match_oracle(monkeypatch):
    """JB_VC_CS: verified-committer windows whose candidates the stepper walks
    in kernel C's place (no W / P writes; its updated rows staged for kernel
    D, which verifies the rest of the window and commits)"""
    from jubatus_amd.models.classifier import LinearClassifier
    from jubatus_amd.ops import hip

    monkeypatch.setenv("JB_VC_CS", "16")
    monkeypatch.setenv("JB_VC_CS_PM", "0")   # every window of 16+ candidates
    rng = random.Random(21)
    data = []
    for _ in range(40 * 512):
        y = rng.randrange(6)
        sv = [[f"s{j}", f"t{y * 131 + rng.randrange(16) if rng.random() < 0.6 else rng.randrange(4000)}"]
              for j in range(6)]
        nv = [[f"n{j}", (y - 3) * 0.05 + rng.gauss(0.0, 1.0)] for j in range(4)]
        data.append((f"L{y}", [sv, nv, []]))
    param = {"regularization_weight": 1.0}
    reqs = [data[i:i + 128] for i in range(0, len(data), 128)]
    g = LinearClassifier("AROW", param, DatumToFvConverter(CONV), device=_device())
    c = LinearClassifier("AROW", param, DatumToFvConverter(CONV))
    for y in range(6):
        g.set_label(f"L{y}")
        c.set_label(f"L{y}")
    hip.stepper_error()
    half = len(reqs) // 2
    wins = 0
    for part in (reqs[:half], reqs[half:]):
        g.train_requests([msgpack.packb([[l, d] for l, d in r], use_bin_type=False) for r in part])
        g.synchronize()
        wins += g._serial.last_batch().get("stepper_windows", 0)
    for r in reqs:
        c.train(r)
    g.pipe.check_errors()
    assert hip.stepper_error() == 0
    assert wins > 0
    _close(g, c)
