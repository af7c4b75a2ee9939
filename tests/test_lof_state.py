"""Incremental LOF state (models/lof_state.py, csrc/hip/lof.hip) vs a
brute-force LOF recomputed from scratch (Breunig et al. 2000; the semantics
of jubatus_core's lof_storage behind anomaly_serv.cpp:157-244).

With reverse_nearest_neighbor_num >= the number of rows every insert reaches
every row, so the incremental state must equal the from-scratch LOF exactly;
updates (a row moves) and removals invalidate and recompute lists on demand.
The GPU variant replays the same operations on DeviceLofState and must agree
with the host state."""
import math
import random

import numpy as np
import pytest

from jubatus_amd.fv_converter.converter import DatumToFvConverter

CONV = {"num_rules": [{"key": "*", "type": "num"}], "hash_max_size": 1 << 16}


def brute_lof(X: dict, q: np.ndarray, k: int, exclude=None, ignore_same=False) -> float:
    """LOF of point q against the stored points X {rid: vec} (q itself
    excluded when it is stored under ``exclude``)"""
    ids = sorted(X)
    slot = {r: i for i, r in enumerate(ids)}

    def knn(v, skip):
        ds = sorted((float(np.float32(np.linalg.norm(X[r] - v))), slot[r]) for r in ids if r != skip)
        return ds[:k]

    def kth(nb):
        d = [x for x, _ in nb]
        if ignore_same:
            d = [x for x in d if x > 0] or [0.0]
        return d[-1] if d else 0.0

    kd = {r: kth(knn(X[r], r)) for r in ids}

    def lrd(nb):
        if not nb:
            return 0.0
        m = sum(max(kd[ids[s]], d) for d, s in nb) / len(nb)
        return math.inf if m <= 0 else 1.0 / m

    nb = knn(q, exclude)
    if not nb:
        return 1.0
    lp = lrd(nb)
    lo = [lrd(knn(X[ids[s]], ids[s])) for _, s in nb]
    mean_lo = math.inf if any(math.isinf(x) for x in lo) else sum(lo) / len(lo)
    if math.isinf(lp):
        return 1.0 if math.isinf(mean_lo) else 0.0
    if lp == 0.0 or math.isinf(mean_lo):
        return math.inf
    return mean_lo / lp


def _lof(device=None, k=4, rnn=1000, method="inverted_index_euclid", ignore=False):
    from jubatus_amd.models.anomaly import LOF
    p = {"method": method, "nearest_neighbor_num": k, "reverse_nearest_neighbor_num": rnn,
         "ignore_kth_same_point": ignore, "parameter": {}}
    return LOF("lof", p, DatumToFvConverter(CONV), device)


def _vec(d):
    return np.asarray([d["x"], d["y"], d["z"]], np.float64)


def _ops(seed, n=60):
    r = random.Random(seed)
    ops = []
    for i in range(n):
        ops.append(("add", str(i), {"x": r.gauss(0, 1), "y": r.gauss(0, 1), "z": r.gauss(0, 1)}))
        if i > 10 and i % 7 == 0:
            ops.append(("overwrite", str(r.randrange(i)), {"x": r.gauss(0, 2), "y": r.gauss(0, 2),
                                                           "z": r.gauss(0, 2)}))
        if i > 10 and i % 11 == 0:
            ops.append(("remove", str(r.randrange(i)), None))
        if i % 5 == 0:
            ops.append(("score", None, {"x": r.gauss(0, 3), "y": r.gauss(0, 3), "z": r.gauss(0, 3)}))
    return ops


def _run(lof, ops, check=None):
    X = {}
    out = []
    for kind, rid, d in ops:
        if kind in ("add", "overwrite"):
            X[rid] = _vec(d)
            s = lof.add(rid, d) if kind == "add" else lof.overwrite(rid, d)
            out.append(s)
            if check:
                check(s, brute_lof(X, X[rid], lof.k, exclude=rid, ignore_same=lof.ignore_kth_same))
        elif kind == "remove":
            if rid in X:
                del X[rid]
            lof.clear_row(rid)
        else:
            s = lof.calc_score(d)
            out.append(s)
            if check:
                check(s, brute_lof(X, _vec(d), lof.k, ignore_same=lof.ignore_kth_same))
    return out


def _close(a, b):
    if math.isinf(b):
        assert math.isinf(a), (a, b)
    else:
        assert a == pytest.approx(b, rel=1e-4, abs=1e-5)


@pytest.mark.parametrize("ignore", [False, True])
def test_incremental_lof_equals_brute_force(ignore):
    lof = _lof(ignore=ignore)
    _run(lof, _ops(1), check=_close)


def test_duplicates_and_bulk_loaded_rows():
    """zero distances (duplicate points) and rows loaded without lists
    (set_rows / MIX): lists are built on demand and scores stay exact"""
    lof = _lof(k=3)
    r = random.Random(3)
    pts = [{"x": float(r.randrange(4)), "y": float(r.randrange(3)), "z": 0.0} for _ in range(40)]
    lof.set_rows([(str(i), p) for i, p in enumerate(pts)])
    X = {str(i): _vec(p) for i, p in enumerate(pts)}
    q = {"x": 1.5, "y": 0.5, "z": 0.2}
    _close(lof.calc_score(q), brute_lof(X, _vec(q), 3))
    X["new"] = _vec(q)
    _close(lof.add("new", q), brute_lof(X, X["new"], 3, exclude="new"))


def test_bounded_rnn_marks_only_neighbourhood():
    """rnn < n: an insert touches only its rnn-nearest rows (the reference's
    update scope); the scores stay finite and ranked"""
    lof = _lof(k=5, rnn=10)
    r = random.Random(5)
    for i in range(200):
        lof.add(str(i), {"x": r.gauss(0, 1), "y": r.gauss(0, 1), "z": r.gauss(0, 1)})
    far = lof.calc_score({"x": 9.0, "y": 9.0, "z": 9.0})
    near = lof.calc_score({"x": 0.0, "y": 0.1, "z": 0.0})
    assert far > 2.0 > near


@pytest.mark.gpu
@pytest.mark.parametrize("method", ["inverted_index_euclid", "euclid_lsh"])
def test_device_lof_state_matches_host(method):
    import torch
    from jubatus_amd.models.lof_state import DeviceLofState
    dev = torch.device("cuda", 0)
    g = _lof(dev, method=method, rnn=12)
    c = _lof(None, method=method, rnn=12)
    if method == "euclid_lsh":
        c.parameter = g.parameter
    ops = _ops(7, n=120)
    sg = _run(g, ops)
    assert isinstance(g._st, DeviceLofState)
    if method == "inverted_index_euclid":
        sc = _run(c, ops)
        for a, b in zip(sg, sc):
            _close(a, b)
        # the device state itself equals the host state
        n = g.rows.nslots
        ok = g._st.ok[:n].cpu().numpy().astype(bool)
        assert (ok == c._st.ok[:n].astype(bool)).all()
        np.testing.assert_array_equal(g._st.nb_slot[:n].cpu().numpy()[ok], c._st.nb_slot[:n][ok])
        np.testing.assert_allclose(g._st.kdist[:n].cpu().numpy()[ok], c._st.kdist[:n][ok],
                                   rtol=1e-5, atol=1e-6)
    else:
        # LSH distances are hash-approximate: exactness is covered above,
        # here the device path must run clean and rank outliers
        far = g.calc_score({"x": 30.0, "y": -30.0, "z": 30.0})
        near = g.calc_score({"x": 0.0, "y": 0.0, "z": 0.0})
        assert all(math.isfinite(s) or s == math.inf for s in sg)
        assert far > near


@pytest.mark.gpu
def test_device_lof_exact_with_full_rnn():
    import torch
    g = _lof(torch.device("cuda", 0), k=4, rnn=127)
    _run(g, _ops(11, n=80), check=_close)


def test_device_bindings_present():
    """the device state's kernel wrappers exist (checked without a GPU)"""
    from jubatus_amd.ops import hip
    for name in ("lof_add", "lof_mark", "lof_set_lists", "lof_score", "pool_scan",
                 "pool_append"):
        assert callable(getattr(hip, name)), name
    for name in ("jb_lof_add", "jb_lof_mark", "jb_lof_set_lists", "jb_lof_score",
                 "jb_pool_scan", "jb_pool_append"):
        assert name in hip._SIGS, name
