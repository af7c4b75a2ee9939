"""clustering engine: model-level checks (compressors, forgetting, k-means /
GMM recovery of separated blobs, MIX of coresets, pack/unpack) and the server
end to end (reference client_test/clustering_test.cpp API coverage)."""
import json
import random

import pytest

from helpers import start_standalone
from jubatus_amd.client import Clustering as ClusteringClient
from jubatus_amd.client import Datum, WeightedDatum
from jubatus_amd.fv_converter.converter import DatumToFvConverter
from jubatus_amd.models.clustering import Clustering, NotPerformed

CONV = {"num_rules": [{"key": "*", "type": "num"}]}
CENTERS = [(0.0, 0.0), (10.0, 10.0), (-10.0, 10.0)]


def blobs(n, seed=0):
    r = random.Random(seed)
    out = []
    for i in range(n):
        cx, cy = CENTERS[i % 3]
        out.append({"x": cx + r.gauss(0, 0.5), "y": cy + r.gauss(0, 0.5)})
    return out


def make(method="kmeans", **p):
    param = {"k": 3, "compressor_method": "simple", "bucket_size": 60,
             "compressed_bucket_size": 30, "bucket_length": 2, "seed": 1}
    param.update(p)
    return Clustering(method, param, DatumToFvConverter(CONV))


def near(center, tol=1.5):
    # centres come back in feature space: num_values keyed by feature names
    nv = dict(center.num_values)
    return min(abs(nv["x@num"] - cx) + abs(nv["y@num"] - cy) for cx, cy in CENTERS) < tol


@pytest.mark.parametrize("method,comp", [("kmeans", "simple"), ("kmeans", "compressive_kmeans"),
                                         ("gmm", "compressive_gmm"), ("gmm", "simple")])
def test_recovers_blobs(method, comp):
    c = make(method, compressor_method=comp)
    with pytest.raises(NotPerformed):
        c.get_k_center()
    c.push(blobs(59))
    assert c.get_revision() == 0
    c.push(blobs(1, seed=9))
    assert c.get_revision() == 1
    c.push(blobs(120, seed=3))
    assert c.get_revision() == 3
    centers = c.get_k_center()
    assert len(centers) == 3 and all(near(x) for x in centers)
    # total coreset weight tracks the number of points seen
    members = c.get_core_members()
    tot = sum(w for m in members for w, _ in m)
    assert 150 <= tot <= 190
    nc = c.get_nearest_center({"x": 9.5, "y": 10.2})
    assert abs(dict(nc.num_values)["x@num"] - 10.0) < 1.5
    nm = c.get_nearest_members({"x": -9.8, "y": 9.9})
    assert nm and all(dict(d.num_values)["x"] < -5 for _, d in nm)


def test_bucket_merge_and_forgetting():
    c = make(bucket_size=20, compressed_bucket_size=10, bucket_length=2,
             forgetting_factor=1.0, forgetting_threshold=0.5)
    c.push(blobs(100))
    assert len(c.buckets) <= 2
    # exp(-1) decays: weights of old coresets shrink, tiny ones are dropped
    assert all(w >= 0.5 for b in c.buckets for w, _, _ in b)


def test_compressive_weights_conserved():
    c = make(compressor_method="compressive_kmeans", bucket_size=50, compressed_bucket_size=10)
    c.push(blobs(50))
    assert sum(w for w, _, _ in c.buckets[0]) == pytest.approx(50.0)
    assert len(c.buckets[0]) <= 10


def test_mix_and_pack():
    a, b = make(), make()
    a.push(blobs(60, seed=1))
    b.push(blobs(60, seed=2))
    mixed = Clustering.mix_diff(a.get_diff(), b.get_diff())
    a.put_diff(mixed)
    b.put_diff(mixed)
    wa = sum(w for m in a.get_core_members() for w, _ in m)
    assert wa == pytest.approx(120.0)
    obj = a.pack()
    c = make()
    c.unpack(obj)
    assert c.get_revision() == a.get_revision()
    assert sum(w for m in c.get_core_members() for w, _ in m) == pytest.approx(120.0)
    c.clear()
    assert c.get_revision() == 0


def test_bad_parameters():
    with pytest.raises(ValueError):
        Clustering("dbscan", {}, DatumToFvConverter(CONV))
    with pytest.raises(ValueError):
        make(compressor_method="nope")
    with pytest.raises(ValueError):
        make(compressed_bucket_size=100, bucket_size=10)


def test_server(tmp_path):
    cfg = json.dumps({"method": "kmeans", "converter": CONV,
                      "parameter": {"k": 3, "compressor_method": "compressive_kmeans",
                                    "bucket_size": 90, "compressed_bucket_size": 30,
                                    "bicriteria_base_size": 10, "bucket_length": 2,
                                    "forgetting_factor": 0.0, "forgetting_threshold": 0.5,
                                    "seed": 0}})
    h = start_standalone("clustering", cfg, tmp_path)
    try:
        with ClusteringClient("127.0.0.1", h.argv.port, "") as c:
            assert c.push([Datum(p) for p in blobs(30)]) is True
            assert c.get_revision() == 0
            with pytest.raises(Exception):
                c.get_k_center()
            assert c.push([Datum(p) for p in blobs(60, seed=5)]) is True
            assert c.get_revision() == 1
            centers = c.get_k_center()
            assert len(centers) == 3 and all(near(x) for x in centers)
            core = c.get_core_members()
            assert len(core) == 3 and all(isinstance(m, WeightedDatum) for g in core for m in g)
            nc = c.get_nearest_center(Datum({"x": 0.2, "y": -0.1}))
            assert abs(dict(nc.num_values)["x@num"]) < 1.5
            nm = c.get_nearest_members(Datum({"x": 10.0, "y": 10.0}))
            assert nm and all(isinstance(m, WeightedDatum) for m in nm)
            c.save("c")
            assert c.clear() is True and c.get_revision() == 0
            assert c.load("c") is True and c.get_revision() == 1
            assert len(c.get_k_center()) == 3
    finally:
        h.stop()
