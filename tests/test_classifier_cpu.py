"""Classifier driver on the host backend (oracle semantics)."""
import random

import numpy as np
import pytest

from jubatus_amd.fv_converter.converter import DatumToFvConverter
from jubatus_amd.models.classifier import ClassifierConfigError, LinearClassifier

CONV = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
        "num_rules": [{"key": "*", "type": "num"}], "hash_max_size": 1 << 14}


def data(n, seed=0, nl=3):
    r = random.Random(seed)
    out = []
    for _ in range(n):
        y = r.randrange(nl)
        out.append((f"c{y}", {"w": f"t{y}{r.randrange(3)}", "x": y + r.random()}))
    return out


@pytest.mark.parametrize("method", ["perceptron", "PA", "PA1", "PA2", "CW", "AROW", "NHERD"])
def test_methods_learn(method):
    c = LinearClassifier(method, {"regularization_weight": 1.0}, DatumToFvConverter(CONV))
    d = data(300)
    assert c.train(d) == 300
    res = c.classify([x for _, x in d[:100]])
    acc = np.mean([max(r, key=lambda t: t[1])[0] == l for r, (l, _) in zip(res, d)])
    assert acc >= 0.9, (method, acc)
    assert sum(c.get_labels().values()) == 300


def test_config_errors():
    with pytest.raises(ClassifierConfigError):
        LinearClassifier("AROW", {}, DatumToFvConverter(CONV))
    with pytest.raises(ClassifierConfigError):
        LinearClassifier("nope", {}, DatumToFvConverter(CONV))
    with pytest.raises(ClassifierConfigError):
        LinearClassifier("AROW", {"regularization_weight": -1}, DatumToFvConverter(CONV))


def test_labels_and_clear():
    c = LinearClassifier("PA", {}, DatumToFvConverter(CONV))
    assert c.set_label("x") and not c.set_label("x")
    assert c.get_labels() == {"x": 0}
    c.train(data(10))
    assert c.delete_label("x") and not c.delete_label("x")
    assert "x" not in c.get_labels()
    c.clear()
    assert c.get_labels() == {}
    assert c.classify([{"w": "a"}]) == [[]]


def test_pack_unpack_roundtrip():
    c = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV))
    d = data(100, seed=2)
    c.train(d)
    blob = c.pack()
    c2 = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV))
    c2.unpack(blob)
    assert c2.get_labels() == c.get_labels()
    np.testing.assert_array_equal(c2.W[:, :3], c.W[:, :3])
    np.testing.assert_array_equal(c2.P[:, :3], c.P[:, :3])


def test_sequential_semantics_order_matters():
    # online learning is order dependent: same data, different order -> different model
    d = data(50, seed=4)
    a = LinearClassifier("PA", {}, DatumToFvConverter(CONV))
    b = LinearClassifier("PA", {}, DatumToFvConverter(CONV))
    a.train(d)
    b.train(list(reversed(d)))
    assert not np.array_equal(a.W, b.W)
