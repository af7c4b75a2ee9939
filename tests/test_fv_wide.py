"""Wide-rule native converter (csrc/native/jb_hostfv_wide.hpp) and its GPU
twin (csrc/hip/fv_wide.hip, ops/fv_wide.py) against the Python converter
(fv_converter/converter.py `_convert`): ngram / space splitters, tf / log_tf
sample weights, idf / bm25 global weights with document frequencies updated
datum by datum, num / log num rules and add / mul combinations - identical
feature order, indices and values, and identical document statistics."""
import json
import os
import random

import msgpack
import numpy as np
import pytest

from helpers import ROOT
from jubatus_amd.fv_converter.converter import DatumToFvConverter
from jubatus_amd.fv_converter.datum import Datum
from jubatus_amd.fv_converter.gpu_path import WideRuleTable, gpu_eligible, wide_eligible

CONFIGS = ["recommender/default.json", "weight/default.json",
           "classifier/arow_combinational_feature.json", "anomaly/default.json"]

EXTRA = {
    "string_types": {"tri": {"method": "ngram", "char_num": "3"}},
    "string_rules": [{"key": "t*", "type": "space", "sample_weight": "log_tf", "global_weight": "bm25"},
                     {"key": "*x", "type": "tri", "sample_weight": "tf", "global_weight": "idf"},
                     {"key": "id", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
    "num_rules": [{"key": "n*", "type": "log"}, {"key": "*", "type": "num"}],
    "combination_types": {"pr": {"method": "mul"}},
    "combination_rules": [{"key_left": "id$*", "key_right": "*@num", "type": "pr"},
                          {"key_left": "*", "key_right": "n1@log", "type": "add"}],
    "hash_max_size": 1 << 16,
}


def _conv(name):
    if name == "extra":
        return DatumToFvConverter(EXTRA)
    with open(os.path.join(ROOT, "config", name)) as f:
        return DatumToFvConverter(json.load(f)["converter"])


def datums(n, seed=0):
    r = random.Random(seed)
    words = ["ab", "abc", "日本語", "héllo", "a b", "x", "", "zzzz", "the cat sat", "cat"]
    out = []
    for _ in range(n):
        sv = [(f"t{r.randrange(3)}", " ".join(r.choice(words) for _ in range(r.randrange(1, 4))))
              for _ in range(r.randrange(0, 4))]
        if r.random() < 0.5:
            sv.append(("tx", r.choice(words) * 2))
        if r.random() < 0.2:          # long text: the hashed token-count path
            sv.append(("t9", " ".join(r.choice(words) for _ in range(40))))
        sv.append(("id", f"u{r.randrange(5)}"))
        nv = [(f"n{r.randrange(3)}", r.choice([0.5, 2.0, 10.0, -3.0, 1.0])) for _ in range(r.randrange(0, 3))]
        d = Datum()
        d.string_values, d.num_values = sv, nv
        out.append(d)
    return out


def native_wide(conv):
    from jubatus_amd._native import native
    rt = WideRuleTable(conv)
    h = native().HostFvWide(rt.srules, rt.n_srules, rt.nrules, rt.n_nrules, rt.crules,
                            rt.n_crules, rt.blob, rt.H)
    if h.needs_weights():
        df, diff, counts = conv.weights.arrays()
        h.set_weights(df.ctypes.data, diff.ctypes.data, counts.ctypes.data)
    return h


def run_native(h, ds, update):
    out = []
    for d in ds:
        body = msgpack.packb([d.to_msgpack()], use_bin_type=False)
        cap = 4096
        idx = np.empty(cap, np.int32)
        val = np.empty(cap, np.float32)
        rp = np.zeros(2, np.int64)
        n, slots, err = h.hash([body], idx.ctypes.data, val.ctypes.data, rp.ctypes.data, 1, cap,
                               update)
        assert err == 0 and n == 1
        out.append((idx[:slots].copy(), val[:slots].copy()))
    return out


def run_python(conv, ds, update):
    out = []
    for d in ds:
        fv = conv.convert_and_update_weight(d) if update else conv.convert(d)
        i, v = conv.hashed(fv)
        out.append((np.asarray(i, np.int32), np.asarray(v, np.float32)))
    return out


@pytest.mark.parametrize("name", CONFIGS + ["extra"])
def test_wide_eligible_configs(name):
    conv = _conv(name)
    assert wide_eligible(conv) and gpu_eligible(conv)


@pytest.mark.parametrize("name", CONFIGS + ["extra"])
def test_native_wide_equals_python_converter(name):
    ds = datums(60, seed=sum(map(ord, name)))
    cpy, cnat = _conv(name), _conv(name)
    h = native_wide(cnat)
    for update in (True, False):
        a = run_python(cpy, ds, update)
        b = run_native(h, ds, update)
        for (ia, va), (ib, vb) in zip(a, b):
            np.testing.assert_array_equal(ia, ib)
            np.testing.assert_allclose(va, vb, rtol=1e-6, atol=1e-7)
    if cpy.uses_global_weight:
        assert cpy.weights.doc_count == cnat.weights.doc_count == 60
        assert cpy.weights.total_len == cnat.weights.total_len
        np.testing.assert_array_equal(cpy.weights.df, cnat.weights.df)
        np.testing.assert_array_equal(cpy.weights.diff, cnat.weights.diff)


def test_weight_manager_mix_and_pack_roundtrip():
    a, b = _conv("recommender/default.json"), _conv("recommender/default.json")
    for d in datums(20, 1):
        a.convert_and_update_weight(d)
    for d in datums(30, 2):
        b.convert_and_update_weight(d)
    m = a.weights.mix(a.weights.get_diff(), b.weights.get_diff())
    a.weights.put_diff(m)
    b.weights.put_diff(m)
    assert a.weights.doc_count == b.weights.doc_count == 50
    np.testing.assert_array_equal(a.weights.df, b.weights.df)
    c = _conv("recommender/default.json")
    c.weights.unpack(msgpack.unpackb(msgpack.packb(a.weights.pack()), strict_map_key=False))
    np.testing.assert_array_equal(c.weights.df, a.weights.df)
    assert c.weights.avg_len() == a.weights.avg_len()
    # older name-keyed statistics load into index space
    d = _conv("recommender/default.json")
    d.weights.unpack([4, 10, {"t$ab@bigram#tf/idf": 2}])
    from jubatus_amd.fv_converter.hashing import feature_index
    assert d.weights.df_of(feature_index("t$ab@bigram#tf/idf", d.hash_max_size)) == 2


def _device_convert(conv, ds, update):
    import torch
    from jubatus_amd.ops.fv_wide import WideDevice
    dev = torch.device("cuda", 0)
    wd = getattr(conv, "_test_wide", None)
    if wd is None:
        wd = conv._test_wide = WideDevice(conv, dev)
    blobs = [msgpack.packb(d.to_msgpack(), use_bin_type=False) for d in ds]
    offs = np.zeros(len(blobs), np.int64)
    np.cumsum([len(b) for b in blobs[:-1]], out=offs[1:])
    buf = b"".join(blobs) + b"\0" * 16
    d_buf = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
    d_off = torch.from_numpy(offs).to(dev)
    d_len = torch.tensor([len(b) for b in blobs], dtype=torch.int32, device=dev)
    rp, idx, val, total = wd.convert(d_buf, len(buf) - 16, d_off, d_len, len(ds), update)
    rp, idx, val = rp.cpu().numpy(), idx[:total].cpu().numpy(), val[:total].cpu().numpy()
    assert int(wd.err.item()) == 0
    out = []
    for i in range(len(ds)):
        a, b = rp[i], rp[i + 1]
        keep = idx[a:b] >= 0
        out.append((idx[a:b][keep], val[a:b][keep]))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", CONFIGS + ["extra"])
def test_device_wide_converter_equals_host(name):
    """csrc/hip/fv_wide.hip + ops/fv_wide.py (DF table in HBM, sequential
    semantics inside a batch) == the native host converter, datum by datum,
    for a training batch (statistics updated) and then a query batch"""
    ds = datums(200, seed=sum(map(ord, name)) + 7)
    chost, cdev = _conv(name), _conv(name)
    h = native_wide(chost)
    for update in (True, False):
        a = run_native(h, ds, update)
        b = _device_convert(cdev, ds, update)
        for (ia, va), (ib, vb) in zip(a, b):
            np.testing.assert_array_equal(ia, ib)
            np.testing.assert_allclose(va, vb, rtol=2e-6, atol=1e-7)
    if chost.uses_global_weight:
        assert cdev.weights.doc_count == chost.weights.doc_count
        np.testing.assert_array_equal(cdev.weights.arrays()[0], chost.weights.df)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["classifier/arow_combinational_feature.json", "idf"])
def test_classifier_trains_on_device_wide_converter(name):
    """a classifier whose converter needs the wide rule set converts on the
    device (fv_path gpu-wide) and, trained as one update stream, equals the
    host engine (the reference's per-sample online update order)"""
    import torch
    from jubatus_amd.models.classifier import LinearClassifier
    if name == "idf":
        cfg = {"method": "AROW", "parameter": {"regularization_weight": 1.0},
               "converter": {"string_types": {"bi": {"method": "ngram", "char_num": "2"}},
                             "string_rules": [{"key": "*", "type": "bi", "sample_weight": "tf",
                                               "global_weight": "idf"}],
                             "num_rules": [{"key": "*", "type": "num"}], "hash_max_size": 1 << 16}}
    else:
        with open(os.path.join(ROOT, "config", name)) as f:
            cfg = json.load(f)
    r = random.Random(3)
    data = []
    for _ in range(300):
        y = r.randrange(3)
        data.append((f"L{y}", {"a": f"w{y}{r.randrange(4)}x", "b": f"v{r.randrange(9)}",
                               "x": y + r.gauss(0, 0.3), "z": r.gauss(0, 1)}))
    g = LinearClassifier(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]),
                         device=torch.device("cuda", 0))
    h = LinearClassifier(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]))
    assert g.get_status()["fv_path"] == "gpu-wide"
    for i in range(0, 300, 100):
        g.train(data[i:i + 100])
        h.train(data[i:i + 100])
    G = g.W.cpu().numpy()[:, :g.labels.size()]
    Hm = h.W[:, :h.labels.size()]
    np.testing.assert_allclose(G, Hm, rtol=1e-3, atol=1e-4)
    test = [d for _, d in data[:50]]
    pg = [max(x, key=lambda e: e[1])[0] for x in g.classify(test)]
    ph = [max(x, key=lambda e: e[1])[0] for x in h.classify(test)]
    assert pg == ph
