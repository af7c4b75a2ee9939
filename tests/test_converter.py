"""Host fv_converter semantics (feature names, weights, filters, matchers)."""
import math

import pytest

from jubatus_amd.fv_converter.converter import ConverterError, DatumToFvConverter, KeyMatcher
from jubatus_amd.fv_converter.datum import Datum
from jubatus_amd.fv_converter.gpu_path import gpu_eligible


def conv(**kw):
    return DatumToFvConverter(kw)


def test_key_matchers():
    assert KeyMatcher("*").match("anything")
    assert KeyMatcher("ab*").match("abc") and not KeyMatcher("ab*").match("xab")
    assert KeyMatcher("*bc").match("abc") and not KeyMatcher("*bc").match("bcx")
    assert KeyMatcher("/^a.c$/").match("abc") and not KeyMatcher("/^a.c$/").match("abcd")
    assert KeyMatcher("abc").match("abc") and not KeyMatcher("abc").match("abcd")


def test_str_and_num_rules():
    c = conv(string_rules=[{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
             num_rules=[{"key": "*", "type": "num"}, {"key": "n*", "type": "log"},
                        {"key": "z", "type": "str"}])
    fv = c.convert(Datum({"name": "taro", "n": 10.0, "z": 3.0}))
    assert ("name$taro@str#bin/bin", 1.0) in fv
    assert ("n@num", 10.0) in fv
    assert ("n@log", pytest.approx(math.log(10.0))) in fv
    assert ("z$3@str", 1.0) in fv


def test_ngram_tf_idf_and_weights():
    c = conv(string_types={"bigram": {"method": "ngram", "char_num": "2"}},
             string_rules=[{"key": "*", "type": "bigram", "sample_weight": "tf", "global_weight": "idf"}])
    c.convert_and_update_weight({"t": "abab"})
    c.convert_and_update_weight({"t": "xy"})
    fv = dict(c.convert({"t": "abab"}))
    # tf(ab)=2, df(ab)=1 of 2 docs
    assert fv["t$ab@bigram#tf/idf"] == pytest.approx(2 * math.log(2.0))
    assert fv["t$ba@bigram#tf/idf"] == pytest.approx(1 * math.log(2.0))


def test_filters_and_combination():
    c = conv(string_filter_types={"detag": {"method": "regexp", "pattern": "<[^>]*>", "replace": ""}},
             string_filter_rules=[{"key": "html", "type": "detag", "suffix": "-detagged"}],
             num_filter_types={"lin": {"method": "linear_normalization", "min": "0", "max": "10"}},
             num_filter_rules=[{"key": "*", "type": "lin", "suffix": "_n"}],
             string_rules=[{"key": "*-detagged", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
             num_rules=[{"key": "*", "type": "num"}],
             combination_rules=[{"key_left": "a@num", "key_right": "b@num", "type": "mul"}])
    fv = dict(c.convert({"html": "<b>hi</b>", "a": 5.0, "b": 20.0}))
    assert fv["html-detagged$hi@str#bin/bin"] == 1.0
    assert fv["a_n@num"] == pytest.approx(0.5) and fv["b_n@num"] == 1.0
    assert fv["a@num&b@num/mul"] == 100.0


def test_errors():
    with pytest.raises(ConverterError):
        conv(string_rules=[{"key": "*", "type": "nope", "sample_weight": "bin", "global_weight": "bin"}])
    with pytest.raises(ConverterError):
        conv(string_rules=[{"key": "*", "type": "str", "sample_weight": "zzz", "global_weight": "bin"}])


def test_gpu_eligibility():
    base = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
            "num_rules": [{"key": "*", "type": "num"}]}
    from jubatus_amd.fv_converter.gpu_path import fast_eligible, wide_eligible
    assert gpu_eligible(DatumToFvConverter(base)) and fast_eligible(DatumToFvConverter(base))
    ng = dict(base, string_types={"u": {"method": "ngram", "char_num": "1"}},
              string_rules=[{"key": "*", "type": "u", "sample_weight": "tf", "global_weight": "idf"}])
    assert not fast_eligible(DatumToFvConverter(ng))
    assert wide_eligible(DatumToFvConverter(ng)) and gpu_eligible(DatumToFvConverter(ng))
    rx = dict(base, string_rules=[{"key": "/x.*/", "type": "str", "sample_weight": "bin",
                                   "global_weight": "bin"}])
    assert not gpu_eligible(DatumToFvConverter(rx))


def test_native_host_hasher_matches_converter():
    """csrc/native/jb_hostfv.hpp (low-latency classify path) == host converter."""
    import random

    import msgpack
    import numpy as np

    from jubatus_amd._native import native
    from jubatus_amd.fv_converter.gpu_path import GpuRuleTable

    conf = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"},
                             {"key": "s1*", "type": "str", "sample_weight": "log_tf",
                              "global_weight": "bin"}],
            "num_rules": [{"key": "*", "type": "num"}, {"key": "*1", "type": "log"}],
            "hash_max_size": 1 << 18}
    conv = DatumToFvConverter(conf)
    rt = GpuRuleTable(conv)
    h = native().HostFvHasher(rt.srules, rt.n_srules, rt.nrules, rt.n_nrules, rt.blob, rt.H)
    rng = random.Random(4)
    data = [{**{f"s{j}": f"v{rng.randrange(50)}" for j in range(3)},
             **{f"n{j}": rng.gauss(0, 5) for j in range(3)}, "big": rng.randrange(1 << 20)}
            for _ in range(20)]
    body = msgpack.packb([Datum(d).to_msgpack() for d in data], use_bin_type=False)
    idx = np.zeros(4096, np.int32)
    val = np.zeros(4096, np.float32)
    rp = np.zeros(64, np.int64)
    n, slots, err = h.hash([body], idx.ctypes.data, val.ctypes.data, rp.ctypes.data, 63, 4096)
    assert (n, err) == (20, 0)
    for s, d in enumerate(data):
        hi, hv = conv.hashed(conv.convert(d))
        gi, gv = idx[rp[s]:rp[s + 1]], val[rp[s]:rp[s + 1]]
        m = gi >= 0
        assert sorted(zip(gi[m].tolist(), np.round(gv[m], 4).tolist())) == \
            sorted(zip(hi, np.round(np.asarray(hv, np.float32), 4).tolist()))
    # capacity: too few slots / samples -> 2 (caller falls back)
    assert h.hash([body], idx.ctypes.data, val.ctypes.data, rp.ctypes.data, 63, 10)[2] == 2
    assert h.hash([body], idx.ctypes.data, val.ctypes.data, rp.ctypes.data, 5, 4096)[2] == 2
    assert h.hash([b"\x93\x01"], idx.ctypes.data, val.ctypes.data, rp.ctypes.data, 5, 4096)[2] == 1
