"""fv_converter dynamic plug-ins through the C ABI (reference
server/fv_converter/{dynamic_loader,so_factory}_test.cpp strategy: real
sample plug-ins built by the same build, every extension point, path search
and error paths)."""
import os

import pytest

from jubatus_amd.fv_converter.converter import DatumToFvConverter
from jubatus_amd.fv_converter.datum import Datum
from jubatus_amd.fv_converter.plugin import PLUGIN_DIR, PluginError, PluginLoader, resolve_path

LIB = "libjubatus_sample_plugins.so"


@pytest.fixture(scope="module", autouse=True)
def built():
    from jubatus_amd import build_ext
    build_ext.build_plugins()


def dyn(fn, **kw):
    return {"method": "dynamic", "path": LIB, "function": fn, **kw}


def test_all_extension_points():
    conf = {
        "string_filter_types": {"up": dyn("create_upper_filter")},
        "string_filter_rules": [{"key": "t", "type": "up", "suffix": "-up"}],
        "num_filter_types": {"aff": dyn("create_affine_filter", scale="2", shift="1")},
        "num_filter_rules": [{"key": "x", "type": "aff", "suffix": "-aff"}],
        "string_types": {"comma": dyn("create_splitter", delimiter=",", min_length="2")},
        "string_rules": [{"key": "t*", "type": "comma", "sample_weight": "tf", "global_weight": "bin"}],
        "num_types": {"bk": dyn("create_bucket_feature", width="10")},
        "num_rules": [{"key": "x*", "type": "bk"}],
        "binary_types": {"hist": dyn("create_byte_histogram")},
        "binary_rules": [{"key": "*", "type": "hist"}],
        "combination_types": {"mx": dyn("create_max_combination")},
        "combination_rules": [{"key_left": "x@raw", "key_right": "x-aff@raw", "type": "mx"}],
    }
    conv = DatumToFvConverter(conf)
    d = Datum({"t": "ab,c,ab,de", "x": 25.0})
    d.binary_values.append(("bin", b"\x01\x01\x02"))
    fv = dict(conv.convert(d))
    assert fv["t$ab@comma#tf/bin"] == 2.0 and fv["t$de@comma#tf/bin"] == 1.0
    assert "t$c@comma#tf/bin" not in fv                         # min_length 2
    assert fv["t-up$AB@comma#tf/bin"] == 2.0                     # string filter + splitter
    assert fv["x@bucket2"] == 1.0 and fv["x@raw"] == 25.0
    assert fv["x-aff@bucket5"] == 1.0 and fv["x-aff@raw"] == 51.0  # 25 * 2 + 1
    assert fv["bin$b1@hist"] == 2.0 and fv["bin$b2@hist"] == 1.0
    assert fv["x@raw&x-aff@raw/mx"] == 51.0


def test_path_search(monkeypatch, tmp_path):
    assert resolve_path(LIB) == os.path.join(PLUGIN_DIR, LIB)
    assert resolve_path(os.path.join(PLUGIN_DIR, LIB)) == os.path.join(PLUGIN_DIR, LIB)
    os.symlink(os.path.join(PLUGIN_DIR, LIB), tmp_path / "mine.so")
    monkeypatch.setenv("JUBATUS_PLUGIN_PATH", str(tmp_path))
    assert resolve_path("mine.so") == str(tmp_path / "mine.so")
    with pytest.raises(PluginError):
        resolve_path("nope.so")


def test_errors():
    ld = PluginLoader()
    with pytest.raises(PluginError):
        ld.create("string_feature", {"path": LIB})                       # no function
    with pytest.raises(PluginError):
        ld.create("string_feature", {"path": LIB, "function": "missing"})
    with pytest.raises(PluginError):
        ld.create("num_filter", {"path": LIB, "function": "create_splitter"})  # wrong kind
    with pytest.raises(PluginError):
        ld.create("string_feature", {"path": "/nonexistent/x.so", "function": "f"})


def test_gpu_path_falls_back_for_plugins():
    from jubatus_amd.fv_converter.gpu_path import gpu_eligible
    conv = DatumToFvConverter({"string_types": {"c": dyn("create_splitter")},
                               "string_rules": [{"key": "*", "type": "c"}]})
    assert not gpu_eligible(conv)


def test_ux_splitter_longest_prefix(tmp_path):
    d = tmp_path / "dict.txt"
    d.write_text("tokyo\ntokyo tower\nto\nkyoto\n\n")
    conv = DatumToFvConverter({
        "string_types": {"ux": {"method": "dynamic", "path": "libjubatus_ux_splitter.so",
                                "function": "create", "dict_path": str(d)}},
        "string_rules": [{"key": "*", "type": "ux", "sample_weight": "tf", "global_weight": "bin"}]})
    fv = dict(conv.convert(Datum({"t": "tokyo towerxkyoto to tokyo"})))
    # longest match wins ("tokyo tower" over "tokyo"); unmatched bytes are skipped
    assert fv == {"t$tokyo tower@ux#tf/bin": 1.0, "t$kyoto@ux#tf/bin": 1.0,
                  "t$to@ux#tf/bin": 1.0, "t$tokyo@ux#tf/bin": 1.0}
    with pytest.raises(PluginError):
        PluginLoader().create("string_feature", {"path": "libjubatus_ux_splitter.so", "function": "create"})


@pytest.fixture(scope="module")
def fake_mecab(tmp_path_factory):
    """a test double of libmecab (tests/fixtures/fake_mecab.cpp): MeCab is not
    installed here, so parity with real MeCab dictionaries is unpinned"""
    import subprocess
    out = tmp_path_factory.mktemp("mecab") / "libfakemecab.so"
    src = os.path.join(os.path.dirname(__file__), "fixtures", "fake_mecab.cpp")
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-o", str(out), src], check=True)
    return str(out)


def _mecab_conv(lib, **params):
    p = {"method": "dynamic", "path": "libjubatus_mecab_splitter.so", "function": "create",
         "libmecab": lib, **params}
    return DatumToFvConverter({"string_types": {"mecab": p},
                               "string_rules": [{"key": "*", "type": "mecab", "sample_weight": "tf",
                                                 "global_weight": "bin"}]})


def test_mecab_splitter_surface_base_ngram_filters(fake_mecab):
    text = "Tokyo is  running fast !"
    fv = dict(_mecab_conv(fake_mecab).convert(Datum({"t": text})))
    assert fv == {f"t${w}@mecab#tf/bin": 1.0 for w in ("Tokyo", "is", "running", "fast", "!")}
    # base form (7th CSV field; the surface where it is "*"), bigrams
    fv = dict(_mecab_conv(fake_mecab, base="true", ngram="2").convert(Datum({"t": text})))
    assert fv == {f"t${w}@mecab#tf/bin": 1.0 for w in ("tokyo,is", "is,runn", "runn,fast", "fast,!")}
    # include nouns and verbs, exclude a feature by regex
    conv = _mecab_conv(fake_mecab, include_features="名詞*|動詞*", exclude_features="/,fast$/")
    fv = dict(conv.convert(Datum({"t": text})))
    assert fv == {f"t${w}@mecab#tf/bin": 1.0 for w in ("Tokyo", "is", "running")}
    # fewer words than n: no feature
    assert dict(_mecab_conv(fake_mecab, ngram="9").convert(Datum({"t": text}))) == {}


def test_mecab_splitter_token_spans(fake_mecab):
    from jubatus_amd.fv_converter.plugin import PluginLoader
    split = PluginLoader().create("string_feature", {
        "path": "libjubatus_mecab_splitter.so", "function": "create", "libmecab": fake_mecab,
        "ngram": "2"})
    assert split("a  bb ccc") == ["a,bb", "bb,ccc"]


def test_mecab_splitter_errors(fake_mecab):
    from jubatus_amd.fv_converter.plugin import PluginLoader
    base = {"path": "libjubatus_mecab_splitter.so", "function": "create"}
    for bad in ({"ngram": "0", "libmecab": fake_mecab}, {"base": "yes", "libmecab": fake_mecab},
                {"include_features": "", "libmecab": fake_mecab},
                {"arg": "--fail", "libmecab": fake_mecab},        # tagger creation fails
                {"libmecab": "/nonexistent/libmecab.so.2"}):      # MeCab not installed
        with pytest.raises(PluginError):
            PluginLoader().create("string_feature", {**base, **bad})
