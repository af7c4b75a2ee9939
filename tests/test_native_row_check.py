"""The native row-engine servers' configuration check (no GPU needed):
every reference recommender / nearest_neighbor config is served natively
(csrc/server/jb_row_server.hpp), and the ones that need the Python
converter are handed over."""
import json
import os
import subprocess

from helpers import ROOT

NATIVE_BIN = os.path.join(ROOT, "jubatus_amd", "native_bin")


def _check(engine, path):
    out = subprocess.run([os.path.join(NATIVE_BIN, f"juba{engine}"), "--native-check", "-f", path],
                         capture_output=True, text=True, timeout=30)
    return out.stdout.strip()


def test_reference_configs_are_native():
    for engine in ("recommender", "nearest_neighbor"):
        d = os.path.join(ROOT, "config", engine)
        for f in sorted(os.listdir(d)):
            assert _check(engine, os.path.join(d, f)) == "native", f


def test_host_converter_configs_go_to_python(tmp_path):
    base = json.load(open(os.path.join(ROOT, "config", "recommender", "euclid_lsh.json")))
    for conv_extra, why in (({"string_filter_rules": [{"key": "*", "type": "x", "suffix": "_f"}],
                              "string_filter_types": {"x": {"method": "regexp", "pattern": "a"}}},
                             "regexp"),   # (the other filter methods convert natively)
                            ({"string_rules": [{"key": "/re/", "type": "str"}]}, "regex")):
        cfg = dict(base)
        cfg["converter"] = {**base["converter"], **conv_extra}
        p = tmp_path / "c.json"
        p.write_text(json.dumps(cfg))
        out = _check("recommender", str(p))
        assert out.startswith("python:") and why in out, out
    cfg = dict(base, method="no_such_method")
    p = tmp_path / "c.json"
    p.write_text(json.dumps(cfg))
    assert _check("recommender", str(p)).startswith("python:")
