"""IDL tooling: parser, generators, and API parity of idl/specs.py with the
reference's service IDLs (jubatus/server/server/*.idl - every method's
argument / return types, routing, request type, aggregator and every message
layout)."""
import glob
import os
import types

import pytest

from helpers import config_path, start_standalone
from jubatus_amd.idl import jdl, jenerator, specs

REF_IDL = "/root/reference/jubatus/server/server"
DEFS = os.path.join(os.path.dirname(jenerator.__file__), "defs")


@pytest.mark.parametrize("engine", sorted(specs.SERVICES))
def test_specs_idl_roundtrip(engine):
    text = jenerator.emit_idl(jenerator.service_from_specs(engine))
    assert jenerator.check(jdl.parse(text), engine) == []
    # the committed defs are current
    with open(os.path.join(DEFS, engine + ".idl")) as f:
        assert f.read() == text


@pytest.mark.skipif(not os.path.isdir(REF_IDL), reason="reference tree not present")
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(REF_IDL, "*.idl"))))
def test_reference_idl_parity(path):
    assert jenerator.check(jdl.parse_file(path)) == []


def test_parser_features_and_errors():
    f = jdl.parse('''
%include "x.hpp"
type alias = list<string>
enum color { 0: red 1: blue }
message m("cpp::type") { 0: map<string, list<int> > a
  1: datum d }
exception oops { 0: string msg }
service s {
  #- does things
  #-   indented
  #@cht(3) #@update #@all_and
  map<string, m> go(0: string id, 1: list<m> xs)
  #@internal #@nolock
  bool hidden()
}''')
    assert f.typedefs == {"alias": "list<string>"} and f.enums["color"] == [(0, "red"), (1, "blue")]
    assert f.messages[0].native == "cpp::type" and f.messages[0].fields[0].type == "map<string,list<int>>"
    assert f.messages[1].exception
    go = f.services[0].methods[0]
    assert (go.routing, go.cht_n, go.lock, go.agg) == ("cht", 3, "update", "all_and")
    assert go.doc == ["does things", "  indented"] and [a.name for a in go.args] == ["id", "xs"]
    with pytest.raises(jdl.IdlError):
        jdl.parse("service s {\n #@random #@bogus\n int f()\n}")
    with pytest.raises(jdl.IdlError):
        jdl.parse("service s {\n #@random\n int f()\n}")          # no request type
    with pytest.raises(jdl.IdlError):
        jdl.parse("message x { 0 string a }")


def test_generated_python_client_talks_to_server(tmp_path):
    src = jenerator.emit_python(jenerator.service_from_specs("classifier"))
    mod = types.ModuleType("gen_classifier")
    import sys
    sys.modules["gen_classifier"] = mod          # dataclasses resolve annotations there
    exec(compile(src, "gen_classifier.py", "exec"), mod.__dict__)
    h = start_standalone("classifier", config_path("classifier/pa.json"), tmp_path)
    try:
        c = mod.ClassifierClient("127.0.0.1", h.argv.port, "")
        from jubatus_amd.client import Datum
        assert c.train([mod.LabeledDatum("pos", Datum({"x": 1.0})),
                        mod.LabeledDatum("neg", Datum({"x": -1.0}))]) == 2
        res = c.classify([Datum({"x": 2.0})])
        assert isinstance(res[0][0], mod.EstimateResult)
        assert max(res[0], key=lambda r: r.score).label == "pos"
        assert c.get_labels() == {"pos": 1, "neg": 1}
        c.close()
    finally:
        h.stop()


@pytest.mark.parametrize("engine", sorted(specs.SERVICES))
def test_generated_sources_compile(engine):
    f = jenerator.service_from_specs(engine)
    compile(jenerator.emit_python(f), f"{engine}_client.py", "exec")
    compile(jenerator.emit_server(f), f"{engine}_serv.py", "exec")
    rst = jenerator.emit_rst(f)
    assert all(f".. mdef:: {m.name}(" in rst for m in specs.SERVICES[engine])
    compile("SERVICES = {\n" + jenerator.emit_spec(f) + "}\n", "spec.py", "exec")


def test_native_proxy_tables_up_to_date():
    """csrc/proxy/jb_proxy_tables.hpp (compiled into the native proxy) is the
    jenerator output of the current specs"""
    from jubatus_amd.idl import jenerator
    with open(jenerator.PROXY_TABLES) as f:
        assert f.read() == jenerator.emit_proxy_tables(), \
            "regenerate: python -m jubatus_amd.idl.jenerator --proxy-tables"
