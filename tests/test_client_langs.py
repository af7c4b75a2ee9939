"""Ruby / Java / Go client generators (jenerator -l ruby|java|go; reference
tools/jenerator/src/{ruby,java,go}.ml, main.ml:45-63).

No Ruby, JDK or Go toolchain exists in this image, so the generated sources
are checked structurally (every public method of every engine, balanced
blocks, wire-order message fields) and pinned to the committed trees;
running them against a server is "parity unpinned"."""
from __future__ import annotations

import re

import pytest

from jubatus_amd.idl import jenerator, specs


def _public(engine):
    return [m for m in jenerator.service_from_specs(engine).services[0].methods
            if m.routing != "internal"]


@pytest.mark.parametrize("engine", specs.ENGINES)
def test_committed_clients_are_current(engine):
    f = jenerator.service_from_specs(engine)
    for lang, path in jenerator.client_paths(engine).items():
        with open(path) as fp:
            assert fp.read() == jenerator.BACKENDS[lang](f), f"{path}: rerun jenerator --clients"


@pytest.mark.parametrize("engine", specs.ENGINES)
def test_ruby_client_shape(engine):
    src = jenerator.emit_ruby(jenerator.service_from_specs(engine))
    for m in _public(engine):
        args = ", ".join(a.name for a in m.args)
        assert f"def {m.name}({args})" in src
        assert f'call("{m.name}"' in src
    opens = len(re.findall(r"^\s*(def|class|module)\b", src, re.M))
    ends = len(re.findall(r"^\s*end\s*$", src, re.M))
    assert opens == ends
    assert src.count("{") == src.count("}")


@pytest.mark.parametrize("engine", specs.ENGINES)
def test_java_client_shape(engine):
    src = jenerator.emit_java(jenerator.service_from_specs(engine))
    cls = jenerator._camel(engine) + "Client"
    assert f"public class {cls} extends ClientBase" in src
    for m in _public(engine):
        assert f"public {jenerator._java_type(m.ret)} {jenerator._java_ident(m.name)}(" in src
        assert f'call("{m.name}", ' in src
    assert src.count("{") == src.count("}")
    assert src.count("(") == src.count(")")
    assert src.count("<") == src.count(">")


@pytest.mark.parametrize("engine", specs.ENGINES)
def test_go_client_shape(engine):
    f = jenerator.service_from_specs(engine)
    src = jenerator.emit_go(f)
    assert src.startswith("// generated")
    assert f"package {engine.replace('_', '')}" in src
    for m in _public(engine):
        assert re.search(rf"func \(c \*\w+Client\) {jenerator._go_ident(m.name)}\(", src)
        assert f'c.Call("{m.name}", &result' in src
    for msg in f.messages:                       # fields in wire order (StructToArray)
        body = re.search(rf"type {jenerator._go_ident(msg.name)} struct {{\n(.*?)\n}}", src, re.S)
        got = [ln.split()[0] for ln in body.group(1).splitlines()]
        assert got == [jenerator._go_ident(fl.name) for fl in msg.fields]
    assert src.count("{") == src.count("}")


def test_type_mapping():
    assert jenerator._go_type("map<string,list<estimate_result>>") == "map[string][]EstimateResult"
    assert jenerator._java_type("map<string,list<ulong>>") == "Map<String, List<Long>>"
    assert jenerator._java_tmpl("list<map<string,double>>") == \
        "Templates.tList(Templates.tMap(Templates.TString, Templates.TDouble))"
    assert jenerator._ruby_conv("list<datum>", set(), "r") == \
        "r.map { |x0| Jubatus::Common::Datum.from_msgpack(x0) }"


def test_cli_lang_choices():
    assert {"ruby", "java", "go"} <= set(jenerator.BACKENDS)
