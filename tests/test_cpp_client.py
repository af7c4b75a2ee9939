"""Header-only C++ client library (reference C35, jubatus/client/*.hpp):
generated per-engine headers compile and talk to live servers."""
import os
import shutil
import subprocess

import pytest

from helpers import config_path, start_standalone
from jubatus_amd.idl import jenerator, specs

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "jubatus_amd", "client_cpp", "include")


@pytest.mark.parametrize("engine", sorted(specs.SERVICES))
def test_generated_headers_current(engine):
    with open(os.path.join(INC, "jubatus_amd", f"{engine}_client.hpp")) as f:
        assert f.read() == jenerator.emit_cpp(jenerator.service_from_specs(engine))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no C++ compiler")
def test_cpp_client_end_to_end(tmp_path):
    exe = tmp_path / "client_test"
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", f"-I{INC}",
                        os.path.join(ROOT, "tests", "cpp", "client_test.cpp"), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    c = start_standalone("classifier", config_path("classifier/arow.json"), tmp_path)
    s = start_standalone("stat", config_path("stat/stat.json"), tmp_path)
    try:
        r = subprocess.run([str(exe), str(c.argv.port), str(s.argv.port)], capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, r.stdout + r.stderr
        assert "cpp client ok" in r.stdout
    finally:
        c.stop()
        s.stop()
