"""roctx ranges behind JUBATUS_ROCTX=1 (csrc/native/jb_roctx.hpp, ops/hip.py
_roctx): the marker library loads on demand and the instrumented paths keep
working; off, nothing is loaded. The ranges themselves are read by
rocprofv3 --marker-trace on the GPU (profiles/r6_roctx_marker_trace.md)."""
import os
import subprocess
import sys

from helpers import ROOT, config_path

BIN = os.path.join(ROOT, "jubatus_amd", "native_bin", "jubaclassifier")


def test_python_marker_library_on_demand():
    code = ("import os, sys; sys.path.insert(0, %r); from jubatus_amd.ops import hip; "
            "lib = hip._roctx(); print('on' if lib is not None else 'off')" % ROOT)
    on = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                        env=dict(os.environ, JUBATUS_ROCTX="1"))
    off = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120,
                         env={k: v for k, v in os.environ.items() if k != "JUBATUS_ROCTX"})
    assert off.stdout.strip() == "off", off.stderr
    assert on.stdout.strip() == ("on" if os.path.exists("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1") else "off")


def test_native_server_serves_with_ranges_on(tmp_path):
    """the RPC server's batch / call ranges and the classifier's kernel-group
    ranges wrap the served calls (here the host backend)"""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_native_server import _start, _stream
    p, c = _start(["-f", config_path("classifier/pa.json"), "-d", str(tmp_path)],
                  env_extra={"JUBATUS_ROCTX": "1"})
    try:
        data = _stream(100, seed=1)
        assert c.call("train", "", data) == 100
        assert len(c.call("classify", "", [d for _, d in data[:5]])) == 5
    finally:
        c.close()
        p.terminate()
        p.wait(timeout=30)
