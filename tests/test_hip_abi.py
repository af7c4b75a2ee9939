"""The ctypes signatures in ops/hip.py match the extern "C" prototypes of
the HIP library sources (parameter counts), so an ABI slip is caught on the
CPU instead of as a TypeError / garbage argument on the GPU box."""
import glob
import os
import re

from jubatus_amd.ops import hip

SRC = os.path.join(os.path.dirname(hip.__file__), "..", "csrc", "hip")


def _prototypes():
    protos = {}
    for f in glob.glob(os.path.join(SRC, "*.hip")):
        text = open(f).read()
        for m in re.finditer(r'extern "C" [\w\s\*]+?\b(jb_\w+)\(([^)]*)\)', text):
            params = [p for p in m.group(2).split(",") if p.strip()]
            protos[m.group(1)] = len(params)
    return protos


def test_ctypes_signatures_match_sources():
    protos = _prototypes()
    assert protos, "no prototypes found"
    for name, sig in hip._SIGS.items():
        assert name in protos, name
        assert len(sig) == protos[name], (name, len(sig), protos[name])
