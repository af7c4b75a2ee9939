"""Loader for the in-tree native components.

``native()`` returns the host C++ runtime module (``_jubatus_native``);
``hip_lib()`` returns the ctypes handle of ``libjubatus_hip.so``.

Both are looked up in the package directory only (in-tree build, see
jubatus_amd/build_ext.py). If a library is missing and the sources are
present, it is built on first use. On a machine with a GPU a missing HIP
library is an error - there is no silent fallback to an eager PyTorch path.
"""
from __future__ import annotations

import ctypes
import importlib
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
_lock = threading.Lock()
_native_mod = None
_hip = None


def native():
    global _native_mod
    if _native_mod is not None:
        return _native_mod
    with _lock:
        if _native_mod is None:
            try:
                _native_mod = importlib.import_module("jubatus_amd._jubatus_native")
            except ImportError:
                from . import build_ext

                build_ext.build_native()
                _native_mod = importlib.import_module("jubatus_amd._jubatus_native")
    return _native_mod


def hip_lib_path() -> str:
    # JUBATUS_HIP_LIB: an alternative in-tree build (kernel experiments)
    alt = os.environ.get("JUBATUS_HIP_LIB")
    return os.path.join(_PKG, alt) if alt else os.path.join(_PKG, "libjubatus_hip.so")


def hip_lib() -> ctypes.CDLL:
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            path = hip_lib_path()
            if not os.path.exists(path):
                from . import build_ext

                build_ext.build_hip()
            _hip = ctypes.CDLL(path)
    return _hip
