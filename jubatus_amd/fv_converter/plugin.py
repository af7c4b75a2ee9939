"""fv_converter plug-in loader (``"method": "dynamic"``).

Reference: jubatus/server/fv_converter/so_factory.cpp:41-106 (six extension
points) and dynamic_loader.cpp:44-94 (path search, version logging). A
config type ``{"method": "dynamic", "path": P, "function": F, ...params}``
loads shared object P and calls factory F with every other parameter; the
plug-in ABI is the C one of csrc/plugins/jb_plugin.h (the reference's is
C++-class based). Search order for P: absolute path / path relative to the
working directory, then ``$JUBATUS_PLUGIN_PATH/P``, then the in-tree plug-in
dir ``jubatus_amd/plugins/P``. Each library's ``version()`` is logged once.

Loaded plug-ins are wrapped as the plain callables the converter uses:
string_feature text -> [token], string_filter str -> str, num_filter
float -> float, num_feature (key, x) -> [(name, value)], binary_feature
(key, bytes) -> [(token, weight)], combination_feature (l, r) -> float.
"""
from __future__ import annotations

import ctypes
import os
import threading

from ..utils import logger

log = logger.get_logger("plugin")

PLUGIN_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "plugins")
ABI = 1
KINDS = {"string_feature": 1, "string_filter": 2, "num_feature": 3, "num_filter": 4,
         "binary_feature": 5, "combination_feature": 6}


class PluginError(RuntimeError):
    pass


class _Token(ctypes.Structure):
    _fields_ = [("begin", ctypes.c_int64), ("length", ctypes.c_int64),
                ("value", ctypes.c_void_p), ("value_len", ctypes.c_int64),
                ("score", ctypes.c_double)]


class _Named(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("value", ctypes.c_double)]


_SF = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64,
                       ctypes.POINTER(_Token), ctypes.c_int)
_STF = ctypes.CFUNCTYPE(ctypes.c_int64, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int64,
                        ctypes.c_char_p, ctypes.c_int64)
_NF = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_double,
                       ctypes.POINTER(_Named), ctypes.c_int)
_NFL = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_void_p, ctypes.c_double)
_BF = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p,
                       ctypes.c_int64, ctypes.POINTER(_Named), ctypes.c_int)
_CF = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_void_p, ctypes.c_double, ctypes.c_double)
_DF = ctypes.CFUNCTYPE(None, ctypes.c_void_p)


class _Plugin(ctypes.Structure):
    _fields_ = [("abi", ctypes.c_int), ("kind", ctypes.c_int), ("self", ctypes.c_void_p),
                ("string_feature", _SF), ("string_filter", _STF), ("num_feature", _NF),
                ("num_filter", _NFL), ("binary_feature", _BF), ("combination", _CF),
                ("destroy", _DF)]


def resolve_path(path: str) -> str:
    """dynamic_loader.cpp:44-94 search order"""
    if os.path.isabs(path) or os.path.exists(path):
        if os.path.exists(path):
            return path
        raise PluginError(f"cannot load dynamic library: {path}")
    for base in (os.environ.get("JUBATUS_PLUGIN_PATH", ""), PLUGIN_DIR):
        if base:
            cand = os.path.join(base, path)
            if os.path.exists(cand):
                return cand
    raise PluginError(f"cannot load dynamic library: {path} (searched $JUBATUS_PLUGIN_PATH and "
                      f"{PLUGIN_DIR})")


class _Handle:
    """owns one plug-in instance; calls are serialised (plug-ins keep their
    output buffers in the instance)"""

    def __init__(self, lib, plug_ptr, kind: str):
        self.lib = lib
        self.ptr = plug_ptr
        self.p = plug_ptr.contents
        self.kind = kind
        self.lock = threading.Lock()

    def __del__(self):
        try:
            if self.p.destroy:
                self.p.destroy(self.p.self)
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass

    # callables -----------------------------------------------------------
    def split(self, text: str) -> list[str]:
        raw = text.encode()
        cap = 64
        with self.lock:
            while True:
                buf = (_Token * cap)()
                n = self.p.string_feature(self.p.self, raw, len(raw), buf, cap)
                if n < 0:
                    raise PluginError("string_feature plug-in failed")
                if n <= cap:
                    break
                cap = n
            out = []
            for t in buf[:n]:
                if t.value:
                    tok = ctypes.string_at(t.value, t.value_len)
                else:
                    tok = raw[t.begin:t.begin + t.length]
                out.append(tok.decode(errors="replace"))
            return out

    def filter_string(self, s: str) -> str:
        raw = s.encode()
        cap = max(64, 2 * len(raw))
        with self.lock:
            while True:
                buf = ctypes.create_string_buffer(cap)
                n = self.p.string_filter(self.p.self, raw, len(raw), buf, cap)
                if n < 0:
                    raise PluginError("string_filter plug-in failed")
                if n <= cap:
                    return buf.raw[:n].decode(errors="replace")
                cap = int(n)

    def filter_num(self, x: float) -> float:
        with self.lock:
            return float(self.p.num_filter(self.p.self, float(x)))

    def _named(self, call) -> list[tuple[str, float]]:
        cap = 16
        while True:
            buf = (_Named * cap)()
            n = call(buf, cap)
            if n < 0:
                raise PluginError(f"{self.kind} plug-in failed")
            if n <= cap:
                return [(b.name.decode(errors="replace"), float(b.value)) for b in buf[:n]]
            cap = n

    def num_feature(self, key: str, x: float) -> list[tuple[str, float]]:
        k = key.encode()
        with self.lock:
            return self._named(lambda buf, cap: self.p.num_feature(self.p.self, k, float(x), buf, cap))

    def binary_feature(self, key: str, data: bytes) -> list[tuple[str, float]]:
        k = key.encode()
        with self.lock:
            return self._named(lambda buf, cap: self.p.binary_feature(self.p.self, k, bytes(data),
                                                                     len(data), buf, cap))

    def combine(self, a: float, b: float) -> float:
        with self.lock:
            return float(self.p.combination(self.p.self, float(a), float(b)))


class PluginLoader:
    def __init__(self):
        self._libs: dict[str, ctypes.CDLL] = {}
        self.handles: list[_Handle] = []

    def _lib(self, path: str):
        real = os.path.realpath(resolve_path(path))
        lib = self._libs.get(real)
        if lib is None:
            try:
                lib = ctypes.CDLL(real)
            except OSError as e:
                raise PluginError(f"cannot load dynamic library: {real}: {e}") from e
            try:
                ver = ctypes.CFUNCTYPE(ctypes.c_char_p)(("version", lib))()
                log.info("plugin loaded: %s version: %s", real, ver.decode() if ver else "?")
            except AttributeError:
                log.warning("plugin %s has no version() symbol", real)
            self._libs[real] = lib
        return lib

    def create(self, kind: str, params: dict):
        params = {str(k): str(v) for k, v in (params or {}).items()}
        path = params.pop("path", None)
        fn = params.pop("function", None)
        if not path or not fn:
            raise PluginError(f"dynamic {kind}: 'path' and 'function' are required")
        if kind not in KINDS:
            raise PluginError(f"unknown plug-in kind: {kind}")
        lib = self._lib(path)
        try:
            factory = getattr(lib, fn)
        except AttributeError as e:
            raise PluginError(f"cannot find symbol {fn} in {path}") from e
        factory.restype = ctypes.POINTER(_Plugin)
        factory.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p),
                            ctypes.c_int]
        keys = [k.encode() for k in params]
        vals = [params[k].encode() for k in params]
        ka = (ctypes.c_char_p * max(1, len(keys)))(*keys)
        va = (ctypes.c_char_p * max(1, len(vals)))(*vals)
        ptr = factory(ka, va, len(keys))
        if not ptr:
            raise PluginError(f"{fn} in {path} returned no plug-in")
        p = ptr.contents
        if p.abi != ABI:
            raise PluginError(f"{fn}: plug-in ABI {p.abi}, expected {ABI}")
        if p.kind != KINDS[kind]:
            raise PluginError(f"{fn} is not a {kind} plug-in (kind {p.kind})")
        h = _Handle(lib, ptr, kind)
        self.handles.append(h)
        return {"string_feature": h.split, "string_filter": h.filter_string,
                "num_filter": h.filter_num, "num_feature": h.num_feature,
                "binary_feature": h.binary_feature, "combination_feature": h.combine}[kind]
