"""Spans: per-RPC / per-kernel-launch / per-MIX timing counters plus roctx
ranges for rocprofv3 timelines.

The reference has no tracer (timing only in log lines). Every
``span(name)`` updates an in-process counter (count, total, max) that
``get_status`` exports as ``trace.<name>.{count,total_ms,max_us}``; with
``JUBATUS_ROCTX=1`` it also pushes a roctx range, so ``rocprofv3
--marker-trace`` shows RPCs, kernel launches and RCCL MIX phases on the GPU
timeline. GPU work is asynchronous: a kernel span measures the host-side
launch, the GPU time comes from the profiler.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from contextlib import contextmanager

_lock = threading.Lock()
_stats: dict[str, list] = {}     # name -> [count, total_ns, max_ns]
_roctx = None
_roctx_tried = False


def _lib():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("JUBATUS_ROCTX") != "1":
        return None
    for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            break
        except OSError:
            continue
    return _roctx


def record(name: str, ns: int) -> None:
    with _lock:
        s = _stats.get(name)
        if s is None:
            _stats[name] = [1, ns, ns]
        else:
            s[0] += 1
            s[1] += ns
            if ns > s[2]:
                s[2] = ns


@contextmanager
def span(name: str):
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter_ns()
    try:
        yield
    finally:
        record(name, time.perf_counter_ns() - t0)
        if lib is not None:
            lib.roctxRangePop()


def stats(prefix: str = "trace.") -> dict[str, str]:
    with _lock:
        items = sorted(_stats.items())
    out = {}
    for name, (n, tot, mx) in items:
        out[f"{prefix}{name}.count"] = str(n)
        out[f"{prefix}{name}.total_ms"] = f"{tot / 1e6:.3f}"
        out[f"{prefix}{name}.max_us"] = f"{mx / 1e3:.1f}"
    return out


def reset() -> None:
    with _lock:
        _stats.clear()
