"""Deterministic fault injection (the reference has none besides
a test-only non-responding socket; the new framework adds a hook).

``JUBATUS_FAULT`` holds ``;``-separated rules ``kind:key=value,...``:

  rpc_delay:method=train,ms=200          sleep before serving the method
  rpc_drop:method=classify,every=2       serve no reply (client times out)
  rpc_error:method=*,after=3             fail the 4th and later calls
  mix_kill:phase=allreduce,at=2          exit the process at the 2nd MIX
                                         reaching that phase (rank failure)
  mix_hang:phase=allreduce,at=1,ms=8000  stall that MIX phase (a rank that
                                         stops answering collectives)

``method`` / ``phase`` accept ``*``; ``every=N`` fires on every N-th match,
``after=N`` on matches beyond the first N, ``at=N`` on exactly the N-th.
Counting is per process and deterministic (no randomness).
"""
from __future__ import annotations

import os
import threading
import time

from . import logger

log = logger.get_logger("fault")


class InjectedFault(RuntimeError):
    pass


class _Rule:
    def __init__(self, kind: str, params: dict[str, str]):
        self.kind = kind
        self.p = params
        self.hits = 0

    def matches(self, **ctx) -> bool:
        for k in ("method", "phase"):
            want = self.p.get(k)
            if want is not None and want != "*" and ctx.get(k) != want:
                return False
        self.hits += 1
        n = self.hits
        if "at" in self.p:
            return n == int(self.p["at"])
        if "after" in self.p:
            return n > int(self.p["after"])
        if "every" in self.p:
            return n % int(self.p["every"]) == 0
        return True


def parse(spec: str) -> list[_Rule]:
    rules = []
    for part in filter(None, (x.strip() for x in spec.split(";"))):
        kind, _, rest = part.partition(":")
        params = {}
        for kv in filter(None, rest.split(",")):
            k, _, v = kv.partition("=")
            params[k.strip()] = v.strip()
        if kind not in ("rpc_delay", "rpc_drop", "rpc_error", "mix_kill", "mix_hang"):
            raise ValueError(f"unknown fault kind: {kind}")
        rules.append(_Rule(kind, params))
    return rules


_lock = threading.Lock()
_rules: list[_Rule] | None = None


def rules() -> list[_Rule]:
    global _rules
    if _rules is None:
        _rules = parse(os.environ.get("JUBATUS_FAULT", ""))
    return _rules


def configure(spec: str) -> None:
    """replace the active rules (tests / operators)"""
    global _rules
    with _lock:
        _rules = parse(spec)


def on_rpc(method: str) -> str | None:
    """-> None (serve normally) | "drop" (send no reply); may sleep or raise"""
    rs = rules()
    if not rs:
        return None
    action = None
    with _lock:
        fired = [r for r in rs if r.kind.startswith("rpc_") and r.matches(method=method)]
    for r in fired:
        if r.kind == "rpc_delay":
            time.sleep(float(r.p.get("ms", "100")) / 1e3)
        elif r.kind == "rpc_drop":
            log.warning("fault injection: dropping %s", method)
            action = "drop"
        elif r.kind == "rpc_error":
            raise InjectedFault(f"injected fault in {method}")
    return action


def on_mix(phase: str) -> None:
    rs = rules()
    if not rs:
        return
    with _lock:
        fired = [r for r in rs if r.kind in ("mix_kill", "mix_hang") and r.matches(phase=phase)]
    for r in fired:
        if r.kind == "mix_hang":
            log.critical("fault injection: stalling MIX phase %s", phase)
            time.sleep(float(r.p.get("ms", "5000")) / 1e3)
    if any(r.kind == "mix_kill" for r in fired):
        log.critical("fault injection: killing this rank at MIX phase %s", phase)
        os._exit(17)
