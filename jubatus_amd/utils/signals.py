"""Signal handling (reference C12: jubatus/server/common/signals.cpp:98-181).

TERM/INT run the registered termination action once, HUP runs the HUP
action (log reload), SIGPIPE is ignored. The reference blocks the signals in
every thread and runs the actions on a dedicated sigwait thread; here the
interpreter's signal handler only *posts* the action to a dedicated action
thread, so actions never run inside arbitrary interrupted code.
"""
from __future__ import annotations

import queue
import signal
import threading
from typing import Callable

_actions: dict[int, Callable[[], None] | None] = {signal.SIGTERM: None, signal.SIGINT: None,
                                                  signal.SIGHUP: None}
_fired_term = False
_q: "queue.Queue[int]" = queue.Queue()
_thread: threading.Thread | None = None
_lock = threading.Lock()


def _runner() -> None:
    global _fired_term
    while True:
        sig = _q.get()
        if sig < 0:
            return
        if sig in (signal.SIGTERM, signal.SIGINT):
            with _lock:
                if _fired_term:
                    continue
                _fired_term = True
            fn = _actions.get(signal.SIGTERM) or _actions.get(signal.SIGINT)
        else:
            fn = _actions.get(sig)
        if fn is not None:
            try:
                fn()
            except Exception:  # noqa: BLE001
                import logging
                logging.getLogger("jubatus").exception("signal action failed")


def _handler(signum, frame) -> None:
    _q.put(signum)


def prepare_signal_handling() -> None:
    """Must be called from the main thread."""
    global _thread
    with _lock:
        if _thread is None:
            _thread = threading.Thread(target=_runner, name="signal-actions", daemon=True)
            _thread.start()
    signal.signal(signal.SIGPIPE, signal.SIG_IGN)
    for s in (signal.SIGTERM, signal.SIGINT, signal.SIGHUP):
        signal.signal(s, _handler)


def set_action_on_term(fn: Callable[[], None]) -> None:
    _actions[signal.SIGTERM] = fn
    _actions[signal.SIGINT] = fn


def set_action_on_hup(fn: Callable[[], None]) -> None:
    _actions[signal.SIGHUP] = fn


def reset_for_tests() -> None:
    global _fired_term
    _fired_term = False
