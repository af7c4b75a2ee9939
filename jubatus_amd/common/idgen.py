"""Global id generators (reference C11: global_id_generator_{standalone,zk}.cpp).

Standalone: an atomic counter. Distributed: ``create_id`` on
``<actor>/id_generator`` (the node's data version). Used by anomaly ``add``
and graph ``create_node`` / ``create_edge``.
"""
from __future__ import annotations

import itertools
import threading

from .membership import build_actor_path


class StandaloneIdGenerator:
    def __init__(self, start: int = 0):
        self._lock = threading.Lock()
        self._next = start

    def generate(self) -> int:
        with self._lock:
            v = self._next
            self._next += 1
            return v

    def set_next(self, v: int) -> None:
        with self._lock:
            self._next = v


class CoordinatorIdGenerator:
    def __init__(self, ls, type_: str, name: str):
        self.ls = ls
        self.path = build_actor_path(type_, name) + "/id_generator"
        ls.create(self.path, "")

    def generate(self) -> int:
        return self.ls.create_id(self.path, 0)

    def set_next(self, v: int) -> None:  # ids are cluster-wide; nothing to reset
        pass


def create_id_generator(argv, ls):
    if argv.is_standalone() or ls is None:
        return StandaloneIdGenerator()
    return CoordinatorIdGenerator(ls, argv.type, argv.name)


_counter = itertools.count()
