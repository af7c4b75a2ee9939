"""Request micro-batching: concurrent RPCs of one method become one launch.

Reference: the request-level parallelism of the servers - ``threadnum``
RPC worker threads (server_util.cpp:155-156) calling into an internally
thread-safe driver (classifier "giant lock" removal, ChangeLog.rst:152).
On a GPU the unit of work is a kernel launch, so the worker threads hand
their request bodies to a leader that submits everything queued at that
moment as ONE batch (one update stream per train request, one fused
classify launch for all queued datums), then hands the per-request results
back. Leader/follower, no extra thread: the first caller leads; a leader
whose own request is answered passes leadership on, so no caller waits
behind an unbounded stream of others.
"""
from __future__ import annotations

import threading
from typing import Any, Callable, Sequence


class MicroBatcher:
    def __init__(self, fn: Callable[[Sequence[Any]], Sequence[Any]], max_items: int = 4096):
        self.fn = fn
        self.max_items = int(max_items)
        self._cv = threading.Condition()
        self._queue: list[list] = []
        self._leader = False
        self.calls = 0
        self.batches = 0

    def submit(self, item: Any) -> Any:
        slot = [item, None, None, False]          # item, result, error, done
        with self._cv:
            self._queue.append(slot)
            self.calls += 1
            while self._leader and not slot[3]:
                self._cv.wait()
            if slot[3]:
                return self._result(slot)
            self._leader = True
        try:
            while not slot[3]:
                with self._cv:
                    batch = self._queue[:self.max_items]
                    del self._queue[:len(batch)]
                if not batch:
                    break
                self._run(batch)
        finally:
            with self._cv:
                self._leader = False
                self._cv.notify_all()
        return self._result(slot)

    def _run(self, batch: list[list]) -> None:
        items = [s[0] for s in batch]
        try:
            res = list(self.fn(items))
            if len(res) != len(items):
                raise RuntimeError("batched call returned a wrong number of results")
            for s, r in zip(batch, res):
                s[1] = r
        except Exception:  # noqa: BLE001 - isolate the failing request(s)
            if len(batch) == 1:
                import sys
                batch[0][2] = sys.exc_info()[1]
            else:
                for s in batch:
                    try:
                        s[1] = self.fn([s[0]])[0]
                    except Exception as e:  # noqa: BLE001
                        s[2] = e
        with self._cv:
            for s in batch:
                s[3] = True
            self.batches += 1
            self._cv.notify_all()

    @staticmethod
    def _result(slot: list) -> Any:
        if slot[2] is not None:
            raise slot[2]
        return slot[1]


def msgpack_array_len(body) -> int:
    """element count of a msgpack array at the head of ``body`` (-1: not an array)"""
    mv = memoryview(body).cast("B")
    if not len(mv):
        return -1
    t = mv[0]
    if 0x90 <= t <= 0x9F:
        return t & 0x0F
    if t == 0xDC and len(mv) >= 3:
        return (mv[1] << 8) | mv[2]
    if t == 0xDD and len(mv) >= 5:
        return (mv[1] << 24) | (mv[2] << 16) | (mv[3] << 8) | mv[4]
    return -1
