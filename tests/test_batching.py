"""Request micro-batching (framework/batching.py): concurrent calls merge
into batched calls; results go back to the right caller; a failing request
does not fail the others."""
import threading
import time

import msgpack
import pytest

from jubatus_amd.framework.batching import MicroBatcher, msgpack_array_len


def test_concurrent_calls_are_batched_and_routed():
    seen = []

    def fn(items):
        seen.append(len(items))
        time.sleep(0.01)               # a "launch": later callers queue up meanwhile
        return [x * 10 for x in items]

    b = MicroBatcher(fn)
    out = {}

    def call(i):
        out[i] = b.submit(i)
    ts = [threading.Thread(target=call, args=(i,)) for i in range(64)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert out == {i: i * 10 for i in range(64)}
    assert b.calls == 64 and sum(seen) == 64
    assert b.batches < 64                # at least some calls were merged


def test_failing_item_is_isolated():
    def fn(items):
        if any(x < 0 for x in items):
            raise ValueError("bad item")
        return [x + 1 for x in items]

    b = MicroBatcher(fn)
    res, errs = {}, {}
    gate = threading.Barrier(8)

    def call(i):
        gate.wait()
        try:
            res[i] = b.submit(-1 if i == 3 else i)
        except ValueError as e:
            errs[i] = e
    ts = [threading.Thread(target=call, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert set(errs) == {3}
    assert res == {i: i + 1 for i in range(8) if i != 3}


@pytest.mark.parametrize("n", [0, 5, 15, 16, 300, 70000])
def test_msgpack_array_len(n):
    assert msgpack_array_len(msgpack.packb(list(range(n)))) == n
    assert msgpack_array_len(b"\xa3abc") == -1
