"""Transport framing (csrc/native/jb_rpc.cpp): the speculative multi-walk
framer must find exactly the message ends of the sequential walk, on
streams delivered in two reads, with payloads full of bytes that look like
msgpack headers (0xc1, 0xdd, ...) and on the train requests of the bench."""
from __future__ import annotations

import random

import msgpack
import pytest

from jubatus_amd._native import native


def _obj(rng: random.Random, depth: int = 0):
    k = rng.random()
    if depth > 3 or k < 0.35:
        c = rng.randrange(9)
        if c == 0:
            return rng.randrange(-2**63, 2**63)
        if c == 1:
            return rng.randrange(-40, 200)
        if c == 2:
            return rng.random() * 1e6
        if c == 3:
            return None if rng.random() < 0.5 else rng.random() < 0.5
        if c == 4:      # binary payload: any byte, long or short
            return rng.randbytes(rng.choice((1, 7, 40, 300, 3000, 70000 if depth == 0 else 5)))
        if c == 5:
            return msgpack.ExtType(rng.randrange(100), rng.randbytes(rng.choice((1, 2, 4, 8, 16, 9))))
        return "".join(chr(rng.randrange(32, 0x2FF)) for _ in range(rng.choice((0, 3, 31, 32, 300))))
    width = (0, 1, 2, 15, 16, 40) if depth < 2 else (0, 1, 2, 3)
    if k < 0.7:
        return [_obj(rng, depth + 1) for _ in range(rng.choice(width))]
    return {str(i): _obj(rng, depth + 1) for i in range(rng.choice(width))}


def _stream(seed: int, nmsg: int) -> tuple[bytes, list[int]]:
    rng = random.Random(seed)
    out, ends = b"", []
    for _ in range(nmsg):
        out += msgpack.packb([0, rng.randrange(2**32), "train", ["", _obj(rng)]], use_bin_type=True)
        ends.append(len(out))
    return out, ends


def _frame(buf: bytes, cut: int, spec: bool):
    ends, rc, pos, rem = native().frame_stream(buf, cut, spec)
    return list(ends), rc, pos, rem


@pytest.mark.parametrize("seed", range(12))
def test_speculative_framer_matches_sequential(seed):
    buf, want = _stream(seed, 30)
    rng = random.Random(100 + seed)
    for cut in [0, len(buf) // 2, rng.randrange(len(buf) + 1), len(buf)]:
        seq = _frame(buf, cut, False)
        spec = _frame(buf, cut, True)
        assert seq == spec
        assert seq[0] == want and seq[1] == 0
    # an incomplete tail: the pending state agrees too
    part = buf[:want[-1] - 5]
    assert _frame(part, len(part) // 3, True) == _frame(part, len(part) // 3, False)


def test_speculative_framer_on_train_requests():
    import bench
    rng = random.Random(7)
    bodies = bench.make_requests(rng, 24, 128, 16, 8, 8, 100000)
    buf, want = b"", []
    for i, body in enumerate(bodies):
        buf += b"\x94\x00\xce" + i.to_bytes(4, "big") + b"\xa5train\x92\xa0" + body
        want.append(len(buf))
    assert len(buf) > 256 << 10
    for cut in (0, 70000, len(buf) - 3):
        assert _frame(buf, cut, True) == (want, 0, 0, 1) == _frame(buf, cut, False)


def test_malformed_byte_on_the_true_chain():
    buf, want = _stream(3, 20)
    # a reserved type byte where the 13th message starts: the ends before it stand
    bad = buf[:want[11]] + b"\xc1" + buf[want[11] + 1:]
    seq = _frame(bad, len(bad), False)
    spec = _frame(bad, len(bad), True)
    assert seq[1] == -1 and spec[1] == -1
    assert seq[0] == spec[0] == want[:12]
