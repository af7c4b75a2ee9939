"""csrc/native/jb_pyrandom.hpp reproduces CPython's random.Random stream:
seeding from ints (incl. negative and > 32 bits), random(), getrandbits,
randbelow, sample(range(n), k) on both of its algorithms, and weighted
choices - the draws the native clustering server must share with the Python
one (models/clustering.py)."""
import random

import pytest

from jubatus_amd._native import native


@pytest.mark.parametrize("seed", [0, 1, 42, -7, 2**40 + 3, 123456789])
def test_stream_matches_cpython(seed):
    c = native().PyRandom(seed)
    r = random.Random(seed)
    for _ in range(50):
        assert c.random() == r.random()
    for k in (1, 5, 31, 32, 33, 63):
        assert c.getrandbits(k) == r.getrandbits(k)
    for n in (1, 2, 7, 1000, 2**33 + 5):
        assert c.randbelow(n) == r._randbelow(n)
    for n, k in ((10, 3), (21, 20), (50, 5), (1000, 100), (1100, 100), (200, 150)):
        assert c.sample_range(n, k) == r.sample(range(n), k)
    w = [r2 * 0.37 for r2 in range(1, 40)]
    for _ in range(20):
        assert c.choice_weighted(w) == r.choices(range(len(w)), weights=w, k=1)[0]
    assert c.random() == r.random()
