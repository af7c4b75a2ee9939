"""MIX schedule and fold logic on the CPU, without a process group.

Mirrors the reference's mixer unit tests:
* skip_mixer_test.cpp:41-80 (filter_candidates for N=2 and N=4),
* linear_mixer_test.cpp:156-169 (the master folds the diffs of all members,
  "(4+(3+(2+1)))").
The peer schedules differ from the reference on purpose: here a pair
exchange is a matched send/recv on both ranks, so each stride's pairing must
be symmetric (rank ^ stride for power-of-two N; parallel/push_mixer.py).
"""
import pytest

from jubatus_amd.framework.mixer import UnsupportedMixables
from jubatus_amd.parallel import mixable
from jubatus_amd.parallel.push_mixer import random_matching, round_robin, skip_peers, skip_strides


def test_skip_strides():
    assert skip_strides(1) == []
    assert skip_strides(2) == [1]
    assert skip_strides(4) == [2, 1]
    assert skip_strides(8) == [4, 2, 1]
    assert skip_strides(6) == [3, 1]


def test_skip_peers_reference_cases():
    # N=2: the one other member (skip_mixer_test.cpp:41-58)
    assert skip_peers(1, 2) == [0]
    # N=4: two peers, the farther stride first (skip_mixer_test.cpp:60-80
    # expects the +2 peer first as well)
    p = skip_peers(1, 4)
    assert len(p) == 2 and p[0] == 3


@pytest.mark.parametrize("n", [2, 4, 8, 16])
def test_skip_peers_symmetric_butterfly(n):
    for r in range(n):
        for i, peer in enumerate(skip_peers(r, n)):
            assert peer != r
            assert skip_peers(peer, n)[i] == r     # matched pairing per stride


@pytest.mark.parametrize("n", [2, 4, 8])
def test_butterfly_pair_averaging_is_exact_mean(n):
    vals = [float(3 * r * r + 1) for r in range(n)]
    want = sum(vals) / n
    for i in range(len(skip_strides(n))):
        nxt = list(vals)
        for r in range(n):
            peer = skip_peers(r, n)[i]
            nxt[r] = (vals[r] + vals[peer]) / 2
        vals = nxt
    assert all(abs(v - want) < 1e-9 for v in vals)


@pytest.mark.parametrize("n", [2, 3, 5, 8])
def test_random_matching(n):
    m = random_matching(n, seed=7)
    assert m == random_matching(n, seed=7)          # every rank derives the same matching
    for a, b in m.items():
        assert a != b and m[b] == a
    assert len(m) == n - (n % 2)


@pytest.mark.parametrize("n", [2, 3, 4, 7])
def test_round_robin_covers_every_pair_once(n):
    seen = set()
    for rnd in round_robin(n):
        for a, b in rnd.items():
            assert rnd[b] == a
            if a < b:
                assert (a, b) not in seen
                seen.add((a, b))
    assert seen == {(a, b) for a in range(n) for b in range(a + 1, n)}


class _StringDriver:
    """linear_mixable with the reference test's string fold (my_string::mix)"""

    def __init__(self):
        self.put = None

    def get_diff(self):
        return ""

    def mix_diff(self, acc, d):
        return f"({d}+{acc})"

    def put_diff(self, mixed):
        self.put = mixed


class _FakeDist:
    def __init__(self, diffs):
        self.diffs = diffs

    def is_initialized(self):
        return True

    def get_world_size(self):
        return len(self.diffs)

    def all_gather_object(self, out, obj):
        out[:] = list(self.diffs)


def test_linear_mix_fold_order(monkeypatch):
    from jubatus_amd.parallel import wire
    monkeypatch.setattr(wire, "all_gather", lambda obj, group=None: ["1", "2", "3", "4"])
    d = _StringDriver()
    st = mixable.linear_mix(d)
    assert d.put == "(4+(3+(2+1)))"
    assert st["seconds"] >= 0


def test_linear_mix_single_member():
    d = _StringDriver()
    mixable.linear_mix(d)
    assert d.put == ""


def test_unsupported_mixables():
    with pytest.raises(UnsupportedMixables):
        mixable.linear_mix(object())


def test_wire_roundtrip_without_pickle(monkeypatch):
    """driver diffs cross the model plane as msgpack (parallel/wire.py):
    numpy values are converted, nothing is pickled"""
    import pickle

    import numpy as np
    from jubatus_amd.parallel import wire
    monkeypatch.setattr(pickle, "dumps", None)
    obj = {"a": [1, 2.5, "x"], 3: {"n": np.float32(1.5), "v": np.arange(3)}, "b": b"\x00\x01"}
    back = wire.decode(wire.encode(obj))
    assert back == {"a": [1, 2.5, "x"], 3: {"n": 1.5, "v": [0, 1, 2]}, "b": b"\x00\x01"}
    assert wire.all_gather(obj) == [obj]          # no process group: identity
