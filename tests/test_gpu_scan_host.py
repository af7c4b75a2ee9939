"""Host-side pieces of the GPU request scan (ops/feature_pipeline.py): the
device label table (open addressing on FNV-1a 64, the hash csrc/hip/scan.hip
recomputes) and the body header pass. CPU only."""
import msgpack
import numpy as np

from jubatus_amd.ops.feature_pipeline import scan_too_big, body_counts, fnv1a64, label_table_arrays


def _probe(th, tm, blob, label: bytes):
    """the device lookup, in Python"""
    cap = th.size
    h = fnv1a64(label)
    i = h & (cap - 1)
    for _ in range(cap):
        lid = tm[3 * i + 2]
        if lid < 0:
            return -1
        if int(th.view(np.uint64)[i]) == h and tm[3 * i + 1] == len(label):
            off = tm[3 * i]
            if bytes(blob[off:off + len(label)]) == label:
                return int(lid)
        i = (i + 1) & (cap - 1)
    return -1


def test_fnv1a64_reference_values():
    # FNV-1a 64 test vectors (the same function as csrc/native/jb_hash.hpp)
    assert fnv1a64(b"") == 0xCBF29CE484222325
    assert fnv1a64(b"a") == 0xAF63DC4C8601EC8C
    assert fnv1a64(b"foobar") == 0x85944171F73967E8


def test_label_table_lookup_and_deleted_labels():
    names = [f"label{i}" for i in range(40)] + ["ラベル", ""]
    alive = [i % 7 != 3 for i in range(len(names))]
    th, tm, blob = label_table_arrays(names, alive)
    cap = th.size
    assert cap & (cap - 1) == 0 and cap >= 2 * sum(alive)
    for i, (n, a) in enumerate(zip(names, alive)):
        got = _probe(th, tm, blob, n.encode())
        assert got == (i if a else -1), (n, got)
    assert _probe(th, tm, blob, b"nope") == -1


def test_body_counts_headers():
    bodies = [msgpack.packb([1] * k) for k in (0, 3, 15, 16, 70000)]
    buf = np.frombuffer(b"".join(bodies), np.uint8)
    offs = np.cumsum([0] + [len(b) for b in bodies[:-1]]).astype(np.int64)
    lens = np.array([len(b) for b in bodies], np.int64)
    np.testing.assert_array_equal(body_counts(buf, offs, lens), [0, 3, 15, 16, 70000])
    # a body that is not an array, or empty: the host scanner reports it
    bad = np.frombuffer(b"\xa1x" + bodies[1], np.uint8)
    assert body_counts(bad, np.array([0, 2]), np.array([2, len(bodies[1])])) is None
    assert body_counts(buf, np.array([0]), np.array([0])) is None


def test_size_rule_matches_the_kernel_limits():
    # the host decides up front what the device scan would reject as too big
    offs = np.array([0, 16, 32], np.int64)
    assert not scan_too_big(offs, np.array([100, 27 * 1024, 5]), np.array([1, 2, 768]))
    assert scan_too_big(offs, np.array([100, 27 * 1024 + 1, 5]), np.array([1, 2, 3]))
    assert scan_too_big(np.array([3]), np.array([27 * 1024 - 2]), np.array([1]))   # aligned window
    assert scan_too_big(offs, np.array([1, 1, 1]), np.array([1, 769, 1]))
