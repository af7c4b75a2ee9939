"""Host-native runtime: CRC32 / MD5 vectors, hashing twins, request scanner."""
import msgpack
import pytest

from jubatus_amd._native import native
from jubatus_amd.fv_converter.hashing import feature_index, fnv1a64


def test_crc32_reference_vector():
    # reference: jubatus/server/common/crc32_test.cpp:25-28
    assert native().crc32(b"jubatus") == 0x41918955


def test_crc32_chaining():
    n = native()
    assert n.crc32(b"batus", n.crc32(b"ju")) == n.crc32(b"jubatus")


def test_md5_rfc1321_vectors():
    n = native()
    assert n.md5_hex("") == "d41d8cd98f00b204e9800998ecf8427e"
    assert n.md5_hex("abc") == "900150983cd24fb0d6963f7d28e17f72"
    assert n.md5_hex("a" * 200) == __import__("hashlib").md5(b"a" * 200).hexdigest()


@pytest.mark.parametrize("name", ["a", "key$value@str#bin/bin", "日本語$x@num", "x" * 300])
@pytest.mark.parametrize("H", [1 << 10, 1 << 20, 1000003])
def test_hash_twins(name, H):
    b = name.encode()
    assert native().fnv1a64(b) == fnv1a64(b)
    assert native().feature_index(b, H) == feature_index(name, H)
    assert 0 <= feature_index(name, H) < H


def _pack_call(bodies, labeled, table, rs=1, rn=1):
    import numpy as np
    n = native()
    staging = np.zeros(1 << 16, np.uint8)
    off = np.zeros(4096, np.int64)
    lab = np.zeros(4096, np.int32)
    row = np.zeros(4097, np.int64)
    sp = np.zeros(len(bodies) + 1, np.int64)
    ln = np.zeros(4096, np.int32)
    r = n.pack_requests(bodies, labeled, rs, rn, table, staging.ctypes.data, staging.nbytes,
                        off.ctypes.data, ln.ctypes.data, lab.ctypes.data if labeled else 0,
                        row.ctypes.data, sp.ctypes.data, 4096, 2)
    return r, staging, off, lab, row, sp


def test_scanner_counts_and_labels():
    n = native()
    t = n.LabelTable()
    b1 = msgpack.packb([["a", [[["k", "v"], ["k2", "w"]], [["x", 1.5]], []]],
                        ["b", [[], [["x", 2], ["y", -3]], []]]], use_bin_type=False)
    b2 = msgpack.packb([["a", [[["k", "v"]], [], []]]], use_bin_type=True)
    (ns, nb, nslots, err, _), staging, off, lab, row, sp = _pack_call([b1, b2], True, t, 2, 1)
    assert err == 0 and ns == 3
    assert row[:4].tolist() == [0, 5, 7, 9]
    assert lab[:3].tolist() == [0, 1, 0]
    assert sp.tolist() == [0, 2, 3]
    assert t.names() == ["a", "b"] and t.count(0) == 2 and t.count(1) == 1
    # datum offsets point at the datum inside staging
    first = msgpack.unpackb(bytes(staging[off[0]:]), raw=False) if False else None
    assert staging[off[0]] == 0x93  # fixarray(3)


@pytest.mark.parametrize("bad", [
    msgpack.packb([["a", [[["k"]], [], []]]]),           # string pair of length 1
    msgpack.packb([["a", [[], [["x", "notnum"]], []]]]),  # non-numeric num value
    msgpack.packb([["a"]]),                                # missing datum
    b"\x91\x92\xa1a\x93\x90",                             # truncated
])
def test_scanner_rejects_malformed(bad):
    t = native().LabelTable()
    (ns, nb, nslots, err, req), *_ = _pack_call([bad], True, t)
    assert err == 1 and req == 0


def test_label_table_delete_and_revive():
    t = native().LabelTable()
    assert t.get_or_add("x") == 0 and t.get_or_add("y") == 1
    assert t.remove("x") and not t.remove("x")
    assert t.lookup("x") == -1 and t.alive() == [False, True]
    assert t.get_or_add("x") == 0 and t.alive() == [True, True]


def test_pack_requests_has_no_side_effects_on_a_bad_batch():
    """a malformed request must leave the label table untouched
    (labels and counts are committed only after every request validated), so
    the per-request retry of the RPC batch path does not double-count."""
    import msgpack
    import numpy as np
    from jubatus_amd._native import native
    nat = native()
    t = nat.LabelTable()
    t.get_or_add("old")
    good = msgpack.packb([["old", [[["a", "x"]], [], []]], ["new1", [[["a", "y"]], [], []]]],
                         use_bin_type=False)
    good2 = msgpack.packb([["new2", [[], [["n", 1.5]], []]]] * 3, use_bin_type=False)
    bad = msgpack.packb([["new3", [[["a"]], [], []]]], use_bin_type=False)    # pair of 1
    cap = 1 << 16
    staging = np.zeros(cap, np.uint8)
    off = np.zeros(64, np.int64)
    ln = np.zeros(64, np.int32)
    lab = np.zeros(64, np.int32)
    rp = np.zeros(65, np.int64)
    sp = np.zeros(8, np.int64)

    def pack(bodies):
        return nat.pack_requests(bodies, 1, 1, 1, t, staging.ctypes.data, cap, off.ctypes.data,
                                 ln.ctypes.data, lab.ctypes.data, rp.ctypes.data, sp.ctypes.data,
                                 64, 2)

    n, nbytes, nslots, err, err_req = pack([good, bad, good2])
    assert err == 1 and err_req == 1
    assert t.names() == ["old"] and t.count(0) == 0          # nothing committed
    n, nbytes, nslots, err, err_req = pack([good, good2])
    assert err == 0 and n == 5
    assert t.names() == ["old", "new1", "new2"]               # order of first appearance
    assert [t.count(i) for i in range(3)] == [1, 1, 3]
    assert lab[:5].tolist() == [0, 1, 2, 2, 2]


def test_csr_normalize_matches_numpy():
    """native per-row sort / merge / norm (query latency path) == the numpy
    normalize_csr of models/similarity.py"""
    import numpy as np
    from jubatus_amd._native import native
    from jubatus_amd.models.similarity import normalize_csr
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 30, 50)
    rp = np.zeros(51, np.int64)
    np.cumsum(lens, out=rp[1:])
    idx = rng.integers(-2, 40, int(rp[-1])).astype(np.int32)
    val = rng.standard_normal(int(rp[-1])).astype(np.float32)
    a = normalize_csr(rp, idx, val)
    b = native().csr_normalize(rp, idx, val)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(np.asarray(x), np.asarray(y))
