"""GPU request scanner (csrc/hip/scan.hip) vs the host scanner
(csrc/native/jb_pack.cpp): identical batch descriptors and feature rows on
the same arena, rejection + host re-run for what the device path does not
take, and the same model through LinearClassifier.train_arena."""
import random

import msgpack
import numpy as np
import pytest

from jubatus_amd.fv_converter.converter import DatumToFvConverter
from jubatus_amd.fv_converter.datum import Datum

pytestmark = pytest.mark.gpu

CONV = {
    "string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"},
                     {"key": "s1*", "type": "str", "sample_weight": "log_tf", "global_weight": "bin"}],
    "num_rules": [{"key": "*", "type": "num"}, {"key": "*1", "type": "log"}],
    "hash_max_size": 1 << 18,
}


def _device():
    import torch
    return torch.device("cuda", 0)


def _sample(rng, y, wide=False):
    d = {f"s{j}": f"v{(y * 7 + rng.randrange(4)) if rng.random() < 0.7 else rng.randrange(500)}"
         for j in range(3)}
    d["long"] = "x" * rng.randrange(30, 300)          # str8 / raw16 encodings (checked path)
    for j in range(3):
        d[f"n{j}"] = (y - 2) * 0.5 + rng.gauss(0, 1)
    d["big"] = rng.randrange(1 << 20)                 # uint32 encoding
    d["neg"] = -rng.randrange(200)                    # negative fixint / int16
    if wide:
        for j in range(40):
            d[f"w{j}"] = f"t{rng.randrange(1000)}"
    return Datum(d).to_msgpack()


def _arena(bodies):
    from jubatus_amd.ops.feature_pipeline import RequestArena
    a = RequestArena(sum(len(b) for b in bodies) + 16 * len(bodies) + 64)
    for b in bodies:
        a.append(b)
    offs, lens = a.spans()
    return a, offs, lens


def _bodies(seed=0, nreq=40, nlabels=5, big_every=7):
    rng = random.Random(seed)
    bodies = []
    for r in range(nreq):
        per = rng.randrange(0, 60)
        wide = r % big_every == 3          # bodies near / above the 27 KB LDS stage
        if wide:
            per = 30
        items = [[f"L{rng.randrange(nlabels)}", _sample(rng, rng.randrange(nlabels), wide)]
                 for _ in range(per)]
        bodies.append(msgpack.packb(items, use_bin_type=False))
    return bodies


def _batch_arrays(b):
    n = b.n
    rp = b.row_ptr[:n + 1].cpu().numpy()
    return (n, rp, b.labels[:n].cpu().numpy(), b.stream_ptr[:b.nstreams + 1].cpu().numpy(),
            b.fidx[:rp[-1]].cpu().numpy(), b.fval[:rp[-1]].cpu().numpy())


@pytest.mark.parametrize("nlabels", [5, 100])
def test_gpu_scan_matches_host_scan(nlabels):
    """5 labels: label table and counts in LDS; 100: the table is read from
    global memory and labels >= 64 are counted with global atomics"""
    import torch
    from jubatus_amd._native import native
    from jubatus_amd.ops.feature_pipeline import FeaturePipeline, ScanCheck

    pipe = FeaturePipeline(DatumToFvConverter(CONV), _device())
    bodies = _bodies(nlabels=nlabels)
    assert 16 * 1024 < max(len(b) for b in bodies) <= 27 * 1024 - 16
    arena, offs, lens = _arena(bodies)
    table = native().LabelTable()
    for y in range(nlabels):
        table.get_or_add(f"L{y}")
    host = _batch_arrays(pipe.from_arena(arena, offs, lens, True, table))
    torch.cuda.synchronize()
    pipe.check_errors()
    chk = ScanCheck(128)
    b = pipe.from_arena_gpu(arena, offs, lens, table, chk)
    torch.cuda.synchronize()
    pipe.check_errors()
    assert int(chk.err[0]) == 0
    dev = _batch_arrays(b)
    assert dev[0] == host[0]
    for h, d, name in zip(host[1:], dev[1:], ("row_ptr", "labels", "stream_ptr", "fidx", "fval")):
        np.testing.assert_array_equal(h, d, err_msg=name)
    # label counts of the batch
    want = np.bincount(host[2], minlength=128)
    np.testing.assert_array_equal(chk.hist[:128], want)


@pytest.mark.parametrize("case", ["unknown_label", "binary_values", "malformed", "too_big"])
def test_gpu_scan_rejects_batch(case):
    import torch
    from jubatus_amd._native import native
    from jubatus_amd.ops.feature_pipeline import FeaturePipeline, ScanCheck

    pipe = FeaturePipeline(DatumToFvConverter(CONV), _device())
    bodies = _bodies(seed=1, nreq=6, big_every=100)
    if case == "unknown_label":
        bodies.append(msgpack.packb([["new", _sample(random.Random(2), 1)]], use_bin_type=False))
    elif case == "binary_values":
        dm = _sample(random.Random(3), 1)
        dm[2] = [["b", b"\x00\x01"]]
        bodies.append(msgpack.packb([["L1", dm]], use_bin_type=True))
    elif case == "malformed":
        good = msgpack.packb([["L1", _sample(random.Random(4), 1)]] * 2, use_bin_type=False)
        bodies.append(good[:len(good) - 7])          # truncated
    else:                                            # larger than the LDS stage: host path
        rng = random.Random(6)
        bodies.append(msgpack.packb([["L1", _sample(rng, 1, True)] for _ in range(200)],
                                    use_bin_type=False))
        assert len(bodies[-1]) > 27 * 1024
    arena, offs, lens = _arena(bodies)
    table = native().LabelTable()
    for y in range(5):
        table.get_or_add(f"L{y}")
    chk = ScanCheck(16)
    b = pipe.from_arena_gpu(arena, offs, lens, table, chk)
    if case == "too_big":                             # decided on the host: no launch
        assert b is None
        return
    torch.cuda.synchronize()
    pipe.check_errors()                               # the stand-in datums parse cleanly
    assert int(chk.err[0]) != 0
    n, rp, labels, *_ = _batch_arrays(b)
    assert (labels == -1).all() and (rp == 0).all()


def test_train_arena_gpu_scan_same_model(monkeypatch):
    """single-request batches (exact sequential updates): the GPU-scanned
    model equals the host-scanned one, new labels included (host re-run)"""
    import torch
    from jubatus_amd.models.classifier import LinearClassifier

    rng = random.Random(5)
    steps = []
    for s in range(6):
        nl = 3 if s < 2 else 6                      # labels L3..L5 first appear in step 2
        items = [[f"L{rng.randrange(nl)}", _sample(rng, rng.randrange(nl))] for _ in range(50)]
        steps.append(_arena([msgpack.packb(items, use_bin_type=False)]))
    models = []
    for gpu_scan in (False, True):
        clf = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV),
                               device=_device())
        clf.gpu_scan = gpu_scan
        for a, offs, lens in steps:
            assert clf.train_arena(a, offs, lens) == 50
        clf.synchronize()
        clf.pipe.check_errors()
        models.append((clf.get_labels(), clf.W.cpu().numpy(), clf.P.cpu().numpy(),
                       clf.labels.names()))
        st = clf.get_status()
        if gpu_scan:   # step 0 has no labels yet (host), new labels in step 2 are re-run
            assert int(st["train_scan.gpu"]) >= 4 and int(st["train_scan.replayed"]) >= 1
            assert int(st["train_scan.host"]) >= 1
    (l0, w0, p0, n0), (l1, w1, p1, n1) = models
    assert l0 == l1 and n0 == n1
    np.testing.assert_allclose(w1, w0, rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(p1, p0, rtol=1e-6, atol=1e-6)


def test_train_arena_concurrent_requests_serial_equivalent():
    """the GPU-scan batch path (csrc/hip/train_batch.hip) with many requests
    per batch in the default exact mode: the model equals the requests
    trained one after another on the host oracle"""
    from jubatus_amd.models.classifier import LinearClassifier

    rng = random.Random(9)
    batches, reqs = [], []
    for b in range(4):
        items_per = []
        for r in range(64):
            items = [[f"L{(y := rng.randrange(5))}", _sample(rng, y)] for _ in range(rng.randrange(1, 30))]
            items_per.append(items)
            reqs.append(items)
        batches.append(_arena([msgpack.packb(it, use_bin_type=False) for it in items_per]))
    g = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV),
                         device=_device())
    c = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV))
    for y in range(5):
        g.set_label(f"L{y}")
        c.set_label(f"L{y}")
    for a, offs, lens in batches:
        g.train_arena(a, offs, lens)
    for items in reqs:
        c.train_requests([msgpack.packb(items, use_bin_type=False)])
    g.synchronize()
    g.pipe.check_errors()
    st = g.get_status()
    assert int(st["train_scan.gpu"]) == 4 and st["train.update_mode"] == "exact"
    assert g.train_stats()["updated"] == c.train_stats()["updated"]
    scale = float(np.abs(c.W).max()) or 1.0
    np.testing.assert_allclose(g.W.cpu().numpy()[:, :c.LC], c.W, rtol=2e-3, atol=2e-3 * scale)
    np.testing.assert_allclose(g.P.cpu().numpy()[:, :c.LC], c.P, rtol=2e-3,
                               atol=2e-3 * float(c.P.max()))
