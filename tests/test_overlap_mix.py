"""Overlapped MIX (LinearClassifier.mix_begin / mix_end) on a 2-rank gloo
group: the cluster mean of the snapshot is folded in while updates made
during the collective survive; a label-layout disagreement falls back to the
synchronous MIX. Compared against a numpy recomputation."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

CONV = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
        "num_rules": [{"key": "*", "type": "num"}], "hash_max_size": 1 << 12}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q, mismatch, grow=False):
    import torch.distributed as dist
    os.environ.setdefault("JUBATUS_FORCE_CPU", "1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier
    clf = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV))
    for lab in ("a", "b"):
        clf.set_label(lab)
    if mismatch and rank == 0:
        clf.set_label("extra")
    data = [(("a" if (i + rank) % 2 else "b"), {"x": f"v{i % 5}", "n": float(i + rank)}) for i in range(20)]
    clf.train(data)
    snapW, snapP = clf.W.copy(), clf.P.copy()
    h = clf.mix_begin()
    late = [("a", {"x": "late", "n": 1.0})] if rank == 1 and not mismatch else []
    if grow and rank == 1:               # 9 labels: the label capacity grows 8 -> 16
        late = [(f"g{i}", {"x": "late", "n": 1.0}) for i in range(7)]
    clf.train(late)                      # keeps going while the collective runs
    W_after, P_after = clf.W.copy(), clf.P.copy()
    clf.mix_end(h)
    if grow:
        # rank 1 replaced its tables during the collective: nothing folded in;
        # the next (synchronous) MIX reconciles both ranks
        stats = dict(clf._last_mix)
        same = bool(np.array_equal(clf.W, W_after))
        clf.mix()
        out = [None, None]
        dist.all_gather_object(out, (stats, same, clf.W.copy(), clf.get_labels()))
        if rank == 0:
            q.put(out)
        dist.destroy_process_group()
        return
    # every rank's snapshot, for the reference computation
    out = [None, None]
    dist.all_gather_object(out, (snapW, snapP, W_after, P_after, clf.W.copy(), clf.P.copy(),
                                 clf.get_labels()))
    if rank == 0:
        q.put(out)
    dist.destroy_process_group()


@pytest.mark.parametrize("mismatch", [False, True])
def test_overlapped_mix(mismatch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, mismatch)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (s0W, s0P, a0W, a0P, f0W, f0P, l0), (s1W, s1P, a1W, a1P, f1W, f1P, l1) = res
    if not mismatch:
        meanW, meanP = (s0W + s1W) / 2, (s0P + s1P) / 2
        np.testing.assert_allclose(f0W, meanW + (a0W - s0W), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(f1W, meanW + (a1W - s1W), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(f1P, meanP + (a1P - s1P), rtol=1e-5, atol=1e-6)
        assert l0 == {"a": 20, "b": 20} and l1 == {"a": 21, "b": 20}   # + rank 1's late sample
    else:
        # fell back to the synchronous MIX: one label layout, identical tables
        assert set(l0) == set(l1) == {"a", "b", "extra"}
        np.testing.assert_allclose(f0W, f1W, rtol=1e-6, atol=1e-7)


def test_overlapped_mix_tables_replaced_during_collective():
    """a train that grows the label capacity while the overlapped
    MIX runs replaces W / P; mix_end must not fold the stale snapshot into
    the new tables (the collectives still complete on both ranks)"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, port, q, False, True)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (st0, same0, W0, l0), (st1, same1, W1, l1) = res
    assert st1["abandoned"] and same1          # rank 1: no fold into the new tables
    assert not st0["abandoned"] and not same0  # rank 0 folded the mean
    assert l0 == l1 and len(l0) == 9
    np.testing.assert_allclose(W0, W1, rtol=1e-6, atol=1e-7)


def _nosync_worker(rank, port, q):
    import torch
    import torch.distributed as dist
    os.environ.setdefault("JUBATUS_FORCE_CPU", "1")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=2)
    from jubatus_amd.parallel.table_mix import TableMix
    H, C = 4096, 8
    W = torch.zeros(H, C)
    touched = torch.zeros(H, dtype=torch.uint8)
    touched[rank * 100:rank * 100 + 50] = 1
    W[touched.bool()] = 1.0 + rank
    calls = []
    real_item, real_nonzero = torch.Tensor.item, torch.nonzero

    def item(self):
        calls.append("item")
        return real_item(self)

    def nonzero(*a, **k):
        calls.append("nonzero")
        return real_nonzero(*a, **k)
    torch.Tensor.item, torch.nonzero = item, nonzero
    try:
        job = TableMix([W], touched, None).begin()      # must not synchronise with the device
    finally:
        torch.Tensor.item, torch.nonzero = real_item, real_nonzero
    job.end()
    q.put((rank, calls, job.stats(), float(W[0, 0]), float(W[100, 0])))
    dist.destroy_process_group()


def test_mix_begin_has_no_host_sync():
    """the union of the touched rows is a MAX all-reduce of the
    bitmaps, sized on the host only once it completed (ready / end) - begin
    itself calls neither .item() nor nonzero"""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_nosync_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, calls, st, w0, w100 in res:
        assert calls == [], calls
        assert st["mode"] == "sparse" and st["rows"] == 100
        assert w0 == 0.5 and w100 == 1.0                  # the mean of the two ranks' rows
