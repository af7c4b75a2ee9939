"""LOF state across a MIX (models/anomaly.py _rows_changed): 2 and 4 gloo
ranks each add their own rows, the row MIX (parallel/row_mix.py) gives every
rank the union, and the LOF scores afterwards equal a single-node oracle that
holds the union of the rows with exact k-NN lists; the state is warm right
after the MIX (every stored row has a valid list: no lazy rebuild inside the
next scores). A small MIX (below REBUILD_ALL_FRACTION of the rows) is applied
incrementally and also leaves every list valid. Reference:
anomaly_serv.cpp:157-211 (the LOF storage is mixed with the rows)."""
import os
import random
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

CONV = {"num_rules": [{"key": "*", "type": "num"}]}
PARAM = {"method": "euclid_lsh", "nearest_neighbor_num": 4, "reverse_nearest_neighbor_num": 12,
         "parameter": {"hash_num": 512}}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine():
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.anomaly import LOF
    return LOF("lof", PARAM, DatumToFvConverter(CONV), None)


def _rows(rank, n, seed=0):
    r = random.Random(1000 * seed + rank)
    return [(f"r{rank}_{i}", {"x": r.gauss(rank * 0.7, 1.0), "y": r.gauss(0, 1.0), "z": r.gauss(0, 2.0)})
            for i in range(n)]


QUERIES = [{"x": 0.1 * i, "y": -0.2 * i, "z": 0.05 * i} for i in range(-6, 7)]


def _valid_lists(eng) -> bool:
    st = eng._state()
    ids = eng.rows.ids
    ok = np.asarray(st.ok[:len(ids)])
    return all(ok[s] for s, r in enumerate(ids) if r is not None)


def _worker(rank, world, port, sizes, q):
    try:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        eng = _engine()
        for rid, d in _rows(rank, sizes[rank]):
            eng.add(rid, d)
        eng.mix()
        warm = _valid_lists(eng)
        scores = [eng.calc_score(d) for d in QUERIES]
        q.put((rank, warm, scores, sorted(r for r in eng.rows.ids if r is not None)))
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, "error", traceback.format_exc(), None))


def _oracle(sizes):
    eng = _engine()
    items = [it for r in range(len(sizes)) for it in _rows(r, sizes[r])]
    for rid, d in items:
        eng.add(rid, d)
    # exact k-NN lists of the whole union
    st = eng._state()
    st.moved([s for s, r in enumerate(eng.rows.ids) if r is not None])
    eng.build_lists()
    return [eng.calc_score(d) for d in QUERIES]


def _run(sizes):
    world = len(sizes)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sizes, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    for _ in range(world):
        r = q.get(timeout=240)
        assert r[1] != "error", r[2]
        res.append(r)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return sorted(res)


@pytest.mark.parametrize("world", [2, 4])
def test_lof_scores_after_mix_equal_single_node_oracle(world):
    sizes = [40] * world
    res = _run(sizes)
    want = _oracle(sizes)
    for rank, warm, scores, ids in res:
        assert warm, f"rank {rank}: lists missing right after the MIX"
        assert ids == res[0][3]
        np.testing.assert_allclose(scores, want, rtol=1e-5, atol=1e-6)


def test_small_mix_applied_incrementally_keeps_state_warm():
    """rank 1 brings 4 rows to rank 0's 60: rank 0 applies them as a batch
    of adds (no full rebuild) and every list stays valid"""
    res = _run([60, 4])
    for rank, warm, scores, ids in res:
        assert warm
        assert all(np.isfinite(scores))
