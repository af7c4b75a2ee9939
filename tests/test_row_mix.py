"""Row-engine MIX over tensor collectives (parallel/row_mix.py) on 2 gloo
ranks: both ranks end with the same rows, versions, datums, document
statistics and index contents, equal to the reference protocol's fold
(get_diff -> mix_diff in rank order -> put_diff, linear_mixer.cpp:422-544),
for the all-gather MIX and for the pairwise (push) MIX - and nothing is
pickled on the way."""
import os
import pickle
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

CONV = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
        "num_rules": [{"key": "*", "type": "num"}]}
CONV_IDF = {"string_rules": [{"key": "*", "type": "bigram", "sample_weight": "tf", "global_weight": "idf"}],
            "string_types": {"bigram": {"method": "ngram", "char_num": "2"}},
            "num_rules": [{"key": "*", "type": "num"}]}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _engine(kind, device=None):
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    if kind == "nn_lsh":
        from jubatus_amd.models.recommender import NearestNeighbor
        return NearestNeighbor("lsh", {"hash_num": 64}, DatumToFvConverter(CONV), device)
    if kind == "rec_ii_idf":
        from jubatus_amd.models.recommender import Recommender
        return Recommender("inverted_index", {}, DatumToFvConverter(CONV_IDF), device)
    if kind == "rec_euclid_lsh":
        from jubatus_amd.models.recommender import Recommender
        return Recommender("euclid_lsh", {"hash_num": 64}, DatumToFvConverter(CONV), device)
    from jubatus_amd.models.anomaly import LOF
    return LOF("lof", {"method": "inverted_index_euclid", "nearest_neighbor_num": 3,
                       "reverse_nearest_neighbor_num": 10, "parameter": {}},
               DatumToFvConverter(CONV), device)


def _write(eng, rank):
    for i in range(12):
        d = {"x": float(i + 10 * rank), "t": f"word{i % 3}{rank}"}
        if hasattr(eng, "add"):
            eng.add(f"r{rank}_{i}", d)
        else:
            eng.update_row(f"r{rank}_{i}", d)
    # a row both ranks write: rank 1 writes it twice (newer version wins)
    for _ in range(rank + 1):
        d = {"x": 100.0 + rank, "t": f"shared{rank}"}
        (eng.add if hasattr(eng, "add") else eng.update_row)("shared", d)
    eng.clear_row(f"r{rank}_3")


def _state(eng):
    rows = {rid: (eng.rows.version[rid], eng.rows.datum[eng.rows.slot(rid)])
            for rid in sorted(eng.rows.slot_of)}
    w = eng.conv.weights
    df = None
    if eng.conv.uses_global_weight:
        df = (w.doc_count, w.total_len, sorted((int(i), int(v)) for i, v in
                                               zip(*__import__("numpy").nonzero(w.df), w.df[w.df != 0])))
    # every row's distance to a probe (slots differ between ranks, so tied
    # distances may list in another order: compare id -> distance)
    q = eng.query_fv(eng.fv_of(__import__("jubatus_amd.fv_converter.datum",
                                           fromlist=["as_datum"]).as_datum({"x": 3.0, "t": "word01"})),
                     len(rows), similar=False)
    return rows, df, {r: round(d, 5) for r, d in q}


def _worker(rank, world, port, kind, how, q, gpu=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _body(rank, world, kind, how, q, gpu)
    except BaseException as e:  # noqa: BLE001 - report to the parent instead of hanging it
        import traceback
        q.put((rank, "error", traceback.format_exc(), 0, 0))
        raise
    finally:
        dist.destroy_process_group()


def _body(rank, world, kind, how, q, gpu=False):
    if True:
        import torch
        eng = _engine(kind, torch.device("cuda", 0) if gpu else None)
        ref = _engine(kind)
        _write(eng, rank)
        _write(ref, rank)
        # reference fold through the pickled get_diff protocol
        diffs = [None] * world
        dist.all_gather_object(diffs, ref.get_diff())
        mixed = diffs[0]
        for d in diffs[1:]:
            mixed = ref.mix_diff(mixed, d)
        ref.put_diff(mixed)
        if eng.conv.uses_global_weight:   # the reference protocol mixes df separately
            wd = [None] * world
            dist.all_gather_object(wd, eng.conv.weights.get_diff())
            m = wd[0]
            for d in wd[1:]:
                m = ref.conv.weights.mix(m, d)
            ref.conv.weights.put_diff(m)
        real_dumps = pickle.dumps
        pickle.dumps = None              # the tensor MIX must not pickle
        try:
            if how == "all":
                nbytes = eng.mix()
            else:
                eng.pair_mix(1 - rank)
                nbytes = eng._last_mix["bytes"]
        finally:
            pickle.dumps = real_dumps
        q.put((rank, _state(eng), _state(ref), nbytes, eng.get_status().get("mix.last_rows_applied")))


def _run(kind, how, gpu=False):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, how, q, gpu))
             for r in range(world)]
    for p in procs:
        p.start()
    res = []
    for _ in range(world):
        r = q.get(timeout=180)
        assert r[1] != "error", r[2]
        res.append(r)
    res.sort(key=lambda r: r[0])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, s0, r0, b0, a0), (_, s1, r1, b1, a1) = res
    return s0, s1, r0, r1, b0, b1, a0


@pytest.mark.parametrize("kind", ["nn_lsh", "rec_ii_idf", "rec_euclid_lsh", "lof"])
@pytest.mark.parametrize("how", ["all", "pair"])
def test_row_mix_equals_reference_fold(kind, how):
    s0, s1, r0, r1, b0, b1, a0 = _run(kind, how)
    assert s0[0] == s1[0] == r0[0] == r1[0]          # rows, versions, datums
    assert s0[0]["shared"][1][0]["t"] == "shared1"   # the newer write won
    assert "r0_3" not in s0[0] and "r1_3" not in s1[0]
    assert s0[1] == s1[1] == r0[1]                   # document statistics
    assert s0[2] == s1[2]                            # index answers
    assert b0 > 0 and b1 > 0 and int(a0) > 0


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["nn_lsh", "rec_ii_idf", "lof"])
def test_row_mix_device_tables_two_ranks_one_gpu(kind):
    """the same MIX with the tables in HBM (signatures exported from / scattered
    into the device table, pool rows appended on the device); 2 ranks share
    the one GPU over gloo. Host-side results must equal the host engines'."""
    s0, s1, r0, r1, b0, b1, a0 = _run(kind, "all", gpu=True)
    assert s0[0] == s1[0] == r0[0] == r1[0]
    assert s0[1] == s1[1] == r0[1]
    assert s0[2].keys() == s1[2].keys()
    assert int(a0) > 0
