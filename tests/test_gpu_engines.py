"""GPU numerics of the regression, LSH signature and scan kernels vs the
host references (models/regression.py train_one, models/similarity.py)."""
import random

import numpy as np
import pytest

from jubatus_amd.fv_converter.converter import DatumToFvConverter

pytestmark = pytest.mark.gpu

CONV = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
        "num_rules": [{"key": "*", "type": "num"}], "hash_max_size": 1 << 18}


def dev():
    import torch
    return torch.device("cuda", 0)


def rows(n, seed=0):
    r = random.Random(seed)
    out = []
    for _ in range(n):
        k = r.randrange(1, 30)
        idx = r.sample(range(1 << 18), k)
        out.append((idx, [r.gauss(0, 1) for _ in range(k)]))
    return out


def test_regression_single_stream_matches_oracle():
    from jubatus_amd.models.regression import PARegression
    g = PARegression("PA", {"sensitivity": 0.1, "regularization_weight": 2.0}, DatumToFvConverter(CONV), dev())
    c = PARegression("PA", {"sensitivity": 0.1, "regularization_weight": 2.0}, DatumToFvConverter(CONV))
    r = random.Random(1)
    data = [[3.0 * x + 1.0 + r.gauss(0, 0.1), {"x": x, "t": f"k{int(x * 3) % 5}"}]
            for x in (r.random() for _ in range(300))]
    for i in range(0, 300, 50):
        g.train(data[i:i + 50])
        c.train(data[i:i + 50])
    np.testing.assert_allclose(g.w.cpu().numpy(), c.w, rtol=1e-3, atol=1e-4)
    np.testing.assert_allclose(g.stats.cpu().numpy(), c.stats, rtol=1e-4)
    q = [d for _, d in data[:20]]
    np.testing.assert_allclose(g.estimate(q), c.estimate(q), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("method", ["lsh", "euclid_lsh", "minhash"])
def test_signatures_match_host(method):
    from jubatus_amd.models.similarity import LshIndex
    g = LshIndex(method, 128, 1091, dev())
    c = LshIndex(method, 128, 1091, None)
    rs = rows(200)
    gb, gn = g._signatures(rs)
    cb, cn = c._signatures(rs)
    gb = gb.cpu().numpy().view(np.uint64)
    agree = np.mean([bin(int(a) ^ int(b)).count("1") == 0 for a, b in zip(gb.ravel(), cb.ravel())])
    # only a projection within fp32 rounding of 0 may flip a bit (the host
    # sums in another order): at most one word in a thousand differs
    assert agree >= 0.999, agree
    bit_diff = np.mean([bin(int(a) ^ int(b)).count("1") for a, b in zip(gb.ravel(), cb.ravel())]) / 64
    assert bit_diff <= 1e-4, bit_diff
    np.testing.assert_allclose(gn.cpu().numpy(), cn, rtol=1e-5)


@pytest.mark.parametrize("method", ["lsh", "euclid_lsh", "minhash"])
def test_scan_and_topk_match_host(method):
    from jubatus_amd.models.similarity import LshIndex
    g = LshIndex(method, 64, 7, dev())
    c = LshIndex(method, 64, 7, None)
    rs = rows(300, seed=2)
    slots = list(range(300))
    g.set_rows(slots, rs)
    c.set_rows(slots, rs)
    g.remove(17)
    c.remove(17)
    # use identical signatures on both sides to compare the scans exactly
    c.bits[:300] = g.bits[:300].cpu().numpy().view(np.uint64)
    c.norms[:300] = g.norms[:300].cpu().numpy()
    q = rows(4, seed=3)
    dg = g.distances(q, 300).cpu().numpy()
    dc = c.distances(q, 300)
    assert np.all(np.isinf(dg[:, 17])) and np.all(np.isinf(dc[:, 17]))
    m = np.isfinite(dc)
    np.testing.assert_allclose(dg[m], dc[m], rtol=1e-4, atol=1e-4)
    tg = g.query(q, 300, 5, similar=True)
    tc = c.query(q, 300, 5, similar=True)
    for a, b in zip(tg, tc):
        np.testing.assert_allclose([s for _, s in a], [s for _, s in b], rtol=1e-4, atol=1e-4)


def test_sparse_scan_matches_host():
    from jubatus_amd.models.similarity import InvertedIndex
    for euclid in (False, True):
        g = InvertedIndex(euclid, dev())
        c = InvertedIndex(euclid, None)
        rs = rows(150, seed=4)
        g.set_rows(range(150), rs)
        c.set_rows(range(150), rs)
        g.remove(3)
        c.remove(3)
        q = rs[10]
        np.testing.assert_allclose(g.scores(q, 150), c.scores(q, 150), rtol=1e-4, atol=1e-4)


def test_engines_on_gpu():
    from jubatus_amd.models.anomaly import LOF
    from jubatus_amd.models.recommender import NearestNeighbor, Recommender
    nn = NearestNeighbor("euclid_lsh", {"hash_num": 64}, DatumToFvConverter(CONV), dev())
    for i in range(50):
        nn.set_row(f"r{i}", {"x": float(i), "y": float(i % 5)})
    res = nn.neighbor_row_from_id("r10", 3)
    assert res[0][0] == "r10"
    rec = Recommender("inverted_index", {}, DatumToFvConverter(CONV), dev())
    for i in range(30):
        rec.update_row(f"u{i}", {"a": float(i % 3), "b": float(i % 3) + 1})
    assert rec.similar_row_from_id("u1", 2)[0][0] in ("u1", "u4", "u7")
    lof = LOF("light_lof", {"method": "euclid_lsh", "parameter": {"hash_num": 64},
                            "nearest_neighbor_num": 5, "reverse_nearest_neighbor_num": 10},
              DatumToFvConverter(CONV), dev())
    for i in range(60):
        lof.add(str(i), {"x": float(i % 6) * 0.1, "y": float(i % 4) * 0.1})
    assert lof.calc_score({"x": 40.0, "y": -30.0}) > lof.calc_score({"x": 0.2, "y": 0.1})


@pytest.mark.parametrize("n,k,d", [(1, 1, 1), (100, 3, 2), (777, 37, 130), (4096, 64, 33)])
def test_sqdist_mfma_matches_fp32(n, k, d):
    import torch
    from jubatus_amd.ops import hip
    g = torch.Generator().manual_seed(n + k + d)
    X = torch.randn(n, d, generator=g)
    C = torch.randn(k, d, generator=g)
    ref = ((X[:, None, :] - C[None, :, :]) ** 2).sum(-1)
    out = hip.sqdist(X.to(dev()), C.to(dev())).cpu()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4 * d)


@pytest.mark.parametrize("gpu_min_elems", [0, 1 << 40])
def test_clustering_on_gpu_matches_cpu(gpu_min_elems):
    """0: every step on the device (single-workgroup k-means++ / Lloyd
    kernels, MFMA sqdist); 1 << 40: the same engine kept on the host"""
    from jubatus_amd.models.clustering import Clustering
    p = {"k": 3, "compressor_method": "compressive_kmeans", "bucket_size": 90,
         "compressed_bucket_size": 30, "seed": 0}
    conv = {"num_rules": [{"key": "*", "type": "num"}]}
    r = random.Random(0)
    pts = [{"x": cx + r.gauss(0, 0.3), "y": cy + r.gauss(0, 0.3)}
           for i in range(180) for cx, cy in [[(0, 0), (8, 8), (-8, 8)][i % 3]]]
    g = Clustering("kmeans", p, DatumToFvConverter(conv), dev())
    g.GPU_MIN_ELEMS = gpu_min_elems
    g.push(pts)
    assert g.centers.is_cuda == (gpu_min_elems == 0)
    cs = sorted(tuple(round(v) for _, v in sorted(c.num_values)) for c in g.get_k_center())
    assert cs == sorted([(0, 0), (8, 8), (-8, 8)])


@pytest.mark.parametrize("n,d,m", [(50, 3, 10), (200, 10, 100), (1000, 10, 100), (1500, 7, 40), (3000, 4, 20)])
def test_kmeanspp_matches_host_draws(n, d, m):
    """csrc/hip/clustering.hip k-means++ (one wave up to 2048 points, the
    workgroup kernel past that) == the host's draws: bisect_right over the
    double running sum of weight x min squared distance, the same uniforms"""
    import bisect

    import numpy as np
    import torch
    from jubatus_amd.ops import hip
    rng = np.random.default_rng(n + d)
    X = (rng.standard_normal((n, d)) * 3).astype(np.float32)
    w = (rng.random(n) + 0.25).astype(np.float32)
    u = rng.random(m)
    got, status = hip.kmeanspp(torch.from_numpy(X).to(dev()), torch.from_numpy(w).to(dev()), list(u), m)
    assert status == 0
    want, d2 = [], np.full(n, np.inf, np.float32)
    wt = w.astype(np.float64)
    for j in range(m):
        cum = np.cumsum(wt)
        c = min(bisect.bisect_right(cum.tolist(), u[j] * cum[-1]), n - 1)
        want.append(c)
        t = X - X[c]
        d2 = np.minimum(d2, np.einsum("ij,ij->i", t, t).astype(np.float32))
        wt = (d2 * w).astype(np.float64)
    assert got == want


@pytest.mark.parametrize("n,k,d", [(300, 3, 4), (1000, 5, 17), (64, 1, 2)])
def test_gmm_em_kernel_matches_fp32_torch(n, k, d):
    """csrc/hip/clustering.hip gmm_em_kernel (one launch for all iterations)
    == the fp32 torch EM of models/clustering.py on the host"""
    import torch
    from jubatus_amd.models.clustering import Clustering
    from jubatus_amd.ops import hip
    g = torch.Generator().manual_seed(n + k + d)
    centers = torch.randn(k, d, generator=g) * 6
    X = centers[torch.arange(n) % k] + torch.randn(n, d, generator=g)
    w = torch.rand(n, generator=g) + 0.5
    C0 = X[:k].clone()
    ref = Clustering._em(Clustering.__new__(Clustering), X, w, C0.clone(), iters=20)
    C, var = C0.clone().to(dev()), torch.ones(k, d, device=dev())
    pi = torch.full((k,), 1.0 / k, device=dev())
    assert hip.gmm_em(X.to(dev()), w.to(dev()), C, var, pi, 20)
    torch.testing.assert_close(C.cpu(), ref[0], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(var.cpu(), ref[1], rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(pi.cpu(), ref[2], rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("method", ["kmeans", "gmm"])
def test_default_clustering_config_runs_on_device(method):
    """config/clustering/{kmeans,gmm}.json (bucket_size 1000, compressed 100,
    k 3): every bucket is compressed and reclustered in HBM; the device
    engine draws the same k-means++ seeds from the same RNG as the host
    engine, so both find the same centres"""
    import json
    import os
    from helpers import ROOT
    from jubatus_amd.models.clustering import Clustering
    with open(os.path.join(ROOT, "config", "clustering", f"{method}.json")) as f:
        cfg = json.load(f)
    r = random.Random(1)
    truth = [(0.0, 0.0, 0.0), (10.0, 10.0, 0.0), (-10.0, 10.0, 5.0)]
    pts = [{"a": c[0] + r.gauss(0, 0.5), "b": c[1] + r.gauss(0, 0.5), "c": c[2] + r.gauss(0, 0.5)}
           for i in range(3000) for c in [truth[i % 3]]]
    g = Clustering(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]), dev())
    h = Clustering(cfg["method"], cfg["parameter"], DatumToFvConverter(cfg["converter"]))
    for b in range(0, 3000, 500):
        g.push(pts[b:b + 500])
        h.push(pts[b:b + 500])
    assert g.centers.is_cuda and g.get_revision() == h.get_revision() == 3
    got = sorted(tuple(round(v) for _, v in sorted(c.num_values)) for c in g.get_k_center())
    assert got == sorted(tuple(round(x) for x in c) for c in truth)
    ref = sorted(tuple(round(v, 2) for _, v in sorted(c.num_values)) for c in h.get_k_center())
    got2 = sorted(tuple(round(v, 2) for _, v in sorted(c.num_values)) for c in g.get_k_center())
    np.testing.assert_allclose(np.asarray(got2), np.asarray(ref), atol=0.05)


@pytest.mark.parametrize("metric,k,nrows,nq,bits", [(0, 10, 100_000, 3, 64), (1, 10, 250_000, 2, 64),
                                                    (2, 1, 5000, 4, 64), (1, 128, 70_000, 2, 64),
                                                    (0, 37, 3000, 5, 64), (1, 100, 50, 1, 64),
                                                    (0, 10, 400_000, 8, 64), (1, 31, 300_000, 8, 100),
                                                    (2, 100, 200_000, 7, 128),
                                                    # topk_mq_kernel (tables of 2M+ rows): one query, 8
                                                    # queries, euclid_lsh with 2 words, a partial last chunk
                                                    (0, 10, 2_200_000, 1, 64), (0, 10, 2_300_000, 8, 64),
                                                    (1, 16, 2_500_000, 3, 128), (2, 5, 2_100_007, 2, 64),
                                                    # one query: no sample launch (the scan starts
                                                    # unbounded, first chunks cut in the kernel)
                                                    (1, 10, 2_400_000, 1, 64), (1, 32, 2_200_000, 1, 128),
                                                    (2, 10, 2_100_000, 1, 64), (0, 32, 2_300_000, 1, 128),
                                                    (1, 16, 500_000, 12, 128), (2, 32, 300_000, 16, 64)])
def test_topk_hamming_matches_full_sort(metric, k, nrows, nq, bits):
    """csrc/hip/topk.hip (fused scan + exact top-k) == full distance matrix
    + stable argsort, including ties (lsh/minhash distances are multiples of
    1/hash_num) and invalid rows. Tables of 2M+ rows with k <= 32, <= 128
    bits and <= 8 queries (4 for euclid_lsh) take the sampled bound + register
    multi-query scan (topk_mq_sample_kernel, topk_mq_kernel); smaller tables
    or more queries the tile kernels (topk_wq_kernel / topk_kernel)."""
    import torch
    from jubatus_amd.ops import hip
    g = torch.Generator().manual_seed(nrows + k)
    words = (bits + 63) // 64
    tb = torch.randint(-2**62, 2**62, (nrows, words), generator=g, dtype=torch.int64)
    qb = torch.randint(-2**62, 2**62, (nq, words), generator=g, dtype=torch.int64)
    if bits % 64:                        # bits past hash_num are zero in a signature
        mask = (1 << (bits % 64)) - 1
        tb[:, -1] &= mask
        qb[:, -1] &= mask
    tn = torch.rand(nrows, generator=g) * 3
    valid = (torch.rand(nrows, generator=g) > 0.1).to(torch.uint8)
    qn = torch.rand(nq, generator=g) * 3
    d = dev()
    tbd, tnd, vd, qbd, qnd = (x.to(d) for x in (tb, tn, valid, qb, qn))
    full = torch.empty((nq, nrows), dtype=torch.float32, device=d)
    hip.hamming_scan(qbd, qnd, nq, tbd, tnd, vd, nrows, bits, metric, full)
    od, oi = hip.topk_hamming(qbd, qnd, nq, tbd, tnd, vd, nrows, bits, metric, k)
    full = full.cpu().numpy()
    od, oi = od.cpu().numpy(), oi.cpu().numpy()
    for q in range(nq):
        order = np.argsort(full[q], kind="stable")[:k]
        ref = full[q][order]
        fin = np.isfinite(ref)
        nf = int(fin.sum())
        if metric == 1:
            # euclid_lsh distances are float expressions: two kernels may round
            # a near tie (measured: 2.4e-7 apart at 1.409) either way, so the
            # rows must carry the k smallest distances, in order, each once
            got = oi[q][:nf]
            assert len(set(got.tolist())) == nf
            np.testing.assert_allclose(full[q][got], ref[fin], rtol=1e-6)
        else:
            np.testing.assert_array_equal(oi[q][:nf], order[fin])
        np.testing.assert_allclose(od[q][:nf], ref[fin], rtol=1e-6)
        assert np.all(np.isinf(od[q][nf:]))


@pytest.mark.parametrize("k", [1, 10, 31, 100])
def test_topk_hamming_heavy_ties(k):
    """a table of 8 distinct signatures over 600k rows: every distance level
    holds ~75k tied rows, so the exact answer is the lowest row indices of
    the nearest level (the scan's tie pruning must keep exactly those)"""
    import torch
    from jubatus_amd.ops import hip
    nrows, nq = 600_000, 3
    g = torch.Generator().manual_seed(k)
    pool = torch.randint(-2**62, 2**62, (8, 1), generator=g, dtype=torch.int64)
    tb = pool[torch.randint(0, 8, (nrows,), generator=g)]
    tn = torch.ones(nrows)
    valid = (torch.rand(nrows, generator=g) > 0.05).to(torch.uint8)
    qb = pool[:nq].clone()
    qb[0, 0] ^= 1                        # no exact match for query 0
    qn = torch.ones(nq)
    d = dev()
    tbd, tnd, vd, qbd, qnd = (x.to(d) for x in (tb, tn, valid, qb, qn))
    full = torch.empty((nq, nrows), dtype=torch.float32, device=d)
    hip.hamming_scan(qbd, qnd, nq, tbd, tnd, vd, nrows, 64, 0, full)
    od, oi = hip.topk_hamming(qbd, qnd, nq, tbd, tnd, vd, nrows, 64, 0, k)
    full = full.cpu().numpy()
    od, oi = od.cpu().numpy(), oi.cpu().numpy()
    for q in range(nq):
        order = np.argsort(full[q], kind="stable")[:k]
        np.testing.assert_array_equal(oi[q], order)
        np.testing.assert_allclose(od[q], full[q][order], rtol=1e-6)


def test_topk_scores_flip():
    import torch
    from jubatus_amd.ops import hip
    s = torch.rand((2, 9000), generator=torch.Generator().manual_seed(1))
    s[0, 5] = float("-inf")
    od, oi = hip.topk_scores(s.to(dev()), 2, 9000, 20, flip=True)
    for q in range(2):
        ref = np.argsort(1.0 - s[q].numpy(), kind="stable")[:20]
        np.testing.assert_array_equal(oi[q].cpu().numpy(), ref)


@pytest.mark.parametrize("method", ["lsh", "euclid_lsh", "minhash"])
def test_direct_set_row_and_query_match_batch_paths(method):
    """latency paths (csrc/hip/lsh.hip: signatures from kernel arguments into
    table slots; query signature + fused top-k into pinned host memory) ==
    the batch paths on the same data"""
    from jubatus_amd.models.recommender import NearestNeighbor
    conv = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin",
                              "global_weight": "bin"}],
            "num_rules": [{"key": "*", "type": "num"}]}
    a = NearestNeighbor(method, {"hash_num": 128}, DatumToFvConverter(conv), dev())
    b = NearestNeighbor(method, {"hash_num": 128}, DatumToFvConverter(conv), dev())
    import random as _r
    rng = _r.Random(3)
    rows_ = [(f"r{i}", {"s": f"t{rng.randrange(30)}", "x": rng.gauss(0, 1), "y": float(i % 7)})
             for i in range(400)]
    for rid, d in rows_:
        a.set_row(rid, d)                       # direct path, one launch per row
    b.set_rows(rows_)                           # bulk path
    na = a.rows.nslots
    assert na == b.rows.nslots
    ba = a.index.bits[:na].cpu().numpy()
    bb = b.index.bits[:na].cpu().numpy()
    sa = [a.rows.slot(r) for r, _ in rows_]
    sb = [b.rows.slot(r) for r, _ in rows_]
    assert (ba[sa] == bb[sb]).all()
    for q in ({"s": "t3", "x": 0.1, "y": 2.0}, {"x": -1.0}):
        ra = a.similar_row_from_datum(q, 10)    # direct query
        fv = a.fv_of(__import__("jubatus_amd.fv_converter.datum", fromlist=["as_datum"]).as_datum(q))
        rb = a.query_fv(fv, 10, True)           # batch query path
        assert [s for _, s in ra] == pytest.approx([s for _, s in rb], rel=1e-5, abs=1e-6)
        assert [r for r, _ in ra] == [r for r, _ in rb]


@pytest.mark.parametrize("case,k", [("random", 1), ("random", 10), ("random", 100),
                                    ("random", 128), ("ties", 10), ("sparse_valid", 20)])
def test_direct_topk_sampled_path(case, k):
    """latency top-k on large tables (sampled threshold -> collect -> exact
    final, csrc/hip/topk.hip) == full distance matrix + stable sort; "ties"
    (every row at the same distance: the candidate buffer overflows) and
    "sparse_valid" (fewer valid rows than k would need) exercise the retry /
    +inf-threshold paths"""
    import torch
    from jubatus_amd.ops import hip
    d = dev()
    n = 2_200_000
    g = torch.Generator().manual_seed(k + len(case))
    tb = torch.randint(-2**62, 2**62, (n, 1), generator=g, dtype=torch.int64)
    tn = torch.rand(n, generator=g)
    valid = torch.ones(n, dtype=torch.uint8)
    if case == "ties":
        tb[:] = 12345
        tn[:] = 0.5
    if case == "sparse_valid":
        valid[:] = 0
        valid[::220000] = 1
    qb = tb[:2].clone()
    qb[1] ^= 0x5555
    qn = tn[:2].clone()
    tbd, tnd, vd, qbd, qnd = (x.to(d) for x in (tb, tn, valid, qb, qn))
    bufs = hip.DirectQueryBuffers(d, 1)
    od, oi = hip.topk_rows_direct(qbd, qnd, 2, tbd, tnd, vd, n, 64, 1, k, bufs)
    full = torch.empty((2, n), dtype=torch.float32, device=d)
    hip.hamming_scan(qbd, qnd, 2, tbd, tnd, vd, n, 64, 1, full)
    full = full.cpu().numpy()
    for q in range(2):
        order = np.argsort(full[q], kind="stable")[:k]
        ref = full[q][order]
        fin = np.isfinite(ref)
        np.testing.assert_array_equal(oi[q][:fin.sum()], order[fin])
        np.testing.assert_allclose(od[q][:fin.sum()], ref[fin], rtol=1e-6)
        assert np.all(np.isinf(od[q][fin.sum():]))


@pytest.mark.parametrize("euclid", [False, True])
def test_device_pool_updates_removals_compaction_match_host(euclid):
    """HBM row pool (csrc/hip/sparse_pool.hip): in-place updates, removals,
    a compaction, and batched queries (up to 8 per pass) == the host oracle"""
    from jubatus_amd.models.similarity import InvertedIndex
    g = InvertedIndex(euclid, dev())
    c = InvertedIndex(euclid, None)
    rs = rows(400, seed=5)
    g.set_rows(range(400), rs)
    c.set_rows(range(400), rs)
    upd = rows(120, seed=6)
    for j, s in enumerate(range(0, 360, 3)):       # rewrite every 3rd row
        g.set_rows([s], [upd[j]])
        c.set_rows([s], [upd[j]])
    for s in (7, 8, 9, 250):
        g.remove(s)
        c.remove(s)
    assert g.pool.end > g.pool.live
    g.pool.compact()
    assert g.pool.end == g.pool.live
    qs = [rs[i] for i in range(11)] + [upd[3]]
    a = g.query(qs, 400, 10, similar=False)
    b = c.query(qs, 400, 10, similar=False)
    for x, y in zip(a, b):
        np.testing.assert_allclose([d for _, d in x], [d for _, d in y], rtol=1e-4, atol=1e-4)
    for q in qs[:3]:
        np.testing.assert_allclose(g.scores(q, 400), c.scores(q, 400), rtol=1e-4, atol=1e-4)
    ids = [0, 1, 2, 300, 301]
    a = g.query_slots(ids, 400, 5, similar=True)
    b = c.query_slots(ids, 400, 5, similar=True)
    for x, y in zip(a, b):
        np.testing.assert_allclose([d for _, d in x], [d for _, d in y], rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("euclid", [False, True])
@pytest.mark.parametrize("k", [1, 10, 31, 128])
def test_pool_direct_query_radix_topk_matches_exact(euclid, k):
    """the latency path (query in the kernel arguments, then the two-level
    radix-select top-k into pinned memory, csrc/hip/topk.hip) on a table
    large enough to take it == the exact top-k of the scan's own scores, for
    CSR queries and stored-row (slot) queries, 1 and several at once"""
    import torch
    from jubatus_amd.models.similarity import InvertedIndex
    from jubatus_amd.ops import hip
    n = 40000
    g = InvertedIndex(euclid, dev())
    rs = rows(n, seed=11)
    g.set_rows(range(n), rs)
    for s in range(0, n, 97):
        g.remove(s)
    qs = [rs[5], rows(1, seed=12)[0], rs[777]]
    for nq in (1, 3):
        rp, idx, val = __import__("jubatus_amd.models.similarity", fromlist=["_rows_to_csr"])._rows_to_csr(qs[:nq])
        got = g.query_direct(idx.astype(np.int32), val, rp, nq, n, k, similar=False)
        ref = g._query_batches(lambda a, b: g._queries_device(qs[a:b]), nq, n, k, similar=False)
        for x, y in zip(got, ref):
            assert [i for i, _ in x] == [i for i, _ in y]
            np.testing.assert_allclose([d for _, d in x], [d for _, d in y], rtol=1e-6)
        # the scan's scores themselves, against torch.topk
        sc = g.scores_device(qs[0], n)
        dist = sc if euclid else (1.0 - sc)
        dist = torch.where(torch.isfinite(sc), dist, torch.full_like(dist, float("inf")))
        tv, ti = torch.topk(dist, k, largest=False, sorted=True)
        np.testing.assert_allclose([d for _, d in got[0]], tv.cpu().numpy(), rtol=1e-6)
    a = g.query_slots([5, 777], n, k, similar=True)
    b = g._query_batches(lambda x, y: g.pool.query_slots_device([5, 777][x:y]), 2, n, k, True)
    for x, y in zip(a, b):
        assert [i for i, _ in x] == [i for i, _ in y]
    assert hip.TOPK_MAX_K >= k


@pytest.mark.parametrize("k", [1, 10, 37])
def test_topk_16_wave_path_matches_full_sort(k):
    """nq 1 over >= 2M rows takes the 16-wave scan blocks (topk.hip
    scan_waves); heavy ties (hash_num 16: 17 distinct distances) must still
    give the stable (distance, row) order of a full sort"""
    import torch
    from jubatus_amd.ops import hip
    n = 2_200_000
    d = dev()
    g = torch.Generator(device=d).manual_seed(k)
    tb = torch.randint(0, 1 << 16, (n, 1), generator=g, device=d, dtype=torch.int64)
    tn = torch.ones(n, dtype=torch.float32, device=d)
    valid = (torch.rand(n, generator=g, device=d) > 0.01).to(torch.uint8)
    qb = torch.randint(0, 1 << 16, (1, 1), generator=g, device=d, dtype=torch.int64)
    qn = torch.ones(1, dtype=torch.float32, device=d)
    dist, row = hip.topk_hamming(qb, qn, 1, tb, tn, valid, n, 16, 0, k)
    x = (tb[:, 0] ^ qb[0, 0]).cpu().numpy().astype(np.uint64)
    ham = np.unpackbits(x.view(np.uint8).reshape(-1, 8)[:, :2], axis=1).sum(1)
    ref = np.where(valid.cpu().numpy() > 0, ham / 16.0, np.inf)
    order = np.argsort(ref, kind="stable")[:k]
    assert row[0].cpu().numpy().tolist() == order.tolist()
    np.testing.assert_allclose(dist[0].cpu().numpy(), ref[order], rtol=1e-6)


@pytest.mark.parametrize("case,k,nq,metric", [("random", 1, 1, 1), ("random", 10, 1, 1),
                                              ("random", 100, 2, 1), ("random", 10, 8, 1),
                                              ("random", 10, 3, 0), ("ties", 10, 2, 1),
                                              ("ties", 100, 1, 1), ("sparse_valid", 20, 2, 1),
                                              ("levels", 10, 4, 0), ("levels", 31, 2, 2)])
@pytest.mark.parametrize("path", [-1, 2, 3, 4])
def test_direct_topk_one_launch_path(case, k, nq, metric, path):
    """latency top-k below the sampled path's 2M rows: ONE launch
    (csrc/hip/topk.hip topk_fused_kernel: distances cached in LDS, two radix
    levels across grid barriers, last-block selection) == full distance
    matrix + stable sort; also the default choice (-1) and the one-pass
    kernel (3, topk_onepass_kernel: register lists, last-block merge; k <= 16
    only) and the LDS radix-select kernel (4, topk_select_kernel: per-block
    exact top-k over (distance, row) composites, last-block select). "ties" (every row at one distance: the candidates
    overflow the LDS ranking and k > 16 retries on the tile path, k <= 16
    selects from L2), "levels" (8 distinct signatures: ~125k rows per
    distance level) and "sparse_valid" (fewer valid rows than k)"""
    import torch
    from jubatus_amd.ops import hip
    if path == 3 and k > 16:
        pytest.skip("the one-pass kernel takes k <= 16")
    d = dev()
    n = 1_000_000
    g = torch.Generator().manual_seed(k + nq + len(case) + metric)
    tb = torch.randint(-2**62, 2**62, (n, 1), generator=g, dtype=torch.int64)
    tn = torch.rand(n, generator=g)
    valid = torch.ones(n, dtype=torch.uint8)
    if case == "ties":
        tb[:] = 12345
        tn[:] = 0.5
    if case == "levels":
        pool = torch.randint(-2**62, 2**62, (8, 1), generator=g, dtype=torch.int64)
        tb = pool[torch.randint(0, 8, (n,), generator=g)]
    if case == "sparse_valid":
        valid[:] = 0
        valid[::110000] = 1
    qb = tb[:nq].clone()
    qb[-1] ^= 0x5555
    qn = tn[:nq].clone()
    tbd, tnd, vd, qbd, qnd = (x.to(d) for x in (tb, tn, valid, qb, qn))
    bufs = hip.DirectQueryBuffers(d, 1)
    full = torch.empty((nq, n), dtype=torch.float32, device=d)
    hip.hamming_scan(qbd, qnd, nq, tbd, tnd, vd, n, 64, metric, full)
    full = full.cpu().numpy()
    for rep in range(2):                 # the second call checks the state the first left behind
        od, oi = hip.topk_rows_direct(qbd, qnd, nq, tbd, tnd, vd, n, 64, metric, k, bufs, path=path)
        for q in range(nq):
            order = np.argsort(full[q], kind="stable")[:k]
            ref = full[q][order]
            fin = np.isfinite(ref)
            np.testing.assert_array_equal(oi[q][:fin.sum()], order[fin])
            np.testing.assert_allclose(od[q][:fin.sum()], ref[fin], rtol=1e-6)
            assert np.all(np.isinf(od[q][fin.sum():]))


@pytest.mark.parametrize("n,k", [(1000, 100), (300, 7), (50, 64), (2000, 33)])
def test_argmin_rows_first_minimum(n, k):
    """csrc/hip/clustering.hip argmin (a thread a row below 32 columns, a
    wave a row past that) == numpy's first minimum, ties included"""
    import numpy as np
    import torch
    from jubatus_amd.ops import hip
    rng = np.random.default_rng(n + k)
    D = rng.integers(0, 6, size=(n, k)).astype(np.float32)   # many ties
    got = hip.argmin_rows(torch.from_numpy(D).to(dev())).cpu().numpy()
    assert (got == D.argmin(1)).all()
