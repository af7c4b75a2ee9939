"""Score-vector top-k of the inverted-index / LOF query tail
(csrc/hip/topk.hip jb_topk_scores_direct: fused radix levels with a
last-block select, collect, rank) against a float64 NumPy oracle ordered by
(distance, row). Covers continuous scores, heavy ties (quantized scores,
thousands of rows at the threshold), fewer nonzero rows than k and several
queries per call."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _oracle(sc, k, flip):
    d = (1.0 - sc.astype(np.float64)) if flip else sc.astype(np.float64)
    d32 = d.astype(np.float32)
    order = np.lexsort((np.arange(d32.size), d32))[:k]
    return d32[order], order.astype(np.int32)


@pytest.mark.parametrize("frac,levels", [(0.01, 0), (0.2, 0), (0.2, 64), (0.00001, 0)])
@pytest.mark.parametrize("nq", [1, 3])
@pytest.mark.parametrize("path", [-1, 1, 2, 3, 4])
def test_scores_topk_matches_oracle(frac, levels, nq, path):
    from jubatus_amd.ops import hip
    dev = torch.device("cuda", 0)
    rows, k = 200_000, 10
    rng = np.random.default_rng(int(frac * 1e5) + levels + nq)
    sc = np.zeros((nq, rows), np.float32)
    for q in range(nq):
        m = rng.random(rows) < frac
        v = rng.random(rows).astype(np.float32)
        if levels:
            v = np.ceil(v * levels) / levels
        sc[q, m] = v[m]
    bufs = hip.DirectQueryBuffers(dev, 1)
    dist, idx = hip.topk_scores_direct(torch.from_numpy(sc).to(dev), nq, rows, k, True, bufs, path=path)
    for q in range(nq):
        rd, ri = _oracle(sc[q], k, True)
        np.testing.assert_allclose(dist[q], rd, atol=1e-6)
        np.testing.assert_array_equal(idx[q], ri)


def test_scores_topk_repeated_calls_reset_counters():
    """the per-level finished-block counters and histograms are zeroed per
    call: back-to-back calls on different vectors stay exact"""
    from jubatus_amd.ops import hip
    dev = torch.device("cuda", 0)
    rows, k = 100_000, 7
    bufs = hip.DirectQueryBuffers(dev, 1)
    rng = np.random.default_rng(5)
    for _ in range(20):
        sc = (rng.random(rows) * (rng.random(rows) < 0.05)).astype(np.float32)[None]
        dist, idx = hip.topk_scores_direct(torch.from_numpy(sc).to(dev), 1, rows, k, False, bufs)
        rd, ri = _oracle(sc[0], k, False)
        np.testing.assert_allclose(dist[0], rd, atol=1e-6)
        np.testing.assert_array_equal(idx[0], ri)


@pytest.mark.parametrize("k,path", [(16, -1), (20, -1), (16, 2), (20, 2), (16, 3), (20, 4), (100, 4)])
def test_scores_topk_ties_list_and_rank_paths(k, path):
    """~1000 rows tied at the threshold: k <= 16 merges register lists, larger
    k ranks the candidates (early exit once a candidate is out of the top k)"""
    from jubatus_amd.ops import hip
    dev = torch.device("cuda", 0)
    rows = 300_000
    rng = np.random.default_rng(k)
    sc = np.zeros((1, rows), np.float32)
    m = rng.random(rows) < 0.2
    sc[0, m] = np.ceil(rng.random(rows)[m] * 60) / 60
    bufs = hip.DirectQueryBuffers(dev, 1)
    dist, idx = hip.topk_scores_direct(torch.from_numpy(sc).to(dev), 1, rows, k, True, bufs, path=path)
    rd, ri = _oracle(sc[0], k, True)
    np.testing.assert_allclose(dist[0], rd, atol=1e-6)
    np.testing.assert_array_equal(idx[0], ri)
