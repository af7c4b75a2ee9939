"""Bulk row ingest (RowEngine.set_rows / MIX put_diff / load): native
hashing of every datum in one pass + one index insert == row-by-row set_row."""
import random

import pytest

from jubatus_amd.fv_converter.converter import DatumToFvConverter
from jubatus_amd.models.recommender import NearestNeighbor, Recommender

CONV = {"string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
        "num_rules": [{"key": "*", "type": "num"}]}


def _rows(n, seed=0):
    rng = random.Random(seed)
    return [(f"r{i % (n - 3)}", {"a": f"t{rng.randrange(20)}", "x": rng.gauss(0, 1),
                                 "y": float(rng.randrange(5))}) for i in range(n)]


@pytest.mark.parametrize("method", ["lsh", "euclid_lsh", "minhash", "inverted_index",
                                    "inverted_index_euclid"])
def test_bulk_equals_sequential(method):
    rows = _rows(120)                       # includes 3 ids written twice
    cls = Recommender if method.startswith("inverted") else NearestNeighbor
    a = cls(method, {"hash_num": 64}, DatumToFvConverter(CONV))
    b = cls(method, {"hash_num": 64}, DatumToFvConverter(CONV))
    for rid, d in rows:
        a.set_row(rid, d) if cls is NearestNeighbor else a.update_row(rid, d)
    if cls is NearestNeighbor:
        assert b.set_rows(rows) == len(rows)
    else:
        # update_row merges into an existing row; bulk set of the merged rows
        b.set_rows([(rid, a.decode_row(rid)) for rid in a.get_all_rows()])
    assert sorted(a.get_all_rows()) == sorted(b.get_all_rows())
    q = {"a": "t3", "x": 0.5, "y": 2.0}
    ra = a.similar_row_from_datum(q, 10)
    rb = b.similar_row_from_datum(q, 10)
    assert [round(s, 5) for _, s in ra] == [round(s, 5) for _, s in rb]


def test_put_diff_uses_bulk_and_matches():
    src = NearestNeighbor("euclid_lsh", {"hash_num": 64}, DatumToFvConverter(CONV))
    src.set_rows(_rows(60, seed=1))
    diff = src.get_diff()
    dst = NearestNeighbor("euclid_lsh", {"hash_num": 64}, DatumToFvConverter(CONV))
    dst.put_diff(diff)
    assert sorted(dst.get_all_rows()) == sorted(src.get_all_rows())
    q = {"a": "t1", "x": 0.0}
    assert src.similar_row_from_datum(q, 5) == dst.similar_row_from_datum(q, 5)
