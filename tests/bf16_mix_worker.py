"""Rank worker of tests/test_gpu_bf16.py::test_hbm_sized_bf16_table_trains_and_mixes_two_ranks
(launched by torch.distributed.run; both ranks on cuda:0 over gloo)."""
import hashlib
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist

    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier

    dist.init_process_group("gloo")
    rank = dist.get_rank()
    dev = torch.device("cuda", 0)
    conv = DatumToFvConverter({
        "string_rules": [{"key": "*", "type": "str", "sample_weight": "bin", "global_weight": "bin"}],
        "num_rules": [{"key": "*", "type": "num"}],
        "hash_max_size": 1 << 26,
    })
    clf = LinearClassifier("AROW", {"regularization_weight": 1.0}, conv, device=dev,
                           concurrent_update="atomic", weight_dtype="bf16")
    rng = random.Random(100 + rank)

    def sample(y):
        d = {f"s{j}": f"w{y}_{rng.randrange(3)}" if rng.random() < 0.8 else f"r{rng.randrange(10 ** 6)}"
             for j in range(4)}
        d["n0"] = (y % 7) * 0.3 + rng.gauss(0, 0.5)
        return (f"L{y}", d)

    # 40 labels known on both ranks in the same order (label capacity 64),
    # then each rank trains its own requests
    for y in range(40):
        clf.train([sample(y)])
    data = [sample(rng.randrange(40)) for _ in range(20000)]
    clf.train(data)
    clf.synchronize()
    nbytes = clf.mix()
    clf.synchronize()
    st = clf._last_mix
    # every row either rank wrote is now the same on both ranks
    W = clf.W.view(torch.int16)
    nz = torch.nonzero((W != 0).any(dim=1)).flatten()
    rows = torch.zeros(clf.H, dtype=torch.uint8, device=dev)
    rows[nz] = 1
    dist.all_reduce(rows, op=dist.ReduceOp.MAX)
    sel = torch.nonzero(rows).flatten()
    mine = clf.W.index_select(0, sel).float().cpu().numpy()
    digest = hashlib.sha256(mine.tobytes()).hexdigest()
    other = [None, None]
    dist.all_gather_object(other, digest)
    test = [sample(rng.randrange(40)) for _ in range(2000)]
    pred = [max(r, key=lambda t: t[1])[0] for r in clf.classify([d for _, d in test])]
    acc = sum(p == l for p, (l, _) in zip(pred, test)) / len(test)
    print(json.dumps({"rank": rank, "LC": clf.LC, "H": clf.H, "w_bytes": clf.W.numel() * clf.W.element_size(),
                      "mix": st, "mix_bytes": nbytes, "rows_equal": other[0] == other[1],
                      "digest": digest, "acc": acc}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
