"""Accuracy of concurrent-stream training vs the hot-row replica settings
(merge interval), on the wild-valued data of
tests/test_gpu_linear.py::test_concurrent_streams_learn."""
import json
import os
import sys

import msgpack
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    import torch
    from test_gpu_linear import CONV, _data, _shared_data
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.fv_converter.datum import Datum
    from jubatus_amd.models.classifier import LinearClassifier
    dev = torch.device("cuda", 0)
    for wild in (True, False):
        data = _data(4096, seed=7, wild=wild)
        bodies = [msgpack.packb([[l, Datum(d).to_msgpack()] for l, d in data[i:i + 32]],
                                use_bin_type=False) for i in range(0, len(data), 32)]
        test = _data(500, seed=8, wild=wild)
        for mode in ("atomic", "hogwild"):
            for hot, merge in ((False, 0), (True, 1), (True, 2), (True, 4), (True, 8)):
                g = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(CONV),
                                     device=dev, concurrent_update=mode)
                g.hot_rows = hot
                g.hot_merge = max(1, merge)
                g.train_requests(bodies)
                res = g.classify([d for _, d in test])
                acc = float(np.mean([max(r, key=lambda t: t[1])[0] == l for r, (l, _) in zip(res, test)]))
                W = g.W.cpu().numpy()
                print(json.dumps({"wild": wild, "mode": mode, "hot": hot, "merge": merge, "acc": acc,
                                  "wmax": float(np.abs(W).max()), "stats": g.train_stats()}), flush=True)


if __name__ == "__main__":
    main()
