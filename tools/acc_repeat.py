"""Accuracy spread of tests/test_gpu_linear.py::test_concurrent_streams_learn
(atomic mode, 1e6-valued features) over repeated runs on one GPU."""
import importlib.util
import json
import os
import sys

import msgpack
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
spec = importlib.util.spec_from_file_location("tgl", os.path.join(ROOT, "tests", "test_gpu_linear.py"))
m = importlib.util.module_from_spec(spec)
spec.loader.exec_module(m)
from jubatus_amd.fv_converter.converter import DatumToFvConverter  # noqa: E402
from jubatus_amd.fv_converter.datum import Datum  # noqa: E402
from jubatus_amd.models.classifier import LinearClassifier  # noqa: E402

accs = []
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    g = LinearClassifier("AROW", {"regularization_weight": 1.0}, DatumToFvConverter(m.CONV),
                         device=m._device(), concurrent_update="atomic")
    data = m._data(4096, seed=7, wild=True)
    bodies = [msgpack.packb([[l, Datum(d).to_msgpack()] for l, d in data[i:i + 32]], use_bin_type=False)
              for i in range(0, len(data), 32)]
    g.train_requests(bodies)
    test = m._data(500, seed=8, wild=True)
    res = g.classify([d for _, d in test])
    accs.append(float(np.mean([max(r, key=lambda t: t[1])[0] == l for r, (l, _) in zip(res, test)])))
print(json.dumps({"lib": os.environ.get("JUBATUS_HIP_LIB", "libjubatus_hip.so"), "accs": accs,
                  "min": min(accs), "mean": round(float(np.mean(accs)), 4)}), flush=True)
