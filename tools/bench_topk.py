"""Micro-benchmark of the similarity scan kernels (1 GPU): full hamming_scan
(distance matrix) vs fused scan + top-k (topk.hip) at various N, k, nq."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jubatus_amd.ops import hip  # noqa: E402


def timeit(fn, iters=30):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / iters, 2)


def main():
    d = torch.device("cuda", 0)
    g = torch.Generator(device=d).manual_seed(0)
    out = {}
    for nrows in (100_000, 1_000_000, 10_000_000):
        tb = torch.randint(-2**62, 2**62, (nrows, 1), device=d, dtype=torch.int64, generator=g)
        tn = torch.rand(nrows, device=d, generator=g)
        valid = torch.ones(nrows, dtype=torch.uint8, device=d)
        for nq in (1, 8):
            qb = tb[:nq].clone()
            qn = tn[:nq].clone()
            full = torch.empty((nq, nrows), dtype=torch.float32, device=d)
            out[f"scan_full_N{nrows}_q{nq}_us"] = timeit(
                lambda: hip.hamming_scan(qb, qn, nq, tb, tn, valid, nrows, 64, 1, full))
            for k in (1, 10, 100):
                out[f"topk_N{nrows}_q{nq}_k{k}_us"] = timeit(
                    lambda: hip.topk_hamming(qb, qn, nq, tb, tn, valid, nrows, 64, 1, k))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
