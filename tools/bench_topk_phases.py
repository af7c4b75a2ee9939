"""Phase breakdown of the one-pass top-k kernel (csrc/hip/topk.hip
topk_onepass_kernel, path 3) from its realtime stamps (100 MHz): per block,
start -> rows done -> block pop -> published; the last block adds the merge
loads, the final pop and the end. Random 64-bit signatures at 1M rows
(euclid_lsh), one query, k = 10. One JSON line: medians over iterations of
the per-launch spans in microseconds."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from jubatus_amd.ops import hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--mode", choices=("lsh", "scores"), default="lsh")
    a = ap.parse_args()
    d = torch.device("cuda", 0)
    n, k = a.rows, a.k
    g = torch.Generator().manual_seed(0)
    blocks = (n + 2047) // 2048
    prof = torch.zeros(blocks * 8 * 4, dtype=torch.int64, device=d)
    bufs = hip.DirectQueryBuffers(d, 1)
    if a.mode == "lsh":
        tb = torch.randint(-2**62, 2**62, (n, 1), generator=g, dtype=torch.int64).to(d)
        tn = torch.rand(n, generator=g).to(d)
        valid = torch.ones(n, dtype=torch.uint8, device=d)
        qb, qn = tb[:1].clone(), tn[:1].clone()
        call = lambda: hip.topk_rows_direct(qb, qn, 1, tb, tn, valid, n, 64, 1, k, bufs, path=3)  # noqa: E731
    else:
        sc = (torch.rand(1, n, generator=g) * (torch.rand(1, n, generator=g) < 0.01)).to(d)
        call = lambda: hip.topk_scores_direct(sc, 1, n, k, True, bufs, path=3)  # noqa: E731
    spans = {x: [] for x in ("rows", "pop", "publish", "blocks_spread", "merge_loads", "final_pop",
                             "end", "total")}
    for it in range(a.iters + 5):
        prof.zero_()
        torch.cuda.synchronize()
        hip._fn("jb_topk_set_prof")(hip._p(prof))
        call()
        hip._fn("jb_topk_set_prof")(None)
        torch.cuda.synchronize()
        if it < 5:
            continue
        p = prof.view(-1, 8).cpu().numpy()
        live = p[:, 0] > 0
        p = p[live]
        t0 = p[:, 0].min()
        last = p[p[:, 6] > 0]
        if len(last) != 1:
            continue
        spans["rows"].append(np.median(p[:, 1] - p[:, 0]) / 100)
        spans["pop"].append(np.median(p[:, 2] - p[:, 1]) / 100)
        spans["publish"].append(np.median(p[:, 3] - p[:, 2]) / 100)
        spans["blocks_spread"].append((p[:, 3].max() - t0) / 100)
        L = last[0]
        spans["merge_loads"].append((L[4] - L[3]) / 100)
        spans["final_pop"].append((L[5] - L[4]) / 100)
        spans["end"].append((L[6] - L[5]) / 100)
        spans["total"].append((L[6] - t0) / 100)
    print(json.dumps({"rows": n, "k": k, "mode": a.mode, "blocks": int(live.sum()),
                      **{f"{x}_us": round(float(np.median(v)), 2) for x, v in spans.items() if v}}), flush=True)


if __name__ == "__main__":
    main()
