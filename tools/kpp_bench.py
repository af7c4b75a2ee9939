"""k-means++ kernel timing per call (csrc/hip/clustering.hip through ops/hip.kmeanspp): n points x d dims, m draws.
Usage: python tools/kpp_bench.py (JB_KMEANSPP_WAVE=1 / JB_KMEANSPP_BLOCK=1 for the other kernels)"""
import os, sys, torch, numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from jubatus_amd.ops import hip
d = torch.device("cuda", 0)
def run(n, dd, m, it=50):
    rng = np.random.default_rng(0)
    X = torch.from_numpy((rng.standard_normal((n, dd)) * 3).astype(np.float32)).to(d)
    w = torch.from_numpy((rng.random(n) + 0.25).astype(np.float32)).to(d)
    u = list(rng.random(m))
    for _ in range(3): hip.kmeanspp(X, w, u, m)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): hip.kmeanspp(X, w, u, m)
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it
for n, dd in ((1000, 10), (200, 10), (1000, 1), (1000, 32)):
    for m in (1, 10, 100):
        print(os.environ.get("JB_KMEANSPP_WAVE", "blk"), n, dd, m, round(run(n, dd, m), 1), "us", flush=True)
