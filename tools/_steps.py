import os, random, sys, time
sys.path.insert(0, os.getcwd())
import bench, torch, numpy as np
from jubatus_amd.fv_converter.converter import DatumToFvConverter
from jubatus_amd.models.classifier import LinearClassifier
from jubatus_amd.ops.feature_pipeline import RequestArena
dev = torch.device("cuda", 0)
cfg = dict(bench.AROW_CONFIG); cfg["converter"] = dict(cfg["converter"], hash_max_size=1 << 20)
clf = LinearClassifier("AROW", cfg["parameter"], DatumToFvConverter(cfg["converter"]), dev)
for y in range(16): clf.set_label(f"label{y}")
pools = []
for i in range(4):
    bodies = bench.make_requests(random.Random(i), 1024, 128, 16, 8, 8, 100000)
    a = RequestArena(sum(len(b) for b in bodies) + 16 * 1024 + 64)
    for b in bodies: a.append(b)
    pools.append((a,) + a.spans())
for i in range(5): clf.train_arena(*pools[i % 4])
clf.synchronize()
for mode in ("gpu", "gpu1"):
    clf.gpu_scan = True
    for i in range(3): clf.train_arena(*pools[i % 4])
    clf.synchronize()
    evs = []; hs = []
    t0 = time.perf_counter()
    for i in range(40):
        h0 = time.perf_counter()
        clf.train_arena(*pools[0 if mode == "gpu1" else i % 4])
        hs.append(time.perf_counter() - h0)
        e = torch.cuda.Event(enable_timing=True); e.record(); evs.append(e)
    clf.synchronize(); wall = (time.perf_counter() - t0) / 40
    d = np.array([evs[i].elapsed_time(evs[i + 1]) for i in range(len(evs) - 1)])
    print(f"{mode}: wall {wall*1e3:.3f} ms/step; gpu step p50 {np.median(d):.3f} p90 {np.percentile(d,90):.3f} max {d.max():.3f}; host p50 {np.median(hs)*1e3:.3f} max {max(hs)*1e3:.3f}")
    print("   gpu deltas:", " ".join(f"{x:.2f}" for x in d[:20]))
    print("   host calls:", " ".join(f"{x*1e3:.2f}" for x in hs[1:21]))
