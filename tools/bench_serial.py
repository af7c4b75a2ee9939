"""Per-batch cost of the serial-equivalent train mode (csrc/hip/serial.hip)
against the atomic mode on the headline bench's data (bench.py FreshStream:
label-correlated AROW requests, 1024 requests x 128 samples per batch).
Every batch is synchronised and timed; one JSON line per (mode, batch
range) with the mean ms per batch and the fraction of samples that updated.

Usage: python tools/bench_serial.py [--batches 60] [--modes exact,atomic]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--modes", default="exact,atomic")
    ap.add_argument("--requests", type=int, default=1024)
    ap.add_argument("--per-request", type=int, default=128)
    ap.add_argument("--worst-case", action="store_true")
    ap.add_argument("--warm", type=int, default=0,
                    help="label-correlated batches trained first (as bench.py's exact records do)")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from jubatus_amd._native import native
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.models.classifier import LinearClassifier

    dev = torch.device("cuda", 0)
    args = argparse.Namespace(requests=a.requests, per_request=a.per_request, labels=16,
                              str_features=8, num_features=8)
    p_corr, vocab = (0.0, (1 << 31) - 1) if a.worst_case else (0.6, 100000)
    t0 = time.perf_counter()
    data = bench.FreshStream(native(), torch, True, args, 12345, a.batches, 16, p_corr, vocab)
    print(f"data {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    for mode in a.modes.split(","):
        cfg = json.loads(json.dumps(bench.AROW_CONFIG))
        cfg["converter"]["hash_max_size"] = 1 << 20
        clf = LinearClassifier("AROW", cfg["parameter"], DatumToFvConverter(cfg["converter"]),
                               device=dev, concurrent_update=mode)
        for y in range(16):
            clf.set_label(f"label{y}")
        if a.warm:
            wd = bench.FreshStream(native(), torch, True, args, 777, a.warm, 16, 0.6, 100000)
            for arena in wd.batches:
                clf.train_arena(arena, np.asarray(arena.offs, np.int64), np.asarray(arena.lens, np.int64))
            clf.synchronize()
            del wd
        times, upd, diag = [], [], []
        sprof = {}
        for b, arena in enumerate(data.batches):
            st0 = clf.train_stats()
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            clf.train_arena(arena, np.asarray(arena.offs, np.int64), np.asarray(arena.lens, np.int64))
            clf.synchronize()
            times.append((time.perf_counter() - t1) * 1e3)
            st1 = clf.train_stats()
            upd.append((st1["updated"] - st0["updated"]) / max(1, st1["trained"] - st0["trained"]))
            if mode == "exact":
                d = clf._serial.last_batch()
                keys = ("segments", "wasted_steps", "refreshes", "committer_updates", "last_segment_rows", "rounds",
                        "exact_rescored", "committed_samples", "windows", "retries", "candidates", "T",
                        "window_len", "saturated_windows", "non_candidates_verified")
                diag.append((d["exact_steps"], (d["end"] - d["tail_start"]) / max(1, d["end"]),
                             {k: v for k, v in d.items() if k.startswith("commit") or k in keys}))
            if os.environ.get("JB_STEPPER_PROF") == "1" and mode == "exact":
                from jubatus_amd.ops import hip as _hip
                sp = _hip.stepper_prof()
                if b >= 2:
                    for k, v in sp.items():
                        sprof[k] = sprof.get(k, 0) + v
            if b % 10 == 9:
                print(f"{mode} batch {b + 1}: {times[-1]:.2f} ms, update fraction {upd[-1]:.4f}"
                      + (f", exact steps {diag[-1][0]}, sequential tail {diag[-1][1]:.3f}, {diag[-1][2]}"
                         if diag else ""), file=sys.stderr, flush=True)
        edges = [0, 5, 20] + list(range(40, len(times) + 1, max(20, len(times) // 10)))
        for lo, hi in zip(edges, edges[1:] + [len(times)]):
            if lo >= len(times) or hi <= lo:
                continue
            rec = {"mode": mode, "batches": [lo, min(hi, len(times))],
                   "ms_per_batch": round(float(np.mean(times[lo:hi])), 3),
                   "update_fraction": round(float(np.mean(upd[lo:hi])), 5),
                   "samples_per_batch": a.requests * a.per_request, "worst_case": a.worst_case}
            if diag:
                rec["exact_steps"] = round(float(np.mean([x[0] for x in diag[lo:hi]])), 1)
                rec["sequential_tail_fraction"] = round(float(np.mean([x[1] for x in diag[lo:hi]])), 4)
                for key in diag[lo][2]:
                    rec[key] = round(float(np.mean([x[2].get(key, 0) for x in diag[lo:hi]])), 1)
            print(json.dumps(rec), flush=True)
        if sprof:
            # stepper wave phases over batches 2+ (shader cycles; per sample)
            ns = max(1, sprof.get("samples", 1))
            counts = ("samples", "stages", "misses", "direct", "lk_iters")
            print(json.dumps({"mode": mode, "stepper_prof": sprof,
                              "cycles_per_sample": {k: round(v / ns, 1) for k, v in sprof.items()
                                                    if k not in counts}}),
                  flush=True)
        del clf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
