"""bench.py's engine records alone (native row servers and clustering over
RPC, one GPU), without the headline training run: prints one JSON line.

Usage: python tools/bench_engine_records.py [--engines anomaly_lof,clustering_gmm] [bench.py flags...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    ap = bench.build_parser() if hasattr(bench, "build_parser") else None
    if ap is None:
        import argparse
        # bench.main builds its parser inline: parse the flags it knows by
        # running its parser construction on a copy of argv
        ap = argparse.ArgumentParser()
        ap.add_argument("--engines", default="all")
        ap.add_argument("--engine-rows", type=int, default=1_000_000)
        ap.add_argument("--lof-rows", type=int, default=100_000)
        ap.add_argument("--engine-seconds", type=float, default=3.0)
        ap.add_argument("--cluster-points", type=int, default=200_000)
    args = ap.parse_args()
    out = bench.engine_records(args, 0)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
