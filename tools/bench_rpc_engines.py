"""The engine records of bench.py alone (native row / clustering servers over
RPC, no headline run): one JSON line. Same cases and fields as the
`engines` block of bench.py's output (bench.py engine_records)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engines", default="all", help="comma-separated case names (bench.ENGINE_CASES, "
                    "clustering_kmeans, clustering_gmm) or all")
    ap.add_argument("--engine-rows", type=int, default=1_000_000)
    ap.add_argument("--lof-rows", type=int, default=100_000)
    ap.add_argument("--engine-seconds", type=float, default=3.0)
    ap.add_argument("--cluster-points", type=int, default=200_000)
    a = ap.parse_args()
    print(json.dumps(bench.engine_records(a, 0)), flush=True)


if __name__ == "__main__":
    main()
