"""The served train path against its RPC layer alone: the native
jubaclassifier under bench.py's served load (jubaloadgen, 64 connections x 32
in flight, 128-sample requests, fresh values), once training and once with
JB_RPC_NULL_TRAIN=1 (every request answered without training: loopback TCP,
msgpack framing and the copies into the pinned arena only). The second run is
the ceiling any training path behind this RPC layer can reach on this host,
and the CPUs it takes; both records carry the server's CPUs per thread name.

Usage: python tools/rpc_ceiling.py [--rpc-seconds 4] > out.json
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from jubatus_amd._native import native
    ap = argparse.ArgumentParser()
    ap.add_argument("--rpc-seconds", type=float, default=4.0)
    ap.add_argument("--update-mode", default="atomic")
    ap.add_argument("--learning-exact", action="store_true",
                    help="only bench.py's learning_stream_exact record (exact mode, 2 %% noise tokens)")
    a = ap.parse_args()
    args = argparse.Namespace(rpc_seconds=a.rpc_seconds, rpc_conns=64, rpc_depth=32, rpc_threads=32,
                              rpc_distinct=512, rpc_fresh=1, per_request=128, labels=16, str_features=8,
                              num_features=8, vocab=100000, hash_bits=20, update_mode=a.update_mode)
    nat = native()
    if a.learning_exact:
        print(json.dumps(bench.served_train_native(args, 0, nat, mode="exact", noise_pm=20, classify=False)),
              flush=True)
        return
    out = {"trained": bench.served_train_native(args, 0, nat, classify=False)}
    os.environ["JB_RPC_NULL_TRAIN"] = "1"
    try:
        out["rpc_only"] = bench.served_train_native(args, 0, nat, classify=False)
    finally:
        del os.environ["JB_RPC_NULL_TRAIN"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
