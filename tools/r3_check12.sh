#!/bin/bash
# native vs in-process clustering push throughput
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_clustering.py --native --method kmeans > gpurun_out/r3_cluster_native.jsonl 2>gpurun_out/r3_cluster_native.err &&
timeout -k 10 200 python tools/bench_clustering.py --native --method gmm >> gpurun_out/r3_cluster_native.jsonl 2>>gpurun_out/r3_cluster_native.err
