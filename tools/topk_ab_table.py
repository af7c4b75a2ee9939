"""Markdown A/B table of tools/bench_topk_mq.py runs (JB_TOPK_MQ=0 vs the
default) plus, optionally, a rocprofv3 kernel-stats CSV of the quick run.

Usage: python tools/topk_ab_table.py OFF.jsonl ON.jsonl [KERNEL_STATS.csv] > OUT.md
"""
import csv
import json
import sys


def rows(path):
    out = {}
    for line in open(path):
        if line.startswith("{"):
            r = json.loads(line)
            out[(r["bits"], r["metric"], r["nq"], r["k"])] = r
    return out


def main():
    off, on = rows(sys.argv[1]), rows(sys.argv[2])
    metric = {0: "lsh", 1: "euclid_lsh", 2: "minhash"}
    print("| bits | metric | queries | k | previous kernels us | r5 us | speed-up | table GB/s (r5) |")
    print("|---:|---|---:|---:|---:|---:|---:|---:|")
    for key in sorted(on):
        o, n = off.get(key), on[key]
        if not o:
            continue
        print(f"| {key[0]} | {metric[key[1]]} | {key[2]} | {key[3]} | {o['us']:.1f} | {n['us']:.1f} | "
              f"{o['us'] / n['us']:.2f}x | {n['table_GBps']:.0f} |")
    if len(sys.argv) > 3:
        print()
        print("Kernels of the quick run (64-bit table, 1 and 8 queries, k 10; rocprofv3 --kernel-trace --stats):")
        print()
        print("| kernel | calls | mean us |")
        print("|---|---:|---:|")
        for r in csv.DictReader(open(sys.argv[3])):
            name = r["Name"].replace("void ", "").split("(")[0]
            if "jb::" not in name:
                continue
            print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} |")


if __name__ == "__main__":
    main()
