"""Summarise a `rocprofv3 --marker-trace --kernel-trace` run (rocpd SQLite
output, one database per traced process) into a markdown table: the roctx
ranges the framework emits behind JUBATUS_ROCTX=1 (csrc/native/jb_roctx.hpp,
ops/hip.py) - count, total, p50 / p99 per range name - and the busiest
kernels beside them.

Usage: python tools/roctx_table.py <rocprofv3 output dir> [--top 15] > table.md
"""
import argparse
import glob
import json
import os
import sqlite3
import sys


def _pct(v, q):
    if not v:
        return 0.0
    v = sorted(v)
    return v[min(len(v) - 1, int(q * len(v)))]


def collect(paths):
    ranges, kernels = {}, {}
    procs = 0
    for p in paths:
        c = sqlite3.connect(p)
        names = {r[0] for r in c.execute("select name from sqlite_master where type in ('table', 'view')")}
        procs += 1
        if "regions" in names:
            for name, dur, ext in c.execute("select name, duration, extdata from regions where duration is not null"):
                try:   # the roctx message (the region's name is the marker API call)
                    name = json.loads(ext).get("message", name)
                except (TypeError, ValueError):
                    pass
                ranges.setdefault(name, []).append(dur / 1e3)
        if "kernels" in names:
            for name, dur in c.execute("select name, duration from kernels"):
                kernels.setdefault(name.split("(")[0], []).append(dur / 1e3)
        c.close()
    return procs, ranges, kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    paths = sorted(glob.glob(os.path.join(a.dir, "**", "*.db"), recursive=True))
    if not paths:
        print(f"no rocpd databases under {a.dir}", file=sys.stderr)
        return 1
    procs, ranges, kernels = collect(paths)
    print(f"# roctx ranges and kernels ({procs} traced process(es))\n")
    print("| range | count | total ms | p50 us | p99 us |")
    print("|---|---:|---:|---:|---:|")
    for name, v in sorted(ranges.items(), key=lambda kv: -sum(kv[1])):
        print(f"| `{name}` | {len(v)} | {sum(v) / 1e3:.2f} | {_pct(v, 0.5):.1f} | {_pct(v, 0.99):.1f} |")
    print("\n| kernel | calls | total ms | p50 us |")
    print("|---|---:|---:|---:|")
    for name, v in sorted(kernels.items(), key=lambda kv: -sum(kv[1]))[:a.top]:
        print(f"| `{name[-90:]}` | {len(v)} | {sum(v) / 1e3:.2f} | {_pct(v, 0.5):.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
