"""Per-kernel execution time and the idle gap before each dispatch, from a
rocprofv3 --kernel-trace CSV (the verified committer's window loop:
how much of a batch is kernels, how much is the launch gaps between them).

Usage: python tools/trace_gaps.py TRACE_DIR OUT.md [--last N]
  TRACE_DIR: searched recursively for *kernel_trace.csv
  --last N: only the last N dispatches (the steady batches of a run)
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict


def _short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:70]


def main() -> int:
    if len(sys.argv) < 3:
        print(__doc__)
        return 2
    d, out = sys.argv[1], sys.argv[2]
    last = 0
    a = sys.argv[3:]
    if "--last" in a:
        last = int(a[a.index("--last") + 1])
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"])))
    rows.sort()
    if last:
        rows = rows[-last:]
    if not rows:
        print("no dispatches")
        return 1
    ex = defaultdict(list)
    gap = defaultdict(list)
    for i, (s, e, k) in enumerate(rows):
        ex[k].append((e - s) / 1e3)
        if i:
            gap[k].append(max(0, s - rows[i - 1][1]) / 1e3)
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(sum(v) for v in ex.values())
    gaps = sum(sum(v) for v in gap.values())
    lines = ["# kernel-trace gaps", "",
             f"{len(rows)} dispatches over {span:,.0f} us: kernels {busy:,.0f} us ({100 * busy / span:.1f} %), "
             f"idle gaps {gaps:,.0f} us ({100 * gaps / span:.1f} %)", "",
             "| kernel | dispatches | exec us total | mean exec us | mean gap before us | short (<2 us) |",
             "|---|---:|---:|---:|---:|---:|"]
    for k in sorted(ex, key=lambda k: -sum(ex[k]) - sum(gap[k])):
        e, g = ex[k], gap[k]
        lines.append(f"| `{k}` | {len(e)} | {sum(e):,.1f} | {sum(e) / len(e):.2f} | "
                     f"{(sum(g) / len(g)) if g else 0:.2f} | {sum(1 for x in e if x < 2.0)} |")
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    return 0


if __name__ == "__main__":
    sys.exit(main())
