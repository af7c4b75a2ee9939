"""Per-configuration kernel times from a rocprofv3 kernel-trace database.

Usage: python tools/prof_sequence.py <results.db> <labels,comma,separated> <calls per label>

Groups the dispatches (in start order, excluding PyTorch set-up kernels) into
consecutive runs of ``calls`` dispatches per label and prints the median
kernel time of each kernel name within each label, for micro-benchmarks
such as tools/bench_topk.py that run one configuration after another.
"""
from __future__ import annotations

import sqlite3
import statistics
import sys

from prof_summary import short


def main(db: str, labels: str, calls: str) -> None:
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels order by start").fetchall()
    rows = [(short(n), d / 1e3) for n, d in rows if n.lstrip("void ").startswith("jb::")]
    per = int(calls)
    at = 0
    for lab in labels.split(","):
        seg = rows[at:at + per]
        at += per
        by: dict[str, list[float]] = {}
        for n, d in seg:
            by.setdefault(n, []).append(d)
        print(lab, {n: round(statistics.median(v), 2) for n, v in by.items()})


if __name__ == "__main__":
    main(*sys.argv[1:])
