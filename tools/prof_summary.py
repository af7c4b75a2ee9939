"""Summarise a rocprofv3 ``--kernel-trace --stats`` database into markdown.

Usage: python tools/prof_summary.py gpurun_out/prof/run_results.db profiles/<name>.md [title]

Writes the per-kernel table (calls, total / average / min / max time, share)
plus the launch resources of each kernel (grid, workgroup, VGPR / AGPR /
SGPR, LDS, scratch) so register or LDS regressions show up in review.
"""
from __future__ import annotations

import re
import sqlite3
import sys


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*\)$", "", name)        # drop the parameter list
    name = name.replace("void ", "")
    return name if len(name) < 90 else name[:87] + "..."


def main(db: str, out: str, title: str = "rocprofv3 kernel summary") -> None:
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), sum(duration), avg(duration), min(duration), max(duration),"
        " max(grid_x), max(grid_y), max(workgroup_x), max(vgpr_count), max(accum_vgpr_count),"
        " max(sgpr_count), max(lds_size), max(scratch_size)"
        " from kernels group by name order by sum(duration) desc").fetchall()
    total = sum(r[2] for r in rows) or 1
    lines = [f"# {title}", "", f"source: `{db}` (durations in microseconds; kernel time only)", "",
             "| kernel | calls | total us | avg us | min us | max us | share |",
             "|---|---:|---:|---:|---:|---:|---:|"]
    for r in rows:
        lines.append(f"| `{short(r[0])}` | {r[1]} | {r[2] / 1e3:.1f} | {r[3] / 1e3:.2f} | "
                     f"{r[4] / 1e3:.2f} | {r[5] / 1e3:.2f} | {100 * r[2] / total:.1f}% |")
    lines += ["", "## launch resources", "",
              "| kernel | grid x,y | wg | VGPR | AGPR | SGPR | LDS B | scratch B |",
              "|---|---|---:|---:|---:|---:|---:|---:|"]
    for r in rows:
        lines.append(f"| `{short(r[0])}` | {r[6]},{r[7]} | {r[8]} | {r[9]} | {r[10]} | {r[11]} | "
                     f"{r[12]} | {r[13]} |")
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:14]))


if __name__ == "__main__":
    main(*sys.argv[1:])
