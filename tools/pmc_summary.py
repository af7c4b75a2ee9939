"""Per-kernel roofline table from rocprofv3 --pmc passes (CSV output).

Each pass directory holds <prefix>_counter_collection.csv (one row per
dispatch x counter, with the dispatch's start / end timestamps). The table
joins the passes by kernel name: mean duration, HBM bytes read / written
(FETCH_SIZE / WRITE_SIZE, KiB), the achieved GB/s and its share of the
MI355X's 8 TB/s HBM3E peak, L2 hit rate (TCC_HIT / (HIT + MISS)) and the
instruction mix per wave (SQ_INSTS_* / SQ_WAVES).

Usage: python tools/pmc_summary.py OUT.md DIR [DIR...] [--match SUBSTR ...]
"""
from __future__ import annotations

import csv
import glob
import os
import sys
from collections import defaultdict

PEAK_GBS = 8000.0


def _short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    n = n.split("(")[0]
    return n if len(n) <= 60 else n[:57] + "..."


def load(dirs: list[str]):
    vals: dict[str, dict[str, list[float]]] = defaultdict(lambda: defaultdict(list))
    dur: dict[str, list[float]] = defaultdict(list)
    for d in dirs:
        # rocprofv3 nests its files (<dir>/<host>/<pid>_...) depending on -o
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    k = _short(r["Kernel_Name"])
                    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return vals, dur


def main() -> int:
    if len(sys.argv) < 3:
        print(__doc__)
        return 2
    out = sys.argv[1]
    args = sys.argv[2:]
    match = []
    if "--match" in args:
        i = args.index("--match")
        match = args[i + 1:]
        args = args[:i]
    vals, dur = load(args)

    def mean(xs):
        return sum(xs) / len(xs) if xs else float("nan")
    rows = []
    for k, c in vals.items():
        if match and not any(m in k for m in match):
            continue
        us = mean(dur[k])
        rd = mean(c.get("FETCH_SIZE", []))
        wr = mean(c.get("WRITE_SIZE", []))
        gbs = ((0 if rd != rd else rd) + (0 if wr != wr else wr)) * 1024 / (us * 1e3) if us > 0 else 0
        hit, miss = mean(c.get("TCC_HIT_sum", [])), mean(c.get("TCC_MISS_sum", []))
        waves = mean(c.get("SQ_WAVES", []))

        def per_wave(name):
            v = mean(c.get(name, []))
            return v / waves if waves and waves == waves and v == v else float("nan")
        rows.append((k, len(dur[k]), us, rd, wr, gbs, 100 * gbs / PEAK_GBS,
                     100 * hit / (hit + miss) if hit == hit and miss == miss and hit + miss else float("nan"),
                     per_wave("SQ_INSTS_VALU"), per_wave("SQ_INSTS_LDS"), per_wave("SQ_INSTS_VMEM_RD"),
                     per_wave("SQ_INSTS_VMEM_WR")))
    rows.sort(key=lambda r: -r[1] * r[2])

    def f(x, nd=1):
        return "-" if x != x else f"{x:,.{nd}f}"
    lines = ["# rocprofv3 PMC roofline", "",
             f"passes: {', '.join(args)}; HBM peak {PEAK_GBS:.0f} GB/s (MI355X HBM3E). "
             "Durations are per dispatch under counter collection.", "",
             "| kernel | dispatches | mean us | HBM read KiB | HBM write KiB | GB/s | % peak | L2 hit % "
             "| VALU/wave | LDS/wave | VMEM rd/wave | VMEM wr/wave |",
             "|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for r in rows:
        lines.append(f"| `{r[0]}` | {r[1]} | {f(r[2])} | {f(r[3], 0)} | {f(r[4], 0)} | {f(r[5], 0)} | "
                     f"{f(r[6])} | {f(r[7])} | {f(r[8])} | {f(r[9])} | {f(r[10])} | {f(r[11])} |")
    # every counter collected, mean per dispatch (the SQ ones per wave too)
    names = sorted({n for c in vals.values() for n in c})
    lines += ["", "## all counters (mean per dispatch; SQ_* / SQ_WAVES in parentheses)", "",
              "| kernel | " + " | ".join(names) + " |", "|---|" + "---:|" * len(names)]
    for r in rows:
        c = vals[r[0]]
        waves = mean(c.get("SQ_WAVES", []))
        cells = []
        for n in names:
            v = mean(c.get(n, []))
            cell = f(v, 0)
            if n.startswith("SQ_") and n != "SQ_WAVES" and waves == waves and waves and v == v:
                cell += f" ({v / waves:,.0f})"
            cells.append(cell)
        lines.append(f"| `{r[0]}` | " + " | ".join(cells) + " |")
    with open(out, "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines[:14]))
    return 0


if __name__ == "__main__":
    sys.exit(main())
