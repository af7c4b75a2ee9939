"""Print a per-step GPU timeline (kernels + memory copies) from a rocprofv3
database: python tools/timeline.py <results.db> [first_ns_offset_steps]"""
import sqlite3
import sys


def main(db: str, limit: int = 60) -> None:
    c = sqlite3.connect(db)
    tables = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
    ev = []
    if "kernels" in tables:
        for name, s, e, q in c.execute("select name, start, end, queue_id from kernels"):
            ev.append((s, e, "K", name.split("(")[0][-40:], q))
    for t in ("memory_copies", "memory_copy"):
        if t in tables:
            cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
            nm = "name" if "name" in cols else cols[1]
            size = "size" if "size" in cols else None
            q = "queue_id" if "queue_id" in cols else "0"
            for row in c.execute(f"select {nm}, start, end, {size or 0}, {q} from {t}"):
                ev.append((row[1], row[2], "C", f"{row[0]} {row[3]}", row[4]))
            break
    ev.sort()
    if not ev:
        print("no events; tables:", tables)
        return
    t0 = ev[max(0, len(ev) - limit)][0]
    for s, e, kind, name, q in ev[-limit:]:
        print(f"{(s - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f} {kind} q{q} {name}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 60)
