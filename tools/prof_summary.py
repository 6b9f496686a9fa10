#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel-trace database (run_results.db) or stats CSV into
profiles/<name>.csv: one row per kernel with calls, total and average duration."""
import csv
import sqlite3
import sys
from pathlib import Path


def from_db(db: Path):
    con = sqlite3.connect(str(db))
    rows = list(con.execute("select name,total_calls,total_duration,average,percentage from top_kernels"))
    return [(r[0], int(r[1]), float(r[2]), float(r[3]), float(r[4])) for r in rows]


def from_csv(path: Path):
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                    float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main():
    src, dst = Path(sys.argv[1]), Path(sys.argv[2])
    rows = from_db(src) if src.suffix == ".db" else from_csv(src)
    dst.parent.mkdir(parents=True, exist_ok=True)
    with open(dst, "w") as f:
        f.write("name,calls,total_us,avg_us,percent\n")
        for r in rows:
            f.write('"%s",%d,%.3f,%.3f,%.3f\n' % r)
    for r in rows[:6]:
        print(f"{r[3]:10.1f} us x{r[1]:4d} {r[4]:5.1f}%  {r[0][:110]}")


if __name__ == "__main__":
    main()
