#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (SQLite .db or kernel_stats.csv) as a markdown table."""
import csv
import sqlite3
import sys
from pathlib import Path


def short(name: str) -> str:
    n = name.split("(")[0]
    if "rocprim" in n:
        return "rocprim::" + ("scan" if "scan" in name else n.split("::")[-1])[:40]
    return n.replace("void ", "")


def from_db(path):
    db = sqlite3.connect(path)
    rows = db.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    return [(short(n), int(c), float(t) / 1e3, float(a) / 1e3, float(p)) for n, c, t, a, p in rows]


def from_csv(path):
    out = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            out.append((short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"]) / 1e6,
                        float(r["AverageNs"]) / 1e6, float(r["Percentage"])))
    return out


def main():
    p = Path(sys.argv[1])
    rows = from_db(p) if p.suffix == ".db" else from_csv(p)
    print("| kernel | calls | total ms | avg ms | % |")
    print("|---|---:|---:|---:|---:|")
    for n, c, t, a, pc in rows:
        if t >= 0.001:
            print(f"| {n} | {c} | {t:.3f} | {a:.3f} | {pc:.1f} |")


if __name__ == "__main__":
    main()
