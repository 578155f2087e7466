#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (SQLite .db or kernel_stats.csv) as a markdown table.

--trace KERNEL_TRACE_CSV --last N --kernels SUB[,SUB...]: also list, for each kernel whose name contains SUB, the
average duration of its LAST N dispatches (the bench's timed steps, after its warm-up dispatches) next to the
average over all of them (round 6: the encoder's warm-up dispatches run slower under the tracer)."""
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


def last_dispatches(trace, subs, last):
    """(kernel, dispatches, avg ms over all, avg ms over the last `last`) from a kernel_trace.csv."""
    per = {}
    with open(trace) as fh:
        for r in csv.DictReader(fh):
            n = short(r["Kernel_Name"])
            if any(s in n for s in subs):
                per.setdefault(n, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = []
    for n, v in per.items():
        v.sort()
        d = [x[1] / 1e6 for x in v]
        tail = d[-last:]
        out.append((n, len(d), sum(d) / len(d), sum(tail) / len(tail)))
    return out


def main():
    p = Path(sys.argv[1])
    rows = from_db(p) if p.suffix == ".db" else from_csv(p)
    print("| kernel | calls | total ms | avg ms | % |")
    print("|---|---:|---:|---:|---:|")
    for n, c, t, a, pc in rows:
        if t >= 0.001:
            print(f"| {n} | {c} | {t:.3f} | {a:.3f} | {pc:.1f} |")
    if "--trace" in sys.argv:
        trace = sys.argv[sys.argv.index("--trace") + 1]
        last = int(sys.argv[sys.argv.index("--last") + 1]) if "--last" in sys.argv else 5
        subs = sys.argv[sys.argv.index("--kernels") + 1].split(",") if "--kernels" in sys.argv else ["k_encode_v4"]
        print()
        print(f"| kernel | dispatches | avg ms (all) | avg ms (last {last}: the timed steps) |")
        print("|---|---:|---:|---:|")
        for n, c, a, t in last_dispatches(trace, subs, last):
            print(f"| {n} | {c} | {a:.3f} | {t:.3f} |")


if __name__ == "__main__":
    main()
