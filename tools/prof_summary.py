#!/usr/bin/env python3
"""Summarise a rocprofv3 output (the SQLite .db of --kernel-trace/--stats,
or a kernel_stats.csv) into the compact table committed under profiles/.

  python tools/prof_summary.py gpurun_out/prof/run_results.db > profiles/x.md
"""
import csv
import re
import sqlite3
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    if name.startswith("void at::native") or "at::native" in name[:60]:
        m = re.match(r"void at::native::([A-Za-z_]+)", name)
        return "torch:" + (m.group(1) if m else "kernel")
    return name.replace("void ", "")[:110]


def rows_from_db(path):
    db = sqlite3.connect(path)
    q = ("select name, total_calls, total_duration, average, percentage "
         "from top_kernels")
    return [(short(r[0]), int(r[1]), float(r[2]), float(r[3]), float(r[4]))
            for r in db.execute(q)]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((short(r["Name"]), int(r["Calls"]),
                        float(r["TotalDurationNs"]) / 1e3,
                        float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
    return out


def main():
    path = sys.argv[1]
    rows = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    print("| kernel | calls | total us | average us | % |")
    print("|---|---:|---:|---:|---:|")
    for name, calls, tot, avg, pct in rows:
        print("| `%s` | %d | %.1f | %.1f | %.2f |" % (name, calls, tot, avg, pct))


if __name__ == "__main__":
    main()
