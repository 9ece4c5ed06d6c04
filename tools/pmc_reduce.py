#!/usr/bin/env python3
"""Shrinks a rocprofv3 output directory in place (run on the GPU box, so
gpurun_out/ stays under its copy-back limit): counter_collection.csv ->
pmc_summary.csv (per kernel and counter: dispatches, mean per dispatch);
kernel_trace.csv -> kernel_warm_stats.csv (per kernel: launches, then the
median / min / mean of the launches after each kernel's first -- the cold
first launch and the profiler's start-up are not what a bench step sees),
then dropped when kernel_stats.csv is present.

  python3 tools/pmc_reduce.py <rocprofv3 -d dir>
"""
import collections
import csv
import glob
import os
import sys


def reduce_counters(path):
    acc = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = (r["Kernel_Name"], r["Counter_Name"])
            acc[k] += float(r["Counter_Value"] or 0)
            disp[k].add(r["Dispatch_Id"])
    out = os.path.join(os.path.dirname(path), "pmc_summary.csv")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Dispatches",
                    "Mean_Per_Dispatch"])
        for (kern, ctr), v in sorted(acc.items()):
            n = len(disp[(kern, ctr)])
            w.writerow([kern, ctr, n, v / max(1, n)])
    os.remove(path)


def warm_stats(path):
    dur = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            dur[r["Kernel_Name"]].append(
                (int(r["Start_Timestamp"]),
                 int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = os.path.join(os.path.dirname(path), "kernel_warm_stats.csv")
    rows = []
    for kern, v in dur.items():
        v.sort()
        warm = sorted(d for _, d in v[1:]) or [v[0][1]]
        m = len(warm)
        med = warm[m // 2] if m % 2 else (warm[m // 2 - 1] + warm[m // 2]) / 2
        rows.append((kern, len(v), med, warm[0], sum(warm) / m, v[0][1]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "WarmMedianNs", "WarmMinNs",
                    "WarmMeanNs", "FirstNs"])
        for r in sorted(rows, key=lambda r: -r[2] * r[1]):
            w.writerow(r)


def main():
    d = sys.argv[1]
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                       recursive=True):
        reduce_counters(p)
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"),
                       recursive=True):
        warm_stats(p)
        stats = glob.glob(os.path.join(os.path.dirname(p), "*kernel_stats.csv"))
        if stats:
            os.remove(p)


if __name__ == "__main__":
    main()
