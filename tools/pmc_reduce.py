#!/usr/bin/env python3
"""Shrinks a rocprofv3 output directory in place (run on the GPU box, so
gpurun_out/ stays under its copy-back limit): counter_collection.csv ->
pmc_summary.csv (per kernel and counter: dispatches, mean per dispatch);
kernel_trace.csv is dropped when kernel_stats.csv is present.

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


def main():
    d = sys.argv[1]
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                       recursive=True):
        reduce_counters(p)
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"),
                       recursive=True):
        stats = glob.glob(os.path.join(os.path.dirname(p), "*kernel_stats.csv"))
        if stats:
            os.remove(p)


if __name__ == "__main__":
    main()
