#!/usr/bin/env python3
"""Per-launch PMC table of the dominant kernel from tools/pmc_bench.sh
output: python3 tools/pmc_table.py <outdir> <kernel substring> [kernel_ms]

SQ cycle counters count quad-cycles (4 clocks); the issue fraction is
ACTIVE_INST_ANY summed over waves, per SIMD, over the per-SIMD wave time."""
import csv
import glob
import os
import sys


def load(d, ks):
    got = {}
    for p in glob.glob(os.path.join(d, "p*", "pmc_summary.csv")):
        with open(p) as f:
            for r in csv.DictReader(f):
                if ks in r["Kernel_Name"]:
                    got[r["Counter_Name"]] = float(r["Mean_Per_Dispatch"])
    return got


def main():
    d, ks = sys.argv[1], sys.argv[2]
    g = load(d, ks)
    for k in sorted(g):
        print("%-24s %16.1f" % (k, g[k]))
    w = g.get("SQ_WAVES")
    if w:
        print("per wave: VALU %.0f  LDS %.0f  SALU %.0f" % (
            g["SQ_INSTS_VALU"] / w, g["SQ_INSTS_LDS"] / w,
            g.get("SQ_INSTS_SALU", 0) / w))
        print("issue (ACTIVE_INST_ANY / WAVE_CYCLES): %.3f per wave" % (
            g["SQ_ACTIVE_INST_ANY"] / g["SQ_WAVE_CYCLES"]))
        print("wait (WAIT_ANY / WAVE_CYCLES): %.3f" % (
            g["SQ_WAIT_ANY"] / g["SQ_WAVE_CYCLES"]))
    if "GRBM_GUI_ACTIVE" in g and "SQ_LDS_IDX_ACTIVE" in g:
        # GRBM_GUI_ACTIVE: GPU clocks summed over the 8 XCDs
        print("LDS array busy: %.3f" % (
            g["SQ_LDS_IDX_ACTIVE"] / 256 / (g["GRBM_GUI_ACTIVE"] / 8)))
    if "FETCH_SIZE" in g and "WRITE_SIZE" in g:
        print("HBM KB fetch %.0f write %.0f" % (g["FETCH_SIZE"], g["WRITE_SIZE"]))


if __name__ == "__main__":
    main()
