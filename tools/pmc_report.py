#!/usr/bin/env python3
"""Per-dispatch averages of the counters collected by tools/pmc_passes.sh
for one kernel, plus the derived figures DESIGN.md quotes.

  python tools/pmc_report.py gpurun_out/pmc k_icm_hmac [packets]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d, kern = sys.argv[1], sys.argv[2]
    pk = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20
    vals = {}
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                              recursive=True)):
        acc = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            if kern not in r["Kernel_Name"]:
                continue
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for k, v in acc.items():
            vals[k] = v / max(1, len(disp[k]))
    # reduced on the box by tools/pmc_reduce.py: per kernel means (kernels
    # matching the substring are summed: e.g. both launches of one step)
    for f in sorted(glob.glob(os.path.join(d, "**", "pmc_summary.csv"),
                              recursive=True)):
        acc = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Mean_Per_Dispatch"])
        vals.update(acc)
    for k in sorted(vals):
        print("%-28s %16.1f" % (k, vals[k]))
    g = vals.get
    print()
    if g("SQ_WAVES"):
        w = g("SQ_WAVES")
        print("per 64 packets (wave-instructions): VALU %.0f  LDS %.0f  "
              "VMEM_RD %.1f  VMEM_WR %.1f" % (
            64 * g("SQ_INSTS_VALU", 0) / pk, 64 * g("SQ_INSTS_LDS", 0) / pk,
            64 * g("SQ_INSTS_VMEM_RD", 0) / pk,
            64 * g("SQ_INSTS_VMEM_WR", 0) / pk))
        if g("SQ_WAVE_CYCLES"):
            wc = g("SQ_WAVE_CYCLES")
            for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                      "SQ_WAIT_INST_LDS"):
                if g(k) is not None:
                    print("  %-22s %5.1f %% of wave-cycles" % (k, 100 * g(k) / wc))
    if g("GRBM_GUI_ACTIVE"):
        cyc = g("GRBM_GUI_ACTIVE") / 8   # summed over 8 XCDs
        print("kernel cycles (per XCD) %.0f" % cyc)
        if g("SQ_LDS_IDX_ACTIVE"):
            print("  LDS array busy %.1f %%" % (
                100 * g("SQ_LDS_IDX_ACTIVE") / (cyc * 256)))
        if g("SQ_INSTS_VALU"):
            print("  VALU issue (2 cyc/instr/SIMD) %.1f %%" % (
                100 * 2 * g("SQ_INSTS_VALU") / (cyc * 1024)))
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        algo_r, algo_w = pk * 1412, pk * 1422
        print("HBM: FETCH_SIZE x2 = %.3f GB (algorithmic read %.3f), "
              "WRITE_SIZE = %.3f GB (algorithmic write %.3f)" % (
                  2 * g("FETCH_SIZE") * 1024 / 1e9, algo_r / 1e9,
                  g("WRITE_SIZE") * 1024 / 1e9, algo_w / 1e9))


if __name__ == "__main__":
    main()
