#!/usr/bin/env python3
"""Writes profiles/<name>.md from a tools/prof_kernels.sh output directory
(kernel-trace stats + the SQ/GRBM counter passes, reduced on the box by
tools/pmc_reduce.py) and the bench.py JSON line of the same workload.

  python3 tools/write_profile.py <name> <prof dir> <bench log> <kernel> <packets> "<command>"
"""
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    name, pdir, blog, kern, pk, cmd = sys.argv[1:7]
    out = [f"# {name}", "", f"Command (on one MI355X, via gpurun): `{cmd}`", ""]
    with open(blog) as f:
        line = [l for l in f.read().splitlines() if l.startswith("{")][-1]
    d = json.loads(line)
    r = d["roofline"]
    out += ["## bench.py line", "", "```json", line, "```", "",
            f"- dominant kernel `{r['kernel']}`: {r['kernel_ms']:.3f} ms per "
            f"launch (HIP events), {r['achieved']:.0f} GB/s algorithmic = "
            f"{r['frac']:.3f} of {r['peak']:.0f} GB/s"]
    if r.get("traffic"):
        out.append(f"- HBM traffic (FETCH_SIZE + WRITE_SIZE, separate PMC "
                   f"passes) {r['traffic'] / 1e9:.3f} GB per launch = "
                   f"{r['traffic'] / r['algorithmic_bytes_per_launch']:.3f}x "
                   f"the algorithmic bytes")
    out.append("")
    stats = glob.glob(os.path.join(pdir, "kt", "*kernel_stats.csv"))
    if stats:
        tab = subprocess.run([sys.executable,
                              os.path.join(ROOT, "tools", "prof_summary.py"),
                              stats[0]], capture_output=True, text=True).stdout
        out += ["## rocprofv3 --kernel-trace --stats (bench.py --steps 3 "
                "--warmup 1, same workload)", "",
                "\n".join(tab.splitlines()[:18]), ""]
    rep = subprocess.run([sys.executable,
                          os.path.join(ROOT, "tools", "pmc_report.py"), pdir,
                          kern, pk], capture_output=True, text=True).stdout
    out += [f"## PMC counters of `{kern}` (per launch; SQ/GRBM passes)", "",
            "```", rep.rstrip(), "```", ""]
    dst = os.path.join(ROOT, "profiles", name + ".md")
    with open(dst, "w") as f:
        f.write("\n".join(out))
    print(dst)


if __name__ == "__main__":
    main()
