#!/bin/bash
# Kernel-trace stats of a short bench.py run (on the GPU box):
#   tools/ktrace.sh <name> [bench args...]  -> gpurun_out/kt_<name>/*kernel_stats.csv
# prints the top kernels (name, calls, average us, total share)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
name=$1; shift
args=${*:-"--steps 5 --warmup 2"}
export TMPDIR=/tmp
out=gpurun_out/kt_$name
rm -rf "$out"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o kt \
    -- python3 bench.py --no-cpu-baseline --traffic off $args > "$out.log" 2>&1 || { tail -5 "$out.log"; exit 1; }
python3 tools/pmc_reduce.py "$out"
python3 - "$out" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(f and open(f)))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("%-60s %6s calls %10.1f us avg %6.2f%%" % (r["Name"][:60], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
PY
