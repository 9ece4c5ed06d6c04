#!/bin/bash
# The one parameterised GPU runner for a round's evidence (replaces the
# per-session scripts of rounds 2-4).  On the GPU box:
#   tools/bench_lines.sh <outdir> <step> [<step> ...]
# steps, run in order, stopping at the first failure (each under its own
# time limit, so a hang or fault ends the call):
#   tests[:<pytest -k expr>]   the GPU suite (or the selected tests)
#   smoke                      __graft_entry__.smoke()
#   line:<name>:<bench args>   one bench.py JSON line -> <outdir>/<name>.json
#   ktrace:<name>:<bench args> rocprofv3 kernel trace + stats -> <outdir>/kt_<name>
#   pmc:<name>:<bench args>    SQ / HBM counter passes -> <outdir>/pmc_<name>
#   e2e:<op>                   tools/e2e_bench (PCIe-inclusive) -> <outdir>/e2e_<op>.json
#   percall:<calls>            bench.py --percall (one packet per call) -> <outdir>/percall.json
# bench args use ',' for spaces: line:g711:--config,g711,--steps,10
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:?outdir}; shift
mkdir -p "$out"
export TMPDIR=/tmp
summ() {   # one bench line -> a short summary
  python3 - "$1" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
iss = r.get("issue") or {}
c = d.get("cpu_baseline") or {}
print(sys.argv[1].split("/")[-1], round(d["value"] / 1e6, 1), "Mpkt/s",
      round(d["ms_per_step"], 4), "ms", r.get("kernel"), round(r.get("kernel_ms") or 0, 4),
      "frac", round(r.get("frac") or 0, 4), "traffic/alg", r.get("traffic_over_algorithmic"),
      "additive", iss.get("additive_frac"), "cpu", c.get("value"))
PY
}
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}
  name=${rest%%:*}; args=${rest#*:}; args=${args//,/ }
  echo "[run] $step"
  case $kind in
    tests)
      k=(); [ "$rest" != tests ] && [ -n "$rest" ] && k=(-k "$rest")
      timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -q --timeout 300 \
          --timeout-method thread "${k[@]}" > "$out/tests.log" 2>&1
      rc=$?; tail -3 "$out/tests.log"; [ $rc = 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 150 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    line)
      timeout -k 10 500 python3 bench.py $args > "$out/$name.json" 2> "$out/$name.err" ||
          { tail -5 "$out/$name.err"; exit 1; }
      summ "$out/$name.json" ;;
    ktrace)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/kt_$name" -o kt \
          -- python3 bench.py --no-cpu-baseline --traffic off $args > "$out/kt_$name.log" 2>&1 ||
          { tail -5 "$out/kt_$name.log"; exit 1; }
      python3 tools/pmc_reduce.py "$out/kt_$name" ;;
    pmc)
      bash tools/pmc_passes.sh "$out/pmc_$name" $args --no-cpu-baseline --traffic off || exit 1 ;;
    e2e)
      timeout -k 10 300 ./tools/e2e_bench $((1<<20)) 1400 5 16 "$rest" > "$out/e2e_$rest.json" \
          2> "$out/e2e_$rest.err" || exit 1
      cat "$out/e2e_$rest.json" ;;
    percall)
      timeout -k 10 400 python3 bench.py --percall --percall-calls "$rest" \
          > "$out/percall.json" 2> "$out/percall.err" ||
          { tail -5 "$out/percall.err"; exit 1; }
      cat "$out/percall.json" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
