#!/bin/bash
# A/B of a runtime switch on the GPU box: the GPU tests selected by -k,
# then bench.py lines with the environment variable off / on, alternated.
#   tools/ab_env.sh <outdir> <VAR> "<pytest -k expr or ->" <reps> <bench args>...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/${1:?outdir}; var=$2; sel=$3; reps=$4; shift 4
mkdir -p "$o"
export TMPDIR=/tmp
if [ "$sel" != "-" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q -k "$sel" \
      --timeout 300 --timeout-method thread > "$o/tests.log" 2>&1 ||
      { tail -30 "$o/tests.log"; exit 1; }
  tail -1 "$o/tests.log"
fi
for r in $(seq 1 "$reps"); do
  for v in 0 1; do
    f="$o/${var}_${v}_$r.json"
    env "$var=$v" timeout -k 10 300 python3 bench.py "$@" --no-cpu-baseline \
        --traffic off > "$f" 2> "${f%.json}.err" || { tail -5 "${f%.json}.err"; exit 1; }
    python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d['value'] / 1e6, 1), 'Mpkt/s',
      round(d['ms_per_step'], 4), 'ms/step', round(d['roofline']['kernel_ms'], 4), 'ms kernel')" "$f"
  done
done
