#!/bin/bash
# bench.py's step and kernel time for the in-tree library and every
# exp_build/<name> variant (timing only; no CPU baseline, no PMC).
# usage (on the GPU box): [OP=unprotect] [VARIANTS="a b"] tools/step_variants.sh <config> [rounds]
# (VARIANTS: only these exp_build names besides the tree)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cfg=${1:-icm128}; rounds=${2:-2}
for r in $(seq $rounds); do
  for so in libsrtp_amd/libsrtp_mi355x.so exp_build/*/libsrtp_mi355x.so; do
    [ -f "$so" ] || continue
    name=$(basename $(dirname $so))
    if [ -n "$VARIANTS" ] && [ "$so" != libsrtp_amd/libsrtp_mi355x.so ] &&
       ! echo " $VARIANTS " | grep -q " $name "; then continue; fi
    LIBSRTP_MI355X_LIB=$PWD/$so timeout -k 10 120 python3 bench.py --config $cfg --op ${OP:-protect} \
        --steps 20 --warmup 3 --no-cpu-baseline --traffic off 2>/dev/null |
      python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms']; print('$name', round(d['ms_per_step'],4), round(k,4), round(d['ms_per_step']-k,4))" || exit 1
  done
done
