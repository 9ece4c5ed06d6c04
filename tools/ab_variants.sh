#!/bin/bash
# A/B timing of exp_build/<name>/libsrtp_mi355x.so builds against the tree on
# the GPU box: for each repetition and config, one bench.py line (no PMC, no
# CPU baseline) per build, back to back; then a short parity run per variant.
# usage (on the GPU box):
#   tools/ab_variants.sh <outdir> "<config[:op]> ..." <reps> [-k <pytest -k>] name...
# e.g. tools/ab_variants.sh ab1 "g711 g711:unprotect" 2 -k fused kh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=gpurun_out/${1:?outdir}; cfgs=$2; reps=$3; shift 3
sel=""
if [ "$1" = "-k" ]; then sel=$2; shift 2; fi
mkdir -p "$out"
export TMPDIR=/tmp
line() {   # name config op rep
  local so=$PWD/libsrtp_amd/libsrtp_mi355x.so
  [ "$1" != tree ] && so=$PWD/exp_build/$1/libsrtp_mi355x.so
  local f="$out/$2_$3_$1_$4.json"
  LIBSRTP_MI355X_LIB=$so timeout -k 10 300 python3 bench.py --config "$2" \
      --op "$3" --no-cpu-baseline --traffic off > "$f" 2> "${f%.json}.err" ||
      { tail -5 "${f%.json}.err"; return 1; }
  python3 -c "
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split('/')[-1], round(d['value'] / 1e6, 1), 'Mpkt/s',
      round(d['ms_per_step'], 4), 'ms/step', round(d['roofline']['kernel_ms'], 4),
      'ms kernel')" "$f"
}
for name in "$@"; do
  if [ -n "$sel" ]; then
    LIBSRTP_MI355X_LIB=$PWD/exp_build/$name/libsrtp_mi355x.so timeout -k 10 600 \
        python3 -u -m pytest tests -m gpu -x -q -k "$sel" --timeout 300 \
        --timeout-method thread > "$out/parity_$name.log" 2>&1 ||
        { tail -5 "$out/parity_$name.log"; exit 1; }
    echo "parity $name: $(tail -1 "$out/parity_$name.log")"
  fi
done
for r in $(seq 1 "$reps"); do
  for c in $cfgs; do
    cfg=${c%%:*}; op=protect; [ "$c" != "$cfg" ] && op=${c#*:}
    line tree "$cfg" "$op" "$r" || exit 1
    for name in "$@"; do line "$name" "$cfg" "$op" "$r" || exit 1; done
  done
done
