#!/bin/bash
# round-4 GPU session 5: trailer-save cost in the fused classify (timing only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
one() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --traffic off $BARGS 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms']; print('$name', round(d['ms_per_step'],4), round(k,4), round(d['ms_per_step']-k,4))"
}
for r in 1 2; do
  BARGS="--config g711" one g711_fused X=1 || exit 1
  BARGS="--config g711" one g711_notsave LIBSRTP_MI355X_LIB=$PWD/exp_build/notsave/libsrtp_mi355x.so || exit 1
  BARGS="--config g711" one g711_sep SRTP_PP_FUSED_OF=0 || exit 1
done
