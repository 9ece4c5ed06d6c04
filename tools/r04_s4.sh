#!/bin/bash
# round-4 GPU session 4: per-lane key reuse (LaneKey::reload) on configs[3]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prepass.py tests/test_gpu_parity.py -x -q --timeout 300 \
    --timeout-method thread -k "prepass or random or six or multi or shapes" > gpurun_out/s4_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s4_tests.log; [ $rc = 0 ] || exit $rc
one() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --traffic off $BARGS 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms']; print('$name', round(d['ms_per_step'],4), round(k,4), round(d['ms_per_step']-k,4))"
}
for r in 1 2; do
  BARGS="--config g711" one g711_fused X=1 || exit 1
  BARGS="--config g711" one g711_fused_nocoop LIBSRTP_MI355X_LIB=$PWD/exp_build/nocoop/libsrtp_mi355x.so || exit 1
  BARGS="--config g711" one g711_sep SRTP_PP_FUSED_OF=0 || exit 1
  BARGS="--config g711" one g711_sep_nocoop SRTP_PP_FUSED_OF=0 LIBSRTP_MI355X_LIB=$PWD/exp_build/nocoop/libsrtp_mi355x.so || exit 1
done
