#!/bin/bash
# round-4 GPU session 2: prepass tests; configs[3] fused vs separate
# classification vs round 3; headline tree vs round 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_prepass.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/s2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s2_tests.log; [ $rc = 0 ] || exit $rc
one() {  # name env... -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --traffic off $BARGS 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms']; print('$name', round(d['ms_per_step'],4), round(k,4), round(d['ms_per_step']-k,4))"
}
for r in 1 2; do
  BARGS="--config g711" one g711_fused SRTP_PP_FUSED_OF=1 || exit 1
  BARGS="--config g711" one g711_sep SRTP_PP_FUSED_OF=0 || exit 1
  BARGS="--config g711" one g711_r3 LIBSRTP_MI355X_LIB=$PWD/exp_build/r3g711/libsrtp_mi355x.so || exit 1
  BARGS="--config icm128" one icm_tree X=1 || exit 1
  BARGS="--config icm128" one icm_r3 LIBSRTP_MI355X_LIB=$PWD/exp_build/r3base/libsrtp_mi355x.so || exit 1
done
