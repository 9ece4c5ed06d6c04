#!/bin/bash
# round-4 GPU session 6: fused classify trailer save -- correctness of the
# fused/declined paths, then configs[3] step time: tree (trailer bytes saved
# inside the classify), exp_build/late (stored after the crypto),
# exp_build/notsave (no save: the cost bound), separate classify
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ -n "$NOTEST" ] || timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_prepass.py tests/test_gpu_plugin.py > gpurun_out/s6_tests.log 2>&1 || { tail -30 gpurun_out/s6_tests.log; exit 1; }
[ -n "$NOTEST" ] || tail -3 gpurun_out/s6_tests.log
[ -z "$LATETEST" ] || LIBSRTP_MI355X_LIB=$PWD/exp_build/late/libsrtp_mi355x.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_prepass.py > gpurun_out/s6_late_tests.log 2>&1 || { tail -30 gpurun_out/s6_late_tests.log; exit 1; }
[ -z "$LATETEST" ] || tail -2 gpurun_out/s6_late_tests.log
one() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --traffic off --config g711 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); k=d['roofline']['kernel_ms']; print('$name', round(d['ms_per_step'],4), round(k,4), round(d['ms_per_step']-k,4))"
}
for r in 1 2; do
  one g711_sep SRTP_PP_FUSED_OF=0 || exit 1
done
VARIANTS="late notsave" tools/step_variants.sh g711 2
