#!/bin/bash
# round-4 GPU session 1: the changed paths' tests, then kernel variants
# (exp_build/) against the tree build, then bench lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
    --timeout-method thread -k "replica or large_uniform or plugin or prepass or reorder or unprotect or jumbo or shapes" \
    > gpurun_out/s1_tests.log 2>&1
rc=$?; tail -5 gpurun_out/s1_tests.log; [ $rc = 0 ] || exit $rc
VARIANTS="r3base rep16 prio lb768 nb4" timeout -k 10 600 bash tools/step_variants.sh icm128 1 \
    > gpurun_out/s1_icm_variants.log 2>&1 || exit 1
cat gpurun_out/s1_icm_variants.log
VARIANTS="r3g711" timeout -k 10 600 bash tools/step_variants.sh g711 2 \
    > gpurun_out/s1_g711_variants.log 2>&1 || exit 1
cat gpurun_out/s1_g711_variants.log
SRTP_PP_FUSED_OF=0 timeout -k 10 200 python3 bench.py --config g711 --steps 20 --warmup 3 \
    --no-cpu-baseline --traffic off 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('tree_nofused', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))" || exit 1
timeout -k 10 200 python3 bench.py --op unprotect --steps 20 --warmup 3 --no-cpu-baseline \
    --traffic off > gpurun_out/s1_bench_unprotect.json 2> gpurun_out/s1_bench_unprotect.err || exit 1
tail -c 700 gpurun_out/s1_bench_unprotect.json
for op in protect unprotect; do
  timeout -k 10 300 ./tools/e2e_bench $((1<<20)) 1400 5 16 $op > gpurun_out/s1_e2e_$op.json 2> gpurun_out/s1_e2e_$op.err || exit 1
  cat gpurun_out/s1_e2e_$op.json
done
