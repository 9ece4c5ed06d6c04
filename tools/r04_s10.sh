#!/bin/bash
# round-4 GPU session 10: packet commit inside the fused kernel -- tests,
# configs[3] step time; the reorder/dup unprotect step's kernel trace; the
# in-place FETCH/WRITE calibration shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_prepass.py tests/test_gpu_plugin.py > gpurun_out/s10_tests.log 2>&1 || { tail -30 gpurun_out/s10_tests.log; exit 1; }
tail -1 gpurun_out/s10_tests.log
VARIANTS=none tools/step_variants.sh g711 3 || exit 1
tools/ktrace.sh unp_reorder --op unprotect --reorder 0.01 --dup 0.001 --steps 5 --warmup 2 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/fcal2_$c -o p \
      -- tools/fetch_cal > gpurun_out/fcal2_$c.log 2>&1 || { tail -5 gpurun_out/fcal2_$c.log; exit 1; }
  python3 tools/pmc_reduce.py gpurun_out/fcal2_$c
  grep -rh "k_" gpurun_out/fcal2_$c --include=pmc_summary.csv || true
done
