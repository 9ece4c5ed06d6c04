#!/bin/bash
# round-4 GPU session 7: fused-path tests (tag sizes, tight capacities),
# then the configs[3] step's kernel trace (where the step's non-crypto time goes)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_prepass.py > gpurun_out/s7_tests.log 2>&1 || { tail -30 gpurun_out/s7_tests.log; exit 1; }
tail -2 gpurun_out/s7_tests.log
tools/ktrace.sh g711_s7 --config g711 --steps 10 --warmup 2
