#!/bin/bash
# round-4 GPU session 7: fused order-free form with per-stream aggregates
# (k_fz_stream: bitmap + counts instead of the per-packet setbits pass) --
# the pre-pass tests, configs[3] step time, and its kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_prepass.py tests/test_gpu_parity.py tests/test_gpu_replica.py tests/test_gpu_kdf.py > gpurun_out/s7_tests.log 2>&1 || { tail -30 gpurun_out/s7_tests.log; exit 1; }
tail -2 gpurun_out/s7_tests.log
tools/step_variants.sh g711 2 || exit 1
tools/ktrace.sh g711_s7 --config g711 --steps 10 --warmup 2
for args in "--op unprotect" "--op unprotect --reorder 0.01 --dup 0.001"; do
  timeout -k 10 300 python3 bench.py $args --steps 10 --warmup 2 --no-cpu-baseline \
      --traffic off > gpurun_out/s7_unprot.json 2> gpurun_out/s7_unprot.err || { tail -5 gpurun_out/s7_unprot.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/s7_unprot.json').read().strip().splitlines()[-1]); print('$args', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['prepass'], d['config'].get('arrival'))"
done
# FETCH_SIZE / WRITE_SIZE calibration against known bytes (tools/fetch_cal.hip)
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d gpurun_out/fcal_$c -o p \
      -- tools/fetch_cal > gpurun_out/fcal_$c.log 2>&1 || { tail -5 gpurun_out/fcal_$c.log; exit 1; }
  python3 tools/pmc_reduce.py gpurun_out/fcal_$c
  grep -rh "k_" gpurun_out/fcal_$c --include=pmc_summary.csv || true
done
tail -1 gpurun_out/fcal_FETCH_SIZE.log
