#!/bin/bash
# round-4 GPU session 14: the receive side's order-free form inside the
# AES-ICM kernel (pp_unprotect_fused) -- tests, then configs[3] unprotect
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_prepass.py tests/test_gpu_unprotect_adv.py tests/test_gpu_replay.py \
    tests/test_gpu_reorder.py tests/test_gpu_parity.py > gpurun_out/s14_tests.log 2>&1 || { tail -30 gpurun_out/s14_tests.log; exit 1; }
tail -1 gpurun_out/s14_tests.log
for v in 1 0; do
  SRTP_PP_FUSED_OF=$v timeout -k 10 300 python3 bench.py --config g711 --op unprotect --steps 10 --warmup 3 \
      --no-cpu-baseline --traffic off > gpurun_out/s14_unp.json 2> gpurun_out/s14_unp.err || { tail -5 gpurun_out/s14_unp.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/s14_unp.json').read().strip().splitlines()[-1]); print('fused_of=$v', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['prepass'])"
done
tools/ktrace.sh g711_unp --config g711 --op unprotect --steps 5 --warmup 2
