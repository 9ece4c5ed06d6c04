#!/bin/bash
# round-4 GPU session 22: large host-buffer batches as pipelined device
# chunks (batch_device_pipelined) -- its test and the batch-API tests, then
# the end-to-end rates
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s22
timeout -k 10 800 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread \
    tests/test_gpu_prepass.py tests/test_gpu_parity.py tests/test_gpu_reorder.py \
    tests/test_gpu_replay.py tests/test_gpu_udp_relay.py tests/test_gpu_unprotect_adv.py \
    > gpurun_out/s22/tests.log 2>&1 || { tail -30 gpurun_out/s22/tests.log; exit 1; }
tail -1 gpurun_out/s22/tests.log
for op in protect unprotect; do
  timeout -k 10 300 ./tools/e2e_bench $((1<<20)) 1400 5 16 $op > gpurun_out/s22/e2e_$op.json 2> gpurun_out/s22/e2e_$op.err || exit 1
  cat gpurun_out/s22/e2e_$op.json
done
