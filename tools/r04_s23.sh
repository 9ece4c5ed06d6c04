#!/bin/bash
# round-4 GPU session 23: staging gather / scatter on up to 16 host threads
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s23
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_prepass.py -k "pipelined or host_buffer or many_tiles" tests/test_gpu_reorder.py \
    > gpurun_out/s23/tests.log 2>&1 || { tail -30 gpurun_out/s23/tests.log; exit 1; }
tail -1 gpurun_out/s23/tests.log
for op in protect unprotect; do
  timeout -k 10 300 ./tools/e2e_bench $((1<<20)) 1400 5 16 $op > gpurun_out/s23/e2e_$op.json 2> gpurun_out/s23/e2e_$op.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/s23/e2e_$op.json')); print('$op', d['host_batch_api'])"
done
