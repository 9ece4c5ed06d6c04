#!/bin/bash
# round-4 GPU session 11: wave-cooperative undo (k_undo_list + k_undo_wave)
# -- every test that undoes speculative output, then the reorder/dup
# unprotect step and its kernel trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_reorder.py tests/test_gpu_unprotect_adv.py tests/test_gpu_prepass.py \
    tests/test_gpu_xhdr.py tests/test_gpu_replay.py > gpurun_out/s11_tests.log 2>&1 || { tail -30 gpurun_out/s11_tests.log; exit 1; }
tail -1 gpurun_out/s11_tests.log
for args in "--op unprotect" "--op unprotect --reorder 0.01 --dup 0.001"; do
  timeout -k 10 300 python3 bench.py $args --steps 10 --warmup 2 --no-cpu-baseline \
      --traffic off > gpurun_out/s11_unprot.json 2> gpurun_out/s11_unprot.err || { tail -5 gpurun_out/s11_unprot.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/s11_unprot.json').read().strip().splitlines()[-1]); print('$args', round(d['value']/1e6,1), round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d['prepass'])"
done
tools/ktrace.sh unp_reorder2 --op unprotect --reorder 0.01 --dup 0.001 --steps 5 --warmup 2
