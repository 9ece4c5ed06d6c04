#!/bin/bash
# round-4 GPU session 16: protect bitmap bits merged per word before the
# atomic (A/B against exp_build/nowmerge), fused-path tests, and the RCCL
# replication path with a one-rank group
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_prepass.py > gpurun_out/s16_tests.log 2>&1 || { tail -30 gpurun_out/s16_tests.log; exit 1; }
tail -1 gpurun_out/s16_tests.log
VARIANTS="nowmerge" tools/step_variants.sh g711 3 || exit 1
SRTP_FORCE_DIST=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port 29555 bench.py --config gcm256 --steps 5 --warmup 2 \
    --no-cpu-baseline --traffic off > gpurun_out/s16_rccl1.json 2> gpurun_out/s16_rccl1.err || { tail -5 gpurun_out/s16_rccl1.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s16_rccl1.json').read().strip().splitlines()[-1]); print('rccl1', round(d['value']/1e6,1), d['session_replication'], d['prepass'])"
