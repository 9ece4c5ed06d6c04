#!/bin/bash
# round-4 GPU session 9: profiles of the round-4 build -- configs[3] and
# configs[1] protect kernel traces + SQ counter passes, and the configs[3]
# bench line with PMC traffic and the CPU baseline
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tools/prof_kernels.sh gpurun_out/s9_g711 --config g711 --steps 3 --warmup 1 --no-cpu-baseline --traffic off || exit 1
tools/prof_kernels.sh gpurun_out/s9_icm128 --steps 3 --warmup 1 --no-cpu-baseline --traffic off || exit 1
timeout -k 10 400 python3 bench.py --config g711 --steps 10 --warmup 3 > gpurun_out/s9_bench_g711.json 2> gpurun_out/s9_bench_g711.err || { tail -5 gpurun_out/s9_bench_g711.err; exit 1; }
tail -c 600 gpurun_out/s9_bench_g711.json
