# per-call path: tests, then the per-call bench (both ciphers) and a
# phase-stamped run of k_one
set -o pipefail
o=gpurun_out/percall; mkdir -p $o
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_percall.py > $o/tests.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --percall --percall-calls 20000 > $o/percall.json 2> $o/percall.err || exit 1
SRTP_ONE_PROFILE=1 timeout -k 10 60 tools/percall_bench 12 icm > $o/icm_prof.txt 2>&1 || exit 1
SRTP_ONE_PROFILE=1 timeout -k 10 60 tools/percall_bench 12 gcm > $o/gcm_prof.txt 2>&1 || exit 1
