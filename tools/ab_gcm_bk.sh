# many-key AES-GCM (bench --config g711gcm): the per-lane fused form against
# key buckets (SRTP_PP_BUCKETS=1: classify, bucket pass, k_gcm_bk)
set -o pipefail
o=gpurun_out/ab_gcm_bk; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_prepass.py -k "configs3 or bucket" > $o/tests.log 2>&1 || exit 1
for op in protect unprotect; do
  timeout -k 10 300 python bench.py --config g711gcm --op $op --steps 5 --warmup 2 --no-cpu-baseline --traffic off > $o/lane_$op.json 2> $o/lane_$op.err || exit 1
  SRTP_PP_BUCKETS=1 timeout -k 10 300 python bench.py --config g711gcm --op $op --steps 5 --warmup 2 --no-cpu-baseline > $o/bk_$op.json 2> $o/bk_$op.err || exit 1
done
