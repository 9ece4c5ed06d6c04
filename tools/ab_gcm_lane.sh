# per-lane AES-GCM with each lane's 4-bit GHASH table in LDS: GCM tests,
# then many-key shapes with 1, 4 and 128 packets a stream (buckets off)
set -o pipefail
o=gpurun_out/gcm_lane; mkdir -p $o
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "gcm or GCM" > $o/tests.log 2>&1 || exit 1
for p in 65536 262144; do
  timeout -k 10 300 python bench.py --config g711gcm --packets $p --steps 20 --no-cpu-baseline > $o/gcm_$p.json 2> $o/gcm_$p.err || exit 1
done
SRTP_PP_BUCKETS=0 timeout -k 10 300 python bench.py --config g711gcm --steps 5 --no-cpu-baseline > $o/gcm_lane_8m.json 2> $o/gcm_lane_8m.err || exit 1
timeout -k 10 300 python bench.py --config g711gcm --steps 10 --no-cpu-baseline --traffic off > $o/gcm_bk_8m.json 2> $o/gcm_bk_8m.err || exit 1
