# per-lane AES-GCM workgroup size A/B: the tree (256 lanes) against
# exp_build/l384 (384 lanes, 160 KiB of LDS): GCM-256 tests on the variant,
# then one / 128 packets a stream (buckets off), twice each
set -o pipefail
o=gpurun_out/gcm_lanes; mkdir -p $o
LIBSRTP_MI355X_LIB=$PWD/exp_build/l384/libsrtp_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu -k "gcm256" > $o/tests_l384.log 2>&1 || exit 1
for rep in 1 2; do
 for v in tree l384; do
  so=$PWD/libsrtp_amd/libsrtp_mi355x.so; [ $v = tree ] || so=$PWD/exp_build/$v/libsrtp_mi355x.so
  LIBSRTP_MI355X_LIB=$so timeout -k 10 300 python bench.py --config g711gcm --packets 65536 --steps 20 --no-cpu-baseline --traffic off > $o/p1_${v}_$rep.json 2>/dev/null || exit 1
  LIBSRTP_MI355X_LIB=$so SRTP_PP_BUCKETS=0 timeout -k 10 300 python bench.py --config g711gcm --steps 5 --no-cpu-baseline --traffic off > $o/p128_${v}_$rep.json 2>/dev/null || exit 1
 done
done
