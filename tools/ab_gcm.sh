# A/B of the order-free AES-GCM forms on the many-stream template shape
# (bench.py --config g711gcm --template): SRTP_PP_FUSED_OF=1 the fused k_gcm
# (classification in the kernel), 0 the pre-pass form
set -o pipefail
o=gpurun_out/ab_gcm; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_prepass.py > $o/tests.log 2>&1 || exit 1
for op in protect unprotect; do
 for f in 1 0; do
  SRTP_PP_FUSED_OF=$f timeout -k 10 240 python bench.py --config g711gcm --template --op $op --steps 5 --warmup 2 --no-cpu-baseline --traffic off > $o/t_${op}_f$f.json 2> $o/t_${op}_f$f.err || exit 1
 done
done
