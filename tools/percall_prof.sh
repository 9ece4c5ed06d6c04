# k_one phase stamps (SRTP_ONE_PROFILE=1) for both ciphers
set -o pipefail
o=gpurun_out/percall_prof; mkdir -p $o
SRTP_ONE_PROFILE=1 timeout -k 10 60 tools/percall_bench 12 icm > $o/icm_prof.txt 2>&1 || exit 1
SRTP_ONE_PROFILE=1 timeout -k 10 60 tools/percall_bench 12 gcm > $o/gcm_prof.txt 2>&1 || exit 1
